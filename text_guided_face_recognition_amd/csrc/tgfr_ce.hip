// All-pairs cosine logits and the bidirectional contrastive cross-entropy.
//
//   cos_logits   logits[b][i] = scale * x_b.y_i / max(|x_b||y_i|, eps)
//                (sent_loss, models/losses.py:38-43; global_loss :338-343),
//                or scale * x_b.y_i un-normalised (ClipLoss :292-296);
//                optional same-class off-diagonal -inf mask (losses.py:21-30,48).
//   ce_stats     per-row log-sum-exp and per-column (max, sum exp) partials of
//                a [rows x cols] logit block; rows are this rank's images,
//                columns the global caption list, so column partials from all
//                ranks combine into the global column LSE (one tiny exchange).
//                With the column LSE final in-launch (one rank), the last block
//                also forms the losses below (one launch per forward).
//   ce_loss      loss0 = mean_b CE(row b, label b+off) and
//                loss1 = mean_i CE(col i, label i) restricted to this rank's
//                diagonal entries (nn.CrossEntropyLoss, losses.py:52-53,131-132).
//   ce_grad      dlogits = g0/N (softmax_row - onehot) + g1/N (softmax_col - onehot),
//                g0/g1 read from device memory (no host sync).
//   cos_logits_bwd  d x_b from dlogits (the y side is detached in the
//                reference, utils/dataset_utils.py:42, but can be requested).
#include "tgfr_common.h"

using namespace tgfr;

namespace {

constexpr int D = 256;

__global__ __launch_bounds__(256) void cos_logits_kernel(
    const float* __restrict__ x, long long ldx, const float* __restrict__ y, long long ldy,
    int n_x, int n_y, int normalize, float scale, float eps, int masked,
    const long long* __restrict__ cls, int row_offset, float* __restrict__ out, long long ldo) {
  const int b = blockIdx.y;
  const int i = blockIdx.x * 256 + threadIdx.x;
  __shared__ float xs[D];
  xs[threadIdx.x] = x[b * ldx + threadIdx.x];
  __syncthreads();
  if (i >= n_y) return;
  float dot = 0.f, nx = 0.f, ny = 0.f;
  const float* yr = y + i * ldy;
#pragma unroll 8
  for (int d = 0; d < D; d += 4) {
    const float4 v = *(const float4*)(yr + d);
    dot += xs[d] * v.x + xs[d + 1] * v.y + xs[d + 2] * v.z + xs[d + 3] * v.w;
    nx += xs[d] * xs[d] + xs[d + 1] * xs[d + 1] + xs[d + 2] * xs[d + 2] + xs[d + 3] * xs[d + 3];
    ny += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
  }
  float v = normalize ? dot / fmaxf(sqrtf(nx) * sqrtf(ny), eps) * scale : scale * dot;
  if (masked && cls[row_offset + b] == cls[i] && row_offset + b != i) v = -INFINITY;
  out[b * ldo + i] = v;
}

// One block per output row b (x side); g is addressed g[b*gs0 + i*gs1].
__global__ __launch_bounds__(256) void cos_logits_bwd_kernel(
    const float* __restrict__ g, long long gs0, long long gs1, const float* __restrict__ x,
    long long ldx, const float* __restrict__ y, long long ldy, int n_x, int n_y,
    int normalize, float scale, float eps, float* __restrict__ dx, long long lddx) {
  extern __shared__ float sm[];      // coef[n_y]
  __shared__ float xs[D];
  __shared__ float red[8];
  const int b = blockIdx.x, tid = threadIdx.x;
  xs[tid] = x[b * ldx + tid];
  __syncthreads();
  float nx2 = xs[tid] * xs[tid];
  nx2 = wave_sum(nx2);
  if (tid % WAVE == 0) red[tid / WAVE] = nx2;
  __syncthreads();
  const float xn = sqrtf(red[0] + red[1] + red[2] + red[3]);
  // pass 1: per column coefficient of y_i, and the x coefficient
  float xcoef = 0.f;
  for (int i = tid; i < n_y; i += 256) {
    const float* yr = y + i * ldy;
    float dot = 0.f, ny = 0.f;
    for (int d = 0; d < D; d += 4) {
      const float4 v = *(const float4*)(yr + d);
      dot += xs[d] * v.x + xs[d + 1] * v.y + xs[d + 2] * v.z + xs[d + 3] * v.w;
      ny += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
    }
    const float gi = g[b * gs0 + i * gs1] * scale;
    float c = gi;
    if (normalize) {
      const float yn = sqrtf(ny);
      const float den = xn * yn;
      if (den >= eps) {
        c = gi / den;
        xcoef -= gi * dot / (xn * xn * den);
      } else {
        c = gi / eps;
      }
    }
    sm[i] = c;
  }
  xcoef = wave_sum(xcoef);
  __syncthreads();
  if (tid % WAVE == 0) red[4 + tid / WAVE] = xcoef;
  __syncthreads();
  xcoef = red[4] + red[5] + red[6] + red[7];
  // pass 2: thread = feature d
  float acc = xcoef * xs[tid];
  for (int i = 0; i < n_y; ++i) acc += sm[i] * y[i * ldy + tid];
  dx[b * lddx + tid] = acc;
}

// Sums of (row LSE - diagonal logit) and (column LSE - diagonal logit) over
// this rank's rows: loss[0], loss[1] (times inv_n).
__device__ __forceinline__ void ce_loss_block(const float* __restrict__ L, long long ld, int n_r,
                                              int row_offset, float inv_n,
                                              const float* __restrict__ row_lse,
                                              const float* __restrict__ col_lse,
                                              float* __restrict__ loss, float* red) {
  float l0 = 0.f, l1 = 0.f;
  for (int b = threadIdx.x; b < n_r; b += 256) {
    const int c = row_offset + b;
    const float v = L[b * ld + c];
    l0 += row_lse[b] - v;
    l1 += col_lse[c] - v;
  }
  l0 = wave_sum(l0);
  l1 = wave_sum(l1);
  __syncthreads();
  if (threadIdx.x % WAVE == 0) {
    red[threadIdx.x / WAVE] = l0;
    red[4 + threadIdx.x / WAVE] = l1;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    loss[0] = (red[0] + red[1] + red[2] + red[3]) * inv_n;
    loss[1] = (red[4] + red[5] + red[6] + red[7]) * inv_n;
  }
}

// blockIdx.y == 0: rows, == 1: columns; one wave per row / column.  With
// `loss` set (single rank: col_lse is final here) the last block also forms
// the two losses, so the forward is one launch.
__global__ __launch_bounds__(256) void ce_stats_kernel(const float* __restrict__ L, long long ld,
                                                       int n_r, int n_c,
                                                       float* __restrict__ row_lse,
                                                       float* __restrict__ col_max,
                                                       float* __restrict__ col_sum,
                                                       float* __restrict__ col_lse,
                                                       int row_offset, float inv_n,
                                                       float* __restrict__ loss,
                                                       unsigned* __restrict__ counter) {
  __shared__ float red[9];
  const int lane = threadIdx.x % WAVE;
  const int idx = blockIdx.x * 4 + threadIdx.x / WAVE;
  if (blockIdx.y == 0) {
    if (idx < n_r) {
      float m = -INFINITY;
      for (int c = lane; c < n_c; c += WAVE) m = fmaxf(m, L[idx * ld + c]);
      m = wave_max(m);
      float s = 0.f;
      for (int c = lane; c < n_c; c += WAVE) s += __expf(L[idx * ld + c] - m);
      s = wave_sum(s);
      if (lane == 0) row_lse[idx] = m + __logf(s);
    }
  } else if (idx < n_c) {
    float m = -INFINITY;
    for (int r = lane; r < n_r; r += WAVE) m = fmaxf(m, L[r * ld + idx]);
    m = wave_max(m);
    float s = 0.f;
    for (int r = lane; r < n_r; r += WAVE) s += __expf(L[r * ld + idx] - m);
    s = wave_sum(s);
    if (lane == 0) {
      col_max[idx] = m;
      col_sum[idx] = s;
      if (col_lse) col_lse[idx] = m + __logf(s);
    }
  }
  if (!loss) return;
  if (!last_arrival(counter, gridDim.x * gridDim.y, (int*)&red[8])) return;
  ce_loss_block(L, ld, n_r, row_offset, inv_n, row_lse, col_lse, loss, red);
}

__global__ __launch_bounds__(256) void ce_loss_kernel(const float* __restrict__ L, long long ld,
                                                      int n_r, int row_offset, float inv_n,
                                                      const float* __restrict__ row_lse,
                                                      const float* __restrict__ col_lse,
                                                      float* __restrict__ loss) {
  __shared__ float red[8];
  ce_loss_block(L, ld, n_r, row_offset, inv_n, row_lse, col_lse, loss, red);
}

__global__ __launch_bounds__(256) void ce_grad_kernel(const float* __restrict__ L, long long ld,
                                                      int n_r, int n_c, int row_offset,
                                                      float inv_n, const float* __restrict__ row_lse,
                                                      const float* __restrict__ col_lse,
                                                      const float* __restrict__ g0p,
                                                      const float* __restrict__ g1p, float w0,
                                                      float w1, float* __restrict__ dL,
                                                      long long ldd) {
  const long long e = blockIdx.x * 256LL + threadIdx.x;
  if (e >= (long long)n_r * n_c) return;
  const int b = e / n_c, c = e % n_c;
  const float v = L[b * ld + c];
  const float onehot = (c == row_offset + b) ? 1.f : 0.f;
  const float g0 = (g0p ? *g0p : 1.f) * w0 * inv_n;
  const float g1 = (g1p ? *g1p : 1.f) * w1 * inv_n;
  dL[b * ldd + c] = g0 * (__expf(v - row_lse[b]) - onehot) + g1 * (__expf(v - col_lse[c]) - onehot);
}

}  // namespace

extern "C" {

int tgfr_cos_logits(const float* x, long long ldx, const float* y, long long ldy, int n_x,
                    int n_y, int d, int normalize, float scale, float eps, int masked,
                    const long long* cls, int row_offset, float* out, long long ldo,
                    void* stream) {
  if (d != D || n_x <= 0 || n_y <= 0 || (masked && !cls)) return 1001;
  hipLaunchKernelGGL(cos_logits_kernel, dim3((n_y + 255) / 256, n_x), dim3(256), 0,
                     (hipStream_t)stream, x, ldx, y, ldy, n_x, n_y, normalize, scale, eps,
                     masked, cls, row_offset, out, ldo);
  return (int)hipGetLastError();
}

int tgfr_cos_logits_bwd(const float* g, long long gs0, long long gs1, const float* x,
                        long long ldx, const float* y, long long ldy, int n_x, int n_y, int d,
                        int normalize, float scale, float eps, float* dx, long long lddx,
                        void* stream) {
  if (d != D || n_x <= 0 || n_y <= 0 || n_y > 8192) return 1001;
  hipLaunchKernelGGL(cos_logits_bwd_kernel, dim3(n_x), dim3(256), n_y * sizeof(float),
                     (hipStream_t)stream, g, gs0, gs1, x, ldx, y, ldy, n_x, n_y, normalize,
                     scale, eps, dx, lddx);
  return (int)hipGetLastError();
}

int tgfr_ce_stats(const float* L, long long ld, int n_r, int n_c, float* row_lse,
                  float* col_max, float* col_sum, float* col_lse, int row_offset, float inv_n,
                  float* loss, unsigned* counters, void* stream) {
  if (n_r <= 0 || n_c <= 0 || (loss && (!col_lse || !counters))) return 1001;
  const int gx = max((n_r + 3) / 4, (n_c + 3) / 4);
  hipLaunchKernelGGL(ce_stats_kernel, dim3(gx, 2), dim3(256), 0, (hipStream_t)stream, L, ld,
                     n_r, n_c, row_lse, col_max, col_sum, col_lse, row_offset, inv_n, loss,
                     counters);
  return (int)hipGetLastError();
}

int tgfr_ce_loss(const float* L, long long ld, int n_r, int row_offset, float inv_n,
                 const float* row_lse, const float* col_lse, float* loss, void* stream) {
  if (n_r <= 0) return 1001;
  hipLaunchKernelGGL(ce_loss_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, L, ld, n_r,
                     row_offset, inv_n, row_lse, col_lse, loss);
  return (int)hipGetLastError();
}

int tgfr_ce_grad(const float* L, long long ld, int n_r, int n_c, int row_offset, float inv_n,
                 const float* row_lse, const float* col_lse, const float* g0, const float* g1,
                 float w0, float w1, float* dL, long long ldd, void* stream) {
  if (n_r <= 0 || n_c <= 0) return 1001;
  const long long n = (long long)n_r * n_c;
  hipLaunchKernelGGL(ce_grad_kernel, dim3((int)((n + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, L, ld, n_r, n_c, row_offset, inv_n, row_lse, col_lse,
                     g0, g1, w0, w1, dL, ldd);
  return (int)hipGetLastError();
}

}  // extern "C"
