// Fused elementwise/reduction kernels for the heads around the hot path.
//
//   l2norm_rows      y = x / max(|x|, eps) per row       (F.normalize, ProjectionHead
//                    models/models.py:112-120; ArcMargin models/metrics.py:44)
//   l2norm_rows_bwd  dx = (dy - y (y.dy)) / max(|x|, eps)   (|x| > eps; else dy / eps)
//   arc_margin       logits = s * (onehot * phi(cos) + (1 - onehot) * cos) with
//                    phi = cos m - sin m, sin = sqrt(clamp(1 - cos^2, 0, 1)),
//                    phi = where(cos > th, phi, cos - mm)   (models/metrics.py:45-57)
//   arc_margin_bwd   d cos from d logits (the where/clamp branches as torch takes them)
//   focal_ce         logp = mean_b CE(logits_b, y_b); loss = (1 - e^-logp)^gamma logp
//                    (a block per row; the last block takes the row-order mean)
//                    (FocalLoss, models/losses.py:313-325)
//   focal_ce_bwd     dlogits = g * dloss/dlogp * (softmax - onehot) / B
//   loss_mix         out[j] = sum_i W[j][i] * loss_i for the trainer's scalar
//                    losses (one launch instead of a chain of scalar ops);
//   loss_mix_bwd     dloss_i = g * W[0][i]
//   bias_grad        db = column sums of dy (after the ReLU mask y > 0 when given,
//                    writing the masked dy for the weight/input GEMMs): the
//                    nn.Linear / 1x1-conv bias gradient, fixed-order reduction
// Each replaces 10-25 PyTorch launches per call with one.
#include "tgfr_common.h"

using namespace tgfr;

namespace {

// one wave per row
__global__ __launch_bounds__(256) void l2norm_rows_kernel(const float* __restrict__ x, long long ldx,
                                                          int rows, int d, float eps,
                                                          float* __restrict__ y, long long ldy,
                                                          float* __restrict__ inv_norm) {
  const long long row = blockIdx.x * 4LL + threadIdx.x / WAVE;
  const int lane = threadIdx.x % WAVE;
  if (row >= rows) return;
  const float* xr = x + row * ldx;
  float ss = 0.f;
  for (int c = lane; c < d; c += WAVE) ss += xr[c] * xr[c];
  ss = wave_sum(ss);
  const float inv = 1.f / fmaxf(sqrtf(ss), eps);
  float* yr = y + row * ldy;
  for (int c = lane; c < d; c += WAVE) yr[c] = xr[c] * inv;
  if (lane == 0) inv_norm[row] = inv;
}

__global__ __launch_bounds__(256) void l2norm_rows_bwd_kernel(
    const float* __restrict__ dy, long long lddy, const float* __restrict__ y, long long ldy,
    const float* __restrict__ inv_norm, int rows, int d, float eps, float* __restrict__ dx,
    long long lddx) {
  const long long row = blockIdx.x * 4LL + threadIdx.x / WAVE;
  const int lane = threadIdx.x % WAVE;
  if (row >= rows) return;
  const float* g = dy + row * lddy;
  const float* yr = y + row * ldy;
  const float inv = inv_norm[row];
  // clamped rows (|x| <= eps) are y = x / eps: a plain scaling, no projection
  const bool clamped = inv >= 1.f / eps;
  float dot = 0.f;
  for (int c = lane; c < d; c += WAVE) dot += yr[c] * g[c];
  dot = clamped ? 0.f : wave_sum(dot);
  float* o = dx + row * lddx;
  for (int c = lane; c < d; c += WAVE) o[c] = (g[c] - yr[c] * dot) * inv;
}

__global__ __launch_bounds__(256) void arc_margin_kernel(const float* __restrict__ cosv,
                                                         const long long* __restrict__ label,
                                                         int rows, int cols, float s, float cos_m,
                                                         float sin_m, float th, float mm,
                                                         int easy, float* __restrict__ out) {
  const long long e = blockIdx.x * 256LL + threadIdx.x;
  if (e >= (long long)rows * cols) return;
  const int b = e / cols, c = e % cols;
  const float cv = cosv[e];
  float v = cv;
  if (c == label[b]) {
    const float sine = sqrtf(fminf(fmaxf(1.f - cv * cv, 0.f), 1.f));
    const float phi = cv * cos_m - sine * sin_m;
    v = easy ? (cv > 0.f ? phi : cv) : (cv > th ? phi : cv - mm);
  }
  out[e] = v * s;
}

__global__ __launch_bounds__(256) void arc_margin_bwd_kernel(const float* __restrict__ cosv,
                                                             const long long* __restrict__ label,
                                                             const float* __restrict__ dout,
                                                             int rows, int cols, float s,
                                                             float cos_m, float sin_m, float th,
                                                             int easy, float* __restrict__ dcos) {
  const long long e = blockIdx.x * 256LL + threadIdx.x;
  if (e >= (long long)rows * cols) return;
  const int b = e / cols, c = e % cols;
  const float g = dout[e] * s;
  float d = g;
  if (c == label[b]) {
    const float cv = cosv[e];
    const bool use_phi = easy ? cv > 0.f : cv > th;
    if (use_phi) {
      const float one_m = 1.f - cv * cv;
      const float sine = sqrtf(fminf(fmaxf(one_m, 0.f), 1.f));
      // d sine / d cos = -cos / sine inside the clamp range, 0 outside
      const float dsine = (one_m >= 0.f && one_m <= 1.f) ? -cv / sine : 0.f;
      d = g * (cos_m - sin_m * dsine);
    }
  }
  dcos[e] = d;
}

// one block per row: ws[b] = row LSE, ws[rows + 1 + b] = row NLL; the last
// block forms ws[rows] = logp = mean NLL (row order) and the focal loss
// blockIdx.y = 1: a second head (L2, ws2, loss2, the next counter word) on
// the same labels, so the trainer's two identity losses take one launch
__global__ __launch_bounds__(256) void focal_ce_kernel(const float* __restrict__ L, int cols,
                                                       const long long* __restrict__ label,
                                                       int rows, float gamma,
                                                       float* __restrict__ ws,
                                                       unsigned* __restrict__ counter,
                                                       float* __restrict__ loss,
                                                       const float* __restrict__ L2,
                                                       float* __restrict__ ws2,
                                                       float* __restrict__ loss2) {
  __shared__ float red[5];
  if (blockIdx.y) {
    L = L2;
    ws = ws2;
    loss = loss2;
    counter += 1;
  }
  const int b = blockIdx.x, wid = threadIdx.x / WAVE, lane = threadIdx.x % WAVE;
  const float* r = L + (long long)b * cols;
  // one pass, online log-sum-exp: 4 loads in flight per thread per step
  float m = -INFINITY, sum = 0.f;
  for (int c0 = threadIdx.x; c0 < cols; c0 += 4 * 256) {
    float v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = c0 + 256 * u < cols ? r[c0 + 256 * u] : -INFINITY;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (v[u] > m) {
        sum = sum * __expf(m - v[u]) + 1.f;
        m = v[u];
      } else if (v[u] != -INFINITY) {
        sum += __expf(v[u] - m);
      }
    }
  }
  // combine (m, sum) over the wave, then over the 4 waves
#pragma unroll
  for (int k = 32; k >= 1; k >>= 1) {
    const float m2 = __shfl_xor(m, k), s2 = __shfl_xor(sum, k);
    const float mm = fmaxf(m, m2);
    sum = (m == -INFINITY ? 0.f : sum * __expf(m - mm)) +
          (m2 == -INFINITY ? 0.f : s2 * __expf(m2 - mm));
    m = mm;
  }
  __shared__ float rm[4];
  if (lane == 0) {
    rm[wid] = m;
    red[wid] = sum;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const float mm = fmaxf(fmaxf(rm[0], rm[1]), fmaxf(rm[2], rm[3]));
    float tot = 0.f;
#pragma unroll
    for (int k = 0; k < 4; ++k) tot += rm[k] == -INFINITY ? 0.f : red[k] * __expf(rm[k] - mm);
    const float lse = mm + __logf(tot);
    ws[b] = lse;
    ws[rows + 1 + b] = lse - r[label[b]];
  }
  if (!last_arrival(counter, rows, (int*)&red[4])) return;
  float acc = 0.f;
  for (int k = threadIdx.x; k < rows; k += 256) acc += ws[rows + 1 + k];
  acc = wave_sum(acc);
  __syncthreads();
  if (lane == 0) red[wid] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float logp = (red[0] + red[1] + red[2] + red[3]) / rows;
    const float p = __expf(-logp);
    ws[rows] = logp;
    loss[0] = powf(1.f - p, gamma) * logp;
  }
}

__global__ __launch_bounds__(256) void focal_ce_bwd_kernel(const float* __restrict__ L, int rows,
                                                           int cols,
                                                           const long long* __restrict__ label,
                                                           float gamma,
                                                           const float* __restrict__ ws,
                                                           const float* __restrict__ gscale,
                                                           float* __restrict__ dL) {
  const long long e = blockIdx.x * 256LL + threadIdx.x;
  if (e >= (long long)rows * cols) return;
  const int b = e / cols, c = e % cols;
  const float logp = ws[rows];
  const float p = __expf(-logp);
  const float q = 1.f - p;
  // d/dlogp [(1 - e^-logp)^gamma logp] = q^gamma + gamma q^(gamma-1) p logp
  float dfl = powf(q, gamma);
  if (gamma != 0.f) dfl += gamma * powf(q, gamma - 1.f) * p * logp;
  const float g = (gscale ? gscale[0] : 1.f) * dfl / rows;
  const float sm = __expf(L[e] - ws[b]);
  dL[e] = g * (sm - (c == label[b] ? 1.f : 0.f));
}

constexpr int BG_ROWS = 256;   // rows per partial-sum block of bias_grad

// grid (ceil(cols / 64), ceil(rows / BG_ROWS)); block = 64 columns x 4 row
// lanes.  Each block stores its column partials; the last block of a column
// group sums the group's partials in block order.
template <bool RELU>
__global__ __launch_bounds__(256) void bias_grad_kernel(
    const float* __restrict__ dy, long long lddy, int rows, int cols, const float* __restrict__ y,
    long long ldy, float* __restrict__ dym, long long lddm, float* __restrict__ part,
    unsigned* __restrict__ counters, float* __restrict__ db) {
  __shared__ float red[4 * 64 + 1];
  const int tx = threadIdx.x & 63, ry = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + tx;
  const int r0 = blockIdx.y * BG_ROWS, r1 = min(rows, r0 + BG_ROWS);
  float acc = 0.f;
  if (c < cols) {
#pragma unroll 4
    for (int r = r0 + ry; r < r1; r += 4) {
      float v = dy[(long long)r * lddy + c];
      if constexpr (RELU) {
        v = y[(long long)r * ldy + c] > 0.f ? v : 0.f;
        dym[(long long)r * lddm + c] = v;
      }
      acc += v;
    }
  }
  red[ry * 64 + tx] = acc;
  __syncthreads();
  if (ry == 0 && c < cols)
    part[(long long)blockIdx.y * cols + c] = red[tx] + red[64 + tx] + red[128 + tx] + red[192 + tx];
  if (!last_arrival(counters + blockIdx.x, gridDim.y, (int*)&red[256])) return;
  float a = 0.f;
  if (c < cols)
    for (int k = ry; k < (int)gridDim.y; k += 4) a += part[(long long)k * cols + c];
  red[ry * 64 + tx] = a;
  __syncthreads();
  if (ry == 0 && c < cols) db[c] = red[tx] + red[64 + tx] + red[128 + tx] + red[192 + tx];
}

// Vector form (cols, strides % 4 == 0, 16-B aligned rows): grid
// (ceil(cols / 256), ceil(rows / BG4_ROWS)), 16 waves; lane = 4 columns (one
// float4), wave w = rows w, w + 16, ... of the block's BG4_ROWS.  Every load
// is unconditional (clamped row / column, value masked afterwards) so all of
// a lane's loads are in flight before the first add.  Block partials are
// stored write-through (agent-scope relaxed stores), so the arrival needs no
// release fence; the last block of a column group sums the group's partials
// in block order with agent-scope loads.
constexpr int BG4_WAVES = 16, BG4_ROWS = 128, BG4_PER_WAVE = BG4_ROWS / BG4_WAVES;

__device__ __forceinline__ void st_agent(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_agent(const float* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void add4(float4& a, const float4& b) {
  a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
}

template <bool RELU>
__global__ __launch_bounds__(64 * BG4_WAVES) void bias_grad4_kernel(
    const float* __restrict__ dy, long long lddy, int rows, int cols, const float* __restrict__ y,
    long long ldy, float* __restrict__ dym, long long lddm, float* __restrict__ part,
    unsigned* __restrict__ counters, float* __restrict__ db) {
  __shared__ float4 red[BG4_WAVES * 64];
  __shared__ int last;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = blockIdx.x * 256 + 4 * lane;
  const bool on = c < cols;
  const int cc = on ? c : 0;
  const int r0 = blockIdx.y * BG4_ROWS + w;
  float4 v[BG4_PER_WAVE], m[BG4_PER_WAVE];
  // 32-bit element offsets (the host checks they fit): SGPR base + VGPR
  // offset addressing, two VGPRs fewer per load
#pragma unroll
  for (int i = 0; i < BG4_PER_WAVE; ++i) {
    const unsigned r = (unsigned)min(r0 + BG4_WAVES * i, rows - 1);
    v[i] = *(const float4*)(dy + (r * (unsigned)lddy + (unsigned)cc));
    if constexpr (RELU) m[i] = *(const float4*)(y + (r * (unsigned)ldy + (unsigned)cc));
  }
  float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int i = 0; i < BG4_PER_WAVE; ++i) {
    const int r = r0 + BG4_WAVES * i;
    const bool ok = on && r < rows;
    if constexpr (RELU) {
      v[i].x = m[i].x > 0.f ? v[i].x : 0.f;
      v[i].y = m[i].y > 0.f ? v[i].y : 0.f;
      v[i].z = m[i].z > 0.f ? v[i].z : 0.f;
      v[i].w = m[i].w > 0.f ? v[i].w : 0.f;
      if (ok) *(float4*)(dym + (long long)r * lddm + c) = v[i];
    }
    if (ok) add4(a, v[i]);
  }
  red[w * 64 + lane] = a;
  __syncthreads();
  if (w == 0 && on) {
    float4 t = red[lane];
#pragma unroll
    for (int k = 1; k < BG4_WAVES; ++k) add4(t, red[k * 64 + lane]);
    float* o = part + (long long)blockIdx.y * cols + c;
    st_agent(o, t.x); st_agent(o + 1, t.y); st_agent(o + 2, t.z); st_agent(o + 3, t.w);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned n = __hip_atomic_fetch_add(counters + blockIdx.x, 1u, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT);
    last = n == gridDim.y - 1;
    if (last)
      __hip_atomic_store(counters + blockIdx.x, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  if (!last) return;
  // the column group's partials: wave w sums blocks w, w + 16, ... (in order)
  const int nb = gridDim.y;
  float4 s4 = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int k0 = w; k0 < nb; k0 += BG4_WAVES * 8) {
    float4 t[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float* q = part + (long long)min(k0 + BG4_WAVES * j, nb - 1) * cols + cc;
      t[j] = make_float4(ld_agent(q), ld_agent(q + 1), ld_agent(q + 2), ld_agent(q + 3));
    }
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (k0 + BG4_WAVES * j < nb) add4(s4, t[j]);
  }
  red[w * 64 + lane] = s4;
  __syncthreads();
  if (w == 0 && on) {
    float4 t = red[lane];
#pragma unroll
    for (int k = 1; k < BG4_WAVES; ++k) add4(t, red[k * 64 + lane]);
    *(float4*)(db + c) = t;
  }
}

constexpr int MIX_N = 16, MIX_M = 4;
struct MixArgs {
  const float* loss[MIX_N];
  float w[MIX_M][MIX_N];
};

__global__ void loss_mix_kernel(MixArgs a, int n, int m, float* __restrict__ out) {
  const int j = threadIdx.x;
  if (j >= m) return;
  float acc = 0.f;
  for (int i = 0; i < n; ++i) acc += a.w[j][i] * *a.loss[i];
  out[j] = acc;
}

__global__ void loss_mix_bwd_kernel(const float* __restrict__ g, MixArgs a, int n,
                                    float* __restrict__ dloss) {
  const int i = threadIdx.x;
  if (i < n) dloss[i] = g[0] * a.w[0][i];
}

// Verification score of a matched pair (utils/modules.py:152-153,
// nn.CosineSimilarity(dim=1, eps)): x.y / max(|x| |y|, eps), one wave per row.
__global__ __launch_bounds__(256) void pair_cosine_kernel(const float* __restrict__ x,
                                                          long long ldx,
                                                          const float* __restrict__ y,
                                                          long long ldy, int rows, int d,
                                                          float eps, float* __restrict__ out) {
  const long long row = blockIdx.x * 4LL + threadIdx.x / WAVE;
  const int lane = threadIdx.x % WAVE;
  if (row >= rows) return;
  const float* a = x + row * ldx;
  const float* b = y + row * ldy;
  float xy = 0.f, xx = 0.f, yy = 0.f;
  for (int c = lane; c < d; c += WAVE) {
    const float u = a[c], v = b[c];
    xy = fmaf(u, v, xy);
    xx = fmaf(u, u, xx);
    yy = fmaf(v, v, yy);
  }
  xy = wave_sum(xy);
  xx = wave_sum(xx);
  yy = wave_sum(yy);
  if (lane == 0) out[row] = xy / fmaxf(sqrtf(xx * yy), eps);
}

}  // namespace

extern "C" {

int tgfr_l2norm_rows(const float* x, long long ldx, int rows, int d, float eps, float* y,
                     long long ldy, float* inv_norm, void* stream) {
  if (rows <= 0 || d <= 0) return 1001;
  hipLaunchKernelGGL(l2norm_rows_kernel, dim3((rows + 3) / 4), dim3(256), 0,
                     (hipStream_t)stream, x, ldx, rows, d, eps, y, ldy, inv_norm);
  return (int)hipGetLastError();
}

int tgfr_pair_cosine(const float* x, long long ldx, const float* y, long long ldy, int rows,
                     int d, float eps, float* out, void* stream) {
  if (rows <= 0 || d <= 0 || !x || !y || !out) return 1001;
  hipLaunchKernelGGL(pair_cosine_kernel, dim3((rows + 3) / 4), dim3(256), 0, (hipStream_t)stream,
                     x, ldx, y, ldy, rows, d, eps, out);
  return (int)hipGetLastError();
}

int tgfr_l2norm_rows_bwd(const float* dy, long long lddy, const float* y, long long ldy,
                         const float* inv_norm, int rows, int d, float eps, float* dx,
                         long long lddx, void* stream) {
  if (rows <= 0 || d <= 0) return 1001;
  hipLaunchKernelGGL(l2norm_rows_bwd_kernel, dim3((rows + 3) / 4), dim3(256), 0,
                     (hipStream_t)stream, dy, lddy, y, ldy, inv_norm, rows, d, eps, dx, lddx);
  return (int)hipGetLastError();
}

int tgfr_arc_margin(const float* cosv, const long long* label, int rows, int cols, float s,
                    float m, int easy, float* out, void* stream) {
  if (rows <= 0 || cols <= 0) return 1001;
  const long long n = (long long)rows * cols;
  const float PI = 3.14159265358979323846f;
  hipLaunchKernelGGL(arc_margin_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, cosv, label, rows, cols, s, cosf(m), sinf(m),
                     cosf(PI - m), sinf(PI - m) * m, easy, out);
  return (int)hipGetLastError();
}

int tgfr_arc_margin_bwd(const float* cosv, const long long* label, const float* dout, int rows,
                        int cols, float s, float m, int easy, float* dcos, void* stream) {
  if (rows <= 0 || cols <= 0) return 1001;
  const long long n = (long long)rows * cols;
  const float PI = 3.14159265358979323846f;
  hipLaunchKernelGGL(arc_margin_bwd_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, cosv, label, dout, rows, cols, s, cosf(m), sinf(m),
                     cosf(PI - m), easy, dcos);
  return (int)hipGetLastError();
}

int tgfr_focal_ce(const float* L, int rows, int cols, const long long* label, float gamma,
                  float* ws, unsigned* counters, float* loss, void* stream) {
  if (rows <= 0 || cols <= 0 || !counters) return 1001;
  hipLaunchKernelGGL(focal_ce_kernel, dim3(rows), dim3(256), 0, (hipStream_t)stream, L, cols,
                     label, rows, gamma, ws, counters, loss, nullptr, nullptr, nullptr);
  return (int)hipGetLastError();
}

int tgfr_focal_ce2(const float* L, const float* L2, int rows, int cols, const long long* label,
                   float gamma, float* ws, float* ws2, unsigned* counters, float* loss,
                   float* loss2, void* stream) {
  if (rows <= 0 || cols <= 0 || !counters || !L2 || !ws2 || !loss2) return 1001;
  hipLaunchKernelGGL(focal_ce_kernel, dim3(rows, 2), dim3(256), 0, (hipStream_t)stream, L, cols,
                     label, rows, gamma, ws, counters, loss, L2, ws2, loss2);
  return (int)hipGetLastError();
}

int tgfr_focal_ce_bwd(const float* L, int rows, int cols, const long long* label, float gamma,
                      const float* ws, const float* gscale, float* dL, void* stream) {
  if (rows <= 0 || cols <= 0) return 1001;
  const long long n = (long long)rows * cols;
  hipLaunchKernelGGL(focal_ce_bwd_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, L, rows, cols, label, gamma, ws, gscale, dL);
  return (int)hipGetLastError();
}

// ws: ceil(rows / 128) * cols floats; counters: ceil(cols / 64) zeroed words.
// y (ReLU output) and dym are both set or both NULL.
int tgfr_bias_grad(const float* dy, long long lddy, int rows, int cols, const float* y,
                   long long ldy, float* dym, long long lddm, float* db, float* ws,
                   unsigned* counters, void* stream) {
  if (rows <= 0 || cols <= 0 || (!y) != (!dym) || !counters) return 1001;
  auto* st = (hipStream_t)stream;
  auto a16 = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
  const long long span = (long long)rows * (lddy > ldy ? lddy : ldy);
  const bool vec = cols % 4 == 0 && lddy % 4 == 0 && a16(dy) && a16(db) && span < (1LL << 31) &&
                   (!y || (ldy % 4 == 0 && lddm % 4 == 0 && a16(y) && a16(dym)));
  if (vec) {
    const dim3 g4((cols + 255) / 256, (rows + BG4_ROWS - 1) / BG4_ROWS);
    if (y)
      hipLaunchKernelGGL(bias_grad4_kernel<true>, g4, dim3(64 * BG4_WAVES), 0, st, dy, lddy, rows, cols, y,
                         ldy, dym, lddm, ws, counters, db);
    else
      hipLaunchKernelGGL(bias_grad4_kernel<false>, g4, dim3(64 * BG4_WAVES), 0, st, dy, lddy, rows, cols,
                         y, ldy, dym, lddm, ws, counters, db);
    return (int)hipGetLastError();
  }
  const dim3 grid((cols + 63) / 64, (rows + BG_ROWS - 1) / BG_ROWS);
  if (y)
    hipLaunchKernelGGL(bias_grad_kernel<true>, grid, dim3(256), 0, st, dy, lddy, rows, cols, y,
                       ldy, dym, lddm, ws, counters, db);
  else
    hipLaunchKernelGGL(bias_grad_kernel<false>, grid, dim3(256), 0, st, dy, lddy, rows, cols, y,
                       ldy, dym, lddm, ws, counters, db);
  return (int)hipGetLastError();
}

// losses: host array of n device pointers (n <= 16); W: host [m][n] row-major
// (m <= 4).  out[j] = sum_i W[j][i] * *losses[i].
int tgfr_loss_mix(int n, const float* const* losses, int m, const float* W, float* out,
                  void* stream) {
  if (n <= 0 || n > MIX_N || m <= 0 || m > MIX_M || !losses || !W) return 1001;
  MixArgs a = {};
  for (int i = 0; i < n; ++i) {
    a.loss[i] = losses[i];
    for (int j = 0; j < m; ++j) a.w[j][i] = W[j * n + i];
  }
  hipLaunchKernelGGL(loss_mix_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, a, n, m, out);
  return (int)hipGetLastError();
}

// dloss[i] = g[0] * W[0][i] (W as for tgfr_loss_mix; only row 0 is read).
int tgfr_loss_mix_bwd(const float* g, int n, const float* W, float* dloss, void* stream) {
  if (n <= 0 || n > MIX_N || !W) return 1001;
  MixArgs a = {};
  for (int i = 0; i < n; ++i) a.w[0][i] = W[i];
  hipLaunchKernelGGL(loss_mix_bwd_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, g, a, n,
                     dloss);
  return (int)hipGetLastError();
}

}  // extern "C"
