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

// ------------------------------------------ data-parallel glue (one rank) ---
// Global column log-sum-exp from the ranks' gathered (max, sum exp(x - max))
// column partials, rank w's [2][n_c] at parts + w * ld (the contrastive CE's
// one exchange; ld > 2 n_c when it rides in a merged exchange buffer): one
// thread per column, the ranks combined in rank order
__global__ __launch_bounds__(256) void col_lse_combine_kernel(const float* __restrict__ parts,
                                                              int world, long long ld, int n_c,
                                                              float* __restrict__ col_lse) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= n_c) return;
  float m = -INFINITY;
  for (int w = 0; w < world; ++w) m = fmaxf(m, parts[(long long)w * ld + c]);
  float s = 0.f;
  for (int w = 0; w < world; ++w) {
    const float* p = parts + (long long)w * ld;
    s += p[n_c + c] * __expf(p[c] - m);
  }
  col_lse[c] = m + __logf(s);
}

// The focal identity losses on the GLOBAL mean cross-entropy (FocalLoss,
// models/losses.py:313-325, on the reference's gathered batch): phase 0 packs
// each head's local NLL sum (rows x its local mean, ws[rows]) into sums[k]
// for the one collective; phase 1 adds the world ranks' sums (rank w's at
// sums + w * ld: an all-gather; world 1: already all-reduced), turns the
// total into logp = sum / n_global, writes it back into ws[rows] (the
// backward's factor) and forms loss_k = (1 - exp(-logp))^gamma logp.  One
// thread per head.
struct FocalHeads {
  float* ws[2];
  float* loss[2];
};
__global__ void focal_global_kernel(int phase, float* __restrict__ sums, int world, long long ld,
                                    int n_heads, int rows, float inv_n, float gamma,
                                    FocalHeads H) {
  const int k = threadIdx.x;
  if (k >= n_heads) return;
  if (phase == 0) {
    sums[k] = H.ws[k][rows] * (float)rows;
    return;
  }
  float tot = 0.f;
  for (int w = 0; w < world; ++w) tot += sums[(long long)w * ld + k];
  const float logp = tot * inv_n;
  H.ws[k][rows] = logp;
  H.loss[k][0] = powf(1.f - __expf(-logp), gamma) * logp;
}

// ------------------------------------- sent_loss + global_loss, one rank ---
// The two contrastive losses of the stage-1 step on the same pair of feature
// sets (sent_loss, models/losses.py:19-57, and global_loss, :329-351: both
// are cos(img_b, sent_i) / max(|img||sent|, eps) logits, the first scaled by
// gamma3 with the same-class mask, the second by temp3 without) when one
// process holds the whole batch (n <= 64): one workgroup forms the n x n
// cosines (split-bf16 MFMA, ~fp32 products; fp32 norms), both logit sets,
// their row / column log-sum-exps and the four cross-entropies; the
// backward is one launch of n row workgroups (softmax gradients of both
// losses folded into one dcos, then the cosine backward to img).
constexpr int SG_N = 64;
constexpr int SGD_MAXR = 2 * SG_N;     // rows per rank of the dist kernels (row tiles of 64)

// 8 fp32 -> bf16x8 hi and lo = bf16(x - hi) by packed conversions
__device__ __forceinline__ void split8(const float4& a, const float4& b, bf16x8& hi, bf16x8& lo) {
  const float v[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
  uint32_t h[4], l[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    h[k] = pk_bf16(v[2 * k], v[2 * k + 1]);
    l[k] = pk_bf16(v[2 * k] - __uint_as_float(h[k] << 16),
                   v[2 * k + 1] - __uint_as_float(h[k] & 0xffff0000u));
  }
  hi = as_bf8(make_uint4(h[0], h[1], h[2], h[3]));
  lo = as_bf8(make_uint4(l[0], l[1], l[2], l[3]));
}

constexpr int SG_LD = D + 4;                 // padded fp32 LDS rows (bank spread)
constexpr int SG_LDS = 2 * SG_N * SG_LD * 4 + SG_N * (SG_N + 1) * 4;
constexpr int SG_T = 1024;                   // 16 waves

// The cosine tile of up to 64 x rows against up to 64 y rows into LDS
// cs[r][c] (pitch SG_N + 1), and the squared norms into nxp / nyp [4][64]
// (k-quarter partials).  1024 threads = 16 waves: staging 4 float4 loads per
// thread and matrix; wave w computes 32 x 32 tile w & 3 over k quarter w >> 2
// on split-bf16 MFMAs (~fp32 products), the quarters summed through LDS.
// Rows past n_x / n_y repeat the last row (their results are never read).
__device__ __forceinline__ void sg_cos_tile(const float* __restrict__ x, long long ldx, int n_x,
                                            const float* __restrict__ y, long long ldy, int n_y,
                                            float eps, float* cs, float (*nxp)[SG_N],
                                            float (*nyp)[SG_N], float* gcos = nullptr) {
  // LDS: x rows | y rows (fp32, padded) | cos [64][65]; the MFMA partials
  // reuse the row area once the products are done
  float* xs = (float*)g_smem;
  float* ys = xs + SG_N * SG_LD;
  float* part = xs;                            // [16 waves][16][64]
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, lr = lane & 31, h = lane >> 5;
  {
    constexpr int NQ = SG_N * D / 4 / SG_T;    // 4 float4 per thread per matrix
    const uint32_t yoff = SG_N * SG_LD * 4;
    uint4 vx[NQ], vy[NQ];
#pragma unroll
    for (int u = 0; u < NQ; ++u) {
      const int i = u * SG_T + tid, k = i % (D / 4);
      vx[u] = *(const uint4*)(x + min(i / (D / 4), n_x - 1) * ldx + 4 * k);
      vy[u] = *(const uint4*)(y + min(i / (D / 4), n_y - 1) * ldy + 4 * k);
    }
#pragma unroll
    for (int u = 0; u < NQ; ++u) {
      const int i = u * SG_T + tid, r = i / (D / 4), k = i % (D / 4);
      const uint32_t o = (uint32_t)(r * SG_LD + 4 * k) * 4;
      lds_st16(o, vx[u]);
      lds_st16(yoff + o, vy[u]);
    }
  }
  __syncthreads();
  const int t = w & 3, kq = w >> 2, rt = t >> 1, ct = t & 1;
  const int ra = 32 * rt + lr, rb = 32 * ct + lr;
  f32x16 acc;
#pragma unroll
  for (int q = 0; q < 16; ++q) acc[q] = 0.f;
  float sx = 0.f, sy = 0.f;
#pragma unroll
  for (int s = 4 * kq; s < 4 * kq + 4; ++s) {
    const int k0 = 16 * s + 8 * h;
    const float4 a0 = *(const float4*)(xs + ra * SG_LD + k0);
    const float4 a1 = *(const float4*)(xs + ra * SG_LD + k0 + 4);
    const float4 b0 = *(const float4*)(ys + rb * SG_LD + k0);
    const float4 b1 = *(const float4*)(ys + rb * SG_LD + k0 + 4);
    sx = fmaf(a0.x, a0.x, fmaf(a0.y, a0.y, fmaf(a0.z, a0.z, fmaf(a0.w, a0.w, sx))));
    sx = fmaf(a1.x, a1.x, fmaf(a1.y, a1.y, fmaf(a1.z, a1.z, fmaf(a1.w, a1.w, sx))));
    sy = fmaf(b0.x, b0.x, fmaf(b0.y, b0.y, fmaf(b0.z, b0.z, fmaf(b0.w, b0.w, sy))));
    sy = fmaf(b1.x, b1.x, fmaf(b1.y, b1.y, fmaf(b1.z, b1.z, fmaf(b1.w, b1.w, sy))));
    bf16x8 ah, al, bh, bl;
    split8(a0, a1, ah, al);
    split8(b0, b1, bh, bl);
    mma<MODE_SPLIT>(acc, ah, al, bh, bl);
  }
  sx += __shfl_xor(sx, 32);
  sy += __shfl_xor(sy, 32);
  if (h == 0 && ct == 0) nxp[kq][ra] = sx;
  if (h == 0 && rt == 0) nyp[kq][rb] = sy;
  __syncthreads();                             // the row area is free now
#pragma unroll
  for (int q = 0; q < 16; ++q) part[(w * 16 + q) * 64 + lane] = acc[q];
  __syncthreads();
  // cos[r][c] = sum of the 4 quarter partials / max(|x_r||y_c|, eps)
  for (int e = tid; e < SG_N * SG_N; e += SG_T) {
    const int r = e >> 6, c = e & 63;
    if (r >= n_x || c >= n_y) continue;
    const int tt = (r >> 5) * 2 + (c >> 5), rr = r & 31;
    const int hh = (rr >> 2) & 1, q = (rr & 3) | ((rr >> 3) << 2), ln = (c & 31) + 32 * hh;
    float v = 0.f;
#pragma unroll
    for (int k4 = 0; k4 < 4; ++k4) v += part[((tt + 4 * k4) * 16 + q) * 64 + ln];
    const float nx = nxp[0][r] + nxp[1][r] + nxp[2][r] + nxp[3][r];
    const float ny = nyp[0][c] + nyp[1][c] + nyp[2][c] + nyp[3][c];
    const float cv = v / fmaxf(sqrtf(nx) * sqrtf(ny), eps);
    cs[r * (SG_N + 1) + c] = cv;
    if (gcos) gcos[r * n_y + c] = cv;          // dense [n_x][n_y] copy (nullable)
  }
  __syncthreads();
}

__global__ __launch_bounds__(SG_T) void sg_fwd_kernel(
    const float* __restrict__ x, long long ldx, const float* __restrict__ y, long long ldy, int n,
    const long long* __restrict__ cls, float s_sent, float s_glob, float eps,
    float* __restrict__ cosv, float* __restrict__ stats, float* __restrict__ nrm,
    float* __restrict__ loss) {
  float* cs = (float*)g_smem + 2 * SG_N * SG_LD;
  __shared__ float nxp[4][SG_N], nyp[4][SG_N];
  __shared__ long long cl[SG_N];
  __shared__ float red[4 * 16];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  if (tid < n) cl[tid] = cls[tid];
  sg_cos_tile(x, ldx, n, y, ldy, n, eps, cs, nxp, nyp, cosv);
  // logit sets ls = 0..3 (sent rows, sent columns, global rows, global
  // columns) in turn; row / column j = 4 w + lane / 16 of the set, 16 lanes
  // (one DPP row) per row, each taking every 16th element
  const int j = 4 * w + (lane >> 4), sub = lane & 15;
#pragma unroll
  for (int ls = 0; ls < 4; ++ls) {
    const bool glob = ls >= 2, col = ls & 1;
    const float sc = glob ? s_glob : s_sent;
    float L[SG_N / 16];
    float m = -INFINITY;
#pragma unroll
    for (int u = 0; u < SG_N / 16; ++u) {
      const int k = sub + 16 * u;
      const int b = col ? k : j, i = col ? j : k;
      const bool ok = j < n && k < n && (glob || cl[b] != cl[i] || b == i);
      L[u] = ok ? sc * cs[b * (SG_N + 1) + i] : -INFINITY;
      m = fmaxf(m, L[u]);
    }
    m = row16_max(m);
    float sum = 0.f;
#pragma unroll
    for (int u = 0; u < SG_N / 16; ++u) sum += L[u] == -INFINITY ? 0.f : __expf(L[u] - m);
    sum = row16_sum(sum);
    float term = 0.f;
    if (j < n && sub == 0) {
      const float lse = m + __logf(sum);
      stats[ls * n + j] = lse;
      term = lse - sc * cs[j * (SG_N + 1) + j];
    }
    term = wave_sum(term);
    if (lane == 0) red[ls * 16 + w] = term;
  }
  if (tid < n) {
    nrm[tid] = sqrtf(nxp[0][tid] + nxp[1][tid] + nxp[2][tid] + nxp[3][tid]);
    nrm[n + tid] = sqrtf(nyp[0][tid] + nyp[1][tid] + nyp[2][tid] + nyp[3][tid]);
  }
  __syncthreads();
  if (tid == 0) {
    float l4[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      l4[k] = 0.f;
#pragma unroll
      for (int v = 0; v < 16; ++v) l4[k] += red[16 * k + v];
    }
    const float inv = 1.f / (float)n;
    loss[0] = l4[0] * inv;                   // sent loss0 (rows)
    loss[1] = l4[1] * inv;                   // sent loss1 (columns)
    loss[2] = (l4[2] + l4[3]) * inv;         // global loss0 + loss1
  }
}

// grid n (row b of img), 256 threads (thread = feature d)
__global__ __launch_bounds__(256) void sg_bwd_kernel(
    const float* __restrict__ gs0, const float* __restrict__ gs1, const float* __restrict__ ggl,
    const float* __restrict__ x, long long ldx, const float* __restrict__ y, long long ldy, int n,
    const long long* __restrict__ cls, float s_sent, float s_glob, float eps,
    const float* __restrict__ cosv, const float* __restrict__ stats, const float* __restrict__ nrm,
    float* __restrict__ dx, long long lddx) {
  __shared__ float cf[SG_N];
  __shared__ float red[4];
  const int b = blockIdx.x, tid = threadIdx.x;
  const float a0 = gs0 ? *gs0 : 0.f, a1 = gs1 ? *gs1 : 0.f, ag = ggl ? *ggl : 0.f;
  const float inv_n = 1.f / (float)n, nxb = nrm[b];
  float xcoef = 0.f;
  if (tid < n) {
    const int i = tid;
    const float cv = cosv[b * n + i];
    const float dg = i == b ? 1.f : 0.f;
    const bool masked = cls[b] == cls[i] && b != i;
    float dls = 0.f;
    if (!masked) {
      const float L = s_sent * cv;
      dls = a0 * (__expf(L - stats[b]) - dg) + a1 * (__expf(L - stats[n + i]) - dg);
    }
    const float Lg = s_glob * cv;
    const float dlg = ag * ((__expf(Lg - stats[2 * n + b]) - dg) + (__expf(Lg - stats[3 * n + i]) - dg));
    const float dcos = (s_sent * dls + s_glob * dlg) * inv_n;
    const float den = nxb * nrm[n + i];
    if (den >= eps) {
      cf[i] = dcos / den;
      xcoef = -dcos * cv / (nxb * nxb);
    } else {
      cf[i] = dcos / eps;
    }
  }
  xcoef = wave_sum(xcoef);
  if ((tid & 63) == 0) red[tid >> 6] = xcoef;
  __syncthreads();
  xcoef = red[0] + red[1] + red[2] + red[3];
  float acc = xcoef * x[b * ldx + tid];
  for (int i = 0; i < n; ++i) acc = fmaf(cf[i], y[i * ldy + tid], acc);
  dx[b * lddx + tid] = acc;
}

// --------------------------- sent_loss + global_loss, rows x global columns ---
// The same two losses when this rank holds n_r <= 128 images (global rows
// row_offset ..) against n_c all-gathered captions (DataParallel over
// processes, or one process with n > 64): three launches and, with a process
// group, ONE all-gather between the first two.
//   sgd_fwd   grid = 64-column tiles x 64-row tiles: the tile's cosines
//             (sg_cos_tile), per (set, row) the tile's online (max, sum exp)
//             partial and per (set, column) the column's (max, sum exp) over
//             the row tile's rows -- the column partials (one set per row
//             tile) are what the ranks exchange
//   sgd_loss  one workgroup: column LSEs from every rank's partials, row LSEs
//             from the tiles', this rank's four CE contributions (/ N_global)
//   sgd_bwd   one workgroup per row: both losses' softmax gradients folded into
//             one dcos per column, then the cosine backward (as sg_bwd)
// Sets: 0 = sent (gamma3, same-class off-diagonal entries masked), 1 = global
// (temp3).  Layouts: rowpart [2][tiles][n_r][2], colpart [row tiles][2][2][n_c]
// (max, sum), stats = row LSE [2][n_r] then column LSE [2][n_c].
__device__ __forceinline__ void lse_push(float& m, float& sum, float L) {
  if (L > m) {
    sum = sum * __expf(m - L) + 1.f;
    m = L;
  } else {
    sum += __expf(L - m);
  }
}
__device__ __forceinline__ void lse_merge(float& m, float& sum, float m2, float s2) {
  const float mm = fmaxf(m, m2);
  sum = (m == -INFINITY ? 0.f : sum * __expf(m - mm)) + (m2 == -INFINITY ? 0.f : s2 * __expf(m2 - mm));
  m = mm;
}

__global__ __launch_bounds__(SG_T) void sgd_fwd_kernel(
    const float* __restrict__ x, long long ldx, int n_r, const float* __restrict__ y,
    long long ldy, int n_c, const long long* __restrict__ cls, int row_offset, float s_sent,
    float s_glob, float eps, float* __restrict__ cosv, float* __restrict__ rowpart,
    float* __restrict__ colpart, float* __restrict__ nrm) {
  float* cs = (float*)g_smem + 2 * SG_N * SG_LD;
  __shared__ float nxp[4][SG_N], nyp[4][SG_N];
  __shared__ long long clr[SG_N], clc[SG_N];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int tile = blockIdx.x, tiles = gridDim.x, c0 = tile * SG_N;
  const int rt = blockIdx.y, r0 = rt * SG_N;            // this block's row tile
  const int n_y = min(SG_N, n_c - c0), n_x = min(SG_N, n_r - r0);
  if (tid < n_x) clr[tid] = cls[row_offset + r0 + tid];
  if (tid < n_y) clc[tid] = cls[c0 + tid];
  sg_cos_tile(x + (long long)r0 * ldx, ldx, n_x, y + (long long)c0 * ldy, ldy, n_y, eps, cs, nxp,
              nyp);
  for (int e = tid; e < n_x * n_y; e += SG_T)
    cosv[(long long)(r0 + e / n_y) * n_c + c0 + e % n_y] = cs[(e / n_y) * (SG_N + 1) + e % n_y];
  // ls = w >> 2: 0 sent rows, 1 sent columns, 2 global rows, 3 global columns;
  // row / column j = 16 (w & 3) + lane / 4, four lanes each
  const int ls = w >> 2, j = 16 * (w & 3) + (lane >> 2), sub = lane & 3;
  const bool glob = ls >= 2, col = ls & 1;
  const float sc = glob ? s_glob : s_sent;
  const int nj = col ? n_y : n_x, nk = col ? n_x : n_y;
  float m = -INFINITY, sum = 0.f;
  if (j < nj) {
    for (int k = sub; k < nk; k += 4) {
      const int b = col ? k : j, i = col ? j : k;
      if (!glob && clr[b] == clc[i] && row_offset + r0 + b != c0 + i) continue;
      lse_push(m, sum, sc * cs[b * (SG_N + 1) + i]);
    }
  }
#pragma unroll
  for (int msk = 1; msk <= 2; msk <<= 1) lse_merge(m, sum, __shfl_xor(m, msk), __shfl_xor(sum, msk));
  if (j < nj && sub == 0) {
    const int set = glob ? 1 : 0;
    if (col) {
      float* cp = colpart + (long long)rt * 4 * n_c;
      cp[(set * 2 + 0) * n_c + c0 + j] = m;
      cp[(set * 2 + 1) * n_c + c0 + j] = sum;
    } else {
      float* rp = rowpart + (((long long)set * tiles + tile) * n_r + r0 + j) * 2;
      rp[0] = m;
      rp[1] = sum;
    }
  }
  if (tile == 0 && tid < n_x)
    nrm[r0 + tid] = sqrtf(nxp[0][tid] + nxp[1][tid] + nxp[2][tid] + nxp[3][tid]);
  if (rt == 0 && tid < n_y)
    nrm[n_r + c0 + tid] = sqrtf(nyp[0][tid] + nyp[1][tid] + nyp[2][tid] + nyp[3][tid]);
}

__global__ __launch_bounds__(SG_T) void sgd_loss_kernel(
    const float* __restrict__ cosv, int n_r, int n_c, int row_offset, float s_sent, float s_glob,
    int tiles, const float* __restrict__ rowpart, const float* __restrict__ colparts, int world,
    long long ld_parts, float inv_n, float* __restrict__ stats, float* __restrict__ loss) {
  __shared__ float rl[2][SGD_MAXR], cl[2][SGD_MAXR];
  __shared__ float red[SG_T / WAVE];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  float* row_lse = stats;
  float* col_lse = stats + 2 * n_r;
  // column LSEs over every rank's partials (rank r's [row tiles][2 sets][2][n_c]
  // at colparts + r * ld_parts; every rank holds n_r rows, so as many tiles)
  const int rtiles = (n_r + SG_N - 1) / SG_N;
  for (int e = tid; e < 2 * n_c; e += SG_T) {
    const int set = e / n_c, c = e % n_c;
    float m = -INFINITY, sum = 0.f;
    for (int r = 0; r < world; ++r)
      for (int t = 0; t < rtiles; ++t) {
        const float* cp = colparts + (long long)r * ld_parts + ((long long)t * 2 + set) * 2 * n_c;
        lse_merge(m, sum, cp[c], cp[n_c + c]);
      }
    const float lse = m + __logf(sum);
    col_lse[set * n_c + c] = lse;
    const int b = c - row_offset;
    if (b >= 0 && b < n_r) cl[set][b] = lse;
  }
  // row LSEs over the column tiles' partials
  if (tid < 2 * n_r) {
    const int set = tid / n_r, b = tid % n_r;
    float m = -INFINITY, sum = 0.f;
    for (int t = 0; t < tiles; ++t) {
      const float* rp = rowpart + (((long long)set * tiles + t) * n_r + b) * 2;
      lse_merge(m, sum, rp[0], rp[1]);
    }
    const float lse = m + __logf(sum);
    row_lse[set * n_r + b] = lse;
    rl[set][b] = lse;
  }
  __syncthreads();
  // this rank's diagonal terms: waves 0-3 sent rows / sent columns / global
  // rows / global columns of rows 0-63, waves 4-7 the same of rows 64-127
  float term = 0.f;
  const int db = lane + SG_N * (w >> 2);
  if (w < 8 && db < n_r) {
    const int set = (w >> 1) & 1;
    const float d = (set ? s_glob : s_sent) * cosv[(long long)db * n_c + row_offset + db];
    term = ((w & 1) ? cl[set][db] : rl[set][db]) - d;
  }
  term = wave_sum(term);
  if (lane == 0) red[w] = term;
  __syncthreads();
  if (tid == 0) {
    loss[0] = (red[0] + red[4]) * inv_n;                        // sent loss0 (rows)
    loss[1] = (red[1] + red[5]) * inv_n;                        // sent loss1 (columns)
    loss[2] = ((red[2] + red[6]) + (red[3] + red[7])) * inv_n;  // global loss0 + loss1
  }
}

// grid n_r (row b), 256 threads (thread = feature d); dcos of the n_c columns in LDS
__global__ __launch_bounds__(256) void sgd_bwd_kernel(
    const float* __restrict__ gs0, const float* __restrict__ gs1, const float* __restrict__ ggl,
    const float* __restrict__ x, long long ldx, int n_r, const float* __restrict__ y,
    long long ldy, int n_c, const long long* __restrict__ cls, int row_offset, float s_sent,
    float s_glob, float eps, float inv_n, const float* __restrict__ cosv,
    const float* __restrict__ stats, const float* __restrict__ nrm, float* __restrict__ dx,
    long long lddx) {
  extern __shared__ float cf[];                // [n_c]
  __shared__ float red[4];
  const int b = blockIdx.x, tid = threadIdx.x, gb = row_offset + b;
  const float a0 = gs0 ? *gs0 : 0.f, a1 = gs1 ? *gs1 : 0.f, ag = ggl ? *ggl : 0.f;
  const float* row_lse = stats;
  const float* col_lse = stats + 2 * n_r;
  const float nxb = nrm[b], rls = row_lse[b], rlg = row_lse[n_r + b];
  const long long cb = cls[gb];
  float xcoef = 0.f;
  for (int i = tid; i < n_c; i += 256) {
    const float cv = cosv[(long long)b * n_c + i];
    const float dg = i == gb ? 1.f : 0.f;
    float dls = 0.f;
    if (!(cb == cls[i] && i != gb)) {
      const float L = s_sent * cv;
      dls = a0 * (__expf(L - rls) - dg) + a1 * (__expf(L - col_lse[i]) - dg);
    }
    const float Lg = s_glob * cv;
    const float dlg = ag * ((__expf(Lg - rlg) - dg) + (__expf(Lg - col_lse[n_c + i]) - dg));
    const float dcos = (s_sent * dls + s_glob * dlg) * inv_n;
    const float den = nxb * nrm[n_r + i];
    if (den >= eps) {
      cf[i] = dcos / den;
      xcoef -= dcos * cv / (nxb * nxb);
    } else {
      cf[i] = dcos / eps;
    }
  }
  xcoef = wave_sum(xcoef);
  if ((tid & 63) == 0) red[tid >> 6] = xcoef;
  __syncthreads();
  xcoef = red[0] + red[1] + red[2] + red[3];
  float acc = xcoef * x[b * ldx + tid];
  for (int i = 0; i < n_c; ++i) acc = fmaf(cf[i], y[i * ldy + tid], acc);
  dx[b * lddx + tid] = acc;
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

int tgfr_sent_global(const float* x, long long ldx, const float* y, long long ldy, int n,
                     const long long* cls, float s_sent, float s_glob, float eps, float* cosv,
                     float* stats, float* nrm, float* loss, void* stream) {
  if (n <= 0 || n > SG_N || !x || !y || !cls || !cosv || !stats || !nrm || !loss || ldx % 4 ||
      ldy % 4 || ((uintptr_t)x & 15) || ((uintptr_t)y & 15))
    return 1001;
  if (const int e = set_max_lds((const void*)sg_fwd_kernel, SG_LDS)) return e;
  hipLaunchKernelGGL(sg_fwd_kernel, dim3(1), dim3(SG_T), SG_LDS, (hipStream_t)stream, x, ldx, y,
                     ldy, n,
                     cls, s_sent, s_glob, eps, cosv, stats, nrm, loss);
  return (int)hipGetLastError();
}

int tgfr_sent_global_bwd(const float* gs0, const float* gs1, const float* ggl, const float* x,
                         long long ldx, const float* y, long long ldy, int n,
                         const long long* cls, float s_sent, float s_glob, float eps,
                         const float* cosv, const float* stats, const float* nrm, float* dx,
                         long long lddx, void* stream) {
  if (n <= 0 || n > SG_N || !x || !y || !cls || !cosv || !stats || !nrm || !dx) return 1001;
  hipLaunchKernelGGL(sg_bwd_kernel, dim3(n), dim3(256), 0, (hipStream_t)stream, gs0, gs1, ggl, x,
                     ldx, y, ldy, n, cls, s_sent, s_glob, eps, cosv, stats, nrm, dx, lddx);
  return (int)hipGetLastError();
}

int tgfr_sent_global_dist_ws(int n_r, int n_c, long long* rowpart, long long* colpart,
                             long long* stats) {
  if (n_r <= 0 || n_r > SGD_MAXR || n_c <= 0 || n_c > 8192 || !rowpart || !colpart || !stats)
    return 1001;
  *rowpart = 2ll * ((n_c + SG_N - 1) / SG_N) * n_r * 2;
  *colpart = 4ll * n_c * ((n_r + SG_N - 1) / SG_N);
  *stats = 2ll * (n_r + n_c);
  return 0;
}

int tgfr_sent_global_dist_fwd(const float* x, long long ldx, int n_r, const float* y,
                              long long ldy, int n_c, const long long* cls, int row_offset,
                              float s_sent, float s_glob, float eps, float* cosv, float* rowpart,
                              float* colpart, float* nrm, void* stream) {
  if (n_r <= 0 || n_r > SGD_MAXR || n_c <= 0 || n_c > 8192 || row_offset < 0 ||
      row_offset + n_r > n_c || !x || !y || !cls || !cosv || !rowpart || !colpart || !nrm ||
      ldx % 4 || ldy % 4 || ((uintptr_t)x & 15) || ((uintptr_t)y & 15))
    return 1001;
  if (const int e = set_max_lds((const void*)sgd_fwd_kernel, SG_LDS)) return e;
  hipLaunchKernelGGL(sgd_fwd_kernel, dim3((n_c + SG_N - 1) / SG_N, (n_r + SG_N - 1) / SG_N),
                     dim3(SG_T), SG_LDS,
                     (hipStream_t)stream, x, ldx, n_r, y, ldy, n_c, cls, row_offset, s_sent,
                     s_glob, eps, cosv, rowpart, colpart, nrm);
  return (int)hipGetLastError();
}

int tgfr_sent_global_dist_loss(const float* cosv, int n_r, int n_c, int row_offset, float s_sent,
                               float s_glob, const float* rowpart, const float* colparts,
                               int world, long long ld_parts, float inv_n, float* stats,
                               float* loss, void* stream) {
  if (n_r <= 0 || n_r > SGD_MAXR || n_c <= 0 || world <= 0 || !cosv || !rowpart || !colparts ||
      !stats || !loss)
    return 1001;
  const long long cp = 4LL * n_c * ((n_r + SG_N - 1) / SG_N);    // one rank's column partials
  if (ld_parts == 0) ld_parts = cp;
  if (ld_parts < cp) return 1001;
  hipLaunchKernelGGL(sgd_loss_kernel, dim3(1), dim3(SG_T), 0, (hipStream_t)stream, cosv, n_r, n_c,
                     row_offset, s_sent, s_glob, (n_c + SG_N - 1) / SG_N, rowpart, colparts,
                     world, ld_parts, inv_n, stats, loss);
  return (int)hipGetLastError();
}

int tgfr_sent_global_dist_bwd(const float* gs0, const float* gs1, const float* ggl,
                              const float* x, long long ldx, int n_r, const float* y,
                              long long ldy, int n_c, const long long* cls, int row_offset,
                              float s_sent, float s_glob, float eps, float inv_n,
                              const float* cosv, const float* stats, const float* nrm, float* dx,
                              long long lddx, void* stream) {
  if (n_r <= 0 || n_r > SGD_MAXR || n_c <= 0 || n_c > 8192 || !x || !y || !cls || !cosv ||
      !stats || !nrm || !dx)
    return 1001;
  hipLaunchKernelGGL(sgd_bwd_kernel, dim3(n_r), dim3(256), n_c * sizeof(float),
                     (hipStream_t)stream, gs0, gs1, ggl, x, ldx, n_r, y, ldy, n_c, cls,
                     row_offset, s_sent, s_glob, eps, inv_n, cosv, stats, nrm, dx, lddx);
  return (int)hipGetLastError();
}

int tgfr_col_lse_combine(const float* parts, int world, long long ld, int n_c, float* col_lse,
                         void* stream) {
  if (world <= 0 || n_c <= 0 || !parts || !col_lse || (world > 1 && ld < 2LL * n_c)) return 1001;
  hipLaunchKernelGGL(col_lse_combine_kernel, dim3((n_c + 255) / 256), dim3(256), 0,
                     (hipStream_t)stream, parts, world, ld, n_c, col_lse);
  return (int)hipGetLastError();
}

int tgfr_focal_global(int phase, float* sums, int world, long long ld, int n_heads, int rows,
                      float inv_n, float gamma, float* ws0, float* ws1, float* loss0,
                      float* loss1, void* stream) {
  if ((phase != 0 && phase != 1) || !sums || n_heads < 1 || n_heads > 2 || rows <= 0 || !ws0 ||
      (n_heads == 2 && !ws1) || (phase == 1 && (!loss0 || (n_heads == 2 && !loss1))) ||
      world <= 0 || (world > 1 && ld < n_heads))
    return 1001;
  FocalHeads H{{ws0, ws1}, {loss0, loss1}};
  hipLaunchKernelGGL(focal_global_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, phase, sums,
                     world, ld, n_heads, rows, inv_n, gamma, H);
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
