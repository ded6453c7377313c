// Per-sample LayerNorm of the IMIM head (models/models.py:388, :401:
// nn.LayerNorm([256, 14, 14]) over all C*H*W elements of each sample, with an
// elementwise affine map of the same shape).
//
// PyTorch launches one block per sample (64 blocks on a 256-CU part, ~100 us
// for the backward).  Here every sample is cut into S slices so the launch has
// >= ~1024 blocks:
//   ln_part     per (sample, slice): count-free (mean_i, M2_i) of the slice
//   ln_apply    combine the S slice moments (Chan, fixed order) -> mean, rstd;
//               y = (x - mean) rstd w + b; block (b, 0) stores mean/rstd
//   ln_bwd_part per (sample, slice): sums of g = dy w and g xhat
//   ln_bwd_dx   dx = rstd (g - mean(g) - xhat mean(g xhat)); per element e the
//               block also sums dy xhat and dy over its group of samples
//   ln_bwd_dw   dw[e] = sum of the group partials, db likewise (fixed order)
// Every reduction has a fixed order, so results are run-to-run identical.
#include "tgfr_common.h"

using namespace tgfr;

namespace {

constexpr int NT = 256;

__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int wid = threadIdx.x / WAVE;
  __syncthreads();
  if (threadIdx.x % WAVE == 0) red[wid] = v;
  __syncthreads();
  return red[0] + red[1] + red[2] + red[3];
}

// The affine map w, b is indexed like x's rows ([E]) or, with ch > 0, stored
// channel-major [ch][E / ch] while x's rows are [E / ch][ch] (IMIM's
// LayerNorm([C, H, W]) on channels-last rows: no permuted copies of w, b).
__device__ __forceinline__ long long aidx(long long e, int ch, long long E) {
  return ch ? (e % ch) * (E / ch) + e / ch : e;
}
// 4 consecutive elements 4 i4 .. +3 (ch % 4 == 0 keeps them in one position)
__device__ __forceinline__ float4 aff4(const float* __restrict__ a, long long i4, int ch,
                                       long long E) {
  if (!ch) return ((const float4*)a)[i4];
  const long long e = i4 * 4, n = E / ch, c = e % ch, p = e / ch;
  return make_float4(a[c * n + p], a[(c + 1) * n + p], a[(c + 2) * n + p], a[(c + 3) * n + p]);
}

struct Slice {
  long long lo, hi;
};
__device__ __forceinline__ Slice slice_of(long long E, int S, int s) {
  const long long len = ((E + S - 1) / S + 3) / 4 * 4;
  const long long lo = min(E, s * len);
  return {lo, min(E, lo + len)};
}

// ws layout: part [rows][S][2] | mean [rows] | rstd [rows]
__global__ __launch_bounds__(NT) void ln_part_kernel(const float* __restrict__ x, long long E,
                                                     int S, float* __restrict__ part) {
  __shared__ float red[4];
  const int b = blockIdx.y, s = blockIdx.x;
  const Slice sl = slice_of(E, S, s);
  const float* xr = x + (long long)b * E;
  float sum = 0.f;
  for (long long e = sl.lo + threadIdx.x; e < sl.hi; e += NT) sum += xr[e];
  const float n = (float)(sl.hi - sl.lo);
  const float mean = n > 0.f ? block_sum(sum, red) / n : 0.f;
  float m2 = 0.f;
  for (long long e = sl.lo + threadIdx.x; e < sl.hi; e += NT) {
    const float d = xr[e] - mean;
    m2 += d * d;
  }
  m2 = block_sum(m2, red);
  if (threadIdx.x == 0) {
    part[((long long)b * S + s) * 2] = mean;
    part[((long long)b * S + s) * 2 + 1] = m2;
  }
}

// Chan's parallel combine of the S slice moments of row b.
__device__ __forceinline__ void ln_stats(const float* part, long long E, int S, int b,
                                         float eps, float& mean, float& rstd) {
  float n = 0.f, mu = 0.f, m2 = 0.f;
  for (int s = 0; s < S; ++s) {
    const Slice sl = slice_of(E, S, s);
    const float nb = (float)(sl.hi - sl.lo);
    if (nb <= 0.f) continue;
    const float mb = part[((long long)b * S + s) * 2], m2b = part[((long long)b * S + s) * 2 + 1];
    const float nn = n + nb, d = mb - mu;
    mu += d * nb / nn;
    m2 += m2b + d * d * n * nb / nn;
    n = nn;
  }
  mean = mu;
  rstd = rsqrtf(m2 / n + eps);   // biased variance, as nn.LayerNorm
}

__global__ __launch_bounds__(NT) void ln_apply_kernel(const float* __restrict__ x, long long E,
                                                      int S, const float* __restrict__ w,
                                                      const float* __restrict__ bias, float eps,
                                                      const float* __restrict__ part,
                                                      float* __restrict__ stats, int rows,
                                                      int ch, float* __restrict__ y) {
  const int b = blockIdx.y;
  float mean, rstd;
  ln_stats(part, E, S, b, eps, mean, rstd);
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    stats[b] = mean;
    stats[rows + b] = rstd;
  }
  const long long n4 = E / 4;
  const float4* x4 = (const float4*)(x + (long long)b * E);
  float4* y4 = (float4*)(y + (long long)b * E);
  for (long long i = blockIdx.x * (long long)NT + threadIdx.x; i < n4; i += gridDim.x * (long long)NT) {
    const float4 v = x4[i], ww = aff4(w, i, ch, E), bb = aff4(bias, i, ch, E);
    y4[i] = make_float4((v.x - mean) * rstd * ww.x + bb.x, (v.y - mean) * rstd * ww.y + bb.y,
                        (v.z - mean) * rstd * ww.z + bb.z, (v.w - mean) * rstd * ww.w + bb.w);
  }
}

// part [rows][S][2]: sums of g = dy w and of g xhat over slice s of row b
__global__ __launch_bounds__(NT) void ln_bwd_part_kernel(const float* __restrict__ dy,
                                                         const float* __restrict__ x, long long E,
                                                         int S, const float* __restrict__ w,
                                                         const float* __restrict__ stats, int rows,
                                                         int ch, float* __restrict__ part) {
  __shared__ float red[4];
  const int b = blockIdx.y, s = blockIdx.x;
  const Slice sl = slice_of(E, S, s);
  const float mean = stats[b], rstd = stats[rows + b];
  const float* xr = x + (long long)b * E;
  const float* gr = dy + (long long)b * E;
  float sg = 0.f, sgx = 0.f;
  for (long long e = sl.lo + threadIdx.x; e < sl.hi; e += NT) {
    const float g = gr[e] * w[aidx(e, ch, E)];
    sg += g;
    sgx += g * (xr[e] - mean) * rstd;
  }
  sg = block_sum(sg, red);
  sgx = block_sum(sgx, red);
  if (threadIdx.x == 0) {
    part[((long long)b * S + s) * 2] = sg;
    part[((long long)b * S + s) * 2 + 1] = sgx;
  }
}

// grid (ceil(E/4 / NT), n_groups): thread owns 4 consecutive elements e and
// loops over the samples of its group; dwp/dbp [n_groups][E] partials.
__global__ __launch_bounds__(NT) void ln_bwd_dx_kernel(
    const float* __restrict__ dy, const float* __restrict__ x, long long E, int S,
    const float* __restrict__ w, const float* __restrict__ stats, int rows,
    const float* __restrict__ part, int per_group, int ch, float* __restrict__ dx,
    float* __restrict__ dwp, float* __restrict__ dbp) {
  __shared__ float coef[3][64];
  const int g0 = blockIdx.y * per_group, g1 = min(rows, g0 + per_group);
  // per-sample coefficients: rstd, mean(g), mean(g xhat)
  for (int b = g0 + threadIdx.x; b < g1; b += NT) {
    float sg = 0.f, sgx = 0.f;
    for (int s = 0; s < S; ++s) {
      sg += part[((long long)b * S + s) * 2];
      sgx += part[((long long)b * S + s) * 2 + 1];
    }
    coef[0][b - g0] = stats[rows + b];
    coef[1][b - g0] = sg / (float)E;
    coef[2][b - g0] = sgx / (float)E;
  }
  __syncthreads();
  const long long i = blockIdx.x * (long long)NT + threadIdx.x;
  if (i >= E / 4) return;
  const float4 ww = aff4(w, i, ch, E);
  float4 dw = make_float4(0.f, 0.f, 0.f, 0.f), db = dw;
  for (int b = g0; b < g1; ++b) {
    const float mean = stats[b], rstd = coef[0][b - g0];
    const float mg = coef[1][b - g0], mgx = coef[2][b - g0];
    const float4 v = ((const float4*)(x + (long long)b * E))[i];
    const float4 d = ((const float4*)(dy + (long long)b * E))[i];
    const float4 xh = make_float4((v.x - mean) * rstd, (v.y - mean) * rstd,
                                  (v.z - mean) * rstd, (v.w - mean) * rstd);
    ((float4*)(dx + (long long)b * E))[i] =
        make_float4(rstd * (d.x * ww.x - mg - xh.x * mgx), rstd * (d.y * ww.y - mg - xh.y * mgx),
                    rstd * (d.z * ww.z - mg - xh.z * mgx), rstd * (d.w * ww.w - mg - xh.w * mgx));
    dw.x += d.x * xh.x; dw.y += d.y * xh.y; dw.z += d.z * xh.z; dw.w += d.w * xh.w;
    db.x += d.x; db.y += d.y; db.z += d.z; db.w += d.w;
  }
  ((float4*)(dwp + (long long)blockIdx.y * E))[i] = dw;
  ((float4*)(dbp + (long long)blockIdx.y * E))[i] = db;
}

__global__ __launch_bounds__(NT) void ln_bwd_dw_kernel(const float* __restrict__ dwp,
                                                       const float* __restrict__ dbp, long long E,
                                                       int groups, int ch, float* __restrict__ dw,
                                                       float* __restrict__ db) {
  const long long e = blockIdx.x * (long long)NT + threadIdx.x;
  if (e >= E) return;
  float a = 0.f, c = 0.f;
  for (int k = 0; k < groups; ++k) {
    a += dwp[k * E + e];
    c += dbp[k * E + e];
  }
  const long long t = aidx(e, ch, E);
  dw[t] = a;
  db[t] = c;
}

int slices_for(int rows, long long E) {
  long long s = (1024 + rows - 1) / rows;
  s = std::min<long long>(s, std::max<long long>(1, E / 1024));
  return (int)std::max<long long>(1, s);
}

}  // namespace

extern "C" {

// *out = workspace floats: rows * S * 2 + 2 * rows for the forward (mean and
// rstd at the end, read by the backward); the backward additionally needs
// 2 * G * E (G = ceil(rows / 8) sample groups).
int tgfr_ln_ws_floats(int rows, long long E, int backward, long long* out) {
  if (rows <= 0 || E <= 0 || !out) return 1001;
  const long long S = slices_for(rows, E);
  long long n = rows * S * 2 + 2LL * rows;
  if (backward) n += 2LL * ((rows + 7) / 8) * E;
  *out = n;
  return 0;
}

int tgfr_ln_fwd(const float* x, int rows, long long E, const float* w, const float* b, float eps,
                int ch, float* y, float* ws, void* stream) {
  if (rows <= 0 || E <= 0 || (E & 3) || rows > 65535 || ch < 0 || (ch && (ch & 3 || E % ch)))
    return 1001;
  const int S = slices_for(rows, E);
  float* part = ws;
  float* stats = ws + (long long)rows * S * 2;
  auto* st = (hipStream_t)stream;
  hipLaunchKernelGGL(ln_part_kernel, dim3(S, rows), dim3(NT), 0, st, x, E, S, part);
  const long long blocks = std::min<long long>((E / 4 + NT - 1) / NT, 64);
  hipLaunchKernelGGL(ln_apply_kernel, dim3((unsigned)blocks, rows), dim3(NT), 0, st, x, E, S, w,
                     b, eps, part, stats, rows, ch, y);
  return (int)hipGetLastError();
}

int tgfr_ln_bwd(const float* dy, const float* x, int rows, long long E, const float* w, int ch,
                float* ws, float* dx, float* dw, float* db, void* stream) {
  if (rows <= 0 || E <= 0 || (E & 3) || rows > 65535 || ch < 0 || (ch && (ch & 3 || E % ch)))
    return 1001;
  const int S = slices_for(rows, E);
  const int per = 8, groups = (rows + per - 1) / per;
  float* part = ws;
  const float* stats = ws + (long long)rows * S * 2;
  float* dwp = ws + (long long)rows * S * 2 + 2LL * rows;
  float* dbp = dwp + (long long)groups * E;
  auto* st = (hipStream_t)stream;
  // the forward's slice moments are no longer needed: reuse their slots
  hipLaunchKernelGGL(ln_bwd_part_kernel, dim3(S, rows), dim3(NT), 0, st, dy, x, E, S, w, stats,
                     rows, ch, part);
  hipLaunchKernelGGL(ln_bwd_dx_kernel, dim3((unsigned)((E / 4 + NT - 1) / NT), groups),
                     dim3(NT), 0, st, dy, x, E, S, w, stats, rows, part, per, ch, dx, dwp, dbp);
  hipLaunchKernelGGL(ln_bwd_dw_kernel, dim3((unsigned)((E + NT - 1) / NT)), dim3(NT), 0, st,
                     dwp, dbp, E, groups, ch, dw, db);
  return (int)hipGetLastError();
}

}  // extern "C"
