// Per-sample LayerNorm of the IMIM head (models/models.py:388, :401:
// nn.LayerNorm([256, 14, 14]) over all C*H*W elements of each sample, with an
// elementwise affine map of the same shape).
//
// PyTorch launches one block per sample (64 blocks on a 256-CU part, ~100 us
// for the backward).  Here every sample is cut into S slices so the launch has
// >= ~1024 blocks:
//   ln_part     per (sample, slice): count-free (mean_i, M2_i) of the slice
//   ln_apply    per (element block, group of samples): combine the S slice
//               moments (Chan, fixed order) -> mean, rstd of the group's
//               samples; y = (x - mean) rstd w + b with w, b loaded once per
//               thread; block (0, g) stores the group's mean/rstd
//   ln_bwd_part per (sample, slice): sums of g = dy w and g xhat
//   ln_bwd_dx   dx = rstd (g - mean(g) - xhat mean(g xhat)); per element e the
//               block also sums dy xhat and dy over its group of samples
//   ln_bwd_dw   dw[e] = sum of the group partials, db likewise (fixed order)
// Every reduction has a fixed order, so results are run-to-run identical.
#include "tgfr_ln.h"

using namespace tgfr;

namespace {

// dw, db scatter back to the reference layout: the affine map is stored
// channel-major [ch][E / ch] while x's rows are [E / ch][ch] (IMIM's
// LayerNorm([C, H, W]) on channels-last rows).
__device__ __forceinline__ long long aidx(long long e, int ch, long long E) {
  return ch ? (e % ch) * (E / ch) + e / ch : e;
}

// The affine values of channels-last elements 4 i4 .. 4 i4 + 3 (one position
// p, channels c .. c + 3) read from the reference's channel-major [ch][n]
// map in place (ch = 0: the map is row-indexed like x).  No per-step
// transposed copy of the map.
__device__ __forceinline__ float4 aff4(const float* __restrict__ a, long long i4, int ch, int n) {
  if (!ch) return ((const float4*)a)[i4];
  const int e = (int)(4 * i4), p = e / ch, c = e - p * ch;
  const float* q = a + (long long)c * n + p;
  return make_float4(q[0], q[n], q[2 * n], q[3 * n]);
}

// grid (ceil(E/4 / NT), ceil(rows / LN_GROUP)); w, b row-indexed ([E]).
__global__ __launch_bounds__(NT) void ln_apply_kernel(const float* __restrict__ x, long long E,
                                                      int S, const float* __restrict__ w,
                                                      const float* __restrict__ bias, int ch,
                                                      float eps, const float* __restrict__ part,
                                                      float* __restrict__ stats, int rows,
                                                      float* __restrict__ y) {
  __shared__ float ms[2][LN_GROUP];
  const int g0 = blockIdx.y * LN_GROUP, g1 = min(rows, g0 + LN_GROUP);
  if (threadIdx.x < g1 - g0) {
    const int b = g0 + threadIdx.x;
    float mean, rstd;
    ln_stats(part, E, S, b, eps, mean, rstd);
    ms[0][threadIdx.x] = mean;
    ms[1][threadIdx.x] = rstd;
    if (blockIdx.x == 0) {
      stats[b] = mean;
      stats[rows + b] = rstd;
    }
  }
  __syncthreads();
  const long long i = blockIdx.x * (long long)NT + threadIdx.x;
  if (i >= E / 4) return;
  const int n = ch ? (int)(E / ch) : 0;
  const float4 ww = aff4(w, i, ch, n), bb = aff4(bias, i, ch, n);
  float4 v[LN_GROUP];
#pragma unroll
  for (int k = 0; k < LN_GROUP; ++k)
    if (g0 + k < g1) v[k] = ((const float4*)(x + (long long)(g0 + k) * E))[i];
#pragma unroll
  for (int k = 0; k < LN_GROUP; ++k) {
    if (g0 + k >= g1) break;
    const float mean = ms[0][k], rstd = ms[1][k];
    ((float4*)(y + (long long)(g0 + k) * E))[i] =
        make_float4((v[k].x - mean) * rstd * ww.x + bb.x, (v[k].y - mean) * rstd * ww.y + bb.y,
                    (v[k].z - mean) * rstd * ww.z + bb.z, (v[k].w - mean) * rstd * ww.w + bb.w);
  }
}

// part [rows][S][2]: sums of g = dy w and of g xhat over slice s of row b
__global__ __launch_bounds__(NT) void ln_bwd_part_kernel(const float* __restrict__ dy,
                                                         const float* __restrict__ x, long long E,
                                                         int S, const float* __restrict__ w,
                                                         int ch, const float* __restrict__ stats,
                                                         int rows, float* __restrict__ part) {
  __shared__ float red[4];
  const int b = blockIdx.y, s = blockIdx.x;
  const Slice sl = slice_of(E, S, s);
  const float mean = stats[b], rstd = stats[rows + b];
  const float4* xr = (const float4*)(x + (long long)b * E);
  const float4* gr = (const float4*)(dy + (long long)b * E);
  const int n = ch ? (int)(E / ch) : 0;
  float sg = 0.f, sgx = 0.f;
  for (long long i = sl.lo / 4 + threadIdx.x; i < sl.hi / 4; i += NT) {
    const float4 d = gr[i], ww = aff4(w, i, ch, n), v = xr[i];
    const float ga = d.x * ww.x, gb = d.y * ww.y, gc = d.z * ww.z, gd = d.w * ww.w;
    sg += (ga + gb) + (gc + gd);
    sgx += (ga * (v.x - mean) + gb * (v.y - mean)) + (gc * (v.z - mean) + gd * (v.w - mean));
  }
  sgx *= rstd;
  sg = block_sum(sg, red);
  sgx = block_sum(sgx, red);
  if (threadIdx.x == 0) {
    part[((long long)b * S + s) * 2] = sg;
    part[((long long)b * S + s) * 2 + 1] = sgx;
  }
}

// grid (ceil(E/4 / NT), n_groups): thread owns 4 consecutive elements e and
// loops over the samples of its group; dwp/dbp [n_groups][E] partials.
// ATT (the IMIM LayerNorm, whose input is the attention output O = x with
// 256 channels): instead of dx in fp32, the attention backward's operands --
// dOb = bf16(dx) and D[row] = sum_c dx[row][c] O[row][c] (one wave = one row
// of 256 channels) -- so the attention backward needs no prep pass.
template <bool ATT>
__global__ __launch_bounds__(NT) void ln_bwd_dx_kernel(
    const float* __restrict__ dy, const float* __restrict__ x, long long E, PartSrc src,
    const float* __restrict__ w, int ch, const float* __restrict__ stats, int rows,
    int per_group, float* __restrict__ dx, float* __restrict__ dwp, float* __restrict__ dbp,
    float* __restrict__ Dout, uint16_t* __restrict__ dOb) {
  __shared__ float coef[3][64];
  const int g0 = blockIdx.y * per_group, g1 = min(rows, g0 + per_group);
  const long long i = blockIdx.x * (long long)NT + threadIdx.x;
  const bool live = i < E / 4;
  // the group's loads all in flight before the arithmetic (per_group <=
  // LN_GROUP), issued ahead of the per-sample coefficients' dependent loads
  // below so that both memory rounds overlap
  float4 vv[LN_GROUP], dd[LN_GROUP];
#pragma unroll
  for (int k = 0; k < LN_GROUP; ++k) {
    const int b = g0 + k;
    if (live && b < g1) {
      vv[k] = ((const float4*)(x + (long long)b * E))[i];
      if constexpr (ATT) {   // dy: the tail backward's bf16 dZ rows
        const uint2 u = ((const uint2*)((const uint16_t*)dy + (long long)b * E))[i];
        dd[k] = make_float4(__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u),
                            __uint_as_float(u.y << 16), __uint_as_float(u.y & 0xffff0000u));
      } else {
        dd[k] = ((const float4*)(dy + (long long)b * E))[i];
      }
    }
  }
  const float4 ww = live ? aff4(w, i, ch, ch ? (int)(E / ch) : 0) : make_float4(0.f, 0.f, 0.f, 0.f);
  // per-sample coefficients: rstd, mean(g), mean(g xhat)
  for (int b = g0 + threadIdx.x; b < g1; b += NT) {
    float sg, sgx;
    src.sums(b, sg, sgx);
    coef[0][b - g0] = stats[rows + b];
    coef[1][b - g0] = sg / (float)E;
    coef[2][b - g0] = sgx / (float)E;
  }
  __syncthreads();
  if (!live) return;
  float4 dw = make_float4(0.f, 0.f, 0.f, 0.f), db = dw;
#pragma unroll
  for (int k = 0; k < LN_GROUP; ++k) {
    const int b = g0 + k;
    if (b >= g1) break;
    const float mean = stats[b], rstd = coef[0][k];
    const float mg = coef[1][k], mgx = coef[2][k];
    const float4 v = vv[k], d = dd[k];
    const float4 xh = make_float4((v.x - mean) * rstd, (v.y - mean) * rstd,
                                  (v.z - mean) * rstd, (v.w - mean) * rstd);
    const float4 o =
        make_float4(rstd * (d.x * ww.x - mg - xh.x * mgx), rstd * (d.y * ww.y - mg - xh.y * mgx),
                    rstd * (d.z * ww.z - mg - xh.z * mgx), rstd * (d.w * ww.w - mg - xh.w * mgx));
    if constexpr (ATT) {
      *(uint2*)(dOb + (long long)b * E + 4 * i) =
          make_uint2(pk_bf16(o.x, o.y), pk_bf16(o.z, o.w));
      const float dsum = wave_sum(o.x * v.x + o.y * v.y + o.z * v.z + o.w * v.w);
      if ((threadIdx.x & 63) == 0) Dout[(long long)b * (E / 256) + (4 * i) / 256] = dsum;
    } else {
      ((float4*)(dx + (long long)b * E))[i] = o;
    }
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

bool ln_args_ok(int rows, long long E, int ch) {
  return rows > 0 && E > 0 && !(E & 3) && rows <= 65535 && ch >= 0 &&
         !(ch && (ch & 3 || E % ch));
}

}  // namespace

extern "C" {

int tgfr_ln_ws_floats(int rows, long long E, int ch, int backward, long long* out) {
  if (!ln_args_ok(rows, E, ch) || !out) return 1001;
  const LnWs o = ln_ws(rows, E, ch);
  *out = backward ? o.total_bwd : o.total_fwd;
  return 0;
}

int tgfr_ln_fwd(const float* x, int rows, long long E, const float* w, const float* b, float eps,
                int ch, float* y, float* ws, void* stream) {
  if (!ln_args_ok(rows, E, ch)) return 1001;
  const int S = slices_for(rows, E);
  const LnWs o = ln_ws(rows, E, ch);
  float* part = ws;
  float* stats = ws + o.stats;
  auto* st = (hipStream_t)stream;
  hipLaunchKernelGGL(ln_part_kernel, dim3(S, rows), dim3(NT), 0, st, x, E, S, part);
  hipLaunchKernelGGL(ln_apply_kernel,
                     dim3((unsigned)((E / 4 + NT - 1) / NT), (rows + LN_GROUP - 1) / LN_GROUP),
                     dim3(NT), 0, st, x, E, S, w, b, ch, eps, part, stats, rows, y);
  return (int)hipGetLastError();
}

// ws: the forward's workspace (its stats and, for ch > 0, its channels-last w
// copy), sized for the backward.
int tgfr_ln_bwd(const float* dy, const float* x, int rows, long long E, const float* w, int ch,
                float* ws, float* dx, float* dw, float* db, void* stream) {
  if (!ln_args_ok(rows, E, ch)) return 1001;
  const int S = slices_for(rows, E);
  const LnWs o = ln_ws(rows, E, ch);
  const int groups = (rows + LN_GROUP - 1) / LN_GROUP;
  float* part = ws;
  const float* stats = ws + o.stats;
  float* dwp = ws + o.bwd;
  float* dbp = dwp + (long long)groups * E;
  auto* st = (hipStream_t)stream;
  // the forward's slice moments are no longer needed: reuse their slots
  hipLaunchKernelGGL(ln_bwd_part_kernel, dim3(S, rows), dim3(NT), 0, st, dy, x, E, S, w, ch,
                     stats, rows, part);
  hipLaunchKernelGGL(ln_bwd_dx_kernel<false>, dim3((unsigned)((E / 4 + NT - 1) / NT), groups),
                     dim3(NT), 0, st, dy, x, E, PartSrc{part, S, 0, 0, 1}, w, ch, stats, rows,
                     LN_GROUP, dx, dwp, dbp, nullptr, nullptr);
  hipLaunchKernelGGL(ln_bwd_dw_kernel, dim3((unsigned)((E + NT - 1) / NT)), dim3(NT), 0, st,
                     dwp, dbp, E, groups, ch, dw, db);
  return (int)hipGetLastError();
}

}  // extern "C"

namespace tgfr {

int ln_part_launch(const float* x, int rows, long long E, float* ws, hipStream_t s) {
  if (!ln_args_ok(rows, E, 0)) return 1001;
  const int S = slices_for(rows, E);
  hipLaunchKernelGGL(ln_part_kernel, dim3(S, rows), dim3(NT), 0, s, x, E, S, ws);
  return (int)hipGetLastError();
}

int ln_bwd_tail_launch(const float* dy, const float* x, int rows, long long E, const float* w_cl,
                       int ch, float* ws, const float* tail_part, int hw, int tm, float* dx,
                       float* D, uint16_t* dOb, float* dw, float* db, hipStream_t s) {
  if (!ln_args_ok(rows, E, ch) || hw < tm || tm <= 0) return 1001;
  if (dOb && (ch != 256 || !D)) return 1001;
  const LnWs o = ln_ws(rows, E, ch);
  const int groups = (rows + LN_GROUP - 1) / LN_GROUP;
  const float* stats = ws + o.stats;
  float* dwp = ws + o.bwd;
  float* dbp = dwp + (long long)groups * E;
  const dim3 grid((unsigned)((E / 4 + NT - 1) / NT), groups);
  const PartSrc src{tail_part, 0, 1, hw, tm};
  if (dOb)
    hipLaunchKernelGGL(ln_bwd_dx_kernel<true>, grid, dim3(NT), 0, s, dy, x, E, src, w_cl, 0,
                       stats, rows, LN_GROUP, nullptr, dwp, dbp, D, dOb);
  else
    hipLaunchKernelGGL(ln_bwd_dx_kernel<false>, grid, dim3(NT), 0, s, dy, x, E, src, w_cl, 0,
                       stats, rows, LN_GROUP, dx, dwp, dbp, nullptr, nullptr);
  if (dw)   // (NULL: the caller reduces the group partials later)
    hipLaunchKernelGGL(ln_bwd_dw_kernel, dim3((unsigned)((E + NT - 1) / NT)), dim3(NT), 0, s,
                       dwp, dbp, E, groups, ch, dw, db);
  return (int)hipGetLastError();
}

}  // namespace tgfr
