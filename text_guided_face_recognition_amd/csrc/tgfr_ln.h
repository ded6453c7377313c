// LayerNorm pieces shared by the per-sample LayerNorm (tgfr_norm.hip) and the
// IMIM tail with the LayerNorm fused into its load (tgfr_tail.hip): slice
// moments, their Chan combine, the workspace layout.
#pragma once
#include "tgfr_common.h"

#include <algorithm>

namespace {

using namespace tgfr;

constexpr int NT = 256;
constexpr int LN_GROUP = 8;   // samples per ln_apply / ln_bwd_dx block

__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int wid = threadIdx.x / WAVE;
  __syncthreads();
  if (threadIdx.x % WAVE == 0) red[wid] = v;
  __syncthreads();
  return red[0] + red[1] + red[2] + red[3];
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
  // slices are whole float4s (slice_of rounds the length to 4, E % 4 == 0)
  const float4* xr = (const float4*)(x + (long long)b * E);
  const long long lo = sl.lo / 4, hi = sl.hi / 4;
  float sum = 0.f;
  for (long long i = lo + threadIdx.x; i < hi; i += NT) {
    const float4 v = xr[i];
    sum += (v.x + v.y) + (v.z + v.w);
  }
  const float n = (float)(sl.hi - sl.lo);
  const float mean = n > 0.f ? block_sum(sum, red) / n : 0.f;
  float m2 = 0.f;
  for (long long i = lo + threadIdx.x; i < hi; i += NT) {
    const float4 v = xr[i];
    const float a = v.x - mean, c = v.y - mean, d = v.z - mean, e = v.w - mean;
    m2 += (a * a + c * c) + (d * d + e * e);
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

// The same combine for moments left by the attention forward (tgfr_attn_fwd_ln):
// nt 32-row tiles of a sample with hw rows of ch channels, tile t holding
// min(32, hw - 32 t) rows; mom = this sample's [nt][2].
__device__ __forceinline__ void ln_stats_tiles(const float* mom, int nt, int hw, int ch,
                                               float eps, float& mean, float& rstd) {
  float n = 0.f, mu = 0.f, m2 = 0.f;
  for (int t = 0; t < nt; ++t) {
    const float nb = (float)(min(32, hw - 32 * t) * ch);
    const float mb = mom[2 * t], m2b = mom[2 * t + 1];
    const float nn = n + nb, d = mb - mu;
    mu += d * nb / nn;
    m2 += m2b + d * d * n * nb / nn;
    n = nn;
  }
  mean = mu;
  rstd = rsqrtf(m2 / n + eps);
}

int slices_for(int rows, long long E) {
  long long s = (1024 + rows - 1) / rows;
  s = std::min<long long>(s, std::max<long long>(1, E / 1024));
  return (int)std::max<long long>(1, s);
}

// Workspace floats: part [rows][S][2] | mean [rows] | rstd [rows] -- written
// by the forward and read by the backward -- then (backward) dw, db group
// partials [2][G][E], G = ceil(rows / LN_GROUP).  (The channel-major affine
// maps are read in place, aff4.)
struct LnWs {
  long long stats, aff, bwd, total_fwd, total_bwd;
};
LnWs ln_ws(int rows, long long E, int ch) {
  const long long S = slices_for(rows, E);
  LnWs o;
  o.stats = rows * S * 2;
  o.aff = o.stats + 2LL * rows;
  o.bwd = o.aff;
  o.total_fwd = o.bwd;
  o.total_bwd = o.bwd + 2LL * ((rows + LN_GROUP - 1) / LN_GROUP) * E;
  return o;
}

// Where ln_bwd_dx finds each sample's sums of g = dy w and g xhat: the
// slices of ln_bwd_part ([rows][S][2], tail = 0), or the per-workgroup
// partials of the IMIM tail backward with the LayerNorm backward's first pass
// fused in (tail = 1): workgroup k owns rows [tm k, tm k + tm) of the
// channels-last [rows * hw][ch] map, i.e. at most two samples (hw >= tm), and
// writes [k][slot][2] for samples tm k / hw + slot.
struct PartSrc {
  const float* p;
  int S, tail, hw, tm;
  __device__ __forceinline__ void sums(int b, float& sg, float& sgx) const {
    sg = sgx = 0.f;
    if (!tail) {
      for (int s = 0; s < S; ++s) {
        sg += p[((long long)b * S + s) * 2];
        sgx += p[((long long)b * S + s) * 2 + 1];
      }
      return;
    }
    const long long k0 = (long long)b * hw / tm, k1 = ((long long)(b + 1) * hw - 1) / tm;
    for (long long k = k0; k <= k1; ++k) {
      const int slot = b - (int)(k * tm / hw);
      sg += p[(k * 2 + slot) * 2];
      sgx += p[(k * 2 + slot) * 2 + 1];
    }
  }
};

}  // namespace

namespace tgfr {
// tgfr_norm.hip: the LayerNorm's slice moments into ws (LnWs layout), and its
// backward (ln_bwd_dx + ln_bwd_dw) from per-sample sums left by the IMIM tail
// backward (PartSrc tail = 1); w_cl: the affine weight as channels-last rows
// [E] (coalesced), ch: the reference's channel count for the dw / db scatter.
int ln_part_launch(const float* x, int rows, long long E, float* ws, hipStream_t s);
// (dOb != NULL: instead of dx, the attention backward's operands dOb =
// bf16(dx) and D[row] = dx . x per 256-channel row, ch == 256)
int ln_bwd_tail_launch(const float* dy, const float* x, int rows, long long E, const float* w_cl,
                       int ch, float* ws, const float* tail_part, int hw, int tm, float* dx,
                       float* D, uint16_t* dOb, float* dw, float* db, hipStream_t s);
}  // namespace tgfr
