// SelfAttention core (models/fusion_nets.py:82-118) for gfx950.
//
// The reference computes, per sample n, with x the image and y the text side:
//   Qr = key_proj(x)^T [HW, C'],  Kr = query_proj(y)^T [HW, C'],  V = value_proj(x)^T [HW, C]
//   P  = softmax_j(Qr Kr^T / sqrt_dim)                  (:103-106)
//   O  = P V  -> permuted to [C, HW]                      (:115-117)
// The products (QK^T, PV, the 1x1 projections and their backward) run on
// tgfr_bgemm (tgfr_gemm.hip); this file holds the row softmax:
//   attn_softmax   P = softmax(scale * S) per row over the valid keys + row LSE.
//   attn_softmax_bwd  dS = scale * P (dP - rowsum(P dP)).
// The attention matrices are HW x HW per sample (196^2 fp32 = 150 KB for IMIM,
// 36^2 for FCFM); on the composed path they are materialised.
//
// Fused self-attention (bf16 mode, IMIM: C' = C = 256, HW <= 224), reading the
// packed fp32 projections [Qr | Kr | V] of each sample in place:
//   attn_fwd      per (sample, 32-query tile), online softmax over the key
//                 tiles.  S^T = Kr Qr^T puts ONE query on each lane (its MFMA
//                 column): the running max / sum are lane-local plus one
//                 cross-half combine, and P^T as it stands is the B operand of
//                 O^T = V^T P^T (the MFMA k axis permuted to the accumulator's
//                 row order; V read through LDS with ds_read_b64_tr_b16 in
//                 the same order).  Writes O [HW][256] and the row LSE.
//   attn_bwd_kv   one 2-wave workgroup per (sample, 32-key tile), each wave
//                 owning half of the d / dv columns.  Per query tile it
//                 recomputes S = Qr Kr^T and dP = dO V^T (lane = key column,
//                 so P^T and dS^T are A operands as they stand), then
//                 dV += P^T dO and dKr += dS^T Qr with dO / Qr read through
//                 LDS transposed; dS (bf16) goes to HBM for
//   attn_bwd_q    one wave per (sample, 32-query tile): dQr = dS Kr, Kr staged
//                 per key tile in LDS.
// No HW x HW fp32 matrix is ever written; D = rowsum(dO * O) comes from
// attn_bwd_prep.
//
// Fused small attention (FCFM: HW = C' = C = 36): attn_small_fwd / _bwd, one
// workgroup per sample with the whole problem in LDS, fp32 MFMA (exact fp32).
#include "tgfr_common.h"

using namespace tgfr;

namespace {

// one wave per row of [rows][n] (row stride ld)
__global__ __launch_bounds__(256) void attn_softmax_kernel(const float* __restrict__ S,
                                                           float* __restrict__ P, float* lse,
                                                           long long rows, int n, long long ld,
                                                           float scale) {
  const long long row = blockIdx.x * 4LL + threadIdx.x / WAVE;
  const int lane = threadIdx.x % WAVE;
  if (row >= rows) return;
  const float* s = S + row * ld;
  float m = -INFINITY;
  for (int j = lane; j < n; j += WAVE) m = fmaxf(m, s[j] * scale);
  m = wave_max(m);
  float sum = 0.f;
  for (int j = lane; j < n; j += WAVE) sum += __expf(s[j] * scale - m);
  sum = wave_sum(sum);
  const float inv = 1.f / sum;
  float* p = P + row * ld;
  for (int j = lane; j < n; j += WAVE) p[j] = __expf(s[j] * scale - m) * inv;
  if (lse && lane == 0) lse[row] = m + __logf(sum);
}

__global__ __launch_bounds__(256) void attn_softmax_bwd_kernel(const float* __restrict__ P,
                                                               const float* __restrict__ dP,
                                                               float* __restrict__ dS,
                                                               long long rows, int n,
                                                               long long ld, float scale) {
  const long long row = blockIdx.x * 4LL + threadIdx.x / WAVE;
  const int lane = threadIdx.x % WAVE;
  if (row >= rows) return;
  const float* p = P + row * ld;
  const float* dp = dP + row * ld;
  float dot = 0.f;
  for (int j = lane; j < n; j += WAVE) dot += p[j] * dp[j];
  dot = wave_sum(dot);
  float* ds = dS + row * ld;
  for (int j = lane; j < n; j += WAVE) ds[j] = scale * p[j] * (dp[j] - dot);
}

// ------------------------------------------------------ fused (IMIM) ---
constexpr int AD = 256;                  // Qr/Kr width = V width
constexpr int AT = 7;                    // max 32-position tiles (HW <= 224)
constexpr int IMG = 32 * AD * 2;         // one 32-row bf16 tile image (16 KiB)

__device__ __attribute__((aligned(16))) uint16_t attn_zero16[8] = {0, 0, 0, 0, 0, 0, 0, 0};

// Tile image: 32 rows x 256 bf16, 512-B rows, 16-B chunk c of row r stored at
// chunk c ^ f(r), f(r) = 4 (r & 3) + ((r >> 2) & 3).  Both read shapes are
// conflict-free on it: a ds_read_b128 operand fragment (16 lanes of a group =
// 16 rows, one logical chunk: f is a bijection on r mod 16) and a
// ds_read_b64_tr_b16 transposed fragment (32 lanes = 4 rows x 4 chunks: the
// rows' high swizzle bits differ).
__device__ __forceinline__ int tsw(int r) { return 4 * (r & 3) + ((r >> 2) & 3); }
__device__ __forceinline__ uint32_t tix(int r, int c) {
  return (uint32_t)(r * (AD * 2) + ((c ^ tsw(r)) << 4));
}
__device__ __forceinline__ bf16x8 zero8() { return as_bf8(make_uint4(0, 0, 0, 0)); }

// Wait until at most `younger` ring stages of 8 DMA pieces (this wave's
// share) are outstanding, then meet the workgroup.
__device__ __forceinline__ void ring_wait8(int younger) {
  switch (younger) {
    case 0: ring_barrier<0>(); break;
    case 1: ring_barrier<8>(); break;
    case 2: ring_barrier<16>(); break;
    case 3: ring_barrier<24>(); break;
    case 4: ring_barrier<32>(); break;
    case 5: ring_barrier<40>(); break;
    default: ring_barrier<48>(); break;
  }
}

// Operand fragment, lane row lr: columns 16 s + 8 h .. +7.
__device__ __forceinline__ bf16x8 frag(uint32_t base, int s, int lane) {
  return as_bf8(lds_ld16(base + tix(lane & 31, 2 * s + (lane >> 5))));
}
// Transposed fragment: lane gets column c0 + lane%32 at rows r0 + 0..3
// (elements 0-3) and r1 + 0..3 (elements 4-7).
__device__ __forceinline__ bf16x8 trf(uint32_t base, int r0, int r1, int c0, int lane) {
  const int i = lane & 15, q = i >> 2, p = i & 3, g = lane >> 4;
  const int col = c0 + 16 * (g & 1) + 4 * p;
  const uint32_t o = ((col >> 2) & 1) * 8;
  return join_tr(lds_tr4(base + tix(r0 + q, col >> 3) + o),
                 lds_tr4(base + tix(r1 + q, col >> 3) + o));
}

// DMA of bf16 rows [row0, row0 + 32) x 256 (row stride ld) into a tile image:
// 16 one-KiB pieces (two image rows each); this wave issues pieces
// wv, wv + nw, ...  Each lane's source is the logical chunk its swizzled slot
// holds; rows >= n read zeros (checked only on a ragged tile: per-piece
// address VALU rivals the MFMA time of these short kernels).
__device__ __forceinline__ void dma_tile(const uint16_t* X, long long ld, int row0, int n,
                                         uint32_t base, int wv, int nw, int lane) {
  const bool full = row0 + 32 <= n;                  // uniform
  const uint16_t* X0 = X + (long long)row0 * ld;
  const int r1 = lane >> 5, l31 = lane & 31;
#pragma unroll 4
  for (int p = wv; p < 16; p += nw) {
    const int r = 2 * p + r1, c = l31 ^ tsw(r);
    const uint16_t* src = X0 + r * (int)ld + 8 * c;
    if (!full && row0 + r >= n) src = attn_zero16;
    glds16(src, base + p * 1024);
  }
}

// Forward: one 4-wave workgroup per (sample, pair of query tiles); wave w
// takes query tile 2 j + (w & 1) over key half w >> 1 (tiles [0, nh) or
// [nh, nt), nh = ceil(nt / 2)), so every SIMD of the CU holds a wave (the
// 2-wave version left half of them idle: 448 waves on 1024 SIMDs at B = 64)
// and each wave's serial chain of key tiles is half as long.  Online softmax
// over the wave's key tiles in a ROLLED loop (a fully unrolled run-once kernel
// of ~40 KB spent its time on instruction-cache misses); at the end the key
// half 1 waves hand (m, l, O) to their half-0 partners through LDS, which
// combine the two partial softmaxes and write O and the row LSE.
// Per key tile: S^T = Kr Qr^T (lane = query, so the running max / sum are
// per lane plus one cross-half combine), then O^T += V^T P^T with P^T the
// accumulator as it stands (k axis in the accumulator's key order, V read
// transposed in the same order) -- O^T keeps the query on the lane too, so the
// online-softmax rescale is one scalar per lane.
// LDS: [0, 2 IMG) the query tiles, then a 2-deep ring of stages; stage i =
// Kr, V of key tile i (half 0) and of key tile nh + i (half 1), each wave
// DMA-ing a quarter of every tile.
constexpr int FWD_STAGE = 4 * IMG;
constexpr int FWD_LDS = 2 * IMG + 2 * FWD_STAGE;       // 160 KiB
constexpr int FWD_XCH = 8 * 16 + 2;                    // floats per lane handed over

__global__ __launch_bounds__(256) void attn_fwd_kernel(const uint16_t* __restrict__ Qp,
                                                       const uint16_t* __restrict__ Kp,
                                                       const uint16_t* __restrict__ Vp,
                                                       long long ld, long long sb, int hw,
                                                       float scale, float* __restrict__ O,
                                                       long long ldo, long long sbo,
                                                       float* __restrict__ lse,
                                                       float* __restrict__ lnm, int lnS) {
  const int tid = threadIdx.x, w = tid / WAVE, lane = tid % WAVE, lr = lane & 31, h = lane >> 5;
  const int qsel = w & 1, half = w >> 1;
  const int nt = (hw + 31) / 32, np = (nt + 1) / 2, nh = (nt + 1) / 2;
  // the workgroups of one sample run on one XCD (its Kr / V stay in that L2)
  const int wid = xcd_remap(blockIdx.x, gridDim.x);
  const int b = wid / np, qt = 2 * (wid % np) + qsel;
  const bool active = qt < nt;                       // uniform per wave
  const uint32_t qimg = qsel * IMG, ring = 2 * IMG;
  const int iters = nh;                              // half 0 has nh tiles, half 1 nt - nh
  auto issue = [&](int i) {                          // stage i -> ring slot i % 2
    const uint32_t base = ring + (i & 1) * FWD_STAGE;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int kt = u ? nh + i : i;
      const int n = kt < nt ? hw : 0;                // a missing half-1 tile: zeros
      dma_tile(Kp + b * sb, ld, 32 * kt, n, base + (2 * u) * IMG, w, 4, lane);
      dma_tile(Vp + b * sb, ld, 32 * kt, n, base + (2 * u + 1) * IMG, w, 4, lane);
    }
  };
  // the query tiles (this wave's quarter of both), then stage 0
  dma_tile(Qp + b * sb, ld, 32 * (2 * (wid % np)), hw, 0, w, 4, lane);
  dma_tile(Qp + b * sb, ld, 32 * (2 * (wid % np) + 1), 2 * (wid % np) + 1 < nt ? hw : 0, IMG, w,
           4, lane);
  issue(0);
  ring_barrier<0>();
  if (iters > 1) issue(1);
  bf16x8 qf[AD / 16];
#pragma unroll
  for (int s = 0; s < AD / 16; ++s) qf[s] = frag(qimg, s, lane);

  const float c = scale * 1.4426950408889634f;
  float m = -INFINITY, l = 0.f;
  f32x16 oacc[AD / 32];
#pragma unroll
  for (int t = 0; t < AD / 32; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) oacc[t][r] = 0.f;
  for (int i = 0; i < iters; ++i) {
    if (i > 0) {
      // stage i landed (16 pieces per wave per stage: stage i+1 may still fly)
      if (i + 1 < iters) {
        ring_barrier<0>();
        issue(i + 1);
      } else {
        ring_barrier<0>();
      }
    }
    const int kt = half ? nh + i : i;
    if (kt >= nt) continue;                          // uniform per wave (half 1, odd nt)
    const uint32_t kbuf = ring + (i & 1) * FWD_STAGE + (2 * half) * IMG, vbuf = kbuf + IMG;
    f32x16 sc;
#pragma unroll
    for (int r = 0; r < 16; ++r) sc[r] = 0.f;
#pragma unroll
    for (int s = 0; s < AD / 16; ++s)
      sc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(frag(kbuf, s, lane), qf[s], sc, 0, 0, 0);
    // keys 32 kt + acc_row(r, h) of query 32 qt + lr
    if (32 * kt + 32 > hw) {                         // ragged last tile (uniform)
#pragma unroll
      for (int r = 0; r < 16; ++r)
        sc[r] = 32 * kt + acc_row(r, h) < hw ? sc[r] : -INFINITY;
    }
    float tmax = sc[0];
#pragma unroll
    for (int r = 1; r < 16; ++r) tmax = fmaxf(tmax, sc[r]);
    tmax = xhalf_max(tmax);
    // lazy rescale: the reference max m only moves when some query's tile
    // max exceeds it by more than 8 / c (P then stays <= 2^8, exact in the
    // fp32 sums and fine in bf16); otherwise O and l keep their scale and the
    // 128-register rescale of O is skipped
    if (i == 0) {
      m = tmax;
    } else if (__builtin_amdgcn_ballot_w64((tmax - m) * c > 8.f)) {
      const float mn = fmaxf(m, tmax);
      const float alpha = __builtin_amdgcn_exp2f((m - mn) * c);
      m = mn;
      l *= alpha;
#pragma unroll
      for (int t = 0; t < AD / 32; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) oacc[t][r] *= alpha;
    }
    float ps = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      sc[r] = __builtin_amdgcn_exp2f((sc[r] - m) * c);
      ps += sc[r];
    }
    l += ps;
    bf16x8 pb[2];
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
      pb[s2] = as_bf8(make_uint4(pk_bf16(sc[8 * s2], sc[8 * s2 + 1]),
                                 pk_bf16(sc[8 * s2 + 2], sc[8 * s2 + 3]),
                                 pk_bf16(sc[8 * s2 + 4], sc[8 * s2 + 5]),
                                 pk_bf16(sc[8 * s2 + 6], sc[8 * s2 + 7])));
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
      for (int t = 0; t < AD / 32; ++t) {
        const bf16x8 va = trf(vbuf, 16 * s2 + 4 * h, 16 * s2 + 8 + 4 * h, 32 * t, lane);
        oacc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(va, pb[s2], oacc[t], 0, 0, 0);
      }
  }
  l = xhalf_sum(l);
  // key half 1 -> its half-0 partner (same query tile) through the ring area
  __syncthreads();                                   // every wave is done with the ring
  const uint32_t xch = ring + (uint32_t)(qsel * 64 + lane) * FWD_XCH * 4;
  if (half == 1) {
#pragma unroll
    for (int t = 0; t < AD / 32; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) lds_stf(xch + (16 * t + r) * 4, oacc[t][r]);
    lds_stf(xch + 128 * 4, m);
    lds_stf(xch + 129 * 4, l);
  }
  __syncthreads();
  if (half == 1 || !active) return;
  const float m1 = lds_ldf(xch + 128 * 4), l1 = lds_ldf(xch + 129 * 4);
  const float mm = fmaxf(m, m1);
  const float a0 = __builtin_amdgcn_exp2f((m - mm) * c);
  const float a1 = m1 == -INFINITY ? 0.f : __builtin_amdgcn_exp2f((m1 - mm) * c);
  const float lt = l * a0 + l1 * a1;
  const int q = 32 * qt + lr;
  const bool qv = q < hw;
  if (qv && h == 0) lse[(long long)b * hw + q] = mm * scale + __logf(lt);
  const float i0 = a0 / lt, i1 = a1 / lt;
  // lane: query q; register r of tile t: column 32 t + acc_row(r, h)
  float* orow = O + b * sbo + (long long)q * ldo;
#pragma unroll
  for (int t = 0; t < AD / 32; ++t)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
#pragma unroll
      for (int k = 0; k < 4; ++k)
        oacc[t][4 * g + k] =
            oacc[t][4 * g + k] * i0 + lds_ldf(xch + (16 * t + 4 * g + k) * 4) * i1;
      if (qv)
        *(float4*)(orow + 32 * t + 8 * g + 4 * h) =
            make_float4(oacc[t][4 * g], oacc[t][4 * g + 1], oacc[t][4 * g + 2],
                        oacc[t][4 * g + 3]);
    }
  if (lnm) {
    // the following per-sample LayerNorm's moments of this query tile (mean,
    // M2 over its valid rows x 256 channels; count implied by the tile),
    // two passes over the registers: lnm[b][qt][2], slot qt of lnS per sample
    float sum = 0.f;
#pragma unroll
    for (int t = 0; t < AD / 32; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) sum += oacc[t][r];
    const float cnt = (float)(min(32, hw - 32 * qt) * AD);
    const float mean = wave_sum(qv ? sum : 0.f) / cnt;
    float m2 = 0.f;
#pragma unroll
    for (int t = 0; t < AD / 32; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float d = oacc[t][r] - mean;
        m2 = fmaf(d, d, m2);
      }
    m2 = wave_sum(qv ? m2 : 0.f);
    if (lane == 0) {
      lnm[((long long)b * lnS + qt) * 2] = mean;
      lnm[((long long)b * lnS + qt) * 2 + 1] = m2;
    }
  }
}

// D[row] = sum_c dO[row][c] O[row][c] and dO in bf16 (the backward's operand);
// one wave per row
__global__ __launch_bounds__(256) void attn_bwd_prep_kernel(const float* __restrict__ dO,
                                                            const float* __restrict__ O,
                                                            long long ld, long long rows,
                                                            float* __restrict__ D,
                                                            uint16_t* __restrict__ dOb) {
  const long long row = blockIdx.x * 4LL + threadIdx.x / WAVE;
  const int lane = threadIdx.x % WAVE;
  if (row >= rows) return;
  const float4 a = *(const float4*)(dO + row * ld + 4 * lane);
  const float4 o = *(const float4*)(O + row * ld + 4 * lane);
  *(uint2*)(dOb + row * AD + 4 * lane) = make_uint2(pk_bf16(a.x, a.y), pk_bf16(a.z, a.w));
  const float v = wave_sum(a.x * o.x + a.y * o.y + a.z * o.z + a.w * o.w);
  if (lane == 0) D[row] = v;
}

// dK / dV: one 4-wave workgroup per (sample, pair of key tiles); wave
// (kk, half) = (w >> 1, w & 1) owns columns [128 half, +128) of dKr and dV
// for key tile 2 j + kk.  Per query tile the pair splits the recompute: wave
// half 0 forms S = Qr Kr^T, half 1 dP = dO V^T (16 MFMAs each instead of 32,
// and each holds only its own key tile's fragments), and they swap the
// 32 x 32 results through LDS.  The Qr and dO tiles of each query tile are
// DMA-staged once for the four waves (double buffer).  LDS: Kr and V images
// of both key tiles [0, 4 IMG), then 2 stages x (Qr, dO) [4 IMG, 8 IMG),
// then lse / D, then the S / dP exchange [4 waves][16][64] fp32.
constexpr int KV_XCH = 8 * IMG + 2 * 32 * AT * 4;
constexpr int KV_LDS = KV_XCH + 4 * 16 * 64 * 4;

__global__ __launch_bounds__(256) void attn_bwd_kv_kernel(
    const uint16_t* __restrict__ Qp, const uint16_t* __restrict__ Kp,
    const uint16_t* __restrict__ Vp, long long ld, long long sb, int hw, float scale,
    const uint16_t* __restrict__ dOb, const float* __restrict__ lse, const float* __restrict__ D,
    uint16_t* __restrict__ dK, uint16_t* __restrict__ dV, long long ldg, long long sbg,
    uint16_t* __restrict__ dS) {
  const int tid = threadIdx.x, w = tid / WAVE, lane = tid % WAVE, lr = lane & 31, h = lane >> 5;
  const int nt = (hw + 31) / 32, kp = 32 * nt, np = (nt + 1) / 2;
  const int wid = xcd_remap(blockIdx.x, gridDim.x);
  const int b = wid / np, kk = w >> 1, half = w & 1, kt = 2 * (wid % np) + kk;
  const uint16_t* Qb = Qp + b * sb;
  const uint16_t* dOs = dOb + (long long)b * hw * AD;
  const uint32_t KI = kk * 2 * IMG, VI = KI + IMG, ST = 4 * IMG, LS = 8 * IMG;
  const int key = 32 * kt + lr;
  const bool kv = key < hw;

  // Kr / V tiles of both key tiles (wave w: tile w >> 1, Kr if w even), then
  // query-tile stage 0
  dma_tile((half ? Vp : Kp) + b * sb, ld, 32 * kt, kt < nt ? hw : 0, KI + half * IMG, 0, 1, lane);
  auto issue = [&](int qt) {
    const uint32_t base = ST + (qt & 1) * 2 * IMG;
    dma_tile(Qb, ld, 32 * qt, hw, base, w, 4, lane);
    dma_tile(dOs, AD, 32 * qt, hw, base + IMG, w, 4, lane);
  };
  issue(0);
  for (int i = tid; i < 32 * nt; i += 256) {
    lds_stf(LS + i * 4, i < hw ? lse[(long long)b * hw + i] : 0.f);
    lds_stf(LS + (32 * AT + i) * 4, i < hw ? D[(long long)b * hw + i] : 0.f);
  }
  f32x16 dk[4], dv[4];
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) dk[t][r] = dv[t][r] = 0.f;
  // this wave's operand fragments (Kr for half 0, V for half 1), held for
  // the whole loop
  bf16x8 kf[AD / 16];

  for (int qt = 0; qt < nt; ++qt) {
    // every outstanding op of this wave is this stage's DMA or older
    ring_barrier<0>();
    if (qt == 0) {
#pragma unroll
      for (int s = 0; s < AD / 16; ++s) kf[s] = frag(half ? VI : KI, s, lane);
    }
    if (qt + 1 < nt) issue(qt + 1);
    const uint32_t QI = ST + (qt & 1) * 2 * IMG, OI = QI + IMG;
    // half 0: S = Qr Kr^T; half 1: dP = dO V^T; then swap with the partner
    f32x16 acc0, acc1;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc0[r] = acc1[r] = 0.f;
    const uint32_t AI = half ? OI : QI;
#pragma unroll
    for (int s = 0; s < AD / 16; s += 2) {     // two chains: half the dependent latency
      acc0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(frag(AI, s, lane), kf[s], acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(frag(AI, s + 1, lane), kf[s + 1], acc1, 0,
                                                     0, 0);
    }
    f32x16 sacc, pacc;
    {
      const uint32_t mine = KV_XCH + (uint32_t)(w * 16 * 64 + lane) * 4;
      const uint32_t other = KV_XCH + (uint32_t)((w ^ 1) * 16 * 64 + lane) * 4;
      f32x16 own;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        own[r] = acc0[r] + acc1[r];
        lds_stf(mine + r * 64 * 4, own[r]);
      }
      __syncthreads();
      f32x16 par;
#pragma unroll
      for (int r = 0; r < 16; ++r) par[r] = lds_ldf(other + r * 64 * 4);
      sacc = half ? par : own;
      pacc = half ? own : par;
    }
    // lane: key column; register r: query 32 qt + acc_row(r, h)
    float pv[16], ds[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int qq = 32 * qt + acc_row(r, h);
      const bool ok = kv && qq < hw;
      const float l = lds_ldf(LS + qq * 4), dd = lds_ldf(LS + (32 * AT + qq) * 4);
      pv[r] = ok ? __builtin_amdgcn_exp2f((sacc[r] * scale - l) * 1.4426950408889634f) : 0.f;
      ds[r] = pv[r] * (pacc[r] - dd) * scale;
    }
    if (half == 0 && kt < nt) {
      uint16_t* dsb = dS + ((long long)b * hw) * kp;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int qq = 32 * qt + acc_row(r, h);
        if (qq < hw) dsb[(long long)qq * kp + key] = bf_bits(ds[r]);
      }
    }
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      uint32_t up[4], us[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        up[j] = pk_bf16(pv[8 * s2 + 2 * j], pv[8 * s2 + 2 * j + 1]);
        us[j] = pk_bf16(ds[8 * s2 + 2 * j], ds[8 * s2 + 2 * j + 1]);
      }
      const bf16x8 pa = as_bf8(make_uint4(up[0], up[1], up[2], up[3]));
      const bf16x8 sa = as_bf8(make_uint4(us[0], us[1], us[2], us[3]));
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int c0 = 128 * half + 32 * t;
        const bf16x8 obf = trf(OI, 16 * s2 + 4 * h, 16 * s2 + 8 + 4 * h, c0, lane);
        const bf16x8 qbf = trf(QI, 16 * s2 + 4 * h, 16 * s2 + 8 + 4 * h, c0, lane);
        dv[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(pa, obf, dv[t], 0, 0, 0);
        dk[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(sa, qbf, dk[t], 0, 0, 0);
      }
    }
  }
  if (kt >= nt) return;
  // lane: column 128 half + 32 t + lr; register r: key 32 kt + acc_row(r, h)
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int kq = 32 * kt + acc_row(r, h);
      if (kq < hw) {
        const long long o = b * sbg + (long long)kq * ldg + 128 * half + 32 * t + lr;
        dK[o] = bf_bits(dk[t][r]);
        dV[o] = bf_bits(dv[t][r]);
      }
    }
}

// dQr = dS Kr: one 4-wave workgroup per (sample, pair of query tiles); wave w
// computes query tile 2 j + (w & 1), output columns [128 (w >> 1), +128) -- all
// four SIMDs busy (the 2-wave version, one query tile per wave, left two idle)
// and half the MFMA chain per wave.  All the sample's Kr tiles are DMA-staged
// at once (7 x 16 KiB), together with each query tile's dS rows (staged by
// its two waves, 464-B rows: conflict-free ds_read_b128).
constexpr int Q_NS = 7;
constexpr int DS_PITCH = 464;
constexpr int Q_LDS = Q_NS * IMG + 2 * 32 * DS_PITCH;

static_assert(Q_NS >= AT, "attn_bwd_q stages every key tile of a sample at once");

__global__ __launch_bounds__(256) void attn_bwd_q_kernel(const uint16_t* __restrict__ Kp,
                                                         long long ld, long long sb, int hw,
                                                         const uint16_t* __restrict__ dS,
                                                         uint16_t* __restrict__ dQ, long long ldg,
                                                         long long sbg) {
  const int tid = threadIdx.x, w = tid / WAVE, lane = tid % WAVE, lr = lane & 31, h = lane >> 5;
  const int qsel = w & 1, dh = w >> 1;
  const int nt = (hw + 31) / 32, kp = 32 * nt, np = (nt + 1) / 2;
  const int wid = xcd_remap(blockIdx.x, gridDim.x);
  const int b = wid / np, qt = 2 * (wid % np) + qsel;
  const uint16_t* Kb = Kp + b * sb;
  const uint32_t dsimg = Q_NS * IMG + qsel * 32 * DS_PITCH;
  // every Kr tile (nt <= AT = Q_NS: the whole sample fits) goes out by DMA
  // first, then the query tile's 32 dS rows (kp bf16 each) -> LDS, half by
  // each of its two waves, with plain loads: both in ONE memory round (the
  // dS stores wait for their loads, the youngest, so every DMA piece has
  // landed too); one barrier then publishes all of it
  for (int st = 0; st < nt; ++st) dma_tile(Kb, ld, 32 * st, hw, st * IMG, w, 4, lane);
  for (int i = lane + 64 * dh; i < 32 * (kp / 8); i += 128) {
    const int r = i / (kp / 8), c8 = i % (kp / 8), q = 32 * qt + r;
    const uint4 v = q < hw ? *(const uint4*)(dS + ((long long)b * hw + q) * kp + 8 * c8)
                           : make_uint4(0, 0, 0, 0);
    lds_st16(dsimg + r * DS_PITCH + 16 * c8, v);
  }
  ring_barrier<0>();
  constexpr int NTD = AD / 32 / 2;                   // d tiles per wave
  f32x16 acc[NTD];
#pragma unroll
  for (int t = 0; t < NTD; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;
  for (int kt = 0; kt < nt; ++kt) {
    const uint32_t buf = kt * IMG;
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      const bf16x8 a = as_bf8(lds_ld16(dsimg + lr * DS_PITCH + 2 * (32 * kt + 16 * s2 + 8 * h)));
#pragma unroll
      for (int t = 0; t < NTD; ++t) {
        const bf16x8 kb =
            trf(buf, 16 * s2 + 8 * h, 16 * s2 + 8 * h + 4, 32 * (NTD * dh + t), lane);
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, kb, acc[t], 0, 0, 0);
      }
    }
  }
  if (qt >= nt) return;
#pragma unroll
  for (int t = 0; t < NTD; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int qq = 32 * qt + acc_row(r, h);
      if (qq < hw)
        dQ[b * sbg + (long long)qq * ldg + 32 * (NTD * dh + t) + lr] = bf_bits(acc[t][r]);
    }
}

// ------------------------------------------- fused small (FCFM, HW <= 64) ---
// One 8-wave workgroup per sample holds the whole problem in LDS (fp32, row
// pitch width + 1): FCFM's cross-attention is HW = 36 positions x C' = C = 36
// channels (fusion_nets.py:217-258 -> SelfAttention(36, scale=1)), a few
// tens of KB per sample, so QK^T, the softmax, PV and the five backward
// products run back to back in one launch each way.  The products run on
// v_mfma_f32_16x16x4_f32 (fp32 operands: exact fp32 products and sums, the
// same as an fmaf chain), one 16x16 output tile per wave at a time, operands
// read straight from LDS with (row, k) strides (so transposed operands need
// no copy).  Every operand is loaded from HBM in one batch per thread (all
// loads in flight before the first LDS store).  P [B][hw][hw] is saved for
// the backward.
constexpr int SM_MAX_HW = 64;
constexpr int SNT = 576;                 // threads per workgroup: 9 waves, one per
                                         // 16x16 tile of a 36 x 36 product
constexpr int SLD = (64 * 64 + SNT - 1) / SNT;   // max elements per thread per operand

// out(m, n) = sum_k A(m, k) B(n, k), A(m, k) = A[m am + k ak], B likewise;
// 16x16 tiles dealt to the waves round robin starting at wave w0.
template <typename Store>
__device__ __forceinline__ void small_product(const float* A, int am, int ak, const float* Bm,
                                              int bn, int bk, int M, int N, int K, int w0,
                                              Store st) {
  const int w = threadIdx.x / WAVE, lane = threadIdx.x % WAVE;
  const int li = lane & 15, lk = lane >> 4;
  const int mt = (M + 15) / 16, nt = (N + 15) / 16;
  for (int t = (w - w0 + SNT / WAVE) % (SNT / WAVE); t < mt * nt; t += SNT / WAVE) {
    const int m = 16 * (t / nt) + li, n = 16 * (t % nt) + li;
    const float* a = A + m * am + lk * ak;
    const float* b = Bm + n * bn + lk * bk;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 3
    for (int k = 0; k < K; k += 4) {
      const bool kin = k + lk < K;
      const float av = kin && m < M ? a[k * ak] : 0.f;
      const float bv = kin && n < N ? b[k * bk] : 0.f;
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc, 0, 0, 0);
    }
    const int col = 16 * (t % nt) + li;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = 16 * (t / nt) + 4 * lk + r;
      if (row < M && col < N) st(row, col, acc[r]);
    }
  }
}

struct SmallOp {
  float* dst;
  int ld;
  const float* src;
  long long sr;
  int rows, cols;
};

// dst[r ld + k] = src[r sr + k] for every operand, all HBM loads issued
// before the first LDS store
template <int NOP>
__device__ __forceinline__ void small_load(const SmallOp (&op)[NOP]) {
  float v[NOP][SLD];
  int r0[NOP], c0[NOP];
#pragma unroll
  for (int o = 0; o < NOP; ++o) {
    const int cols = op[o].cols, total = op[o].rows * cols;
    const int dr = SNT / cols, dc = SNT - dr * cols;
    int r = threadIdx.x / cols, c = threadIdx.x - r * cols;
    r0[o] = r;
    c0[o] = c;
#pragma unroll
    for (int u = 0; u < SLD; ++u) {
      v[o][u] = (int)threadIdx.x + u * SNT < total ? op[o].src[r * op[o].sr + c] : 0.f;
      r += dr;
      c += dc;
      if (c >= cols) {
        c -= cols;
        ++r;
      }
    }
  }
#pragma unroll
  for (int o = 0; o < NOP; ++o) {
    const int cols = op[o].cols, total = op[o].rows * cols;
    const int dr = SNT / cols, dc = SNT - dr * cols;
    int r = r0[o], c = c0[o];
#pragma unroll
    for (int u = 0; u < SLD; ++u) {
      if ((int)threadIdx.x + u * SNT < total) op[o].dst[r * op[o].ld + c] = v[o][u];
      r += dr;
      c += dc;
      if (c >= cols) {
        c -= cols;
        ++r;
      }
    }
  }
}

// dst[r sd + k] = src[r ld + k] (LDS -> HBM, coalesced over the whole group)
__device__ __forceinline__ void small_store(float* dst, long long sd, const float* src, int ld,
                                            int rows, int cols) {
  const int total = rows * cols, dr = SNT / cols, dc = SNT - dr * cols;
  int r = threadIdx.x / cols, c = threadIdx.x - r * cols;
  for (int idx = threadIdx.x; idx < total; idx += SNT) {
    dst[r * sd + c] = src[r * ld + c];
    r += dr;
    c += dc;
    if (c >= cols) {
      c -= cols;
      ++r;
    }
  }
}

__global__ __launch_bounds__(SNT) void attn_small_fwd_kernel(
    const float* __restrict__ X, long long sxn, long long sxr, const float* __restrict__ Y,
    long long syn, long long syr, int hw, int cq, int ck, int cv, int c, float scale,
    float* __restrict__ O, long long son, long long sor, float* __restrict__ P) {
  extern __shared__ float sm[];
  const int lq = cq + 1, lv = c + 1, lp = hw + 1;
  float* sQ = sm;
  float* sK = sQ + hw * lq;
  float* sV = sK + hw * lq;
  float* sP = sV + hw * lv;
  const long long n = blockIdx.x;
  const float* x = X + n * sxn;
  const SmallOp ops[3] = {{sQ, lq, x, sxr, hw, cq},
                          {sK, lq, Y + n * syn + ck, syr, hw, cq},
                          {sV, lv, x + cv, sxr, hw, c}};
  small_load(ops);
  __syncthreads();
  small_product(sQ, lq, 1, sK, lq, 1, hw, hw, cq, 0,
                [&](int i, int j, float v) { sP[i * lp + j] = v * scale; });
  __syncthreads();
  // softmax: 16 lanes per row (one DPP row), up to 4 keys per lane
  for (int i = threadIdx.x / 16; i < hw; i += SNT / 16) {
    float* row = sP + i * lp;
    const int j0 = threadIdx.x % 16;
    float v[SM_MAX_HW / 16];
    float m = -INFINITY;
#pragma unroll
    for (int u = 0; u < SM_MAX_HW / 16; ++u) {
      v[u] = j0 + 16 * u < hw ? row[j0 + 16 * u] : -INFINITY;
      m = fmaxf(m, v[u]);
    }
    m = row16_max(m);
    float sum = 0.f;
#pragma unroll
    for (int u = 0; u < SM_MAX_HW / 16; ++u) {
      v[u] = __expf(v[u] - m);
      sum += v[u];
    }
    const float inv = 1.f / row16_sum(sum);
#pragma unroll
    for (int u = 0; u < SM_MAX_HW / 16; ++u)
      if (j0 + 16 * u < hw) row[j0 + 16 * u] = v[u] * inv;
  }
  __syncthreads();
  small_store(P + n * hw * hw, hw, sP, lp, hw, hw);
  float* o = O + n * son;
  small_product(sP, lp, 1, sV, 1, lv, hw, c, hw, 0,
                [&](int i, int cc, float v) { o[i * sor + cc] = v; });
}

// dP = dO V^T, dS = scale P (dP - rowsum(P dP)), dQ = dS K, dK = dS^T Q,
// dV = P^T dO; dQ / dV into dX's columns [0, cq) / [cv, cv + c), dK into dY's
// [ck, ck + cq) (dY = dX for self-attention).
__global__ __launch_bounds__(SNT) void attn_small_bwd_kernel(
    const float* __restrict__ X, long long sxn, long long sxr, const float* __restrict__ Y,
    long long syn, long long syr, int hw, int cq, int ck, int cv, int c, float scale,
    const float* __restrict__ P, const float* __restrict__ dO, long long sdn, long long sdr,
    float* dX, long long sgn, long long sgr, float* dY, long long skn, long long skr) {
  extern __shared__ float sm[];
  const int lq = cq + 1, lv = c + 1, lp = hw + 1;
  float* sQ = sm;
  float* sK = sQ + hw * lq;
  float* sV = sK + hw * lq;
  float* sO = sV + hw * lv;
  float* sP = sO + hw * lv;
  float* sS = sP + hw * lp;
  const long long n = blockIdx.x;
  const float* x = X + n * sxn;
  const SmallOp ops[5] = {{sQ, lq, x, sxr, hw, cq},
                          {sK, lq, Y + n * syn + ck, syr, hw, cq},
                          {sV, lv, x + cv, sxr, hw, c},
                          {sO, lv, dO + n * sdn, sdr, hw, c},
                          {sP, lp, P + n * hw * hw, hw, hw, hw}};
  small_load(ops);
  __syncthreads();
  small_product(sO, lv, 1, sV, lv, 1, hw, hw, c, 0,
                [&](int i, int j, float v) { sS[i * lp + j] = v; });
  __syncthreads();
  for (int i = threadIdx.x / 16; i < hw; i += SNT / 16) {   // 16 lanes per row
    const float* pr = sP + i * lp;
    float* sr = sS + i * lp;
    const int j0 = threadIdx.x % 16;
    float p[SM_MAX_HW / 16], dp[SM_MAX_HW / 16];
    float dot = 0.f;
#pragma unroll
    for (int u = 0; u < SM_MAX_HW / 16; ++u) {
      const bool in = j0 + 16 * u < hw;
      p[u] = in ? pr[j0 + 16 * u] : 0.f;
      dp[u] = in ? sr[j0 + 16 * u] : 0.f;
      dot = fmaf(p[u], dp[u], dot);
    }
    dot = row16_sum(dot);
#pragma unroll
    for (int u = 0; u < SM_MAX_HW / 16; ++u)
      if (j0 + 16 * u < hw) sr[j0 + 16 * u] = scale * p[u] * (dp[u] - dot);
  }
  __syncthreads();
  float* gx = dX + n * sgn;
  float* gy = dY + n * skn + ck;
  // the three products' tiles continue each other's round robin over the waves
  const int tq = ((hw + 15) / 16) * ((cq + 15) / 16);
  small_product(sS, lp, 1, sK, 1, lq, hw, cq, hw, 0,
                [&](int i, int k, float v) { gx[i * sgr + k] = v; });
  small_product(sS, 1, lp, sQ, 1, lq, hw, cq, hw, tq % (SNT / WAVE),
                [&](int j, int k, float v) { gy[j * skr + k] = v; });
  small_product(sP, 1, lp, sO, 1, lv, hw, c, hw, (2 * tq) % (SNT / WAVE),
                [&](int j, int cc, float v) { gx[j * sgr + cv + cc] = v; });
}

}  // namespace

extern "C" {

int tgfr_attn_softmax(const float* S, float* P, float* lse, long long rows, int n, long long ld,
                      float scale, void* stream) {
  if (rows <= 0 || n <= 0) return 1001;
  hipLaunchKernelGGL(attn_softmax_kernel, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0,
                     (hipStream_t)stream, S, P, lse, rows, n, ld, scale);
  return (int)hipGetLastError();
}

int tgfr_attn_softmax_bwd(const float* P, const float* dP, float* dS, long long rows, int n,
                          long long ld, float scale, void* stream) {
  if (rows <= 0 || n <= 0) return 1001;
  hipLaunchKernelGGL(attn_softmax_bwd_kernel, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0,
                     (hipStream_t)stream, P, dP, dS, rows, n, ld, scale);
  return (int)hipGetLastError();
}

// Fused IMIM self-attention (bf16 operands, fp32 accumulate): Qr, Kr, V are
// [B][hw][256] bf16 views (row stride ld, sample stride sb, 16-B aligned
// rows) -- the column slices of the packed projection; O [B][hw][256] fp32
// (ldo, sbo); lse [B*hw].
int tgfr_attn_fwd(const uint16_t* Q, const uint16_t* K, const uint16_t* V, long long ld,
                  long long sb, int B, int hw, float scale, float* O, long long ldo,
                  long long sbo, float* lse, void* stream) {
  if (B <= 0 || hw <= 0 || hw > 32 * AT || (ld & 7) || (sb & 7) || (ldo & 3)) return 1001;
  if (((uintptr_t)Q | (uintptr_t)K | (uintptr_t)V | (uintptr_t)O) & 15) return 1001;
  const int np = ((hw + 31) / 32 + 1) / 2;
  if (const int e = set_max_lds((const void*)attn_fwd_kernel, FWD_LDS)) return e;
  hipLaunchKernelGGL(attn_fwd_kernel, dim3(B * np), dim3(256), FWD_LDS, (hipStream_t)stream, Q, K,
                     V, ld, sb, hw, scale, O, ldo, sbo, lse, nullptr, 0);
  return (int)hipGetLastError();
}

// tgfr_attn_fwd that also leaves, for the LayerNorm([256, H, W]) that follows
// (tgfr_ln_tail_fwd_att), each 32-query tile's moments [B][ceil(hw/32)][2] at
// the start of ln_ws (the tgfr_ln_tail_ws buffer): no separate statistics pass.
int tgfr_attn_fwd_ln(const uint16_t* Q, const uint16_t* K, const uint16_t* V, long long ld,
                     long long sb, int B, int hw, float scale, float* O, float* lse,
                     float* ln_ws, void* stream) {
  if (B <= 0 || hw <= 0 || hw > 32 * AT || (ld & 7) || (sb & 7) || !ln_ws) return 1001;
  if (((uintptr_t)Q | (uintptr_t)K | (uintptr_t)V | (uintptr_t)O) & 15) return 1001;
  const int nt = (hw + 31) / 32, np = (nt + 1) / 2;
  if (const int e = set_max_lds((const void*)attn_fwd_kernel, FWD_LDS)) return e;
  hipLaunchKernelGGL(attn_fwd_kernel, dim3(B * np), dim3(256), FWD_LDS, (hipStream_t)stream, Q, K,
                     V, ld, sb, hw, scale, O, (long long)AD, (long long)hw * AD, lse, ln_ws, nt);
  return (int)hipGetLastError();
}

int tgfr_attn_bwd_ws(int B, int hw, long long* bytes) {
  if (B <= 0 || hw <= 0 || !bytes) return 1001;
  const long long rows = (long long)B * hw, kp = 32LL * ((hw + 31) / 32);
  // D (fp32), dO (bf16), dS (bf16), each 16-B aligned
  *bytes = (rows * 4 + 15) / 16 * 16 + rows * AD * 2 + rows * kp * 2;
  return 0;
}

// Gradients into dQ / dK / dV [B][hw][256] bf16 (ldg, sbg; typically the
// column slices of one packed [B][hw][768] gradient -- the operand of the
// projection's weight-gradient GEMM), overwritten.  O and dO dense fp32
// [B][hw][256].
int tgfr_attn_bwd(const uint16_t* Q, const uint16_t* K, const uint16_t* V, long long ld,
                  long long sb, int B, int hw, float scale, const float* O, const float* dO,
                  long long ldo, long long sbo, const float* lse, uint16_t* dQ, uint16_t* dK,
                  uint16_t* dV, long long ldg, long long sbg, void* ws, void* stream) {
  if (B <= 0 || hw <= 0 || hw > 32 * AT || (ld & 7) || (sb & 7) || !ws) return 1001;
  if (ldo != AD || sbo != (long long)hw * AD) return 1001;     // dO / O dense rows
  if (((uintptr_t)Q | (uintptr_t)K | (uintptr_t)V | (uintptr_t)O | (uintptr_t)dO |
       (uintptr_t)ws) & 15)
    return 1001;
  const int nt = (hw + 31) / 32, np = (nt + 1) / 2;
  auto* s = (hipStream_t)stream;
  const long long rows = (long long)B * hw;
  float* D = (float*)ws;
  auto* dOb = (uint16_t*)((char*)ws + (rows * 4 + 15) / 16 * 16);
  uint16_t* dS = dOb + rows * AD;
  hipLaunchKernelGGL(attn_bwd_prep_kernel, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, s, dO,
                     O, (long long)AD, rows, D, dOb);
  if (const int e = set_max_lds((const void*)attn_bwd_kv_kernel, KV_LDS)) return e;
  hipLaunchKernelGGL(attn_bwd_kv_kernel, dim3(B * np), dim3(256), KV_LDS, s, Q, K, V, ld, sb, hw,
                     scale, dOb, lse, D, dK, dV, ldg, sbg, dS);
  if (const int e = set_max_lds((const void*)attn_bwd_q_kernel, Q_LDS)) return e;
  hipLaunchKernelGGL(attn_bwd_q_kernel, dim3(B * np), dim3(256), Q_LDS, s, K, ld, sb, hw, dS, dQ,
                     ldg, sbg);
  return (int)hipGetLastError();
}

// tgfr_attn_bwd with its prep pass already done by the caller: ws holds D
// [rows] and dO [rows][256] bf16 in tgfr_attn_bwd's layout (the IMIM LayerNorm
// backward writes them, tgfr_ln_tail_bwd_att).
int tgfr_attn_bwd_prepped(const uint16_t* Q, const uint16_t* K, const uint16_t* V, long long ld,
                          long long sb, int B, int hw, float scale, const float* lse,
                          uint16_t* dQ, uint16_t* dK, uint16_t* dV, long long ldg, long long sbg,
                          void* ws, void* stream) {
  if (B <= 0 || hw <= 0 || hw > 32 * AT || (ld & 7) || (sb & 7) || !ws) return 1001;
  if (((uintptr_t)Q | (uintptr_t)K | (uintptr_t)V | (uintptr_t)ws) & 15) return 1001;
  const int nt = (hw + 31) / 32, np = (nt + 1) / 2;
  auto* s = (hipStream_t)stream;
  const long long rows = (long long)B * hw;
  const float* D = (const float*)ws;
  auto* dOb = (const uint16_t*)((char*)ws + (rows * 4 + 15) / 16 * 16);
  uint16_t* dS = (uint16_t*)dOb + rows * AD;
  if (const int e = set_max_lds((const void*)attn_bwd_kv_kernel, KV_LDS)) return e;
  hipLaunchKernelGGL(attn_bwd_kv_kernel, dim3(B * np), dim3(256), KV_LDS, s, Q, K, V, ld, sb, hw,
                     scale, dOb, lse, D, dK, dV, ldg, sbg, dS);
  if (const int e = set_max_lds((const void*)attn_bwd_q_kernel, Q_LDS)) return e;
  hipLaunchKernelGGL(attn_bwd_q_kernel, dim3(B * np), dim3(256), Q_LDS, s, K, ld, sb, hw, dS, dQ,
                     ldg, sbg);
  return (int)hipGetLastError();
}

static int small_check(int B, int hw, int cq, int ck, int cv, int c) {
  if (B <= 0 || hw <= 0 || hw > SM_MAX_HW || cq <= 0 || cq > SM_MAX_HW || c <= 0 ||
      c > SM_MAX_HW || ck < 0 || cv < 0)
    return 1001;
  return 0;
}

// FCFM-sized fused attention (HW <= 64): X [B][hw][*] fp32 rows holding Qr
// at columns [0, cq) and V at [cv, cv + c); Y (NULL = X) holding Kr at
// [ck, ck + cq).  O [B][hw][c] (son, sor); P [B][hw][hw] dense, written.
int tgfr_attn_small_fwd(const float* X, long long sxn, long long sxr, const float* Y,
                        long long syn, long long syr, int B, int hw, int cq, int ck, int cv,
                        int c, float scale, float* O, long long son, long long sor, float* P,
                        void* stream) {
  if (const int e = small_check(B, hw, cq, ck, cv, c)) return e;
  if (!X || !O || !P) return 1001;
  if (!Y) {
    Y = X;
    syn = sxn;
    syr = sxr;
  }
  const int lds = 4 * (2 * hw * (cq + 1) + hw * (c + 1) + hw * (hw + 1));
  if (lds > 160 * 1024) return 1001;
  if (const int e = set_max_lds((const void*)attn_small_fwd_kernel, lds)) return e;
  hipLaunchKernelGGL(attn_small_fwd_kernel, dim3(B), dim3(SNT), lds, (hipStream_t)stream, X, sxn,
                     sxr, Y, syn, syr, hw, cq, ck, cv, c, scale, O, son, sor, P);
  return (int)hipGetLastError();
}

// Its backward: dO [B][hw][c] (sdn, sdr); dQr / dV overwrite dX's columns
// [0, cq) / [cv, cv + c), dKr overwrites dY's [ck, ck + cq) (dY NULL = dX:
// the three column ranges must then be disjoint).
int tgfr_attn_small_bwd(const float* X, long long sxn, long long sxr, const float* Y,
                        long long syn, long long syr, int B, int hw, int cq, int ck, int cv,
                        int c, float scale, const float* P, const float* dO, long long sdn,
                        long long sdr, float* dX, long long sgn, long long sgr, float* dY,
                        long long skn, long long skr, void* stream) {
  if (const int e = small_check(B, hw, cq, ck, cv, c)) return e;
  if (!X || !P || !dO || !dX) return 1001;
  if (!Y) {
    Y = X;
    syn = sxn;
    syr = sxr;
  }
  if (!dY) {
    const bool qk = ck < cq;                                    // [0,cq) vs [ck,ck+cq)
    const bool qv = cv < cq;                                    // [0,cq) vs [cv,cv+c)
    const bool kv = ck < cv + c && cv < ck + cq;                // [ck,..) vs [cv,..)
    if (qk || qv || kv) return 1001;
    dY = dX;
    skn = sgn;
    skr = sgr;
  } else if (cv < cq) {
    return 1001;
  }
  const int lds = 4 * (2 * hw * (cq + 1) + 2 * hw * (c + 1) + 2 * hw * (hw + 1));
  if (lds > 160 * 1024) return 1001;
  if (const int e = set_max_lds((const void*)attn_small_bwd_kernel, lds)) return e;
  hipLaunchKernelGGL(attn_small_bwd_kernel, dim3(B), dim3(SNT), lds, (hipStream_t)stream, X, sxn,
                     sxr, Y, syn, syr, hw, cq, ck, cv, c, scale, P, dO, sdn, sdr, dX, sgn, sgr,
                     dY, skn, skr);
  return (int)hipGetLastError();
}

}  // extern "C"
