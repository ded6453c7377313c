// SelfAttention core (models/fusion_nets.py:82-118) for gfx950.
//
// The reference computes, per sample n, with x the image and y the text side:
//   Qr = key_proj(x)^T [HW, C'],  Kr = query_proj(y)^T [HW, C'],  V = value_proj(x)^T [HW, C]
//   P  = softmax_j(Qr Kr^T / sqrt_dim)                  (:103-106)
//   O  = P V  -> permuted to [C, HW]                      (:115-117)
// The 1x1 projections are plain GEMMs (host side); this file holds the core:
//   bgemm          batched C = alpha A B (+C) on v_mfma_f32_32x32x16_bf16, any
//                  element strides (so every transpose of the backward is a
//                  stride swap, never a copy); fp32-split or bf16 operands.
//   attn_softmax   P = softmax(scale * S) per row over the valid keys + row LSE.
//   attn_softmax_bwd  dS = scale * P (dP - rowsum(P dP)).
// The attention matrices are HW x HW per sample (196^2 fp32 = 150 KB for IMIM,
// 36^2 for FCFM), so they are materialised instead of recomputed.
#include "tgfr_common.h"

using namespace tgfr;

namespace {

constexpr int BM = 64, BN = 64, BK = 32;
constexpr int HALF = 64 * 64;                 // bytes of one 64x32 bf16 tile
constexpr int STAGE = 4 * HALF;               // A hi, A lo, B hi, B lo

// Operand layouts: LAY_K = k-contiguous (unit k stride), LAY_MN = m- (or n-)
// contiguous, LAY_ANY = neither (scalar gathers).  Each layout is staged in
// the LDS layout its global reads coalesce into:
//   LAY_K / LAY_ANY  [64 mn][32 k]  64-B rows, read with ds_read_b128
//   LAY_MN           [32 k][64 mn] 128-B rows, read with ds_read_b64_tr_b16
// so a transposed operand costs neither a copy nor uncoalesced loads.
enum { LAY_K = 0, LAY_MN = 1, LAY_ANY = 2 };

// Split-K partial tiles are combined in-launch by the last-arriving slice only
// while the serial slab read stays small (<= 4 x 16 KB per tile); beyond that a
// chip-wide reduce launch is cheaper.
constexpr int KSPLIT_INLAUNCH = 4;

// [64 mn][32 k]: 16-B chunk swizzle keeps ds_read_b128 lane groups conflict-free.
__device__ __forceinline__ uint32_t toff(int row, int chunk) {
  return row * 64 + ((chunk ^ ((row >> 2) & 3)) << 4);
}
// [32 k][64 mn]: rows 2 apart land 64 B apart, so the 4 rows of one
// transposed read hit disjoint banks.
__device__ __forceinline__ uint32_t moff(int krow, int chunk) {
  return krow * 128 + ((chunk ^ (((krow >> 1) & 1) << 2)) << 4);
}

struct Frag8 {
  float v[8];
};

// Staging role of thread tid for one 64x32 operand tile:
//   LAY_K/ANY: mn row tid/4, k 8*(tid%4) .. +7
//   LAY_MN:    k row tid/8,  mn 8*(tid%8) .. +7
template <int LAY>
__device__ __forceinline__ void load_tile(Frag8& f, const float* base, long long s_mn,
                                          long long s_k, int tid, int k0, int mn_lim, int K) {
  if constexpr (LAY == LAY_MN) {
    const int k = k0 + (tid >> 3), mn = (tid & 7) * 8;
    const float* p = base + (long long)k * s_k + mn;
    if (k < K && mn + 8 <= mn_lim && (((uintptr_t)p & 15) == 0)) {
      const float4 a = *(const float4*)p;
      const float4 b = *(const float4*)(p + 4);
      f.v[0] = a.x; f.v[1] = a.y; f.v[2] = a.z; f.v[3] = a.w;
      f.v[4] = b.x; f.v[5] = b.y; f.v[6] = b.z; f.v[7] = b.w;
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) f.v[e] = (k < K && mn + e < mn_lim) ? p[e] : 0.f;
    }
  } else {
    const int row = tid >> 2, k = k0 + (tid & 3) * 8;
    const float* p = base + (long long)row * s_mn + (long long)k * s_k;
    if (LAY == LAY_K && row < mn_lim && k + 8 <= K && (((uintptr_t)p & 15) == 0)) {
      const float4 a = *(const float4*)p;
      const float4 b = *(const float4*)(p + 4);
      f.v[0] = a.x; f.v[1] = a.y; f.v[2] = a.z; f.v[3] = a.w;
      f.v[4] = b.x; f.v[5] = b.y; f.v[6] = b.z; f.v[7] = b.w;
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e)
        f.v[e] = (row < mn_lim && k + e < K) ? p[(long long)e * s_k] : 0.f;
    }
  }
}

template <int MODE, int LAY>
__device__ __forceinline__ void store_tile(uint32_t base, const Frag8& f, int tid) {
  bf16x8 hi, lo;
  frag8<MODE>(f.v, hi, lo);
  const uint32_t off =
      base + (LAY == LAY_MN ? moff(tid >> 3, tid & 7) : toff(tid >> 2, tid & 3));
  lds_st16(off, __builtin_bit_cast(uint4, hi));
  if (MODE == MODE_SPLIT) lds_st16(off + HALF, __builtin_bit_cast(uint4, lo));
}

// MFMA operand fragment: lane (lr, h) gets element [mn = mn0 + lr][k = 16 s + 8 h .. +7].
template <int LAY>
__device__ __forceinline__ bf16x8 frag_read(uint32_t base, int mn0, int s, int lane) {
  if constexpr (LAY == LAY_MN) {
    // 16-lane group g: mn block 16 (g & 1), k rows 16 s + 8 (g >> 1) (+4);
    // lane 4q+p addresses k row q, mn columns 4p .. 4p+3
    const int i = lane & 15, q = i >> 2, p = i & 3, g = lane >> 4;
    const int col = mn0 + 16 * (g & 1) + 4 * p;
    const int kr = 16 * s + 8 * (g >> 1) + q;
    const uint32_t a = base + moff(kr, col >> 3) + (col & 7) * 2;
    const uint32_t b = base + moff(kr + 4, col >> 3) + (col & 7) * 2;
    return join_tr(lds_tr4(a), lds_tr4(b));
  } else {
    return as_bf8(lds_ld16(base + toff(mn0 + (lane & 31), 2 * s + (lane >> 5))));
  }
}

template <int MODE, int LA, int LB>
__global__ __launch_bounds__(256) void bgemm_kernel(
    const float* __restrict__ A, long long sAb, long long sAm, long long sAk,
    const float* __restrict__ B, long long sBb, long long sBk, long long sBn,
    float* __restrict__ Cm, long long sCb, long long sCm, long long sCn, int M, int N, int Kfull,
    float alpha, int accumulate, const float* __restrict__ bias, int relu, int ksplit,
    float* __restrict__ slab, unsigned* __restrict__ counters) {
  const int n0 = blockIdx.x * BN, m0 = blockIdx.y * BM;
  const int bt = blockIdx.z / ksplit, kz = blockIdx.z % ksplit;
  // split-K: this block reduces k in [kb, kb + K) (possibly empty)
  const int kc = ((Kfull + ksplit - 1) / ksplit + BK - 1) / BK * BK;
  const int kb = kz * kc;
  const int K = max(0, min(Kfull - kb, kc));
  const int tid = threadIdx.x, wid = tid / WAVE, lane = tid % WAVE;
  const int lr = lane & 31, h = lane >> 5;
  const int wm = wid >> 1, wn = wid & 1;
  const float* Ab = A + bt * sAb + m0 * sAm + (long long)kb * sAk;
  const float* Bb = B + bt * sBb + n0 * sBn + (long long)kb * sBk;
  Frag8 fa, fb;
  f32x16 acc;
#pragma unroll
  for (int q = 0; q < 16; ++q) acc[q] = 0.f;

  const int nk = (K + BK - 1) / BK;
  if (nk > 0) {
    load_tile<LA>(fa, Ab, sAm, sAk, tid, 0, M - m0, K);
    load_tile<LB>(fb, Bb, sBn, sBk, tid, 0, N - n0, K);
    store_tile<MODE, LA>(0, fa, tid);
    store_tile<MODE, LB>(2 * HALF, fb, tid);
  }
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const uint32_t sb = (kt & 1) * STAGE;
    if (kt + 1 < nk) {
      load_tile<LA>(fa, Ab, sAm, sAk, tid, (kt + 1) * BK, M - m0, K);
      load_tile<LB>(fb, Bb, sBn, sBk, tid, (kt + 1) * BK, N - n0, K);
    }
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const bf16x8 ahi = frag_read<LA>(sb, 32 * wm, s, lane);
      const bf16x8 bhi = frag_read<LB>(sb + 2 * HALF, 32 * wn, s, lane);
      const bf16x8 alo = MODE == MODE_SPLIT ? frag_read<LA>(sb + HALF, 32 * wm, s, lane) : ahi;
      const bf16x8 blo =
          MODE == MODE_SPLIT ? frag_read<LB>(sb + 3 * HALF, 32 * wn, s, lane) : bhi;
      mma<MODE>(acc, ahi, alo, bhi, blo);
    }
    if (kt + 1 < nk) {
      const uint32_t nb = ((kt + 1) & 1) * STAGE;
      store_tile<MODE, LA>(nb, fa, tid);
      store_tile<MODE, LB>(nb + 2 * HALF, fb, tid);
    }
    __syncthreads();
  }
  if (ksplit > 1) {
    // every K slice stores its tile slab (lane-major, 64 B per lane); with few
    // slices the last arriving slice of the tile sums all slabs in slice order
    // (deterministic), otherwise bgemm_reduce_kernel does it chip-wide
    const long long tile = ((long long)bt * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x;
    float4* mine = (float4*)(slab + ((tile * ksplit + kz) * 256 + tid) * 16);
#pragma unroll
    for (int v = 0; v < 4; ++v)
      mine[v] = make_float4(acc[4 * v], acc[4 * v + 1], acc[4 * v + 2], acc[4 * v + 3]);
    if (ksplit > KSPLIT_INLAUNCH) return;
    if (!last_arrival(counters + tile, ksplit, (int*)(g_smem + 2 * STAGE))) return;
#pragma unroll
    for (int q = 0; q < 16; ++q) acc[q] = 0.f;
    for (int z = 0; z < ksplit; ++z) {
      const float4* src = (const float4*)(slab + ((tile * ksplit + z) * 256 + tid) * 16);
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const float4 t = src[v];
        acc[4 * v] += t.x; acc[4 * v + 1] += t.y; acc[4 * v + 2] += t.z; acc[4 * v + 3] += t.w;
      }
    }
  }
  const int n = n0 + 32 * wn + lr;
  if (n >= N) return;
  float* Cb = Cm + bt * sCb;
  const float bn = bias ? bias[n] : 0.f;
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int m = m0 + 32 * wm + acc_row(q, h);
    if (m < M) {
      float* o = Cb + m * sCm + n * sCn;
      float v = alpha * acc[q] + bn;
      if (accumulate) v += *o;
      *o = relu ? fmaxf(v, 0.f) : v;
    }
  }
}

// Chip-wide split-K combine: one thread per (tile, lane, 4-register group);
// slabs summed in slice order, then the bgemm epilogue.
__global__ __launch_bounds__(256) void bgemm_reduce_kernel(
    const float* __restrict__ slab, int ksplit, int mt, int nt, long long n_tiles, float* Cm,
    long long sCb, long long sCm, long long sCn, int M, int N, float alpha, int accumulate,
    const float* __restrict__ bias, int relu) {
  const long long e = blockIdx.x * 256LL + threadIdx.x;
  if (e >= n_tiles * 1024) return;
  const long long tile = e >> 10;
  const int r = (int)(e & 1023), tid = r >> 2, v = r & 3;
  float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int z = 0; z < ksplit; ++z) {
    const float4 t = ((const float4*)(slab + ((tile * ksplit + z) * 256 + tid) * 16))[v];
    a.x += t.x; a.y += t.y; a.z += t.z; a.w += t.w;
  }
  const int tn = (int)(tile % nt), tm = (int)((tile / nt) % mt), bt = (int)(tile / ((long long)nt * mt));
  const int wid = tid / WAVE, lane = tid % WAVE, wm = wid >> 1, wn = wid & 1;
  const int n = tn * BN + 32 * wn + (lane & 31);
  if (n >= N) return;
  const float bn = bias ? bias[n] : 0.f;
  const float vals[4] = {a.x, a.y, a.z, a.w};
  float* Cb = Cm + bt * sCb;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int m = tm * BM + 32 * wm + acc_row(4 * v + j, lane >> 5);
    if (m < M) {
      float* o = Cb + m * sCm + n * sCn;
      float val = alpha * vals[j] + bn;
      if (accumulate) val += *o;
      *o = relu ? fmaxf(val, 0.f) : val;
    }
  }
}

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

}  // namespace

extern "C" {

int tgfr_bgemm(const float* A, long long sAb, long long sAm, long long sAk, const float* B,
               long long sBb, long long sBk, long long sBn, float* C, long long sCb,
               long long sCm, long long sCn, int batch, int M, int N, int K, float alpha,
               int accumulate, const float* bias, int relu, int ksplit, float* slab,
               unsigned* counters, int mode, void* stream) {
  if (batch <= 0 || M <= 0 || N <= 0 || K <= 0 || ksplit <= 0) return 1001;
  if (ksplit > 1 && (!slab || !counters)) return 1001;
  if (mode != MODE_SPLIT && mode != MODE_BF16) return 1002;
  const dim3 grid((N + BN - 1) / BN, (M + BM - 1) / BM, batch * ksplit);
  auto* s = (hipStream_t)stream;
  const int la = sAk == 1 ? LAY_K : sAm == 1 ? LAY_MN : LAY_ANY;
  const int lb = sBk == 1 ? LAY_K : sBn == 1 ? LAY_MN : LAY_ANY;
  using Fn = void (*)(const float*, long long, long long, long long, const float*, long long,
                      long long, long long, float*, long long, long long, long long, int, int,
                      int, float, int, const float*, int, int, float*, unsigned*);
#define TGFR_BG(MD, A_, B_) &bgemm_kernel<MD, A_, B_>
#define TGFR_BG_ROW(MD, A_) TGFR_BG(MD, A_, LAY_K), TGFR_BG(MD, A_, LAY_MN), TGFR_BG(MD, A_, LAY_ANY)
  static const Fn table[2][3][3] = {
      {{TGFR_BG_ROW(MODE_BF16, LAY_K)}, {TGFR_BG_ROW(MODE_BF16, LAY_MN)},
       {TGFR_BG_ROW(MODE_BF16, LAY_ANY)}},
      {{TGFR_BG_ROW(MODE_SPLIT, LAY_K)}, {TGFR_BG_ROW(MODE_SPLIT, LAY_MN)},
       {TGFR_BG_ROW(MODE_SPLIT, LAY_ANY)}}};
#undef TGFR_BG_ROW
#undef TGFR_BG
  hipLaunchKernelGGL(table[mode][la][lb], grid, dim3(256), 2 * STAGE + 16, s, A, sAb, sAm, sAk,
                     B, sBb, sBk, sBn, C, sCb, sCm, sCn, M, N, K, alpha, accumulate, bias, relu,
                     ksplit, slab, counters);
  if (ksplit > KSPLIT_INLAUNCH) {
    const long long tiles = (long long)grid.x * grid.y * batch;
    hipLaunchKernelGGL(bgemm_reduce_kernel, dim3((unsigned)((tiles * 1024 + 255) / 256)),
                       dim3(256), 0, s, slab, ksplit, (int)grid.y, (int)grid.x, tiles, C, sCb,
                       sCm, sCn, M, N, alpha, accumulate, bias, relu);
  }
  return (int)hipGetLastError();
}

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

}  // extern "C"
