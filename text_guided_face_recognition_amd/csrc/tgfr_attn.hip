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
constexpr int HALF = 64 * 64;                 // bytes of one [64][32] bf16 tile
constexpr int STAGE = 4 * HALF;               // A hi, A lo, B hi, B lo

// [64 rows][32 k] bf16 tile with 64-B rows; chunk swizzle keeps the
// ds_read_b128 lane groups conflict-free.
__device__ __forceinline__ uint32_t toff(int row, int chunk) {
  return row * 64 + ((chunk ^ ((row >> 2) & 3)) << 4);
}

struct Frag8 {
  float v[8];
};

// Load 8 consecutive-k elements of row `row` (a tile row) into f.
__device__ __forceinline__ void load8(Frag8& f, const float* base, long long s_row,
                                      long long s_k, int row, int k0, int rows, int K) {
  const bool vec = (s_k == 1) && (((uintptr_t)(base + row * s_row + k0) & 15) == 0) &&
                   (k0 + 8 <= K) && (row < rows);
  if (vec) {
    const float4 a = *(const float4*)(base + row * s_row + k0);
    const float4 b = *(const float4*)(base + row * s_row + k0 + 4);
    f.v[0] = a.x; f.v[1] = a.y; f.v[2] = a.z; f.v[3] = a.w;
    f.v[4] = b.x; f.v[5] = b.y; f.v[6] = b.z; f.v[7] = b.w;
  } else {
#pragma unroll
    for (int e = 0; e < 8; ++e)
      f.v[e] = (row < rows && k0 + e < K) ? base[row * s_row + (k0 + e) * s_k] : 0.f;
  }
}

template <int MODE>
__device__ __forceinline__ void store8(uint32_t off_hi, const Frag8& f) {
  bf16x8 hi, lo;
  frag8<MODE>(f.v, hi, lo);
  lds_st16(off_hi, __builtin_bit_cast(uint4, hi));
  if (MODE == MODE_SPLIT) lds_st16(off_hi + HALF, __builtin_bit_cast(uint4, lo));
}

template <int MODE>
__global__ __launch_bounds__(256) void bgemm_kernel(
    const float* __restrict__ A, long long sAb, long long sAm, long long sAk,
    const float* __restrict__ B, long long sBb, long long sBk, long long sBn,
    float* __restrict__ Cm, long long sCb, long long sCm, long long sCn, int M, int N, int Kfull,
    float alpha, int accumulate, const float* __restrict__ bias, int relu, int ksplit,
    long long sCsplit) {
  const int n0 = blockIdx.x * BN, m0 = blockIdx.y * BM;
  const int bt = blockIdx.z / ksplit, kz = blockIdx.z % ksplit;
  // split-K: this block reduces k in [kb, kb + K) into its own output slab
  const int kc = ((Kfull + ksplit - 1) / ksplit + BK - 1) / BK * BK;
  const int kb = kz * kc;
  const int K = min(Kfull - kb, kc);
  if (K <= 0) {
    // empty tail slice: its slab must still hold zeros
    const int n = n0 + 32 * (threadIdx.x / WAVE & 1) + (threadIdx.x & 31);
    float* Cb = Cm + bt * sCb + kz * sCsplit;
    for (int q = 0; q < 16; ++q) {
      const int m = m0 + 32 * ((threadIdx.x / WAVE) >> 1) + acc_row(q, (threadIdx.x & 63) >> 5);
      if (m < M && n < N) Cb[m * sCm + n * sCn] = 0.f;
    }
    return;
  }
  A += (long long)kb * sAk;
  B += (long long)kb * sBk;
  const int tid = threadIdx.x, wid = tid / WAVE, lane = tid % WAVE;
  const int lr = lane & 31, h = lane >> 5;
  const int wm = wid >> 1, wn = wid & 1;
  const float* Ab = A + bt * sAb + m0 * sAm;
  const float* Bb = B + bt * sBb + n0 * sBn;
  // staging role: tile row = tid / 4, 8-k chunk = tid % 4
  const int srow = tid >> 2, sch = tid & 3;
  Frag8 fa, fb;
  f32x16 acc;
#pragma unroll
  for (int q = 0; q < 16; ++q) acc[q] = 0.f;

  const int nk = (K + BK - 1) / BK;
  load8(fa, Ab, sAm, sAk, srow, sch * 8, M - m0, K);
  load8(fb, Bb, sBn, sBk, srow, sch * 8, N - n0, K);
  store8<MODE>(toff(srow, sch), fa);
  store8<MODE>(2 * HALF + toff(srow, sch), fb);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const uint32_t sb = (kt & 1) * STAGE;
    if (kt + 1 < nk) {
      const int k0 = (kt + 1) * BK + sch * 8;
      load8(fa, Ab, sAm, sAk, srow, k0, M - m0, K);
      load8(fb, Bb, sBn, sBk, srow, k0, N - n0, K);
    }
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int ch = 2 * s + h;
      const uint32_t ao = sb + toff(32 * wm + lr, ch);
      const uint32_t bo = sb + 2 * HALF + toff(32 * wn + lr, ch);
      const bf16x8 ahi = as_bf8(lds_ld16(ao));
      const bf16x8 bhi = as_bf8(lds_ld16(bo));
      const bf16x8 alo = MODE == MODE_SPLIT ? as_bf8(lds_ld16(ao + HALF)) : ahi;
      const bf16x8 blo = MODE == MODE_SPLIT ? as_bf8(lds_ld16(bo + HALF)) : bhi;
      mma<MODE>(acc, ahi, alo, bhi, blo);
    }
    if (kt + 1 < nk) {
      const uint32_t nb = ((kt + 1) & 1) * STAGE;
      store8<MODE>(nb + toff(srow, sch), fa);
      store8<MODE>(nb + 2 * HALF + toff(srow, sch), fb);
    }
    __syncthreads();
  }
  const int n = n0 + 32 * wn + lr;
  if (n >= N) return;
  float* Cb = Cm + bt * sCb + kz * sCsplit;
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
               int accumulate, const float* bias, int relu, int ksplit, long long sCsplit,
               int mode, void* stream) {
  if (batch <= 0 || M <= 0 || N <= 0 || K <= 0 || ksplit <= 0) return 1001;
  if (ksplit > 1 && (bias || relu || accumulate)) return 1001;
  const dim3 grid((N + BN - 1) / BN, (M + BM - 1) / BM, batch * ksplit);
  auto* s = (hipStream_t)stream;
  if (mode == MODE_SPLIT)
    hipLaunchKernelGGL(bgemm_kernel<MODE_SPLIT>, grid, dim3(256), 2 * STAGE, s, A, sAb, sAm,
                       sAk, B, sBb, sBk, sBn, C, sCb, sCm, sCn, M, N, K, alpha, accumulate,
                       bias, relu, ksplit, sCsplit);
  else if (mode == MODE_BF16)
    hipLaunchKernelGGL(bgemm_kernel<MODE_BF16>, grid, dim3(256), 2 * STAGE, s, A, sAb, sAm,
                       sAk, B, sBb, sBk, sBn, C, sCb, sCm, sCn, M, N, K, alpha, accumulate,
                       bias, relu, ksplit, sCsplit);
  else
    return 1002;
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
