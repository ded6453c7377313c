// Batched GEMM for the IMIM / FCFM heads and the attention products
// (models/fusion_nets.py:103, :115; models/models.py:386-404; the 1x1 convs,
// Linear layers and their backward):
//
//   C[b] = epi(alpha * A[b] B[b] (+ C[b]) + bias),  epi = optional ReLU,
//
// fp32 operands of ANY element strides (every transpose of the backward is a
// stride swap), fp32 accumulation on v_mfma_f32_32x32x16_bf16, operands
// carried as bf16 (MODE_BF16) or as a bf16 hi/lo pair (MODE_SPLIT, ~fp32).
//
// Two kernels:
//   bgemm_glds  the main path.  fp32 tiles go global -> LDS by global_load_lds
//               (no staging registers) through an NS-deep ring, so NS-1 tiles
//               are in flight while one is computed; the bf16 (hi/lo)
//               conversion happens at fragment-read time.  Per operand the LDS
//               image follows the operand's unit-stride axis:
//                 LAY_K   [rows][32 k]  128-B rows, 16-B quads XOR-swizzled by
//                         row so the two ds_read_b128 of a fragment are
//                         conflict-free
//                 LAY_MN  [32 k][rows] (unit stride along m / n), read with 8
//                         ds_read_b32 per fragment (consecutive lanes =
//                         consecutive banks)
//               Block tile (64 WM) x (64 WN), 4 waves in 2 x 2, each wave
//               (32 WM) x (32 WN) = WM x WN accumulators; the host picks the
//               largest tile that still fills the chip.  Block ids are remapped
//               so the tiles that share an A row block run on one XCD (L2).
//   bgemm_regs  register-staged fallback for operands the DMA cannot fetch
//               (no unit-stride axis, 16-B misalignment, ragged quads).
//
// Split-K: each K slice stores its partial tile to a slab; the slices are
// summed in slice order (deterministic) by the tile's last-arriving slice
// (few slices) or by one chip-wide reduce launch (many slices).
#include "tgfr_common.h"

#include <stdlib.h>

#include <algorithm>

using namespace tgfr;

namespace {

constexpr int BK = 32;
enum { LAY_K = 0, LAY_MN = 1, LAY_ANY = 2 };
constexpr int KSPLIT_INLAUNCH = 4;

__device__ __attribute__((aligned(16))) float g_zero16[4] = {0.f, 0.f, 0.f, 0.f};

struct Frag8 {
  float v[8];
};

// ------------------------------------------------------------- epilogues ---
// Stores one 32x32 accumulator (rows m0.., cols n0..) with the bgemm epilogue.
__device__ __forceinline__ void store_acc(const f32x16& acc, float* Cb, long long sCm,
                                          long long sCn, int m0, int n0, int M, int N,
                                          float alpha, int accumulate, const float* bias,
                                          int relu, int lane) {
  const int n = n0 + (lane & 31);
  if (n >= N) return;
  const float bn = bias ? bias[n] : 0.f;
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int m = m0 + acc_row(q, lane >> 5);
    if (m < M) {
      float* o = Cb + m * sCm + n * sCn;
      float v = alpha * acc[q] + bn;
      if (accumulate) v += *o;
      *o = relu ? fmaxf(v, 0.f) : v;
    }
  }
}

// Slab of one split-K slice: the tile in natural [TM][TN] order.
__device__ __forceinline__ void store_slab(const f32x16& acc, float* tile_slab, int TN, int mm0,
                                           int nn0, int lane) {
#pragma unroll
  for (int q = 0; q < 16; ++q)
    tile_slab[(mm0 + acc_row(q, lane >> 5)) * TN + nn0 + (lane & 31)] = acc[q];
}
__device__ __forceinline__ void sum_slabs(f32x16& acc, const float* slab0, long long slab_stride,
                                          int ksplit, int TN, int mm0, int nn0, int lane) {
#pragma unroll
  for (int q = 0; q < 16; ++q) acc[q] = 0.f;
  for (int z = 0; z < ksplit; ++z) {
    const float* t = slab0 + z * slab_stride;
#pragma unroll
    for (int q = 0; q < 16; ++q) acc[q] += t[(mm0 + acc_row(q, lane >> 5)) * TN + nn0 + (lane & 31)];
  }
}

// Chip-wide split-K combine: thread = (tile, row, 4 columns); slabs summed in
// slice order, then the epilogue.
__global__ __launch_bounds__(256) void bgemm_reduce_kernel(
    const float* __restrict__ slab, int ksplit, int TM, int TN, int mt, int nt, long long n_tiles,
    float* Cm, long long sCb, long long sCm, long long sCn, int M, int N, float alpha,
    int accumulate, const float* __restrict__ bias, int relu) {
  const int per_tile = TM * TN / 4;
  const long long e = blockIdx.x * 256LL + threadIdx.x;
  if (e >= n_tiles * per_tile) return;
  const long long tile = e / per_tile;
  const int r = (int)(e % per_tile), mm = r / (TN / 4), nn = (r % (TN / 4)) * 4;
  const float4* src = (const float4*)(slab + tile * ksplit * (long long)(TM * TN) + mm * TN + nn);
  const long long zs = TM * TN / 4;
  float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll 8
  for (int z = 0; z < ksplit; ++z) {
    const float4 t = src[z * zs];
    a.x += t.x; a.y += t.y; a.z += t.z; a.w += t.w;
  }
  const int tn = (int)(tile % nt), tm = (int)((tile / nt) % mt);
  const int bt = (int)(tile / ((long long)nt * mt));
  const int m = tm * TM + mm;
  if (m >= M) return;
  float* Cb = Cm + bt * sCb + m * sCm;
  const float vals[4] = {a.x, a.y, a.z, a.w};
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int n = tn * TN + nn + j;
    if (n < N) {
      float* o = Cb + n * sCn;
      float v = alpha * vals[j] + (bias ? bias[n] : 0.f);
      if (accumulate) v += *o;
      *o = relu ? fmaxf(v, 0.f) : v;
    }
  }
}

// ------------------------------------------------------- glds main path ---
// LDS image of one fp32 operand tile (R rows x 32 k) per layout.
template <int LAY, int R>
struct Img {
  static constexpr int BYTES = R * BK * 4;
  static constexpr int PIECES = BYTES / 1024;     // one wave instruction = 1 KiB
};

// Quad swizzle of the [rows][32 k] fp32 image: 16 consecutive rows of one
// logical quad hit 16 distinct (row parity, quad) bank groups.
__device__ __forceinline__ int kswz(int row, int q) { return q ^ ((row >> 1) & 7); }

// Issue this wave's share of the DMA pieces of one operand tile.
// base: element (mn = 0, k = 0) of the tile; mn_lim / k_lim: valid extents.
template <int LAY, int R, int NW = 4>
__device__ __forceinline__ void issue_tile(const float* base, long long s_mn, long long s_k,
                                           int mn_lim, int k_lim, uint32_t lds_off, int wid,
                                           int lane) {
  constexpr int P = Img<LAY, R>::PIECES;
#pragma unroll
  for (int p = wid; p < P; p += NW) {
    const float* src;
    if constexpr (LAY == LAY_K) {
      const int row = p * 8 + (lane >> 3);
      const int q = kswz(row, lane & 7);
      const bool ok = row < mn_lim && 4 * q < k_lim;
      src = ok ? base + row * s_mn + 4 * q : g_zero16;
    } else {
      constexpr int ROWB = R * 4;                 // bytes per k row
      const int byte = p * 1024 + lane * 16;
      const int kr = byte / ROWB, mn = (byte % ROWB) / 4;
      const bool ok = mn < mn_lim && kr < k_lim;
      src = ok ? base + kr * s_k + mn : g_zero16;
    }
    glds16(src, lds_off + p * 1024);
  }
}

// Fragment (lane: row mn0 + lane%32, k = 16 s + 8 (lane/32) .. +7) as fp32.
template <int LAY, int R>
__device__ __forceinline__ void read_frag(Frag8& f, uint32_t off, int mn0, int s, int lane) {
  const int row = mn0 + (lane & 31), k0 = 16 * s + 8 * (lane >> 5);
  if constexpr (LAY == LAY_K) {
    const int q = k0 >> 2;
    const float4 a = __builtin_bit_cast(float4, lds_ld16(off + row * 128 + (kswz(row, q) << 4)));
    const float4 b =
        __builtin_bit_cast(float4, lds_ld16(off + row * 128 + (kswz(row, q + 1) << 4)));
    f.v[0] = a.x; f.v[1] = a.y; f.v[2] = a.z; f.v[3] = a.w;
    f.v[4] = b.x; f.v[5] = b.y; f.v[6] = b.z; f.v[7] = b.w;
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) f.v[j] = lds_ldf(off + (k0 + j) * (R * 4) + row * 4);
  }
}


template <int MODE, int LA, int LB, int WM, int WN, int NS>
__global__ __launch_bounds__(256) void bgemm_glds_kernel(
    const float* __restrict__ A, long long sAb, long long sAm, long long sAk,
    const float* __restrict__ B, long long sBb, long long sBk, long long sBn,
    float* __restrict__ Cm, long long sCb, long long sCm, long long sCn, int M, int N, int Kfull,
    float alpha, int accumulate, const float* __restrict__ bias, int relu, int ksplit,
    float* __restrict__ slab, unsigned* __restrict__ counters) {
  constexpr int TM = 64 * WM, TN = 64 * WN;
  constexpr int SA = Img<LA, TM>::BYTES, SB = Img<LB, TN>::BYTES, STG = SA + SB;
  constexpr int PER = (Img<LA, TM>::PIECES + Img<LB, TN>::PIECES) / 4;   // DMA ops / wave / stage
  // XCD-aware tile order over the whole (batch x slice, row, col) grid:
  // consecutive work ids -- the tiles of one A row block, all tiles of one
  // batch item, the K slices of one tile -- run on one XCD and share its L2
  const int gx = gridDim.x, gy = gridDim.y;
  const int w = xcd_remap((blockIdx.z * gy + blockIdx.y) * gx + blockIdx.x, gx * gy * gridDim.z);
  const int tn = w % gx, tm = (w / gx) % gy, z = w / (gx * gy);
  const int n0 = tn * TN, m0 = tm * TM;
  const int bt = z / ksplit, kz = z % ksplit;
  const int kc = ((Kfull + ksplit - 1) / ksplit + BK - 1) / BK * BK;
  const int kb = kz * kc;
  const int K = max(0, min(Kfull - kb, kc));
  const int tid = threadIdx.x, wid = tid / WAVE, lane = tid % WAVE;
  const int wm = wid >> 1, wn = wid & 1;
  const float* Ab = A + bt * sAb + m0 * sAm + (long long)kb * sAk;
  const float* Bb = B + bt * sBb + n0 * sBn + (long long)kb * sBk;
  f32x16 acc[WM][WN];
#pragma unroll
  for (int i = 0; i < WM; ++i)
#pragma unroll
    for (int j = 0; j < WN; ++j)
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[i][j][q] = 0.f;

  const int nk = (K + BK - 1) / BK;
  auto issue = [&](int kt) {
    const uint32_t o = (kt % NS) * STG;
    const int k0 = kt * BK;
    issue_tile<LA, TM>(Ab + (long long)k0 * sAk, sAm, sAk, M - m0, K - k0, o, wid, lane);
    issue_tile<LB, TN>(Bb + (long long)k0 * sBk, sBn, sBk, N - n0, K - k0, o + SA, wid, lane);
  };
#pragma unroll
  for (int st = 0; st < NS - 1; ++st)
    if (st < nk) issue(st);
  for (int kt = 0; kt < nk; ++kt) {
    // this wave's pieces of tile kt have landed once at most (NS-2) younger
    // stages are outstanding; the barrier makes every wave's pieces visible
    // and retires the reads of tile kt-1, whose buffer is refilled next
    if (kt + NS - 2 < nk) ring_barrier<(NS - 2) * PER>();
    else ring_barrier<0>();
    if (kt + NS - 1 < nk) issue(kt + NS - 1);
    const uint32_t o = (kt % NS) * STG;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8 bh[WN], bl[WN];
#pragma unroll
      for (int j = 0; j < WN; ++j) {
        Frag8 f;
        read_frag<LB, TN>(f, o + SA, wn * 32 * WN + 32 * j, s, lane);
        frag8<MODE>(f.v, bh[j], bl[j]);
      }
#pragma unroll
      for (int i = 0; i < WM; ++i) {
        Frag8 f;
        bf16x8 ah, al;
        read_frag<LA, TM>(f, o, wm * 32 * WM + 32 * i, s, lane);
        frag8<MODE>(f.v, ah, al);
#pragma unroll
        for (int j = 0; j < WN; ++j) {
          mma<MODE>(acc[i][j], ah, al, bh[j], bl[j]);
        }
      }
    }
  }

  if (ksplit > 1) {
    const long long tile = ((long long)bt * gy + tm) * gx + tn;
    float* mine = slab + (tile * ksplit + kz) * (long long)(TM * TN);
#pragma unroll
    for (int i = 0; i < WM; ++i)
#pragma unroll
      for (int j = 0; j < WN; ++j)
        store_slab(acc[i][j], mine, TN, wm * 32 * WM + 32 * i, wn * 32 * WN + 32 * j, lane);
    if (ksplit > KSPLIT_INLAUNCH) return;
    if (!last_arrival(counters + tile, ksplit, (int*)(g_smem + NS * STG))) return;
#pragma unroll
    for (int i = 0; i < WM; ++i)
#pragma unroll
      for (int j = 0; j < WN; ++j)
        sum_slabs(acc[i][j], slab + tile * ksplit * (long long)(TM * TN), TM * TN, ksplit, TN,
                  wm * 32 * WM + 32 * i, wn * 32 * WN + 32 * j, lane);
  }
  float* Cb = Cm + bt * sCb;
#pragma unroll
  for (int i = 0; i < WM; ++i)
#pragma unroll
    for (int j = 0; j < WN; ++j)
      store_acc(acc[i][j], Cb, sCm, sCn, m0 + wm * 32 * WM + 32 * i, n0 + wn * 32 * WN + 32 * j,
                M, N, alpha, accumulate, bias, relu, lane);
}

// ------------------------------------------------- register-staged path ---
constexpr int HALF = 64 * 64;                 // bytes of one 64x32 bf16 tile
constexpr int STAGE = 4 * HALF;               // A hi, A lo, B hi, B lo

// [64 mn][32 k] bf16: 16-B chunk swizzle keeps ds_read_b128 lane groups conflict-free.
__device__ __forceinline__ uint32_t toff(int row, int chunk) {
  return row * 64 + ((chunk ^ ((row >> 2) & 3)) << 4);
}
// [32 k][64 mn] bf16: rows 2 apart land 64 B apart, so the 4 rows of one
// transposed read hit disjoint banks.
__device__ __forceinline__ uint32_t moff(int krow, int chunk) {
  return krow * 128 + ((chunk ^ (((krow >> 1) & 1) << 2)) << 4);
}

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
__global__ __launch_bounds__(256) void bgemm_regs_kernel(
    const float* __restrict__ A, long long sAb, long long sAm, long long sAk,
    const float* __restrict__ B, long long sBb, long long sBk, long long sBn,
    float* __restrict__ Cm, long long sCb, long long sCm, long long sCn, int M, int N, int Kfull,
    float alpha, int accumulate, const float* __restrict__ bias, int relu, int ksplit,
    float* __restrict__ slab, unsigned* __restrict__ counters) {
  const int n0 = blockIdx.x * 64, m0 = blockIdx.y * 64;
  const int bt = blockIdx.z / ksplit, kz = blockIdx.z % ksplit;
  const int kc = ((Kfull + ksplit - 1) / ksplit + BK - 1) / BK * BK;
  const int kb = kz * kc;
  const int K = max(0, min(Kfull - kb, kc));
  const int tid = threadIdx.x, wid = tid / WAVE, lane = tid % WAVE;
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
    const long long tile = ((long long)bt * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x;
    store_slab(acc, slab + (tile * ksplit + kz) * 4096LL, 64, 32 * wm, 32 * wn, lane);
    if (ksplit > KSPLIT_INLAUNCH) return;
    if (!last_arrival(counters + tile, ksplit, (int*)(g_smem + 2 * STAGE))) return;
    sum_slabs(acc, slab + tile * ksplit * 4096LL, 4096, ksplit, 64, 32 * wm, 32 * wn, lane);
  }
  store_acc(acc, Cm + bt * sCb, sCm, sCn, m0 + 32 * wm, n0 + 32 * wn, M, N, alpha, accumulate,
            bias, relu, lane);
}

// ------------------------------------------ weight-resident row stream ---
// C = epi(alpha A B + bias) for a tall A [M][K] (k-contiguous rows) and a
// small B [K][N] with K = 128 or 256 (a Linear / 1x1 conv weight): every
// forward Linear of the head and the backward dX products (A = dY).
// bgemm_glds re-reads a B tile for every 64-row block of A, which on these
// shapes moves more bytes than A itself.  Here a persistent block owns a
// 128-column slice of B, converts it to bf16 ONCE into an LDS image, and
// streams its share of A's 64-row tiles through an NS-deep DMA ring that runs
// continuously across tiles (the epilogue of tile i overlaps the DMA of tile
// i+1).  Blocks of one A tile's slices are consecutive after the XCD remap,
// so they read A through one L2.  8 waves (2 x 4 of 32 x 32) per block: two
// per SIMD hide each other's LDS / convert latency.  The epilogue reads no
// global memory (bias preloaded, no accumulate): a plain load in the loop
// would make hipcc drain the DMA ring (vmcnt(0)) at every use.  bf16 mode
// only (the split image would not fit beside the ring).  On the step's
// shapes 20-25 % faster than bgemm_glds (tools/gemm_wres_ab.py).
constexpr int WR_TM = 64, WR_TN = 128, WR_NS = 6, WR_NW = 8;
constexpr int WR_STG = WR_TM * BK * 4;                 // one fp32 A stage
constexpr int WR_PER = WR_STG / 1024 / WR_NW;          // DMA ops per wave per stage

// B image [128 n][K] bf16, 16-B chunks XOR-swizzled by n.
__device__ __forceinline__ uint32_t wres_off(int n, int c, int K) {
  return (uint32_t)(n * K * 2 + ((c ^ (n & (K / 8 - 1))) << 4));
}

// Item = (n, 8-k chunk c) of the B slice: consecutive threads take
// consecutive c for k-contiguous B (W[n][k], the forward: two float4 per
// item) and consecutive n for n-contiguous B (W[k][n], the dX products: eight
// coalesced dwords).  Separate instantiations: a runtime layout branch per
// item made hipcc merge both into eight scalar loads.
template <int K, bool KC>
__device__ __forceinline__ void wres_load_b(const float* __restrict__ B, long long sBk,
                                            long long sBn, int n0, int N, int tid) {
  constexpr int ITEMS = WR_TN * (K / 8) / (64 * WR_NW), PASS = ITEMS < 8 ? ITEMS : 8;
#pragma unroll
  for (int p0 = 0; p0 < ITEMS; p0 += PASS) {
    float v[PASS][8];
#pragma unroll
    for (int i = 0; i < PASS; ++i) {
      const int idx = tid + 64 * WR_NW * (p0 + i);
      const int nl = KC ? idx / (K / 8) : idx % WR_TN;
      const int c = KC ? idx % (K / 8) : idx / WR_TN;
      const int n = min(n0 + nl, N - 1);
      if constexpr (KC) {
        const float* src = B + (long long)n * sBn + 8 * c;
        const float4 a = *(const float4*)src, b = *(const float4*)(src + 4);
        v[i][0] = a.x; v[i][1] = a.y; v[i][2] = a.z; v[i][3] = a.w;
        v[i][4] = b.x; v[i][5] = b.y; v[i][6] = b.z; v[i][7] = b.w;
      } else {
        const float* src = B + (long long)n * sBn + (long long)(8 * c) * sBk;
#pragma unroll
        for (int e = 0; e < 8; ++e) v[i][e] = src[e * sBk];
      }
    }
#pragma unroll
    for (int i = 0; i < PASS; ++i) {
      const int idx = tid + 64 * WR_NW * (p0 + i);
      const int nl = KC ? idx / (K / 8) : idx % WR_TN;
      const int c = KC ? idx % (K / 8) : idx / WR_TN;
      if (n0 + nl >= N) {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[i][e] = 0.f;
      }
      bf16x8 hi, lo;
      frag8<MODE_BF16>(v[i], hi, lo);
      lds_st16(wres_off(nl, c, K), __builtin_bit_cast(uint4, hi));
    }
  }
}

// ABF: A is bf16 (e.g. BatchNorm's xhat in bf16 mode): a ring stage then
// holds 64 k instead of 32 in the same 128-B-per-row swizzled image (8-bf16
// chunks where the fp32 image has 4-float quads), and a fragment is one
// ds_read_b128 with no conversion.
template <int K, bool OBF = false, bool ABF = false>
__global__ __launch_bounds__(64 * WR_NW) void bgemm_wres_kernel(
    const float* __restrict__ A, long long sAm, const float* __restrict__ B, long long sBk,
    long long sBn, float* __restrict__ Cm, long long sCm, long long sCn, int M, int N,
    float alpha, const float* __restrict__ bias, int relu, int n_slices, int per_slice) {
  constexpr int WB = WR_TN * K * 2;                     // B image bytes
  constexpr int KS = ABF ? 2 * BK : BK;                 // k per ring stage
  constexpr int NK = K / KS;
  const int tid = threadIdx.x, wid = tid / WAVE, lane = tid % WAVE;
  const int wm = wid >> 2, wn = wid & 3;              // 2 x 4 waves of 32 x 32
  // block -> (slice, g): consecutive remapped ids = the slices of one A tile
  const int total = gridDim.x;
  const int w = xcd_remap(blockIdx.x, total);
  const int slice = w % n_slices, g = w / n_slices;
  const int n0 = slice * WR_TN;
  const int m_tiles = (M + WR_TM - 1) / WR_TM;
  // this block's A tiles: g, g + per_slice, ...
  const int my_tiles = g < m_tiles ? (m_tiles - 1 - g) / per_slice + 1 : 0;
  const int T = my_tiles * NK;                          // k-steps in the stream

  auto issue = [&](int t) {
    const int j = t / NK, kt = t % NK;
    const int m0 = (g + j * per_slice) * WR_TM;
    if constexpr (ABF)   // bf16 rows seen as float pairs: same piece geometry
      issue_tile<LAY_K, WR_TM, WR_NW>(
          (const float*)((const uint16_t*)A + (long long)m0 * sAm + kt * KS), sAm / 2, 1,
          M - m0, (K - kt * KS) / 2, WB + (t % WR_NS) * WR_STG, wid, lane);
    else
      issue_tile<LAY_K, WR_TM, WR_NW>(A + (long long)m0 * sAm + kt * BK, sAm, 1, M - m0,
                                      K - kt * BK, WB + (t % WR_NS) * WR_STG, wid, lane);
  };
#pragma unroll
  for (int t = 0; t < WR_NS - 1; ++t)
    if (t < T) issue(t);

  // B slice -> bf16 image (plain loads, all of a pass in flight at once;
  // overlaps the ring's first stages).
  if (sBk == 1)
    wres_load_b<K, true>(B, sBk, sBn, n0, N, tid);
  else
    wres_load_b<K, false>(B, sBk, sBn, n0, N, tid);

  constexpr int NJ = WR_TN / 32 / (WR_NW / 2);          // 32-col tiles per wave
  // The products are formed transposed, C^T = B^T A^T (the weights as the
  // MFMA's A operand): a lane then holds, per accumulator quad, 4 consecutive
  // output columns of ONE row, so the epilogue stores 8-byte (bf16) or 16-byte
  // (fp32) row pieces instead of one 2- / 4-byte element per register.
  f32x16 acc[NJ];
  // the epilogue's bias values (column n = 8 g + 4 h + i of the wave's tile
  // j), loaded once: no plain global load may sit in the loop beside the DMA
  // ring (hipcc would drain the ring with vmcnt(0) before every use of it)
  float bcol[NJ][16];
#pragma unroll
  for (int j = 0; j < NJ; ++j)
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int n = n0 + wn * 32 * NJ + 32 * j + acc_row(q, lane >> 5);
      bcol[j][q] = bias && n < N ? bias[n] : 0.f;
      acc[j][q] = 0.f;
    }

  for (int t = 0; t < T; ++t) {
    // stage t has landed once at most NS-2 younger stages (and the stores of
    // an epilogue) are outstanding; the barrier also publishes the B image
    if (t + WR_NS - 2 < T) ring_barrier<(WR_NS - 2) * WR_PER>();
    else ring_barrier<0>();
    if (t + WR_NS - 1 < T) issue(t + WR_NS - 1);
    const uint32_t o = WB + (t % WR_NS) * WR_STG;
    const int kt = t % NK;
#pragma unroll
    for (int s = 0; s < KS / 16; ++s) {
      bf16x8 ah, al;
      if constexpr (ABF) {
        const int row = wm * 32 + (lane & 31), q = 2 * s + (lane >> 5);
        ah = al = as_bf8(lds_ld16(o + row * 128 + (kswz(row, q) << 4)));
      } else {
        Frag8 f;
        read_frag<LAY_K, WR_TM>(f, o, wm * 32, s, lane);
        frag8<MODE_BF16>(f.v, ah, al);
      }
      const int c = (kt * KS + 16 * s) / 8 + (lane >> 5);
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int nl = wn * 32 * NJ + 32 * j + (lane & 31);
        const bf16x8 bh = as_bf8(lds_ld16(wres_off(nl, c, K)));
        mma<MODE_BF16>(acc[j], bh, bh, ah, al);          // C^T tile (see above)
      }
    }
    if (kt == NK - 1) {
      const int m0 = (g + (t / NK) * per_slice) * WR_TM;
      const int m = m0 + wm * 32 + (lane & 31);
      // 4-column pieces as one store when rows are 16-B aligned
      const bool vec = sCn == 1 && (sCm & 3) == 0 && (((uintptr_t)Cm & 15) == 0);
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
#pragma unroll
        for (int gq = 0; gq < 4; ++gq) {
          const int nb = n0 + wn * 32 * NJ + 32 * j + 8 * gq + 4 * (lane >> 5);
          float v[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            v[i] = alpha * acc[j][4 * gq + i] + bcol[j][4 * gq + i];
            v[i] = relu ? fmaxf(v[i], 0.f) : v[i];
          }
          if (m < M) {
            if (vec && nb + 3 < N) {
              if constexpr (OBF)
                *(uint2*)((uint16_t*)Cm + m * sCm + nb) =
                    make_uint2(pk_bf16(v[0], v[1]), pk_bf16(v[2], v[3]));
              else
                *(float4*)(Cm + m * sCm + nb) = make_float4(v[0], v[1], v[2], v[3]);
            } else {
#pragma unroll
              for (int i = 0; i < 4; ++i) {
                if (nb + i >= N) continue;
                if constexpr (OBF)
                  ((uint16_t*)Cm)[m * sCm + (nb + i) * sCn] = bf_bits(v[i]);
                else
                  Cm[m * sCm + (nb + i) * sCn] = v[i];
              }
            }
          }
        }
#pragma unroll
        for (int q = 0; q < 16; ++q) acc[j][q] = 0.f;
      }
    }
  }
}

using GemmFn = void (*)(const float*, long long, long long, long long, const float*, long long,
                        long long, long long, float*, long long, long long, long long, int, int,
                        int, float, int, const float*, int, int, float*, unsigned*);

template <int MODE, int LA, int LB>
GemmFn glds_fn(int cfg) {
  switch (cfg) {
    case 0: return &bgemm_glds_kernel<MODE, LA, LB, 1, 1, 4>;
    case 1: return &bgemm_glds_kernel<MODE, LA, LB, 2, 1, 3>;
    case 2: return &bgemm_glds_kernel<MODE, LA, LB, 1, 2, 3>;
    default: return &bgemm_glds_kernel<MODE, LA, LB, 2, 2, 4>;
  }
}
constexpr int CFG_WM[4] = {1, 2, 1, 2}, CFG_WN[4] = {1, 1, 2, 2}, CFG_NS[4] = {4, 3, 3, 4};

template <int MODE>
GemmFn pick_glds(int la, int lb, int cfg) {
  if (la == LAY_K)
    return lb == LAY_K ? glds_fn<MODE, LAY_K, LAY_K>(cfg) : glds_fn<MODE, LAY_K, LAY_MN>(cfg);
  return lb == LAY_K ? glds_fn<MODE, LAY_MN, LAY_K>(cfg) : glds_fn<MODE, LAY_MN, LAY_MN>(cfg);
}

template <int MODE>
GemmFn pick_regs(int la, int lb) {
  static const GemmFn t[3][3] = {
      {&bgemm_regs_kernel<MODE, LAY_K, LAY_K>, &bgemm_regs_kernel<MODE, LAY_K, LAY_MN>,
       &bgemm_regs_kernel<MODE, LAY_K, LAY_ANY>},
      {&bgemm_regs_kernel<MODE, LAY_MN, LAY_K>, &bgemm_regs_kernel<MODE, LAY_MN, LAY_MN>,
       &bgemm_regs_kernel<MODE, LAY_MN, LAY_ANY>},
      {&bgemm_regs_kernel<MODE, LAY_ANY, LAY_K>, &bgemm_regs_kernel<MODE, LAY_ANY, LAY_MN>,
       &bgemm_regs_kernel<MODE, LAY_ANY, LAY_ANY>}};
  return t[la][lb];
}

bool al16(const void* p) { return ((uintptr_t)p & 15) == 0; }

// Can the DMA fetch this operand as whole 16-B quads?
bool dma_ok(const float* p, int lay, long long sb, long long s_mn, long long s_k, int mn, int k,
            int batch) {
  if (lay == LAY_ANY || !al16(p) || (batch > 1 && (sb & 3))) return false;
  if (lay == LAY_K) return (s_mn & 3) == 0 && (k & 3) == 0;
  return (s_k & 3) == 0 && (mn & 3) == 0;
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
  auto* s = (hipStream_t)stream;
  const int la = sAk == 1 ? LAY_K : sAm == 1 ? LAY_MN : LAY_ANY;
  const int lb = sBk == 1 ? LAY_K : sBn == 1 ? LAY_MN : LAY_ANY;
  // weight-resident row stream
  if (mode == MODE_BF16 && batch == 1 && ksplit == 1 && !accumulate && la == LAY_K &&
      (K == 128 || K == 256) && M >= 2048 && dma_ok(A, LAY_K, 0, sAm, 1, M, K, 1) &&
      (sBk != 1 || (al16(B) && (sBn & 3) == 0))) {
    const int n_slices = (N + WR_TN - 1) / WR_TN;
    const int m_tiles = (M + WR_TM - 1) / WR_TM;
    // ~one block per CU: per_slice blocks stream each B slice's A tiles
    const int per_slice = std::max(1, std::min(m_tiles, 256 / n_slices));
    const int lds = WR_TN * K * 2 + WR_NS * WR_STG;
    auto fn = K == 256 ? &bgemm_wres_kernel<256> : &bgemm_wres_kernel<128>;
    if (const int e = set_max_lds((const void*)fn, lds)) return e;
    hipLaunchKernelGGL(fn, dim3(n_slices * per_slice), dim3(64 * WR_NW), lds, s, A, sAm, B, sBk,
                       sBn, C,
                       sCm, sCn, M, N, alpha, bias, relu, n_slices, per_slice);
    return (int)hipGetLastError();
  }
  const bool dma = dma_ok(A, la, sAb, sAm, sAk, M, K, batch) &&
                   dma_ok(B, lb, sBb, sBn, sBk, N, K, batch);
  int TM = 64, TN = 64;
  dim3 grid;
  if (dma) {
    // largest tile that still gives >= 1 block per CU (two fit); the 128x128 tile
    // (cfg 3) is never picked: at K <= 768 it loses to 128x64 / 64x128 on
    // every head shape (measured in round 1)
    int cfg = 0;
    for (int c = 2; c >= 1; --c) {
      const long long blocks = (long long)((M + 64 * CFG_WM[c] - 1) / (64 * CFG_WM[c])) *
                               ((N + 64 * CFG_WN[c] - 1) / (64 * CFG_WN[c])) * batch * ksplit;
      if (blocks >= 256) { cfg = c; break; }
    }
    TM = 64 * CFG_WM[cfg];
    TN = 64 * CFG_WN[cfg];
    grid = dim3((N + TN - 1) / TN, (M + TM - 1) / TM, batch * ksplit);
    const int stg = (TM + TN) * BK * 4;
    const int lds = CFG_NS[cfg] * stg + 16;
    GemmFn fn = mode == MODE_SPLIT ? pick_glds<MODE_SPLIT>(la, lb, cfg)
                                   : pick_glds<MODE_BF16>(la, lb, cfg);
    if (const int e = set_max_lds((const void*)fn, lds)) return e;
    hipLaunchKernelGGL(fn, grid, dim3(256), lds, s, A, sAb, sAm, sAk, B, sBb, sBk, sBn, C, sCb,
                       sCm, sCn, M, N, K, alpha, accumulate, bias, relu, ksplit, slab, counters);
  } else {
    grid = dim3((N + 63) / 64, (M + 63) / 64, batch * ksplit);
    GemmFn fn = mode == MODE_SPLIT ? pick_regs<MODE_SPLIT>(la, lb) : pick_regs<MODE_BF16>(la, lb);
    hipLaunchKernelGGL(fn, grid, dim3(256), 2 * STAGE + 16, s, A, sAb, sAm, sAk, B, sBb, sBk,
                       sBn, C, sCb, sCm, sCn, M, N, K, alpha, accumulate, bias, relu, ksplit,
                       slab, counters);
  }
  if (ksplit > KSPLIT_INLAUNCH) {
    const long long tiles = (long long)grid.x * grid.y * batch;
    hipLaunchKernelGGL(bgemm_reduce_kernel,
                       dim3((unsigned)((tiles * (TM * TN / 4) + 255) / 256)), dim3(256), 0, s,
                       slab, ksplit, TM, TN, (int)grid.y, (int)grid.x, tiles, C, sCb, sCm, sCn,
                       M, N, alpha, accumulate, bias, relu);
  }
  return (int)hipGetLastError();
}

// C = A W^T + bias with a bf16 output (the packed attention projection of
// IMIM in bf16 mode, read by tgfr_attn_fwd / _bwd as bf16): A [M][K] fp32
// rows (K = 128 or 256, 16-B aligned, sAm % 4 == 0), W [N][K] fp32
// (row stride sWn), C [M][N] bf16 (row stride sCm).
int tgfr_linear_bf16io(const uint16_t* A, long long sAm, int M, int K, const float* W,
                       long long sWn, const float* bias, int N, uint16_t* C, long long sCm,
                       void* stream) {
  if (M <= 0 || N <= 0 || (K != 128 && K != 256) || !al16(A) || (sAm & 7) || !al16(W) ||
      (sWn & 3))
    return 1001;
  const int n_slices = (N + WR_TN - 1) / WR_TN;
  const int m_tiles = (M + WR_TM - 1) / WR_TM;
  const int per_slice = std::max(1, std::min(m_tiles, 256 / n_slices));
  const int lds = WR_TN * K * 2 + WR_NS * WR_STG;
  auto fn = K == 256 ? &bgemm_wres_kernel<256, true, true> : &bgemm_wres_kernel<128, true, true>;
  if (const int e = set_max_lds((const void*)fn, lds)) return e;
  hipLaunchKernelGGL(fn, dim3(n_slices * per_slice), dim3(64 * WR_NW), lds, (hipStream_t)stream,
                     (const float*)A, sAm, W, (long long)1, sWn, (float*)C, sCm, (long long)1, M,
                     N, 1.f, bias, 0, n_slices, per_slice);
  return (int)hipGetLastError();
}

int tgfr_linear_bf16out(const float* A, long long sAm, int M, int K, const float* W,
                        long long sWn, const float* bias, int N, uint16_t* C, long long sCm,
                        void* stream) {
  if (M <= 0 || N <= 0 || (K != 128 && K != 256) || !dma_ok(A, LAY_K, 0, sAm, 1, M, K, 1) ||
      !al16(W) || (sWn & 3))
    return 1001;
  const int n_slices = (N + WR_TN - 1) / WR_TN;
  const int m_tiles = (M + WR_TM - 1) / WR_TM;
  const int per_slice = std::max(1, std::min(m_tiles, 256 / n_slices));
  const int lds = WR_TN * K * 2 + WR_NS * WR_STG;
  auto fn = K == 256 ? &bgemm_wres_kernel<256, true> : &bgemm_wres_kernel<128, true>;
  if (const int e = set_max_lds((const void*)fn, lds)) return e;
  hipLaunchKernelGGL(fn, dim3(n_slices * per_slice), dim3(64 * WR_NW), lds, (hipStream_t)stream,
                     A, sAm, W, (long long)1, sWn, (float*)C, sCm, (long long)1, M, N, 1.f, bias,
                     0, n_slices, per_slice);
  return (int)hipGetLastError();
}

}  // extern "C"
