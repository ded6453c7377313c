// IMIM tail (models/models.py:399-405 + ProjectionHead :98-120) fused for
// gfx950, bf16 operands with fp32 accumulation:
//
//   H1 = relu(Z W1^T + b1)      conv1x1_1, 256 -> 128   (:399-400)
//   H2 = relu(H1 W2^T + b2)     conv1x1_2, 128 -> 256   (:402)
//   P  = H2 Wp^T + bp           project_local.projection (:403, :116)
//   R  = P / max(|P|, eps)      F.normalize               (:117)
//
// over the channels-last rows of the LayerNorm output Z [rows = B*196][256].
// One workgroup owns 32 rows and runs the whole chain: the intermediate
// activations never leave LDS, only the bf16 copies the backward needs (Z, H1,
// H2) and R go to HBM.  Layers 1 and 2 are computed transposed
// (Out^T = W In^T): the MFMA accumulator of a lane then holds 4 consecutive
// output features of ONE row per register quad, which is one ds_write_b64
// into the next layer's [row][feature] operand image (no 2-byte scatter).
// The last layer is computed upright so that its fp32 result is stored as
// 128-B row segments and its row norms reduce across lanes (rs16).
//
// 32-row workgroups at ~120 registers per lane put several workgroups on a
// CU, which hides the operand latency better than 64-row workgroups with the
// weight fragments prefetched into registers (13 / 19 us against 17 / 25 us
// forward / backward at 12544 rows, tools/lab/tail_ablate.py); the weights'
// fragment-order pack keeps each fragment load one coalesced KiB.
//
// Backward (one workgroup per 32 rows again):
//   dP  = (dR - R (R.dR)) / max(|P|, eps)        (clamped rows: dR / eps)
//   dH2 = (dP Wp) * [H2 > 0],  dH1 = (dH2 W2) * [H1 > 0],  dZ = dH1 W1
// writing dZ in fp32 (the LayerNorm backward's input) and dP, dH2, dH1 in
// bf16 for the weight gradients, which tail_dw computes as
//   dWp = dP^T H2, dW2 = dH2^T H1, dW1 = dH1^T Z  (+ the bias column sums)
// in one launch: row slices per workgroup, operands transposed at LDS read
// time by ds_read_b64_tr_b16, slice partials summed in slice order by
// tail_dw_reduce (deterministic).
#include "tgfr_fold.h"
#include "tgfr_ln.h"

#include <algorithm>
#include <type_traits>

using namespace tgfr;

namespace {

constexpr int TC = 256;   // IMIM channels (LayerNorm / conv1x1_1 input, conv1x1_2 output)
constexpr int TH = 128;   // conv1x1_1 output
constexpr int TD = 256;   // projection dim (aux_feat_dim_per_granularity)
constexpr int TM = 32;    // rows per workgroup
constexpr int MT = TM / 32;  // 32-row MFMA tiles per workgroup

// packed bf16 weights (uint16 element offsets)
constexpr int OFF_W1 = 0;                     // W1  [TH][TC]
constexpr int OFF_W2 = OFF_W1 + TH * TC;      // W2  [TC][TH]
constexpr int OFF_WP = OFF_W2 + TC * TH;      // Wp  [TD][TC]
constexpr int OFF_W1T = OFF_WP + TD * TC;     // W1^T [TC][TH]
constexpr int OFF_W2T = OFF_W1T + TC * TH;    // W2^T [TH][TC]
constexpr int OFF_WPT = OFF_W2T + TH * TC;    // Wp^T [TC][TD]
constexpr int PACK_ELEMS = OFF_WPT + TC * TD;

// [TM rows][K] bf16 operand image, 16-B chunks XOR-swizzled by row: the 32
// rows of a fragment read land on 32 distinct chunks (conflict-free
// ds_read_b128 lane groups).
template <int K>
__device__ __forceinline__ uint32_t img(int m, int c) {
  return (uint32_t)(m * K * 2 + ((c ^ (m & (K / 8 - 1))) << 4));
}
// byte offset of feature n (multiple of 4) of row m
template <int K>
__device__ __forceinline__ uint32_t img_at(int m, int n) {
  return img<K>(m, n >> 3) + (n & 7) * 2;
}

__device__ __forceinline__ bf16x8 gld16(const uint16_t* p) {
  return as_bf8(*(const uint4*)p);
}

__device__ __forceinline__ uint2 pk4(float a, float b, float c, float d) {
  return make_uint2(pk_bf16(a, b), pk_bf16(c, d));
}

// image -> HBM rows [row0 + m][K] (ld elements), rows < n_rows only
template <int K>
__device__ __forceinline__ void copy_out(uint32_t base, uint16_t* dst, long long ld, int row0,
                                         int n_rows, int tid) {
  constexpr int CH = K / 8;
#pragma unroll
  for (int i = tid; i < TM * CH; i += 256) {
    const int m = i / CH, c = i % CH;
    if (row0 + m < n_rows)
      *(uint4*)(dst + (long long)(row0 + m) * ld + 8 * c) = lds_ld16(base + img<K>(m, c));
  }
}

// --------------------------------------------------------------- pack ---
// Each packed matrix M [rows][K] is stored in MFMA fragment order: the 64
// lanes' 16-B operand pieces of one (32-row tile rt, 16-k step s) are one
// contiguous KiB, lane l holding M[32 rt + l%32][16 s + 8 (l/32) .. +7].  A
// wave's fragment load is then one coalesced KiB instead of 64 scattered
// 16-B pieces (one cache line each), which made the weight reads of the
// first version cost a third of the kernel.
__device__ __forceinline__ const uint16_t* frag_ptr(const uint16_t* pk, int off, int K, int rt,
                                                    int s, int lane) {
  return pk + off + ((rt * (K / 16) + s) * 64 + lane) * 8;
}

constexpr int PACK_UNITS = PACK_ELEMS / 8;    // one lane fragment (8 bf16) per thread

// fragment u (elements 8u .. 8u + 7) of the fragment-order pack: M[r][k .. k + 7]
// of one lane, M = W or W^T.  All 8 loads are issued before the conversion
// (two float4 loads of a W row, or 8 column loads that are coalesced across
// the lanes' consecutive r), then one 16-byte store.
__device__ __forceinline__ void pack_frag(const float* __restrict__ W1,
                                          const float* __restrict__ W2,
                                          const float* __restrict__ Wp, uint16_t* __restrict__ pk,
                                          int u) {
  const int e = 8 * u;
  const float* W;
  int off, K, ld, tr;
  if (e < OFF_W2) { W = W1; off = OFF_W1; K = TC; ld = TC; tr = 0; }
  else if (e < OFF_WP) { W = W2; off = OFF_W2; K = TH; ld = TH; tr = 0; }
  else if (e < OFF_W1T) { W = Wp; off = OFF_WP; K = TC; ld = TC; tr = 0; }
  else if (e < OFF_W2T) { W = W1; off = OFF_W1T; K = TH; ld = TC; tr = 1; }
  else if (e < OFF_WPT) { W = W2; off = OFF_W2T; K = TC; ld = TH; tr = 1; }
  else { W = Wp; off = OFF_WPT; K = TD; ld = TC; tr = 1; }
  const int f = e - off, lane = (f >> 3) & 63, piece = f >> 9;
  const int s = piece % (K / 16), rt = piece / (K / 16);
  const int r = 32 * rt + (lane & 31), k = 16 * s + 8 * (lane >> 5);   // M[r][k ..]
  float v[8];
  if (!tr) {
    const float4 a = *(const float4*)(W + r * ld + k), b = *(const float4*)(W + r * ld + k + 4);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
    v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = W[(k + j) * ld + r];
  }
  uint4 o;
  o.x = bf_bits(v[0]) | ((uint32_t)bf_bits(v[1]) << 16);
  o.y = bf_bits(v[2]) | ((uint32_t)bf_bits(v[3]) << 16);
  o.z = bf_bits(v[4]) | ((uint32_t)bf_bits(v[5]) << 16);
  o.w = bf_bits(v[6]) | ((uint32_t)bf_bits(v[7]) << 16);
  *(uint4*)(pk + e) = o;
}

// (aff != NULL: also the IMIM LayerNorm's affine maps, stored [C][H W] by the
// reference, as channels-last rows aff[0 | 1][p][c] = (w | b)[c][p] for the
// LayerNorm fused into tail_fwd / tail_bwd: coalesced loads there)
__global__ __launch_bounds__(256) void tail_pack_kernel(const float* __restrict__ W1,
                                                        const float* __restrict__ W2,
                                                        const float* __restrict__ Wp,
                                                        uint16_t* __restrict__ pk,
                                                        const float* __restrict__ lnw,
                                                        const float* __restrict__ lnb, int hw,
                                                        float* __restrict__ aff) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= PACK_UNITS) {
    const int f = e - PACK_UNITS, n = hw * TC;
    if (!aff || f >= 2 * n) return;
    const int j = f / n, r = f % n, p = r / TC, c = r % TC;
    aff[f] = (j ? lnb : lnw)[(long long)c * hw + p];
    return;
  }
  pack_frag(W1, W2, Wp, pk, e);
}

// IMIM's whole per-step weight preparation in one launch: blocks [0, nf)
// fold bn_img into the packed q/k/v projection (one wave per row, as
// bn_fold_kernel), the rest run tail_pack_kernel's elements (weights and the
// LayerNorm affine maps).
struct ImimPackArgs {
  Parts P;
  int O, C;
  const float *gamma, *beta;
  float *Wf, *bf;
  uint16_t* Wfb;       // nullable: the folded q/k/v weights also in bf16
  int nf;
  const float *W1, *W2, *Wp;
  uint16_t* pk;
  const float *lnw, *lnb;
  int hw;
  float* aff;
};
__device__ __forceinline__ void imim_pack_block(const ImimPackArgs& A, int bid) {
  if (bid < A.nf) {
    const int o = bid * 4 + threadIdx.x / WAVE;
    if (o < A.O)
      bn_fold_row(A.P, o, A.C, A.gamma, A.beta, A.Wf, A.bf, threadIdx.x % WAVE, A.Wfb);
    return;
  }
  const int e = (bid - A.nf) * 256 + threadIdx.x;
  if (e >= PACK_UNITS) {
    const int f = e - PACK_UNITS, n = A.hw * TC;
    if (f >= 2 * n) return;
    const int j = f / n, r = f % n, p = r / TC, c = r % TC;
    A.aff[f] = (j ? A.lnb : A.lnw)[(long long)c * A.hw + p];
    return;
  }
  pack_frag(A.W1, A.W2, A.Wp, A.pk, e);
}
__global__ __launch_bounds__(256) void imim_pack_kernel(ImimPackArgs A) {
  imim_pack_block(A, blockIdx.x);
}

// The same with IMIM's BatchNorm batch statistics as its first C workgroups
// (bn_stats_block): the whole per-step preparation of the head in ONE launch
// (the fold does not depend on the statistics; tgfr_bn_qkv_bf16 reads both).
struct BnStatsArgs {
  const float* x;
  int N, C, HW;
  float eps, momentum;
  int training;
  float *running_mean, *running_var;
  long long* nbt;
  float *mean, *rstd;
};
__global__ __launch_bounds__(256) void imim_prep_kernel(BnStatsArgs S, ImimPackArgs A) {
  __shared__ float red[4];
  if ((int)blockIdx.x < S.C) {
    bn_stats_block(S.x, S.N, S.C, S.HW, S.eps, S.momentum, S.training, S.running_mean,
                   S.running_var, S.nbt, S.mean, S.rstd, blockIdx.x, red);
    return;
  }
  imim_pack_block(A, blockIdx.x - S.C);
}

// ------------------------------------------------------------ forward ---
// LDS: [0, 32K) Z image (later the H2 image), [32K, 48K) H1 image,
//      [48K, 49K) row sum-of-squares partials [4 waves][64], [49K, 49.25K) 1/norm
constexpr int F_Z = 0, F_H2 = 0, F_H1 = TM * TC * 2, F_SS = F_H1 + TM * TH * 2,
              F_INV = F_SS + 4 * TM * 4;
constexpr int F_LDS = F_INV + TM * 4;

// The IMIM LayerNorm fused into the tail (LN = true): Z = (X - mean_b) rstd_b
// w + b for sample b = row / hw of the attention output X (models/models.py
// :401), from ln_part's slice moments (combined here, Chan, fixed order) and
// the channels-last affine rows of tail_pack; the first workgroup of each
// sample stores its (mean, rstd) for the backward.
struct LnFwd {
  const float* part;      // ln_part moments [n][S][2], or (tiles) the attention's [n][S][2]
  float* stats;           // mean [n] | rstd [n]
  const float* aff;       // w rows [hw][TC] | b rows [hw][TC]
  long long E;            // hw * TC
  int S, hw, n;
  float eps;
  int tiles;              // 1: the S entries are 32-row tile moments (tgfr_attn_fwd_ln)
};
constexpr int F_LN = F_LDS;                 // LN: mean, rstd of the two samples
constexpr int F_MOM = F_LDS + 16;           // LN: their slice moments [2][S][2], S <= 64
constexpr int F_LDS_LN = F_MOM + 2 * 64 * 2 * 4;

template <bool LN>
__global__ __launch_bounds__(256) void tail_fwd_kernel(
    const float* __restrict__ Z, long long ldz, int rows, const uint16_t* __restrict__ pk,
    const float* __restrict__ b1, const float* __restrict__ b2, const float* __restrict__ bp,
    float eps, float* __restrict__ R, long long ldr, uint16_t* __restrict__ Zb,
    uint16_t* __restrict__ H1b, uint16_t* __restrict__ H2b, float* __restrict__ inv_out,
    uint16_t* __restrict__ Rrows, float* __restrict__ Rnorm, int rows_per_item, int rows_pad,
    int rows_f16, LnFwd L) {
  const int tid = threadIdx.x, w = tid / WAVE, lane = tid % WAVE;
  const int lr = lane & 31, h = lane >> 5;
  const int row0 = blockIdx.x * TM;

  // Z rows -> bf16 image (and the bf16 copy for dW1); rows past the end are 0
  constexpr int NI = TM * (TC / 8) / 256;
  float4 va[NI], vb[NI];
#pragma unroll
  for (int u = 0; u < NI; ++u) {
    const int i = tid + 256 * u, m = i / (TC / 8), c = i % (TC / 8);
    va[u] = vb[u] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (row0 + m < rows) {
      const float* src = Z + (long long)(row0 + m) * ldz + 8 * c;
      va[u] = *(const float4*)src;
      vb[u] = *(const float4*)(src + 4);
    }
  }
  if constexpr (LN) {
    // affine values of the same elements (loads in flight with X's), then
    // the two samples' statistics
    float4 wa[NI], wb[NI], ba[NI], bb[NI];
#pragma unroll
    for (int u = 0; u < NI; ++u) {
      const int i = tid + 256 * u, m = i / (TC / 8), c = i % (TC / 8);
      const int p = min(row0 + m, rows - 1) % L.hw;
      const float* wr = L.aff + (long long)p * TC + 8 * c;
      wa[u] = *(const float4*)wr;
      wb[u] = *(const float4*)(wr + 4);
      ba[u] = *(const float4*)(wr + L.E);
      bb[u] = *(const float4*)(wr + L.E + 4);
    }
    // the two samples' slice moments: one load per thread (all in flight),
    // staged in LDS, then combined (Chan, slice order) by two threads
    const int s0 = row0 / L.hw;
    float* mom = (float*)(g_smem + F_MOM);          // [2][S][2]
    if (tid < 4 * L.S) {
      const int sl = tid / (2 * L.S), r = tid % (2 * L.S), b = s0 + sl;
      mom[tid] = b < L.n ? L.part[(long long)b * L.S * 2 + r] : 0.f;
    }
    __syncthreads();
    if (tid < 2) {
      const int b = s0 + tid;
      float mean = 0.f, rstd = 0.f;
      if (b < L.n) {
        if (L.tiles)
          ln_stats_tiles(mom + tid * 2 * L.S, L.S, L.hw, TC, L.eps, mean, rstd);
        else
          ln_stats(mom + tid * 2 * L.S - (long long)b * L.S * 2, L.E, L.S, b, L.eps, mean, rstd);
        if ((long long)b * L.hw >= row0 && (long long)b * L.hw < row0 + TM) {
          L.stats[b] = mean;
          L.stats[L.n + b] = rstd;
        }
      }
      lds_stf(F_LN + 8 * tid, mean);
      lds_stf(F_LN + 8 * tid + 4, rstd);
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < NI; ++u) {
      const int i = tid + 256 * u, m = i / (TC / 8);
      const int sl = min(row0 + m, rows - 1) / L.hw - s0;
      const float mean = lds_ldf(F_LN + 8 * sl), rstd = lds_ldf(F_LN + 8 * sl + 4);
      // (x - mean) rstd w + b, as ln_apply_kernel
      va[u] = make_float4((va[u].x - mean) * rstd * wa[u].x + ba[u].x,
                          (va[u].y - mean) * rstd * wa[u].y + ba[u].y,
                          (va[u].z - mean) * rstd * wa[u].z + ba[u].z,
                          (va[u].w - mean) * rstd * wa[u].w + ba[u].w);
      vb[u] = make_float4((vb[u].x - mean) * rstd * wb[u].x + bb[u].x,
                          (vb[u].y - mean) * rstd * wb[u].y + bb[u].y,
                          (vb[u].z - mean) * rstd * wb[u].z + bb[u].z,
                          (vb[u].w - mean) * rstd * wb[u].w + bb[u].w);
    }
  }
#pragma unroll
  for (int u = 0; u < NI; ++u) {
    const int i = tid + 256 * u, m = i / (TC / 8), c = i % (TC / 8);
    uint4 v = make_uint4(0, 0, 0, 0);
    if (row0 + m < rows) {
      const float4 a = va[u], b = vb[u];
      v = make_uint4(pk_bf16(a.x, a.y), pk_bf16(a.z, a.w), pk_bf16(b.x, b.y), pk_bf16(b.z, b.w));
      *(uint4*)(Zb + (long long)(row0 + m) * TC + 8 * c) = v;
    }
    lds_st16(F_Z + img<TC>(m, c), v);
  }
  __syncthreads();

  // layer 1, transposed: H1^T[i][m] = sum_c W1[i][c] Z[m][c]; wave w: i in [32w, 32w+32)
  {
    f32x16 acc[MT];
#pragma unroll
    for (int t = 0; t < MT; ++t)
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[t][q] = 0.f;
#pragma unroll
    for (int s = 0; s < TC / 16; ++s) {
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const bf16x8 b = as_bf8(lds_ld16(F_Z + img<TC>(32 * mt + lr, 2 * s + h)));
        acc[mt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(gld16(frag_ptr(pk, OFF_W1, TC, w, s, lane)), b, acc[mt], 0, 0, 0);
      }
    }
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int i0 = 32 * w + 8 * g + 4 * h;
      const float4 bb = *(const float4*)(b1 + i0);
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const f32x16& a = acc[mt];
        lds_st8(F_H1 + img_at<TH>(32 * mt + lr, i0),
                pk4(fmaxf(a[4 * g] + bb.x, 0.f), fmaxf(a[4 * g + 1] + bb.y, 0.f),
                    fmaxf(a[4 * g + 2] + bb.z, 0.f), fmaxf(a[4 * g + 3] + bb.w, 0.f)));
      }
    }
  }
  __syncthreads();
  copy_out<TH>(F_H1, H1b, TH, row0, rows, tid);

  // layer 2, transposed: H2^T[j][m] = sum_i W2[j][i] H1[m][i]; wave w: j in [64w, 64w+64)
  {
    f32x16 acc[2][MT];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int u = 0; u < MT; ++u)
#pragma unroll
        for (int q = 0; q < 16; ++q) acc[t][u][q] = 0.f;
#pragma unroll
    for (int s = 0; s < TH / 16; ++s) {
      bf16x8 b[MT];
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
        b[mt] = as_bf8(lds_ld16(F_H1 + img<TH>(32 * mt + lr, 2 * s + h)));
#pragma unroll
      for (int jt = 0; jt < 2; ++jt)
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
          acc[jt][mt] =
              __builtin_amdgcn_mfma_f32_32x32x16_bf16(gld16(frag_ptr(pk, OFF_W2, TH, 2 * w + jt, s, lane)), b[mt], acc[jt][mt], 0, 0, 0);
    }
    // the Z image is dead (every wave passed the barrier after layer 1): H2 reuses it
#pragma unroll
    for (int jt = 0; jt < 2; ++jt)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int j0 = 64 * w + 32 * jt + 8 * g + 4 * h;
        const float4 bb = *(const float4*)(b2 + j0);
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
          const f32x16& a = acc[jt][mt];
          lds_st8(F_H2 + img_at<TC>(32 * mt + lr, j0),
                  pk4(fmaxf(a[4 * g] + bb.x, 0.f), fmaxf(a[4 * g + 1] + bb.y, 0.f),
                      fmaxf(a[4 * g + 2] + bb.z, 0.f), fmaxf(a[4 * g + 3] + bb.w, 0.f)));
        }
      }
  }
  __syncthreads();
  copy_out<TC>(F_H2, H2b, TC, row0, rows, tid);

  // layer 3, upright: P[m][n] = sum_j H2[m][j] Wp[n][j] + bp[n]; wave w: n in [64w, 64w+64)
  f32x16 acc[MT][2];
#pragma unroll
  for (int t = 0; t < MT; ++t)
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[t][u][q] = 0.f;
#pragma unroll
  for (int s = 0; s < TC / 16; ++s) {
    bf16x8 a[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
      a[mt] = as_bf8(lds_ld16(F_H2 + img<TC>(32 * mt + lr, 2 * s + h)));
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int nt = 0; nt < 2; ++nt)
        acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[mt], gld16(frag_ptr(pk, OFF_WP, TC, 2 * w + nt, s, lane)), acc[mt][nt], 0, 0, 0);
  }
  // bias, then the row sums of squares: lane-local over this wave's two
  // column tiles, then over the 32 columns of each half-wave (rs16)
#pragma unroll
  for (int nt = 0; nt < 2; ++nt) {
    const float bb = bp[64 * w + 32 * nt + lr];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[mt][nt][q] += bb;
  }
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    float sq[16];
#pragma unroll
    for (int q = 0; q < 16; ++q)
      sq[q] = acc[mt][0][q] * acc[mt][0][q] + acc[mt][1][q] * acc[mt][1][q];
    const float tot = rs16(sq, lr);
    if (!(lr & 1))
      lds_stf(F_SS + (w * TM + 32 * mt + acc_row(rs16_index(lr), h)) * 4, tot);
  }
  __syncthreads();
  if (tid < TM) {
    const float ss = lds_ldf(F_SS + tid * 4) + lds_ldf(F_SS + (TM + tid) * 4) +
                     lds_ldf(F_SS + (2 * TM + tid) * 4) + lds_ldf(F_SS + (3 * TM + tid) * 4);
    const float nrm = sqrtf(ss);
    const float iv = 1.f / fmaxf(nrm, eps);
    lds_stf(F_INV + tid * 4, iv);
    if (row0 + tid < rows) {
      inv_out[row0 + tid] = iv;
      // |R_row| for the word<->region kernels (tgfr_prep_rows' norms)
      if (Rnorm) {
        const int it = (row0 + tid) / rows_per_item, ri = (row0 + tid) % rows_per_item;
        Rnorm[(long long)it * rows_pad + ri] = nrm * iv;
      }
    }
  }
  __syncthreads();
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int m = 32 * mt + acc_row(q, h);
      if (row0 + m < rows) {
        const float iv = lds_ldf(F_INV + m * 4);
        float* o = R + (long long)(row0 + m) * ldr + 64 * w + lr;
        o[0] = acc[mt][0][q] * iv;
        o[32] = acc[mt][1][q] * iv;
      }
    }
  if (Rrows) {
    // R rows in the contraction's operand layout: [item][rows_pad][256] bf16
    // (or fp16), what tgfr_prep_rows would make of R.  Lanes lr, lr ^ 1 hold
    // adjacent columns: they swap one value so each stores a 4-byte pair --
    // the even lane row acc_row(q), the odd lane row acc_row(q + 1)
    const bool odd = lr & 1;
    auto bits = [&](float x) { return rows_f16 ? f16_bits(x) : bf_bits(x); };
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int q = 0; q < 16; q += 2) {
        const int m0 = 32 * mt + acc_row(q, h), m1 = 32 * mt + acc_row(q + 1, h);
        const float i0 = lds_ldf(F_INV + m0 * 4), i1 = lds_ldf(F_INV + m1 * 4);
        const int m = odd ? m1 : m0;
        const int it = (row0 + m) / rows_per_item, ri = (row0 + m) % rows_per_item;
        uint16_t* d = Rrows + ((long long)it * rows_pad + ri) * TD + 64 * w + (lr & ~1);
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) {
          const float a = acc[mt][nt][q] * i0, b = acc[mt][nt][q + 1] * i1;
          const float y = __shfl_xor(odd ? a : b, 1);
          const uint32_t pk = odd ? pack2(bits(y), bits(b)) : pack2(bits(a), bits(y));
          if (row0 + m < rows) *(uint32_t*)(d + 32 * nt) = pk;
        }
      }
    // the padding rows (rows_per_item .. rows_pad) of every item whose last
    // row this workgroup holds: zero rows, zero norms
    for (int m = 0; m < TM; ++m) {
      const int row = row0 + m;
      if (row >= rows || row % rows_per_item != rows_per_item - 1) continue;
      const int it = row / rows_per_item, npad = rows_pad - rows_per_item;
      uint16_t* d = Rrows + ((long long)it * rows_pad + rows_per_item) * TD;
      for (int i = tid; i < npad * (TD / 8); i += 256) *(uint4*)(d + 8 * i) = make_uint4(0, 0, 0, 0);
      if (Rnorm && tid < npad) Rnorm[(long long)it * rows_pad + rows_per_item + tid] = 0.f;
    }
  }
}

// ----------------------------------------------------------- backward ---
// LDS: [0, 32K) dP image (later the dH1 image), [32K, 64K) dH2 image
constexpr int B_DP = 0, B_DH1 = 0, B_DH2 = TM * TD * 2, B_LDS = 2 * TM * TD * 2;

// LN = true: the IMIM LayerNorm's backward needs, per sample, the sums of
// g = dZ w and g xhat (xhat = (X - mean) rstd): each workgroup adds its rows'
// terms (two sample slots: 32 rows span at most two samples of hw >= 32) and
// writes part[blockIdx.x][slot][2] (PartSrc tail layout) -- no separate pass
// over dZ and X.
struct LnBwd {
  const float* X;         // the LayerNorm input rows [rows][TC]
  const float* stats;     // mean [n] | rstd [n] (tail_fwd<true>)
  const float* w;         // affine w as channels-last rows [hw][TC]
  float* part;            // [gridDim.x][2][2]
  int hw, n;
  int dzb;                // dZ rows in bf16 (the attention path's LayerNorm dx reads them)
};
constexpr int B_RED = B_LDS, B_LDS_LN = B_LDS + 4 * 4 * 4;

template <bool LN>
__global__ __launch_bounds__(256) void tail_bwd_kernel(
    const float* __restrict__ dR, long long lddr, const float* __restrict__ R, long long ldr,
    const float* __restrict__ inv, int rows, float eps, const uint16_t* __restrict__ pk,
    const uint16_t* __restrict__ H1b, const uint16_t* __restrict__ H2b, float* __restrict__ dZ,
    long long lddz, uint16_t* __restrict__ dPb, uint16_t* __restrict__ dH2b,
    uint16_t* __restrict__ dH1b, LnBwd L) {
  const int tid = threadIdx.x, w = tid / WAVE, lane = tid % WAVE;
  const int lr = lane & 31, h = lane >> 5;
  const int row0 = blockIdx.x * TM;

  // F.normalize backward, one row per wave pass (lane: 4 columns)
#pragma unroll 2
  for (int r = 0; r < TM / 4; ++r) {
    const int m = (TM / 4) * w + r, row = row0 + m;
    float4 g = make_float4(0.f, 0.f, 0.f, 0.f), y = g;
    float iv = 0.f;
    if (row < rows) {
      g = *(const float4*)(dR + (long long)row * lddr + 4 * lane);
      y = *(const float4*)(R + (long long)row * ldr + 4 * lane);
      iv = inv[row];
    }
    float dot = wave_sum(g.x * y.x + g.y * y.y + g.z * y.z + g.w * y.w);
    if (iv >= 1.f / eps) dot = 0.f;          // clamped row: y = x / eps
    const uint2 v = pk4((g.x - y.x * dot) * iv, (g.y - y.y * dot) * iv,
                        (g.z - y.z * dot) * iv, (g.w - y.w * dot) * iv);
    lds_st8(B_DP + img_at<TD>(m, 4 * lane), v);
    if (row < rows) *(uint2*)(dPb + (long long)row * TD + 4 * lane) = v;
  }
  // LN: the X / affine values (and the two samples' statistics) the epilogue's
  // LayerNorm sums read, issued here so that their latency hides behind the
  // three GEMMs instead of trailing the kernel (64 registers; the LDS already
  // limits the CU to two workgroups, whose register budget this fits)
  float lx[MT][16][2], lw[MT][16][2], lm0 = 0.f, lr0 = 0.f, lm1 = 0.f, lr1 = 0.f;
  if constexpr (LN) {
    const int s0 = row0 / L.hw;
    lm0 = L.stats[s0];
    lr0 = L.stats[L.n + s0];
    if (s0 + 1 < L.n) {
      lm1 = L.stats[s0 + 1];
      lr1 = L.stats[L.n + s0 + 1];
    }
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int row = min(row0 + 32 * mt + acc_row(q, h), rows - 1), p = row % L.hw;
#pragma unroll
        for (int ct = 0; ct < 2; ++ct) {
          const int c = 64 * w + 32 * ct + lr;
          lx[mt][q][ct] = L.X[(long long)row * TC + c];
          lw[mt][q][ct] = L.w[(long long)p * TC + c];
        }
      }
  }
  __syncthreads();

  // dH2^T[j][m] = sum_n Wp[n][j] dP[m][n] (A = Wp^T rows); wave w: j in [64w, 64w+64)
  bf16x8 g2[TC / 16];
  {
    // relu masks first: H2[m][j0..j0+3] for this lane's accumulator quads
    uint2 msk[2][MT][4];
#pragma unroll
    for (int jt = 0; jt < 2; ++jt)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int row = row0 + 32 * mt + lr, j0 = 64 * w + 32 * jt + 8 * g + 4 * h;
          msk[jt][mt][g] = row < rows ? *(const uint2*)(H2b + (long long)row * TC + j0)
                                      : make_uint2(0, 0);
        }
    f32x16 acc[2][MT];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int u = 0; u < MT; ++u)
#pragma unroll
        for (int q = 0; q < 16; ++q) acc[t][u][q] = 0.f;
#pragma unroll
    for (int s = 0; s < TD / 16; ++s) {
      bf16x8 b[MT];
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
        b[mt] = as_bf8(lds_ld16(B_DP + img<TD>(32 * mt + lr, 2 * s + h)));
#pragma unroll
      for (int jt = 0; jt < 2; ++jt)
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
          acc[jt][mt] =
              __builtin_amdgcn_mfma_f32_32x32x16_bf16(gld16(frag_ptr(pk, OFF_WPT, TD, 2 * w + jt, s, lane)), b[mt], acc[jt][mt], 0, 0, 0);
    }
    // the next GEMM's W2^T fragments, loaded across this phase's barrier
#pragma unroll
    for (int s = 0; s < TC / 16; ++s) g2[s] = gld16(frag_ptr(pk, OFF_W2T, TC, w, s, lane));
#pragma unroll
    for (int jt = 0; jt < 2; ++jt)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int j0 = 64 * w + 32 * jt + 8 * g + 4 * h;
          const uint2 mk = msk[jt][mt][g];
          const f32x16& a = acc[jt][mt];
          // bf16 bits > 0 as a signed 16-bit value <=> the activation is positive
          const float v0 = (short)(mk.x & 0xffff) > 0 ? a[4 * g] : 0.f;
          const float v1 = (short)(mk.x >> 16) > 0 ? a[4 * g + 1] : 0.f;
          const float v2 = (short)(mk.y & 0xffff) > 0 ? a[4 * g + 2] : 0.f;
          const float v3 = (short)(mk.y >> 16) > 0 ? a[4 * g + 3] : 0.f;
          lds_st8(B_DH2 + img_at<TC>(32 * mt + lr, j0), pk4(v0, v1, v2, v3));
        }
  }
  __syncthreads();
  copy_out<TC>(B_DH2, dH2b, TC, row0, rows, tid);

  // dH1^T[i][m] = sum_j W2[j][i] dH2[m][j] (A = W2^T rows); wave w: i in [32w, 32w+32)
  bf16x8 g1[TH / 16][2];
  {
    uint2 msk[MT][4];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int row = row0 + 32 * mt + lr, i0 = 32 * w + 8 * g + 4 * h;
        msk[mt][g] = row < rows ? *(const uint2*)(H1b + (long long)row * TH + i0)
                                : make_uint2(0, 0);
      }
    f32x16 acc[MT];
#pragma unroll
    for (int t = 0; t < MT; ++t)
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[t][q] = 0.f;
#pragma unroll
    for (int s = 0; s < TC / 16; ++s) {
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const bf16x8 b = as_bf8(lds_ld16(B_DH2 + img<TC>(32 * mt + lr, 2 * s + h)));
        acc[mt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(g2[s], b, acc[mt], 0, 0, 0);
      }
    }
#pragma unroll
    for (int s = 0; s < TH / 16; ++s)
#pragma unroll
      for (int ct = 0; ct < 2; ++ct) g1[s][ct] = gld16(frag_ptr(pk, OFF_W1T, TH, 2 * w + ct, s, lane));
    // the dP image is dead (every wave passed the barrier before this GEMM)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int i0 = 32 * w + 8 * g + 4 * h;
        const uint2 mk = msk[mt][g];
        const f32x16& a = acc[mt];
        const float v0 = (short)(mk.x & 0xffff) > 0 ? a[4 * g] : 0.f;
        const float v1 = (short)(mk.x >> 16) > 0 ? a[4 * g + 1] : 0.f;
        const float v2 = (short)(mk.y & 0xffff) > 0 ? a[4 * g + 2] : 0.f;
        const float v3 = (short)(mk.y >> 16) > 0 ? a[4 * g + 3] : 0.f;
        lds_st8(B_DH1 + img_at<TH>(32 * mt + lr, i0), pk4(v0, v1, v2, v3));
      }
  }
  __syncthreads();
  copy_out<TH>(B_DH1, dH1b, TH, row0, rows, tid);

  // dZ[m][c] = sum_i dH1[m][i] W1[i][c] (B = W1^T rows); wave w: c in [64w, 64w+64)
  f32x16 acc[MT][2];
#pragma unroll
  for (int t = 0; t < MT; ++t)
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[t][u][q] = 0.f;
#pragma unroll
  for (int s = 0; s < TH / 16; ++s) {
    bf16x8 a[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
      a[mt] = as_bf8(lds_ld16(B_DH1 + img<TH>(32 * mt + lr, 2 * s + h)));
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int ct = 0; ct < 2; ++ct)
        acc[mt][ct] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[mt], g1[s][ct], acc[mt][ct], 0, 0, 0);
  }
  if (LN && L.dzb) {
    // bf16 rows (stride lddz elements): lanes lr, lr ^ 1 trade one value so
    // that the even lane stores row q's column pair and the odd lane row q + 1's
    uint16_t* dzb = (uint16_t*)dZ;
    const bool odd = lr & 1;
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int q = 0; q < 16; q += 2) {
        const int row = row0 + 32 * mt + acc_row(odd ? q + 1 : q, h);
#pragma unroll
        for (int ct = 0; ct < 2; ++ct) {
          const float a = acc[mt][ct][q], b = acc[mt][ct][q + 1];
          const float y = __shfl_xor(odd ? a : b, 1);
          if (row < rows)
            *(uint32_t*)(dzb + (long long)row * lddz + 64 * w + 32 * ct + (lr & ~1)) =
                odd ? pk_bf16(y, b) : pk_bf16(a, y);
        }
      }
  } else {
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int row = row0 + 32 * mt + acc_row(q, h);
        if (row < rows) {
          float* o = dZ + (long long)row * lddz + 64 * w + lr;
          o[0] = acc[mt][0][q];
          o[32] = acc[mt][1][q];
        }
      }
  }
  if constexpr (LN) {
    const int s0 = row0 / L.hw;
    float sg[2] = {0.f, 0.f}, sgx[2] = {0.f, 0.f};
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int row = row0 + 32 * mt + acc_row(q, h);
        if (row >= rows) continue;
        const int sl = row / L.hw - s0;
        const float mean = sl ? lm1 : lm0, rstd = sl ? lr1 : lr0;
#pragma unroll
        for (int ct = 0; ct < 2; ++ct) {
          const float g = acc[mt][ct][q] * lw[mt][q][ct];
          const float xh = (lx[mt][q][ct] - mean) * rstd;
          if (sl) { sg[1] += g; sgx[1] += g * xh; }
          else { sg[0] += g; sgx[0] += g * xh; }
        }
      }
    float* red = (float*)(g_smem + B_RED);
    const float t0 = wave_sum(sg[0]), t1 = wave_sum(sgx[0]);
    const float t2 = wave_sum(sg[1]), t3 = wave_sum(sgx[1]);
    if (lane == 0) {
      red[4 * w] = t0;
      red[4 * w + 1] = t1;
      red[4 * w + 2] = t2;
      red[4 * w + 3] = t3;
    }
    __syncthreads();
    if (tid < 4)
      L.part[(long long)blockIdx.x * 4 + tid] =
          (red[tid] + red[4 + tid]) + (red[8 + tid] + red[12 + tid]);
  }
}

// ------------------------------------------------- weight gradients ---
// dW[n][k] = sum_rows X[row][n] Y[row][k] and db[n] = sum_rows X[row][n] for
// the three products of the tail; X, Y bf16 rows.  Workgroup = (product,
// 128 x 128 output block, row slice); 4 waves of 64 x 64 (2 x 2 tiles).  Row
// chunks of 32 are staged in LDS as rows with a 64-B pad per row (row pitch
// = 64 mod 256 B: the 4 rows x 64 B of one ds_read_b64_tr_b16 lane half hit
// distinct banks); the MFMA operands (X^T and Y with rows as the reduction
// axis) come out of the transposing read.
constexpr int DW_NB = 128, DW_CH = 32;
constexpr int DW_PITCH = DW_NB * 2 + 64;               // bytes per staged row
constexpr int DW_IMG = DW_CH * DW_PITCH;               // one operand chunk
constexpr int DW_LDS = 6 * DW_IMG;                     // X, Y, three buffers

struct DwProb {
  const uint16_t* X;
  const void* Y;     // bf16, or fp32 when yf32 (converted while staging)
  int yf32;
  int N, K;          // X row width (= ld), Y row width (= ld)
  int nb_n, nb_k;    // 128-blocks
  int first;         // first workgroup of this product
  long long slab;    // float offset of this product's slabs in the workspace
};
constexpr int DW_MAXP = 4;   // products per launch
struct DwArgs {
  DwProb p[DW_MAXP];
  int rows, slices, rows_per;
  int bf16slab;      // 1: the dW slabs in bf16 (half the slab bytes), column sums fp32
};

// operand fragment from a staged chunk: lane (col c = col0 + lane%32, rows
// 16 s + 8 h .. +7), as the bf16x8 of a 32x32x16 MFMA operand
__device__ __forceinline__ bf16x8 tr_frag(uint32_t base, int col0, int s, int lane) {
  const int i = lane & 15, q = i >> 2, p = i & 3, g = lane >> 4;
  const int col = col0 + 16 * (g & 1) + 4 * p;
  const int r = 16 * s + 8 * (g >> 1) + q;
  const uint32_t a = base + r * DW_PITCH + col * 2;
  return join_tr(lds_tr4(a), lds_tr4(a + 4 * DW_PITCH));
}

// raw Y staging registers: fp32 Y is kept as loaded until it is stored to
// LDS (converting at load time would wait on the load and defeat the
// prefetch ring)
struct YF32Piece {
  float4 a, b;
};
template <bool YF32>
using YPiece = typename std::conditional<YF32, YF32Piece, uint4>::type;

template <bool YF32>
__global__ __launch_bounds__(256) void tail_dw_kernel(DwArgs A, float* __restrict__ ws) {
  const int tid = threadIdx.x, wv = tid / WAVE, lane = tid % WAVE;
  const int total = gridDim.x;
  // consecutive ids after the remap: the blocks of one (product, slice) on one XCD
  const int wgi = xcd_remap(blockIdx.x, total);
  int pi = 0;
#pragma unroll
  for (int i = 1; i < DW_MAXP; ++i)
    if (wgi >= A.p[i].first) pi = i;
  const DwProb P = A.p[pi];
  const int local = wgi - P.first;
  const int nblk = P.nb_n * P.nb_k;
  const int slice = local / nblk, blk = local % nblk;
  const int bn = blk / P.nb_k, bk = blk % P.nb_k;
  const int r_begin = slice * A.rows_per, r_end = min(A.rows, r_begin + A.rows_per);
  const int n_chunks = max(0, (r_end - r_begin + DW_CH - 1) / DW_CH);
  const int wn = wv >> 1, wk = wv & 1;

  f32x16 acc[2][2];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[t][u][q] = 0.f;
  float cs[2] = {0.f, 0.f};

  // staging: thread t loads 16 B of X and 16 B of Y per pass; 2 passes per chunk
  using YP = YPiece<YF32>;
  auto load = [&](int c, uint4 (&vx)[2], YP (&vy)[2]) {
#pragma unroll
    for (int ps = 0; ps < 2; ++ps) {
      const int i = tid + 256 * ps, r = i / 16, c16 = i % 16;
      const int row = r_begin + c * DW_CH + r;
      const long long yo = (long long)row * P.K + bk * DW_NB + 8 * c16;
      const bool ok = row < r_end;
      vx[ps] = ok ? *(const uint4*)(P.X + (long long)row * P.N + bn * DW_NB + 8 * c16)
                  : make_uint4(0, 0, 0, 0);
      if constexpr (YF32) {
        const float* yp = (const float*)P.Y + yo;
        vy[ps].a = ok ? *(const float4*)yp : make_float4(0.f, 0.f, 0.f, 0.f);
        vy[ps].b = ok ? *(const float4*)(yp + 4) : make_float4(0.f, 0.f, 0.f, 0.f);
      } else {
        vy[ps] = ok ? *(const uint4*)((const uint16_t*)P.Y + yo) : make_uint4(0, 0, 0, 0);
      }
    }
  };
  auto store = [&](int buf, const uint4 (&vx)[2], const YP (&vy)[2]) {
#pragma unroll
    for (int ps = 0; ps < 2; ++ps) {
      const int i = tid + 256 * ps, r = i / 16, c16 = i % 16;
      lds_st16(buf * 2 * DW_IMG + r * DW_PITCH + 16 * c16, vx[ps]);
      uint4 y;
      if constexpr (YF32)
        y = make_uint4(pk_bf16(vy[ps].a.x, vy[ps].a.y), pk_bf16(vy[ps].a.z, vy[ps].a.w),
                       pk_bf16(vy[ps].b.x, vy[ps].b.y), pk_bf16(vy[ps].b.z, vy[ps].b.w));
      else
        y = vy[ps];
      lds_st16(buf * 2 * DW_IMG + DW_IMG + r * DW_PITCH + 16 * c16, y);
    }
  };
  auto compute = [&](int buf) {
    const uint32_t bx = buf * 2 * DW_IMG, by = bx + DW_IMG;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8 a[2], b[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) a[t] = tr_frag(bx, 64 * wn + 32 * t, s, lane);
#pragma unroll
      for (int u = 0; u < 2; ++u) b[u] = tr_frag(by, 64 * wk + 32 * u, s, lane);
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int u = 0; u < 2; ++u)
          acc[t][u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[t], b[u], acc[t][u], 0, 0, 0);
      if (wk == 0 && bk == 0) {
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
          for (int j = 0; j < 8; ++j) cs[t] += (float)a[t][j];
      }
    }
  };
  // three chunks in flight: chunk c sits in register slot c % 3 from its load
  // (issued three steps ahead) until it is stored to LDS buffer c % 3 one
  // step before it is used
  uint4 rx[3][2];
  YP ry[3][2];
#pragma unroll
  for (int j = 0; j < 3; ++j)
    if (j < n_chunks) load(j, rx[j], ry[j]);
  if (n_chunks > 0) store(0, rx[0], ry[0]);
  __syncthreads();
  auto step = [&](auto J, int c) {
    constexpr int j = decltype(J)::value, j1 = (j + 1) % 3;
    if (c + 1 < n_chunks) store(j1, rx[j1], ry[j1]);
    if (c + 3 < n_chunks) load(c + 3, rx[j], ry[j]);
    compute(j);
    __syncthreads();
  };
  for (int c = 0; c < n_chunks; c += 3) {
    step(std::integral_constant<int, 0>{}, c);
    if (c + 1 < n_chunks) step(std::integral_constant<int, 1>{}, c + 1);
    if (c + 2 < n_chunks) step(std::integral_constant<int, 2>{}, c + 2);
  }

  // slab [slice][N][K] (+ [slice][N] column sums after all products' dW slabs)
  if (A.bf16slab) {
    // bf16 slab: lanes lr, lr ^ 1 hold adjacent k: they swap one value so each
    // stores a 4-byte pair -- the even lane row acc_row(q), the odd lane row
    // acc_row(q + 1)
    uint16_t* slab = (uint16_t*)(ws + P.slab) + (long long)slice * P.N * P.K;
    const bool odd = lane & 1;
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int q = 0; q < 16; q += 2) {
          const float a = acc[t][u][q], b = acc[t][u][q + 1];
          const float y = __shfl_xor(odd ? a : b, 1);
          const int n = bn * DW_NB + 64 * wn + 32 * t + acc_row(odd ? q + 1 : q, lane >> 5);
          const int k = bk * DW_NB + 64 * wk + 32 * u + ((lane & 31) & ~1);
          *(uint32_t*)(slab + (long long)n * P.K + k) = odd ? pk_bf16(y, b) : pk_bf16(a, y);
        }
  } else {
    float* slab = ws + P.slab + (long long)slice * P.N * P.K;
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          const int n = bn * DW_NB + 64 * wn + 32 * t + acc_row(q, lane >> 5);
          const int k = bk * DW_NB + 64 * wk + 32 * u + (lane & 31);
          slab[(long long)n * P.K + k] = acc[t][u][q];
        }
  }
  if (wk == 0 && bk == 0) {
    float* cslab = ws + P.slab + (long long)A.slices * P.N * P.K / (A.bf16slab ? 2 : 1) +
                   (long long)slice * P.N;
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const float v = xhalf_sum(cs[t]);
      if (lane < 32) cslab[bn * DW_NB + 64 * wn + 32 * t + lane] = v;
    }
  }
}

struct DwOut {
  float* dW[DW_MAXP];
  float* db[DW_MAXP];
  // optional (lnE > 0): the IMIM LayerNorm's weight / bias gradients from the
  // group partials its backward left (ln_bwd_dx: dw [lng][lnE] then db
  // [lng][lnE], channels-last e = p * 256 + c), summed in group order like
  // ln_bwd_dw and scattered to the reference's [256][hw] maps
  const float* lnp;
  long long lnE;
  int lng, lnhw;
  float* dlnw;
  float* dlnb;
};

// out = sum over slices, in slice order; thread = 2 consecutive outputs (a
// grid of ~2 workgroups per CU) with 8 slice loads in flight.  Threads past
// the products' e_total outputs reduce the LayerNorm partials (O.lnE > 0).
__global__ __launch_bounds__(256) void tail_dw_reduce_kernel(DwArgs A, DwOut O,
                                                             const float* __restrict__ ws,
                                                             long long e_total) {
  const long long e4 = (blockIdx.x * 256LL + threadIdx.x) * 2;
  if (e4 >= e_total) {
    long long off = e4 - e_total;      // (e_total and lnE are even: pairs never straddle)
    if (off >= 2 * O.lnE) return;
    const bool bias = off >= O.lnE;
    if (bias) off -= O.lnE;
    const float* src = O.lnp + (bias ? (long long)O.lng * O.lnE : 0) + off;
    float2 s = make_float2(0.f, 0.f);
    for (int k = 0; k < O.lng; ++k) {
      const float2 v = *(const float2*)(src + k * O.lnE);
      s.x += v.x;
      s.y += v.y;
    }
    float* dst = bias ? O.dlnb : O.dlnw;
    // channels-last e -> channel-major [TC][hw] (e and e + 1: channels c, c + 1)
    const long long p = off / TC;
    const int c = (int)(off % TC);
    dst[(long long)c * O.lnhw + p] = s.x;
    dst[(long long)(c + 1) * O.lnhw + p] = s.y;
    return;
  }
  // which product / region: products laid out as [dW N*K][db N] each
  long long off = e4;
  int pi = 0;
  for (; pi < DW_MAXP - 1; ++pi) {
    const long long sz = (long long)A.p[pi].N * A.p[pi].K + A.p[pi].N;
    if (off < sz) break;
    off -= sz;
  }
  const DwProb P = A.p[pi];
  const long long nk = (long long)P.N * P.K;
  if (A.bf16slab && off < nk) {
    // bf16 dW slabs: one 4-byte pair per slice
    const uint32_t* bsrc = (const uint32_t*)((const uint16_t*)(ws + P.slab) + off);
    float2 s = make_float2(0.f, 0.f);
#pragma unroll 8
    for (int z = 0; z < A.slices; ++z) {
      const uint32_t v = bsrc[(long long)z * (nk / 2)];
      s.x += __uint_as_float(v << 16);
      s.y += __uint_as_float(v & 0xffff0000u);
    }
    *(float2*)(O.dW[pi] + off) = s;
    return;
  }
  const float* src;
  long long stride;
  float* dst;
  if (off < nk) {
    src = ws + P.slab + off;
    stride = nk;
    dst = O.dW[pi] + off;
  } else {
    src = ws + P.slab + A.slices * nk / (A.bf16slab ? 2 : 1) + (off - nk);
    stride = P.N;
    dst = O.db[pi] + (off - nk);
  }
  float2 s = make_float2(0.f, 0.f);
#pragma unroll 8
  for (int z = 0; z < A.slices; ++z) {
    const float2 v = *(const float2*)(src + z * stride);
    s.x += v.x;
    s.y += v.y;
  }
  *(float2*)dst = s;
}

// n products (N[i] x K[i], multiples of 128) over `rows` rows; wg_budget:
// workgroups to aim for (the slabs, slices x sum N K floats, are written and
// read back once more by the reduce, so fewer slices trade chip fill for
// traffic)
void dw_plan_n(int rows, int n, const int* NS, const int* KS, int wg_budget, DwArgs& A,
               long long& ws_floats, int& n_wg, bool bf16slab = false) {
  int blocks = 0;
  for (int i = 0; i < n; ++i) blocks += (NS[i] / DW_NB) * (KS[i] / DW_NB);
  const int want = std::max(1, wg_budget / blocks);
  const int max_slices = std::max(1, rows / (4 * DW_CH));
  A.slices = std::min(want, max_slices);
  A.rows_per = ((rows + A.slices - 1) / A.slices + DW_CH - 1) / DW_CH * DW_CH;
  A.rows = rows;
  A.bf16slab = bf16slab ? 1 : 0;
  long long slab = 0;
  int first = 0;
  for (int i = 0; i < n; ++i) {
    DwProb& p = A.p[i];
    p.N = NS[i];
    p.K = KS[i];
    p.nb_n = NS[i] / DW_NB;
    p.nb_k = KS[i] / DW_NB;
    p.first = first;
    p.slab = slab;
    p.yf32 = 0;
    first += p.nb_n * p.nb_k * A.slices;
    slab += (long long)A.slices * (p.N * (long long)p.K / (bf16slab ? 2 : 1) + p.N);
  }
  for (int i = n; i < DW_MAXP; ++i) {  // unused: no workgroup, nothing to reduce
    A.p[i] = DwProb{nullptr, nullptr, 0, 0, 0, 0, 0, first, slab};
  }
  ws_floats = slab;
  n_wg = first;
}

void dw_plan(int rows, DwArgs& A, long long& ws_floats, int& n_wg) {
  // slices: one workgroup per CU (the slabs, slices x 0.53 MB written here
  // and read back by the reduce, are then ~half the 32 MB of operands at the
  // step's 12544 rows); at least 4 chunks per slice
  const int NS[3] = {TD, TC, TH}, KS[3] = {TC, TH, TC};   // dWp, dW2, dW1
  dw_plan_n(rows, 3, NS, KS, 256, A, ws_floats, n_wg);
}

int dw_launch(const DwArgs& A, int n_wg, const DwOut& O, float* ws, hipStream_t s) {
  const bool yf32 = A.p[0].yf32 != 0;      // uniform over the launch's products
  auto fn = yf32 ? &tail_dw_kernel<true> : &tail_dw_kernel<false>;
  if (const int e = set_max_lds((const void*)fn, DW_LDS)) return e;
  hipLaunchKernelGGL(fn, dim3(n_wg), dim3(256), DW_LDS, s, A, ws);
  long long e_total = 0;
  for (int i = 0; i < DW_MAXP; ++i) e_total += (long long)A.p[i].N * A.p[i].K + A.p[i].N;
  const long long e_all = e_total + 2 * O.lnE;
  hipLaunchKernelGGL(tail_dw_reduce_kernel, dim3((unsigned)((e_all / 2 + 255) / 256)),
                     dim3(256), 0, s, A, O, ws, e_total);
  return (int)hipGetLastError();
}

}  // namespace

extern "C" {

int tgfr_tail_pack_elems(void) { return PACK_ELEMS; }

int tgfr_tail_pack(const float* W1, const float* W2, const float* Wp, uint16_t* pk,
                   void* stream) {
  if (!W1 || !W2 || !Wp || !pk) return 1001;
  hipLaunchKernelGGL(tail_pack_kernel, dim3((PACK_UNITS + 255) / 256), dim3(256), 0,
                     (hipStream_t)stream, W1, W2, Wp, pk, nullptr, nullptr, 0, nullptr);
  return (int)hipGetLastError();
}

int tgfr_tail_fwd(const float* Z, long long ldz, int rows, const uint16_t* pk, const float* b1,
                  const float* b2, const float* bp, float eps, float* R, long long ldr,
                  uint16_t* Zb, uint16_t* H1b, uint16_t* H2b, float* inv, uint16_t* Rrows,
                  float* Rnorm, int rows_per_item, int rows_pad, int rows_f16, void* stream) {
  if (rows <= 0 || ldz < TC || ldr < TD || (ldz & 3) || (ldr & 3)) return 1001;
  if (((uintptr_t)Z & 15) || !pk || !b1 || !b2 || !bp || !R || !Zb || !H1b || !H2b || !inv)
    return 1001;
  if ((Rrows || Rnorm) && (rows_per_item <= 0 || rows_pad < rows_per_item ||
                           rows % rows_per_item || ((uintptr_t)Rrows & 15)))
    return 1001;
  hipLaunchKernelGGL(tail_fwd_kernel<false>, dim3((rows + TM - 1) / TM), dim3(256), F_LDS,
                     (hipStream_t)stream, Z, ldz, rows, pk, b1, b2, bp, eps, R, ldr, Zb, H1b, H2b,
                     inv, Rrows, Rnorm, rows_per_item > 0 ? rows_per_item : 1, rows_pad,
                     rows_f16 ? 1 : 0, LnFwd{});
  return (int)hipGetLastError();
}

int tgfr_tail_bwd(const float* dR, long long lddr, const float* R, long long ldr,
                  const float* inv, int rows, float eps, const uint16_t* pk, const uint16_t* H1b,
                  const uint16_t* H2b, float* dZ, long long lddz, uint16_t* dPb, uint16_t* dH2b,
                  uint16_t* dH1b, void* stream) {
  if (rows <= 0 || lddr < TD || ldr < TD || lddz < TC || (lddr & 3) || (ldr & 3)) return 1001;
  if (((uintptr_t)dR & 15) || ((uintptr_t)R & 15) || !inv || !pk || !H1b || !H2b || !dZ ||
      !dPb || !dH2b || !dH1b)
    return 1001;
  hipLaunchKernelGGL(tail_bwd_kernel<false>, dim3((rows + TM - 1) / TM), dim3(256), B_LDS,
                     (hipStream_t)stream, dR, lddr, R, ldr, inv, rows, eps, pk, H1b, H2b, dZ,
                     lddz, dPb, dH2b, dH1b, LnBwd{});
  return (int)hipGetLastError();
}

// ---- the tail with IMIM's LayerNorm fused in (bf16 / fp16 step path) ----
// ws floats: the attention's 32-row tile moments [n][ceil(hw / 32)][2]
// (tgfr_attn_fwd_ln writes them at the start of the buffer) | the LayerNorm
// workspace (LnWs of n = rows / hw samples, E = hw * 256) | tail_bwd<true>'s
// per-workgroup sums [ceil(rows / TM)][2][2] | the affine maps as
// channels-last rows [2][hw][256] (tgfr_tail_pack_ln)
struct LnTailWs {
  long long ln, tp, aff, total;
  int n;
  long long E;
};
static LnTailWs ln_tail_ws(int rows, int hw) {
  LnTailWs o;
  o.n = rows / hw;
  o.E = (long long)hw * TC;
  o.ln = ((long long)o.n * ((hw + 31) / 32) * 2 + 3) & ~3LL;
  const LnWs l = ln_ws(o.n, o.E, TC);
  o.tp = o.ln + l.total_bwd;
  o.aff = o.tp + 4LL * ((rows + TM - 1) / TM);
  o.total = o.aff + 2 * o.E;
  return o;
}
static bool ln_tail_ok(int rows, int hw) {
  // (the tail's load combines at most 64 slice moments per sample)
  return rows > 0 && hw >= TM && rows % hw == 0 && rows / hw <= 65535 &&
         slices_for(rows / hw, (long long)hw * TC) <= 64;
}

int tgfr_ln_tail_ws(int rows, int hw, long long* floats) {
  if (!ln_tail_ok(rows, hw) || !floats) return 1001;
  *floats = ln_tail_ws(rows, hw).total;
  return 0;
}

int tgfr_tail_pack_ln(const float* W1, const float* W2, const float* Wp, const float* lnw,
                      const float* lnb, int rows, int hw, uint16_t* pk, float* ws, void* stream) {
  if (!W1 || !W2 || !Wp || !pk || !lnw || !lnb || !ws || !ln_tail_ok(rows, hw)) return 1001;
  const LnTailWs o = ln_tail_ws(rows, hw);
  const long long n = PACK_UNITS + 2 * o.E;
  hipLaunchKernelGGL(tail_pack_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, W1, W2, Wp, pk, lnw, lnb, hw, ws + o.aff);
  return (int)hipGetLastError();
}

int tgfr_imim_pack(const float* const* Wqkv, const float* const* bqkv, int rows_qkv, int C,
                   const float* gamma, const float* beta, float* Wf, float* bf, const float* W1,
                   const float* W2, const float* Wp, const float* lnw, const float* lnb,
                   int rows, int hw, uint16_t* pk, float* ws, void* stream) {
  if (!Wqkv || !Wqkv[0] || !Wqkv[1] || !Wqkv[2] || rows_qkv <= 0 || C <= 0 || !gamma || !beta ||
      !Wf || !bf || !W1 || !W2 || !Wp || !pk || !lnw || !lnb || !ws || !ln_tail_ok(rows, hw))
    return 1001;
  const Parts P{Wqkv[0], Wqkv[1], Wqkv[2],
                bqkv ? bqkv[0] : nullptr, bqkv ? bqkv[1] : nullptr, bqkv ? bqkv[2] : nullptr,
                rows_qkv};
  const int O = 3 * rows_qkv, nf = (O + 3) / 4;
  const LnTailWs o = ln_tail_ws(rows, hw);
  const long long n = PACK_UNITS + 2 * o.E;
  const ImimPackArgs A{P, O, C, gamma, beta, Wf, bf, nullptr, nf, W1, W2, Wp, pk, lnw, lnb, hw,
                       ws + o.aff};
  hipLaunchKernelGGL(imim_pack_kernel, dim3((unsigned)(nf + (n + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, A);
  return (int)hipGetLastError();
}

int tgfr_imim_prep(const float* x, int N, int HW, float bn_eps, float momentum, int training,
                   float* running_mean, float* running_var, long long* nbt, float* mean,
                   float* rstd, const float* const* Wqkv, const float* const* bqkv, int rows_qkv,
                   int C, const float* gamma, const float* beta, float* Wf, uint16_t* Wfb,
                   float* bf, const float* W1, const float* W2, const float* Wp,
                   const float* lnw, const float* lnb, int rows, int hw, uint16_t* pk, float* ws,
                   void* stream) {
  if (!x || N <= 0 || HW <= 0 || !mean || !rstd || (!training && (!running_mean || !running_var)))
    return 1001;
  if (!Wqkv || !Wqkv[0] || !Wqkv[1] || !Wqkv[2] || rows_qkv <= 0 || C <= 0 || !gamma || !beta ||
      !Wf || !bf || !W1 || !W2 || !Wp || !pk || !lnw || !lnb || !ws || !ln_tail_ok(rows, hw))
    return 1001;
  const Parts P{Wqkv[0], Wqkv[1], Wqkv[2],
                bqkv ? bqkv[0] : nullptr, bqkv ? bqkv[1] : nullptr, bqkv ? bqkv[2] : nullptr,
                rows_qkv};
  const int O = 3 * rows_qkv, nf = (O + 3) / 4;
  const LnTailWs o = ln_tail_ws(rows, hw);
  const long long n = PACK_UNITS + 2 * o.E;
  const ImimPackArgs A{P, O, C, gamma, beta, Wf, bf, Wfb, nf, W1, W2, Wp, pk, lnw, lnb, hw,
                       ws + o.aff};
  const BnStatsArgs S{x, N, C, HW, bn_eps, momentum, training, running_mean, running_var, nbt,
                      mean, rstd};
  hipLaunchKernelGGL(imim_prep_kernel, dim3((unsigned)(C + nf + (n + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, S, A);
  return (int)hipGetLastError();
}

static int ln_tail_fwd(const float* X, int rows, int hw, float ln_eps, float* ws,
                       const uint16_t* pk, const float* b1, const float* b2, const float* bp,
                       float eps, float* R, long long ldr, uint16_t* Zb, uint16_t* H1b,
                       uint16_t* H2b, float* inv, uint16_t* Rrows, float* Rnorm,
                       int rows_per_item, int rows_pad, int rows_f16, bool tiles,
                       void* stream) {
  if (!ln_tail_ok(rows, hw) || !ws || ldr < TD || (ldr & 3) || ((uintptr_t)X & 15)) return 1001;
  if (!pk || !b1 || !b2 || !bp || !R || !Zb || !H1b || !H2b || !inv) return 1001;
  if ((Rrows || Rnorm) && (rows_per_item <= 0 || rows_pad < rows_per_item ||
                           rows % rows_per_item || ((uintptr_t)Rrows & 15)))
    return 1001;
  const LnTailWs o = ln_tail_ws(rows, hw);
  auto* s = (hipStream_t)stream;
  const int S = slices_for(o.n, o.E), nt = (hw + 31) / 32;
  if (tiles && nt > 64) return 1001;         // (the load combines at most 64 moments)
  if (!tiles)
    if (const int e = ln_part_launch(X, o.n, o.E, ws + o.ln, s)) return e;
  const LnWs l = ln_ws(o.n, o.E, TC);
  const LnFwd L{tiles ? ws : ws + o.ln, ws + o.ln + l.stats, ws + o.aff, o.E, tiles ? nt : S,
                hw, o.n, ln_eps, tiles ? 1 : 0};
  hipLaunchKernelGGL(tail_fwd_kernel<true>, dim3((rows + TM - 1) / TM), dim3(256), F_LDS_LN, s,
                     X, (long long)TC, rows, pk, b1, b2, bp, eps, R, ldr, Zb, H1b, H2b, inv,
                     Rrows, Rnorm, rows_per_item > 0 ? rows_per_item : 1, rows_pad,
                     rows_f16 ? 1 : 0, L);
  return (int)hipGetLastError();
}

static int ln_tail_bwd(const float* dR, const float* R, const float* inv, int rows, float eps,
                       const uint16_t* pk, const uint16_t* H1b, const uint16_t* H2b,
                       const float* X, int hw, float* ws, float* dZ, uint16_t* dPb,
                       uint16_t* dH2b, uint16_t* dH1b, float* dX, float* D, uint16_t* dOb,
                       float* dlnw, float* dlnb, void* stream) {
  if (!ln_tail_ok(rows, hw) || !ws || ((uintptr_t)dR & 15) || ((uintptr_t)R & 15) ||
      ((uintptr_t)X & 15) || ((uintptr_t)dZ & 15) || ((uintptr_t)dX & 15) ||
      ((uintptr_t)dOb & 7))
    return 1001;
  // (dlnw and dlnb both NULL: the LayerNorm's dw / db group partials stay in
  // ws for tgfr_imim_dw_ln's reduce)
  if (!inv || !pk || !H1b || !H2b || !dZ || !dPb || !dH2b || !dH1b || !(dX || (D && dOb)) ||
      !dlnw != !dlnb)
    return 1001;
  const LnTailWs o = ln_tail_ws(rows, hw);
  const LnWs l = ln_ws(o.n, o.E, TC);
  auto* s = (hipStream_t)stream;
  const LnBwd L{X, ws + o.ln + l.stats, ws + o.aff, ws + o.tp, hw, o.n, dOb ? 1 : 0};
  hipLaunchKernelGGL(tail_bwd_kernel<true>, dim3((rows + TM - 1) / TM), dim3(256), B_LDS_LN, s,
                     dR, (long long)TD, R, (long long)TD, inv, rows, eps, pk, H1b, H2b, dZ,
                     (long long)TC, dPb, dH2b, dH1b, L);
  if (const int e = (int)hipGetLastError()) return e;
  return ln_bwd_tail_launch(dZ, X, o.n, o.E, ws + o.aff, TC, ws + o.ln, ws + o.tp, hw, TM, dX, D, dOb,
                            dlnw, dlnb, s);
}

int tgfr_ln_tail_fwd(const float* X, int rows, int hw, float ln_eps, float* ws,
                     const uint16_t* pk, const float* b1, const float* b2, const float* bp,
                     float eps, float* R, long long ldr, uint16_t* Zb, uint16_t* H1b,
                     uint16_t* H2b, float* inv, uint16_t* Rrows, float* Rnorm,
                     int rows_per_item, int rows_pad, int rows_f16, void* stream) {
  return ln_tail_fwd(X, rows, hw, ln_eps, ws, pk, b1, b2, bp, eps, R, ldr, Zb, H1b, H2b, inv,
                     Rrows, Rnorm, rows_per_item, rows_pad, rows_f16, false, stream);
}

int tgfr_ln_tail_fwd_att(const float* X, int rows, int hw, float ln_eps, float* ws,
                         const uint16_t* pk, const float* b1, const float* b2, const float* bp,
                         float eps, float* R, long long ldr, uint16_t* Zb, uint16_t* H1b,
                         uint16_t* H2b, float* inv, uint16_t* Rrows, float* Rnorm,
                         int rows_per_item, int rows_pad, int rows_f16, void* stream) {
  return ln_tail_fwd(X, rows, hw, ln_eps, ws, pk, b1, b2, bp, eps, R, ldr, Zb, H1b, H2b, inv,
                     Rrows, Rnorm, rows_per_item, rows_pad, rows_f16, true, stream);
}

int tgfr_ln_tail_bwd(const float* dR, const float* R, const float* inv, int rows, float eps,
                     const uint16_t* pk, const uint16_t* H1b, const uint16_t* H2b,
                     const float* X, int hw, float* ws, float* dZ, uint16_t* dPb,
                     uint16_t* dH2b, uint16_t* dH1b, float* dX, float* dlnw, float* dlnb,
                     void* stream) {
  if (!dX) return 1001;
  return ln_tail_bwd(dR, R, inv, rows, eps, pk, H1b, H2b, X, hw, ws, dZ, dPb, dH2b, dH1b, dX,
                     nullptr, nullptr, dlnw, dlnb, stream);
}

int tgfr_ln_tail_bwd_att(const float* dR, const float* R, const float* inv, int rows, float eps,
                         const uint16_t* pk, const uint16_t* H1b, const uint16_t* H2b,
                         const float* X, int hw, float* ws, float* dZ, uint16_t* dPb,
                         uint16_t* dH2b, uint16_t* dH1b, void* att_ws, float* dlnw, float* dlnb,
                         void* stream) {
  if (!att_ws || ((uintptr_t)att_ws & 15)) return 1001;
  // tgfr_attn_bwd's workspace: D [rows] fp32, then dO [rows][256] bf16 (16-B aligned)
  float* D = (float*)att_ws;
  auto* dOb = (uint16_t*)((char*)att_ws + ((long long)rows * 4 + 15) / 16 * 16);
  return ln_tail_bwd(dR, R, inv, rows, eps, pk, H1b, H2b, X, hw, ws, dZ, dPb, dH2b, dH1b,
                     nullptr, D, dOb, dlnw, dlnb, stream);
}

int tgfr_tail_dw_ws(int rows, long long* floats) {
  if (rows <= 0 || !floats) return 1001;
  DwArgs A;
  int n_wg;
  dw_plan(rows, A, *floats, n_wg);
  return 0;
}

// dWp = dP^T H2, dW2 = dH2^T H1, dW1 = dH1^T Z and the bias sums; outputs
// overwritten, row-major [out][in] like the reference weights.
int tgfr_tail_dw(const uint16_t* dPb, const uint16_t* H2b, const uint16_t* dH2b,
                 const uint16_t* H1b, const uint16_t* dH1b, const uint16_t* Zb, int rows,
                 float* dWp, float* dbp, float* dW2, float* db2, float* dW1, float* db1, float* ws,
                 void* stream) {
  if (rows <= 0 || !dPb || !H2b || !dH2b || !H1b || !dH1b || !Zb || !dWp || !dbp || !dW2 ||
      !db2 || !dW1 || !db1 || !ws)
    return 1001;
  DwArgs A;
  long long wsf;
  int n_wg;
  dw_plan(rows, A, wsf, n_wg);
  A.p[0].X = dPb;  A.p[0].Y = H2b;
  A.p[1].X = dH2b; A.p[1].Y = H1b;
  A.p[2].X = dH1b; A.p[2].Y = Zb;
  DwOut O = {};
  O.dW[0] = dWp; O.db[0] = dbp;
  O.dW[1] = dW2; O.db[1] = db2;
  O.dW[2] = dW1; O.db[2] = db1;
  return dw_launch(A, n_wg, O, ws, (hipStream_t)stream);
}

// IMIM's two weight-gradient sets in ONE launch (+ one reduce): the tail's
// dWp, dW2, dW1 (tgfr_tail_dw) and the packed q/k/v projection's dW = dX^T Y,
// db = colsum(dX) (tgfr_dw_bf16 with bf16 Y: X [rows][Nq], Y [rows][Kq]).
// Budget 512 workgroups (24 row slices at config 2: two 61-KB workgroups per
// CU hide each other's staging latency; the larger slab read by the reduce
// costs less): 0.440-0.450 -> 0.434-0.437 ms per step against 256 (128: 0.46;
// tools/lab/lib_ab.sh, profiles/r04/fork_ab.txt).
static void imim_dw_plan(int rows, int Nq, int Kq, DwArgs& A, long long& wsf, int& n_wg) {
  const int NS[4] = {TD, TC, TH, Nq}, KS[4] = {TC, TH, TC, Kq};
  // bf16 dW slabs (fp32 slabs: the lab variant dwf32slab, tools/lab/variants.py)
  dw_plan_n(rows, 4, NS, KS, 512, A, wsf, n_wg, true);
}

int tgfr_imim_dw_ws(int rows, int Nq, int Kq, long long* floats) {
  if (rows <= 0 || Nq <= 0 || Kq <= 0 || Nq % DW_NB || Kq % DW_NB || !floats) return 1001;
  DwArgs A;
  int n_wg;
  imim_dw_plan(rows, Nq, Kq, A, *floats, n_wg);
  return 0;
}

int tgfr_imim_dw(const uint16_t* dPb, const uint16_t* H2b, const uint16_t* dH2b,
                 const uint16_t* H1b, const uint16_t* dH1b, const uint16_t* Zb, int rows,
                 float* dWp, float* dbp, float* dW2, float* db2, float* dW1, float* db1,
                 const uint16_t* Xq, const uint16_t* Yq, int Nq, int Kq, float* dWq, float* dbq,
                 float* ws, void* stream) {
  if (rows <= 0 || !dPb || !H2b || !dH2b || !H1b || !dH1b || !Zb || !dWp || !dbp || !dW2 ||
      !db2 || !dW1 || !db1 || !Xq || !Yq || !dWq || !dbq || !ws || Nq <= 0 || Kq <= 0 ||
      Nq % DW_NB || Kq % DW_NB)
    return 1001;
  DwArgs A;
  long long wsf;
  int n_wg;
  imim_dw_plan(rows, Nq, Kq, A, wsf, n_wg);
  A.p[0].X = dPb;  A.p[0].Y = H2b;
  A.p[1].X = dH2b; A.p[1].Y = H1b;
  A.p[2].X = dH1b; A.p[2].Y = Zb;
  A.p[3].X = Xq;   A.p[3].Y = Yq;
  DwOut O = {};
  O.dW[0] = dWp; O.db[0] = dbp;
  O.dW[1] = dW2; O.db[1] = db2;
  O.dW[2] = dW1; O.db[2] = db1;
  O.dW[3] = dWq; O.db[3] = dbq;
  return dw_launch(A, n_wg, O, ws, (hipStream_t)stream);
}

// tgfr_imim_dw with the IMIM LayerNorm's dw / db reduce as extra workgroups of
// its slab reduce: lnws is the tail workspace that tgfr_ln_tail_bwd_att,
// called with dlnw = dlnb = NULL, left the LayerNorm's group partials in
// (one launch less on the step's critical path; same sums, same order as
// ln_bwd_dw).  dlnw / dlnb: the reference's [256][hw] maps.
int tgfr_imim_dw_ln(const uint16_t* dPb, const uint16_t* H2b, const uint16_t* dH2b,
                    const uint16_t* H1b, const uint16_t* dH1b, const uint16_t* Zb, int rows,
                    float* dWp, float* dbp, float* dW2, float* db2, float* dW1, float* db1,
                    const uint16_t* Xq, const uint16_t* Yq, int Nq, int Kq, float* dWq,
                    float* dbq, const float* lnws, int hw, float* dlnw, float* dlnb, float* ws,
                    void* stream) {
  if (rows <= 0 || !dPb || !H2b || !dH2b || !H1b || !dH1b || !Zb || !dWp || !dbp || !dW2 ||
      !db2 || !dW1 || !db1 || !Xq || !Yq || !dWq || !dbq || !ws || Nq <= 0 || Kq <= 0 ||
      Nq % DW_NB || Kq % DW_NB || !lnws || !dlnw || !dlnb || !ln_tail_ok(rows, hw))
    return 1001;
  DwArgs A;
  long long wsf;
  int n_wg;
  imim_dw_plan(rows, Nq, Kq, A, wsf, n_wg);
  A.p[0].X = dPb;  A.p[0].Y = H2b;
  A.p[1].X = dH2b; A.p[1].Y = H1b;
  A.p[2].X = dH1b; A.p[2].Y = Zb;
  A.p[3].X = Xq;   A.p[3].Y = Yq;
  DwOut O = {};
  O.dW[0] = dWp; O.db[0] = dbp;
  O.dW[1] = dW2; O.db[1] = db2;
  O.dW[2] = dW1; O.db[2] = db1;
  O.dW[3] = dWq; O.db[3] = dbq;
  const LnTailWs o = ln_tail_ws(rows, hw);
  const LnWs l = ln_ws(o.n, o.E, TC);
  O.lnp = lnws + o.ln + l.bwd;
  O.lnE = o.E;
  O.lng = (o.n + LN_GROUP - 1) / LN_GROUP;
  O.lnhw = hw;
  O.dlnw = dlnw;
  O.dlnb = dlnb;
  return dw_launch(A, n_wg, O, ws, (hipStream_t)stream);
}

// Generic weight gradient of a row-wise linear map with bf16 operands:
// dW[n][k] = sum_rows X[row][n] Y[row][k], db[n] = sum_rows X[row][n], for
// dense X [rows][N] bf16 and Y [rows][K] (bf16, or fp32 when y_f32: rounded
// to bf16 while staged); N, K multiples of 128.  dW [N][K] and db [N] fp32,
// overwritten; ws: tgfr_dw_bf16_ws floats.  (IMIM's packed q/k/v projection:
// X = the attention's bf16 gradient, Y = the BN output.)
static int dw_generic_plan(int rows, int N, int K, DwArgs& A, long long& wsf, int& n_wg) {
  if (rows <= 0 || N <= 0 || K <= 0 || N % DW_NB || K % DW_NB) return 1001;
  const int NS[1] = {N}, KS[1] = {K};
  dw_plan_n(rows, 1, NS, KS, 256, A, wsf, n_wg);
  return 0;
}

int tgfr_dw_bf16_ws(int rows, int N, int K, long long* floats) {
  if (!floats) return 1001;
  DwArgs A;
  int n_wg;
  return dw_generic_plan(rows, N, K, A, *floats, n_wg);
}

int tgfr_dw_bf16(const uint16_t* X, const void* Y, int y_f32, int rows, int N, int K, float* dW,
                 float* db, float* ws, void* stream) {
  if (!X || !Y || !dW || !db || !ws) return 1001;
  DwArgs A;
  long long wsf;
  int n_wg;
  if (const int e = dw_generic_plan(rows, N, K, A, wsf, n_wg)) return e;
  A.p[0].X = X;
  A.p[0].Y = Y;
  A.p[0].yf32 = y_f32 ? 1 : 0;
  DwOut O = {};
  O.dW[0] = dW;
  O.db[0] = db;
  return dw_launch(A, n_wg, O, ws, (hipStream_t)stream);
}

}  // extern "C"
