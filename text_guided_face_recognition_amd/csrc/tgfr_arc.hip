// ArcMarginProduct (models/metrics.py:17-60) as two fused launches:
//
//   arc_fwd   logits[b][c] = s * margin(cos), cos = normalize(x_b) .
//             normalize(W_c) (F.linear of the two F.normalize, :43-44) with the
//             additive angular margin on the label column (:45-57) -- one
//             launch instead of two row normalisations, a GEMM and the margin
//   arc_bwd   dcos from dlogits through the margin; dW_c = d normalize(W_c)
//             applied to dWn_c = sum_b dcos[b][c] xn_b (the l2-norm backward
//             fused in); dcs[b][c] = dcos[b][c] / |W_c| for the input side
//             (dxn = dcs W, a plain GEMM, then the x l2-norm backward)
//
// fp32 FMA throughout (the products are 64 x 4500 x 256: far from MFMA-bound
// and the fp32 sums match the reference more closely than bf16).  Block = 16
// classes (32 in the forward); the class tile of W and a chunk of x rows sit in LDS (rows padded
// by 4 floats so the 16 classes of a 16-lane group read distinct banks).
#include "tgfr_common.h"
#include "../../include/tgfr.h"

#include <math.h>

#include <algorithm>

using namespace tgfr;

namespace {

constexpr int CB = 16;          // classes per block
constexpr int NT = 256;

__device__ __forceinline__ float group16_sum(float v) { return row16_sum(v); }

__device__ __forceinline__ float4 ld4(const float* p) { return *(const float4*)p; }
__device__ __forceinline__ float4 lds4(uint32_t off) {
  return __builtin_bit_cast(float4, lds_ld16(off));
}

// Rows [r0, r0 + n) of a [rows][D] matrix -> LDS rows of stride (D + 4)
// floats, zero rows past `rows`.  Eight loads per thread are issued before
// the first LDS store (a load-store loop would pay one L2 round trip per
// float4).
__device__ __forceinline__ void stage_rows(const float* __restrict__ src, long long ld, int r0,
                                           int n, int rows, int D, uint32_t off) {
  constexpr int U = 8;
  const int q = D / 4, total = n * q;
  for (int base = threadIdx.x; base < total; base += NT * U) {
    float4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = min(base + u * NT, total - 1);
      const int r = i / q, k = i % q;
      const int row = min(r0 + r, rows - 1);
      v[u] = ld4(src + (long long)row * ld + 4 * k);
      if (r0 + r >= rows) v[u] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = base + u * NT;
      if (i < total) {
        const int r = i / q, k = i % q;
        lds_st16(off + (uint32_t)((r * (D + 4) + 4 * k) * 4), __builtin_bit_cast(uint4, v[u]));
      }
    }
  }
}

// Split form of stage_rows for tiles that fit one pass (n D / 4 <= U NT):
// load_rows issues the thread's U float4 loads into registers, store_rows
// writes them to LDS later, so several tiles' loads (and a next chunk's) are
// in flight together.
template <int U>
__device__ __forceinline__ void load_rows(float4 (&v)[U], const float* __restrict__ src,
                                          long long ld, int r0, int n, int rows, int D) {
  const int q = D / 4, total = n * q;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int i = min((int)threadIdx.x + u * NT, total - 1);
    const int r = i / q, k = i % q;
    const int row = min(r0 + r, rows - 1);
    v[u] = ld4(src + (long long)row * ld + 4 * k);
    if (r0 + r >= rows) v[u] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
}
template <int U>
__device__ __forceinline__ void store_rows(const float4 (&v)[U], int n, int D, uint32_t off) {
  const int q = D / 4, total = n * q;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int i = threadIdx.x + u * NT;
    if (i < total) {
      const int r = i / q, k = i % q;
      lds_st16(off + (uint32_t)((r * (D + 4) + 4 * k) * 4), __builtin_bit_cast(uint4, v[u]));
    }
  }
}

// 1 / max(|row|, eps) of n LDS rows (16 lanes per row) -> out[r]
__device__ __forceinline__ void row_inv_norms(uint32_t off, int n, int D, float eps, float* out) {
  const int g = threadIdx.x & 15;
  for (int r = threadIdx.x >> 4; r < n; r += NT / 16) {
    float ss = 0.f;
    for (int k = g; k < D / 4; k += 16) {
      const float4 v = lds4(off + (uint32_t)((r * (D + 4) + 4 * k) * 4));
      ss += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
    }
    ss = group16_sum(ss);
    if (g == 0) out[r] = 1.f / fmaxf(sqrtf(ss), eps);
  }
}

struct Margin {
  float s, cos_m, sin_m, th, mm;
  int easy;
};

__device__ __forceinline__ float margin_fwd(float cv, bool target, const Margin& M) {
  float v = cv;
  if (target) {
    const float sine = sqrtf(fminf(fmaxf(1.f - cv * cv, 0.f), 1.f));
    const float phi = cv * M.cos_m - sine * M.sin_m;
    v = M.easy ? (cv > 0.f ? phi : cv) : (cv > M.th ? phi : cv - M.mm);
  }
  return v * M.s;
}

__device__ __forceinline__ float margin_bwd(float g, float cv, bool target, const Margin& M) {
  g *= M.s;
  if (target && (M.easy ? cv > 0.f : cv > M.th)) {
    const float one_m = 1.f - cv * cv;
    const float sine = sqrtf(fminf(fmaxf(one_m, 0.f), 1.f));
    const float dsine = (one_m >= 0.f && one_m <= 1.f) ? -cv / sine : 0.f;
    g *= M.cos_m - M.sin_m * dsine;
  }
  return g;
}

// Block = (32-class tile, 64-row x chunk).  D is walked in FK-wide k chunks:
// LDS holds only W [CBF][FK+4] and x [64][FK+4] (~51 KB at FK = 128, several
// blocks per CU), the row sums of squares accumulate in registers across chunks.
// LDS: W chunk | x chunk (also the k-half exchange) | inv_nw [CBF] |
// inv_nx [64] | labels [64] (column within the block or -1).
constexpr int CBF = 32;         // classes per forward block
constexpr int FRB = 64;         // x rows per forward block
// FK: k chunk (256 when D <= 256 and B <= 64: one chunk, no re-staging barriers;
// 128 else, so that several blocks share a CU)
// Second head (blockIdx.z == 1) of a two-head launch: the trainer's image and
// text identity classifiers (src/train_encoders_bert.py:293-306) share
// (B, D, C) and run as one grid.
struct ArcHead2 {
  const float* x;
  const float* W;
  float* logits;
  float* cosv;
  float* xn;
  float* inv_nx;
  float* inv_nw;
  Margin M;
};

template <int FK>
__global__ __launch_bounds__(NT) void arc_fwd_kernel(
    const float* __restrict__ x, long long ldx, int B, int D, const float* __restrict__ W,
    long long ldw, int C, const long long* __restrict__ label, Margin M, float eps,
    float* __restrict__ logits, float* __restrict__ cosv, float* __restrict__ xn,
    float* __restrict__ inv_nx, float* __restrict__ inv_nw, ArcHead2 h2) {
  if (blockIdx.z) {
    x = h2.x;
    W = h2.W;
    logits = h2.logits;
    cosv = h2.cosv;
    xn = h2.xn;
    inv_nx = h2.inv_nx;
    inv_nw = h2.inv_nw;
    M = h2.M;
  }
  float* lds_f = (float*)g_smem;
  const uint32_t w_off = 0, x_off = CBF * (FK + 4) * 4;
  float* nw = lds_f + (CBF + FRB) * (FK + 4);
  float* nx = nw + CBF;
  int* lab = (int*)(nx + FRB);
  const int c0 = blockIdx.x * CBF, b0 = blockIdx.y * FRB, nb = min(FRB, B - b0);
  const int tid = threadIdx.x, g = tid & 15;
  if (tid < nb) {
    const long long l = label[b0 + tid];
    lab[tid] = l >= c0 && l < c0 + CBF ? (int)(l - c0) : -1;
  }
  // cos on v_mfma_f32_32x32x2_f32 (fp32 operands, fp32 sums): wave w owns
  // row tile rt = w & 1 (32 rows; rows past B are staged as zeros) and k half
  // kh = w >> 1 of each chunk; one float4 LDS read per operand feeds two MFMAs
  // (lane half h uses elements h and h + 2).
  const int w = tid >> 6, lane = tid & 63, rt = w & 1, kh = w >> 1, h = lane >> 5;
  f32x16 acc;
#pragma unroll
  for (int q = 0; q < 16; ++q) acc[q] = 0.f;
  float sw[2] = {0.f, 0.f}, sx[4] = {0.f, 0.f, 0.f, 0.f};
  // both operands' chunk loads in one batch; chunk j + 1's loads are issued
  // right after chunk j is in LDS, so they fly during chunk j's MFMAs
  constexpr int UW = CBF * FK / 4 / NT, UX = FRB * FK / 4 / NT;
  float4 vw[UW], vx[UX];
  load_rows(vw, W, ldw, c0, CBF, C, min(FK, D));
  load_rows(vx, x, ldx, b0, FRB, B, min(FK, D));
  for (int k0 = 0; k0 < D; k0 += FK) {
    const int kc = min(FK, D - k0);      // multiple of 8 (D % 8 == 0)
    __syncthreads();                     // previous chunk's readers are done
    store_rows(vw, CBF, kc, w_off);
    store_rows(vx, FRB, kc, x_off);
    __syncthreads();
    if (k0 + FK < D) {
      const int kn = min(FK, D - k0 - FK);
      load_rows(vw, W + k0 + FK, ldw, c0, CBF, C, kn);
      load_rows(vx, x + k0 + FK, ldx, b0, FRB, B, kn);
    }
    // running sums of squares: 16 lanes per row, rows tid / 16 + 16 i
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = (tid >> 4) + 16 * i;
#pragma unroll
      for (int j = 0; j < FK / 64; ++j) {
        const int k = g + 16 * j;
        if (k < kc / 4) {
          const float4 v = lds4(x_off + (uint32_t)((r * (kc + 4) + 4 * k) * 4));
          sx[i] += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
          if (i < 2) {
            const float4 u = lds4(w_off + (uint32_t)((r * (kc + 4) + 4 * k) * 4));
            sw[i] += u.x * u.x + u.y * u.y + u.z * u.z + u.w * u.w;
          }
        }
      }
    }
    const uint32_t xa = x_off + (uint32_t)((32 * rt + (lane & 31)) * (kc + 4) * 4);
    const uint32_t wa = w_off + (uint32_t)((lane & 31) * (kc + 4) * 4);
    const int k_lo = kh * (kc / 2), k_hi = k_lo + kc / 2;
#pragma unroll 4
    for (int k = k_lo; k < k_hi; k += 4) {
      const float4 av = lds4(xa + 4 * k), bv = lds4(wa + 4 * k);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(h ? av.y : av.x, h ? bv.y : bv.x, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(h ? av.w : av.z, h ? bv.w : bv.z, acc, 0, 0, 0);
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float ssx = group16_sum(sx[i]);
    if (g == 0) nx[(tid >> 4) + 16 * i] = 1.f / fmaxf(sqrtf(ssx), eps);
    if (i < 2) {
      const float ssw = group16_sum(sw[i]);
      if (g == 0) nw[(tid >> 4) + 16 * i] = 1.f / fmaxf(sqrtf(ssw), eps);
    }
  }
  // k halves: waves 2, 3 hand their sums to waves 0, 1 through LDS (the x
  // chunk's space is free once every wave has passed the barrier)
  __syncthreads();
  float* xs = (float*)(g_smem + x_off);
  if (kh == 1) {
#pragma unroll
    for (int q = 0; q < 16; ++q) xs[(rt * 16 + q) * 64 + lane] = acc[q];
  }
  __syncthreads();
  if (kh == 0) {
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int r = 32 * rt + acc_row(q, h), cc = lane & 31;
      const float v = acc[q] + xs[(rt * 16 + q) * 64 + lane];
      if (r < nb && c0 + cc < C) {
        const float cv = v * nx[r] * nw[cc];
        const long long e = (long long)(b0 + r) * C + c0 + cc;
        cosv[e] = cv;
        logits[e] = margin_fwd(cv, lab[r] == cc, M);
      }
    }
  }
  if (blockIdx.x == 0) {                 // the normalised rows, for the backward
    const int q = D / 4;
    for (int i = tid; i < nb * q; i += NT) {
      const int r = i / q, k = i % q;
      float4 v = ld4(x + (long long)(b0 + r) * ldx + 4 * k);
      const float sc = nx[r];
      v.x *= sc; v.y *= sc; v.z *= sc; v.w *= sc;
      *(float4*)(xn + (long long)(b0 + r) * D + 4 * k) = v;
    }
    for (int r = tid; r < nb; r += NT) inv_nx[b0 + r] = nx[r];
  }
  if (blockIdx.y == 0 && tid < CBF && c0 + tid < C) inv_nw[c0 + tid] = nw[tid];
}

// dW_c = (dWn - wn (wn . dWn)) / |W_c| for one class row held by a 16-lane
// group (lane g owns dims 4 g + 64 j); acc = dWn, wv = the raw W row slice.
template <int MAXJ>
__device__ __forceinline__ void arc_dw_epilogue(const float4 (&acc)[MAXJ],
                                                const float4 (&wv)[MAXJ], int nj, float inv,
                                                float eps, int g, float* __restrict__ dWrow) {
  const bool clamped = inv >= 1.f / eps;   // |W_c| <= eps: y = W / eps, no projection
  float4 wn[MAXJ];
  float dot = 0.f;
#pragma unroll
  for (int j = 0; j < MAXJ; ++j) {
    if (j < nj) {
      const float4 w = wv[j];
      wn[j] = make_float4(w.x * inv, w.y * inv, w.z * inv, w.w * inv);
      dot += wn[j].x * acc[j].x + wn[j].y * acc[j].y + wn[j].z * acc[j].z + wn[j].w * acc[j].w;
    }
  }
  dot = clamped ? 0.f : group16_sum(dot);
#pragma unroll
  for (int j = 0; j < MAXJ; ++j) {
    if (j < nj) {
      const float4 o = make_float4((acc[j].x - wn[j].x * dot) * inv, (acc[j].y - wn[j].y * dot) * inv,
                                   (acc[j].z - wn[j].z * dot) * inv, (acc[j].w - wn[j].w * dot) * inv);
      *(float4*)(dWrow + 4 * g + 64 * j) = o;
    }
  }
}

// LDS: dcos [rows_per][CB] | xn chunk [RB][D+4]
// thread: class c = tid / 16, d-group g = tid % 16 owns dims 4 g + 64 j
// The head's focal loss (models/losses.py:313-325) as the source of the logit
// gradient (dlogits == NULL): dlogits[b][c] = g f'(logp) / B (softmax(L_b)[c]
// - [c == label_b]) formed in place from the logits L, the focal workspace
// (ws[b] = row LSE, ws[B] = logp) and the upstream gradient g (nullable = 1).
struct FocalSrc {
  const float* L;
  const float* ws;
  const float* g;
  float gamma;
};
struct ArcBwd2 {
  const float* cosv;
  const float* xn;
  const float* W;
  const float* inv_nw;
  float* dW;
  float* dcs;
  FocalSrc F;
  Margin M;
};

template <int NJ>   // float4 columns per thread: D = 64 NJ (NJ = 0: any D <= 1024)
__global__ __launch_bounds__(NT) void arc_bwd_kernel(
    const float* __restrict__ dlogits, const float* __restrict__ cosv,
    const long long* __restrict__ label, const float* __restrict__ xn,
    const float* __restrict__ W, long long ldw, const float* __restrict__ inv_nw, int B, int D,
    int C, Margin M, float eps, int RB, float* __restrict__ dW, long long lddw,
    float* __restrict__ dcs, int rows_per, float* __restrict__ part, FocalSrc F, ArcBwd2 h2) {
  if (blockIdx.z) {
    cosv = h2.cosv;
    xn = h2.xn;
    W = h2.W;
    inv_nw = h2.inv_nw;
    dW = h2.dW;
    dcs = h2.dcs;
    F = h2.F;
    M = h2.M;
  }
  float fscale = 0.f;
  if (!dlogits) {
    const float logp = F.ws[B], p = __expf(-logp), q = 1.f - p;
    float dfl = powf(q, F.gamma);
    if (F.gamma != 0.f) dfl += F.gamma * powf(q, F.gamma - 1.f) * p * logp;
    fscale = (F.g ? F.g[0] : 1.f) * dfl / (float)B;
  }
  // block row y owns rows [rb0, rb1); with gridDim.y > 1 the raw sums go to
  // part[y][C][D] and arc_bwd_finish_kernel applies the l2-norm backward
  const int rb0 = blockIdx.y * rows_per, rb1 = min(B, rb0 + rows_per), nbs = rb1 - rb0;
  float* dc = (float*)g_smem;
  const uint32_t x_off = (uint32_t)(rows_per * CB * 4);
  const int c0 = blockIdx.x * CB, tid = threadIdx.x;
  const int c = tid >> 4, g = tid & 15, col = c0 + c;
  constexpr int MAXJ = NJ ? NJ : 16;       // D <= 1024
  const int nj = NJ ? NJ : D / 64 + ((D % 64) > 4 * g ? 1 : 0);
  // this thread's W row slice, needed only at the end: loaded first so its
  // latency hides under the rest
  float4 wv[MAXJ];
  {
    const float* wr = W + (long long)min(col, C - 1) * ldw + 4 * g;
#pragma unroll
    for (int j = 0; j < MAXJ; ++j)
      wv[j] = j < nj ? ld4(wr + 64 * j) : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  // dcos of the block's columns (all loads of a thread issued together)
  for (int base = tid; base < nbs * CB; base += NT * 4) {
    float gl[4], cv[4], iw[4];
    bool tg[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int i = min(base + u * NT, nbs * CB - 1);
      const int b = rb0 + i / CB, col = min(c0 + i % CB, C - 1);
      const long long e = (long long)b * C + col;
      gl[u] = dlogits ? dlogits[e]
                      : fscale * (__expf(F.L[e] - F.ws[b]) - (label[b] == col ? 1.f : 0.f));
      cv[u] = cosv[e];
      iw[u] = inv_nw[col];
      tg[u] = label[b] == col;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int i = base + u * NT;
      if (i < nbs * CB) {
        const int b = rb0 + i / CB, col = c0 + i % CB;
        float d = 0.f;
        if (col < C) {
          d = margin_bwd(gl[u], cv[u], tg[u], M);
          if (dcs) dcs[(long long)b * C + col] = d * iw[u];
        }
        dc[i] = d;
      }
    }
  }
  float4 acc[MAXJ];
#pragma unroll
  for (int j = 0; j < MAXJ; ++j) acc[j] = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int b0 = rb0; b0 < rb1; b0 += RB) {
    const int nb = min(RB, rb1 - b0);
    __syncthreads();
    stage_rows(xn, D, b0, nb, B, D, x_off);
    __syncthreads();
    for (int r = 0; r < nb; ++r) {
      const float a = dc[(b0 - rb0 + r) * CB + c];
#pragma unroll
      for (int j = 0; j < MAXJ; ++j) {
        if (j < nj) {
          const float4 v = lds4(x_off + (uint32_t)((r * (D + 4) + 4 * g + 64 * j) * 4));
          acc[j].x = fmaf(a, v.x, acc[j].x);
          acc[j].y = fmaf(a, v.y, acc[j].y);
          acc[j].z = fmaf(a, v.z, acc[j].z);
          acc[j].w = fmaf(a, v.w, acc[j].w);
        }
      }
    }
  }
  if (col >= C) return;                    // whole 16-lane groups leave together
  if (gridDim.y > 1) {
    float* pr = part + ((long long)blockIdx.y * C + col) * D + 4 * g;
#pragma unroll
    for (int j = 0; j < MAXJ; ++j)
      if (j < nj) *(float4*)(pr + 64 * j) = acc[j];
    return;
  }
  arc_dw_epilogue<MAXJ>(acc, wv, nj, inv_nw[col], eps, g, dW + (long long)col * lddw);
}

// The same backward with dWn = dcos^T xn on the matrix core: block = 32
// classes; v_mfma_f32_32x32x2f32 (fp32 operands, exact products) with A =
// dcos [rows][32 classes] and B = xn [rows][d] read straight from LDS (lane
// l takes row l / 32 of the k pair and class / d column l % 32: no
// transposes); wave w owns d tiles w NTW .. w NTW + NTW - 1 (D = 128 NTW).
// The l2-norm backward's per-class dot is reduced across lanes and waves
// through LDS.  LDS: dcos [rows_per + RB][33] (rows past the slice zero) |
// xn chunk [RB][D + 4]; for slices of <= 64 rows at D <= 256, the whole
// slice: dcos [rows_per][33] | xn [rows_per][D + 4], with every HBM load of
// the block (xn rows, then logits / cos / labels) in flight at once.
constexpr int CBM = 32;
constexpr int RBM = 16;         // xn rows per staged chunk
constexpr int ARC_WHOLE = 64;   // slices of at most this many rows are staged whole
template <int NTW>
__global__ __launch_bounds__(NT) void arc_bwd_mma_kernel(
    const float* __restrict__ dlogits, const float* __restrict__ cosv,
    const long long* __restrict__ label, const float* __restrict__ xn,
    const float* __restrict__ W, long long ldw, const float* __restrict__ inv_nw, int B, int D,
    int C, Margin M, float eps, float* __restrict__ dW, long long lddw, float* __restrict__ dcs,
    int rows_per, float* __restrict__ part, FocalSrc F, ArcBwd2 h2) {
  if (blockIdx.z) {
    cosv = h2.cosv;
    xn = h2.xn;
    W = h2.W;
    inv_nw = h2.inv_nw;
    dW = h2.dW;
    dcs = h2.dcs;
    F = h2.F;
    M = h2.M;
  }
  float fscale = 0.f;
  if (!dlogits) {
    const float logp = F.ws[B], p = __expf(-logp), q = 1.f - p;
    float dfl = powf(q, F.gamma);
    if (F.gamma != 0.f) dfl += F.gamma * powf(q, F.gamma - 1.f) * p * logp;
    fscale = (F.g ? F.g[0] : 1.f) * dfl / (float)B;
  }
  constexpr int LDC = CBM + 1;
  const int rb0 = blockIdx.y * rows_per, rb1 = min(B, rb0 + rows_per), nbs = rb1 - rb0;
  // whole: the slice's xn rows (<= ARC_WHOLE) staged at once, their loads
  // issued before the dcos loads so both are in flight together; else RBM-row
  // chunks
  const bool whole = NTW <= 2 && rows_per <= ARC_WHOLE;
  const int dc_rows = whole ? (rows_per + 1) & ~1 : rows_per + RBM;
  float* dc = (float*)g_smem;
  const uint32_t x_off = (uint32_t)((dc_rows * LDC * 4 + 15) & ~15);
  const float* xs = (const float*)(g_smem + x_off);
  const int c0 = blockIdx.x * CBM, tid = threadIdx.x;
  const int lane = tid & 63, w = tid >> 6, lr = lane & 31, h = lane >> 5;
  constexpr int UXN = NTW <= 2 ? ARC_WHOLE * 32 * NTW / NT : 1;   // float4 per thread (D = 128 NTW)
  float4 vx[UXN];
  if (whole) load_rows(vx, xn, D, rb0, dc_rows, B, D);
  // dcos of the block's columns; rows past the slice (up to one chunk) zero
  for (int base = tid; base < dc_rows * CBM; base += NT * 4) {
    float gl[4], cv[4], iw[4];
    bool tg[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int i = min(base + u * NT, max(nbs * CBM - 1, 0));
      const int b = rb0 + i / CBM, col = min(c0 + i % CBM, C - 1);
      const long long e = (long long)b * C + col;
      const long long lb = label[b];
      gl[u] = dlogits ? dlogits[e]
                      : fscale * (__expf(F.L[e] - F.ws[b]) - (lb == col ? 1.f : 0.f));
      cv[u] = cosv[e];
      iw[u] = inv_nw[col];
      tg[u] = lb == col;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int i = base + u * NT;
      if (i < dc_rows * CBM) {
        const int r = i / CBM, cc = i % CBM, col = c0 + cc;
        float d = 0.f;
        if (r < nbs && col < C) {
          d = margin_bwd(gl[u], cv[u], tg[u], M);
          if (dcs) dcs[(long long)(rb0 + r) * C + col] = d * iw[u];
        }
        dc[r * LDC + cc] = d;
      }
    }
  }
  f32x16 acc[NTW];
#pragma unroll
  for (int t = 0; t < NTW; ++t)
#pragma unroll
    for (int q = 0; q < 16; ++q) acc[t][q] = 0.f;
  const int dbase = 32 * NTW * w + lr;
  // the epilogue's W values (lane: classes acc_row(q, h), its d columns),
  // loaded now so they arrive during the MFMAs
  float wv[16][NTW];
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const float* wr = W + (long long)min(c0 + acc_row(q, h), C - 1) * ldw + dbase;
#pragma unroll
    for (int t = 0; t < NTW; ++t) wv[q][t] = wr[32 * t];
  }
  if (whole) {
    store_rows(vx, dc_rows, D, x_off);   // rows past B are zeros
    __syncthreads();
    for (int k = 0; k < nbs; k += 2) {
      const float a = dc[(k + h) * LDC + lr];
      const float* xr = xs + (k + h) * (D + 4) + dbase;
#pragma unroll
      for (int t = 0; t < NTW; ++t)
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, xr[32 * t], acc[t], 0, 0, 0);
    }
  } else {
    for (int b0 = rb0; b0 < rb1; b0 += RBM) {
      const int nb = min(RBM, rb1 - b0);
      __syncthreads();
      stage_rows(xn, D, b0, RBM, B, D, x_off);   // rows past B staged as zeros
      __syncthreads();
      for (int k = 0; k < nb; k += 2) {
        const float a = dc[(b0 - rb0 + k + h) * LDC + lr];
        const float* xr = xs + (k + h) * (D + 4) + dbase;
#pragma unroll
        for (int t = 0; t < NTW; ++t)
          acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, xr[32 * t], acc[t], 0, 0, 0);
      }
    }
  }
  if (gridDim.y > 1) {                       // raw dWn partials: part[y][C][D]
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int col = c0 + acc_row(q, h);
      if (col < C) {
        float* pr = part + ((long long)blockIdx.y * C + col) * D + dbase;
#pragma unroll
        for (int t = 0; t < NTW; ++t) pr[32 * t] = acc[t][q];
      }
    }
    return;
  }
  // l2-norm backward: dW_c = (dWn_c - wn_c (wn_c . dWn_c)) / |W_c|
  __syncthreads();                           // dc / xs no longer read
  float* red = (float*)g_smem;               // [4 waves][32 classes]
  float part_dot[16];
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    float sdot = 0.f;
#pragma unroll
    for (int t = 0; t < NTW; ++t) sdot = fmaf(wv[q][t], acc[t][q], sdot);
    part_dot[q] = x16_sum(row16_sum(sdot));  // over the 32 d columns of the half
  }
  if (lr == 0) {
#pragma unroll
    for (int q = 0; q < 16; ++q) red[w * CBM + acc_row(q, h)] = part_dot[q];
  }
  __syncthreads();
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int cc = acc_row(q, h), col = c0 + cc;
    if (col >= C) continue;
    const float inv = inv_nw[col];
    const bool clamped = inv >= 1.f / eps;   // |W_c| <= eps: y = W / eps, no projection
    const float dot = clamped ? 0.f
                              : inv * (red[cc] + red[CBM + cc] + red[2 * CBM + cc] + red[3 * CBM + cc]);
    float* o = dW + (long long)col * lddw + dbase;
#pragma unroll
    for (int t = 0; t < NTW; ++t) o[32 * t] = (acc[t][q] - wv[q][t] * inv * dot) * inv;
  }
}

// Sums the block rows' partial dWn in fixed order and applies the l2-norm
// backward; the thread layout of arc_bwd_kernel (16 classes x 16 lanes).
template <int NJ>
__global__ __launch_bounds__(NT) void arc_bwd_finish_kernel(
    const float* __restrict__ part, int S, const float* __restrict__ W, long long ldw,
    const float* __restrict__ inv_nw, int D, int C, float eps, float* __restrict__ dW,
    long long lddw) {
  const int tid = threadIdx.x, g = tid & 15, col = blockIdx.x * CB + (tid >> 4);
  if (col >= C) return;                    // whole 16-lane groups leave together
  constexpr int MAXJ = NJ ? NJ : 16;
  const int nj = NJ ? NJ : D / 64 + ((D % 64) > 4 * g ? 1 : 0);
  float4 wv[MAXJ], acc[MAXJ];
  const float* wr = W + (long long)col * ldw + 4 * g;
#pragma unroll
  for (int j = 0; j < MAXJ; ++j) {
    wv[j] = j < nj ? ld4(wr + 64 * j) : make_float4(0.f, 0.f, 0.f, 0.f);
    acc[j] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
  for (int y = 0; y < S; ++y) {
    const float* pr = part + ((long long)y * C + col) * D + 4 * g;
#pragma unroll
    for (int j = 0; j < MAXJ; ++j) {
      if (j < nj) {
        const float4 v = ld4(pr + 64 * j);
        acc[j].x += v.x; acc[j].y += v.y; acc[j].z += v.z; acc[j].w += v.w;
      }
    }
  }
  arc_dw_epilogue<MAXJ>(acc, wv, nj, inv_nw[col], eps, g, dW + (long long)col * lddw);
}

Margin make_margin(float s, float m, int easy) {
  const float PI = 3.14159265358979323846f;
  return Margin{s, cosf(m), sinf(m), cosf(PI - m), sinf(PI - m) * m, easy};
}

bool a16(const void* p) { return ((uintptr_t)p & 15) == 0; }

// block rows of the dW backward: one up to 64 batch rows, then <= 64 rows each
int arc_bwd_slices(int B) { return B <= 64 ? 1 : (B + 63) / 64; }

// rows per x chunk so that the LDS stays under 128 KiB
int chunk_rows(int B, int D, int fixed_floats) {
  const int budget = 32768 - fixed_floats;
  return std::max(1, std::min(B, budget / (D + 4)));
}

// The MFMA backward for D in {128, 256, 512, 640}: returns -1 when D has no
// instance (the caller takes the VALU kernel), else the launch status.
int launch_arc_bwd_mma(const float* dlogits, const float* cosv, const long long* label,
                       const float* xn, const float* W, long long ldw, const float* inv_nw,
                       int B, int D, int C, Margin M, float eps, float* dW, long long lddw,
                       float* dcs, int S, int rows_per, float* part, FocalSrc F, ArcBwd2 h2,
                       int n_heads, void* stream) {
  using Fn = decltype(&arc_bwd_mma_kernel<1>);
  Fn fn = D == 128 ? &arc_bwd_mma_kernel<1> : D == 256 ? &arc_bwd_mma_kernel<2>
        : D == 512 ? &arc_bwd_mma_kernel<4> : D == 640 ? &arc_bwd_mma_kernel<5> : nullptr;
  if (!fn || ldw % 4 || lddw % 4) return -1;
  const bool whole = D <= 256 && rows_per <= ARC_WHOLE;
  const int dc_rows = whole ? (rows_per + 1) & ~1 : rows_per + RBM;
  const int lds = ((dc_rows * (CBM + 1) * 4 + 15) & ~15) + (whole ? dc_rows : RBM) * (D + 4) * 4;
  if (lds > 160 * 1024) return -1;
  if (const int e = set_max_lds((const void*)fn, lds)) return e;
  hipLaunchKernelGGL(fn, dim3((C + CBM - 1) / CBM, S, n_heads), dim3(NT), lds,
                     (hipStream_t)stream, dlogits, cosv, label, xn, W, ldw, inv_nw, B, D, C, M,
                     eps, dW, lddw, dcs, rows_per, part, F, h2);
  return (int)hipGetLastError();
}

}  // namespace

extern "C" {

int tgfr_arc_fwd(const float* x, long long ldx, int B, int D, const float* W, long long ldw,
                 int C, const long long* label, float s, float m, int easy, float eps,
                 float* logits, float* cosv, float* xn, float* inv_nx, float* inv_nw,
                 void* stream) {
  if (B <= 0 || B > 4096 || C <= 0 || D <= 0 || D % 8 || D > 1024 || ldx % 4 || ldw % 4 ||
      !a16(x) || !a16(W) || !a16(xn))
    return 1001;
  const int fk = D <= 256 && B <= FRB ? 256 : 128;   // one row block: LDS per block is free
  const int lds = ((CBF + FRB) * (fk + 4) + CBF + 2 * FRB) * 4;
  auto fn = fk == 256 ? &arc_fwd_kernel<256> : &arc_fwd_kernel<128>;
  if (const int e = set_max_lds((const void*)fn, lds)) return e;
  hipLaunchKernelGGL(fn, dim3((C + CBF - 1) / CBF, (B + FRB - 1) / FRB), dim3(NT),
                     lds, (hipStream_t)stream, x, ldx, B, D, W, ldw, C, label,
                     make_margin(s, m, easy), eps, logits, cosv, xn, inv_nx, inv_nw, ArcHead2{});
  return (int)hipGetLastError();
}

int tgfr_arc_bwd(const float* dlogits, const float* cosv, const long long* label,
                 const float* xn, const float* W, long long ldw, const float* inv_nw, int B,
                 int D, int C, float s, float m, int easy, float eps, float* dW, long long lddw,
                 float* dcs, float* ws, void* stream) {
  if (B <= 0 || C <= 0 || D <= 0 || D % 4 || D > 1024 || ldw % 4 || lddw % 4 || !a16(W) ||
      !a16(dW) || !a16(xn) || B > 4096 || (!ws && B * CB > 16384) || (ws && !a16(ws)))
    return 1001;
  // B > 64 with a workspace: block rows of <= 64 batch rows each (partial
  // dWn to ws, summed by the finish launch) and small x chunks, so several
  // blocks share a CU instead of one block walking all B rows
  const int S = ws ? arc_bwd_slices(B) : 1;
  const int rows_per = (B + S - 1) / S;
  const int RB = S > 1 ? std::min(16, rows_per) : chunk_rows(B, D, B * CB);
  const int lds = (rows_per * CB + RB * (D + 4)) * 4;
  if (const int e = launch_arc_bwd_mma(dlogits, cosv, label, xn, W, ldw, inv_nw, B, D, C,
                                       make_margin(s, m, easy), eps, dW, lddw, dcs, S, rows_per,
                                       ws, FocalSrc{}, ArcBwd2{}, 1, stream);
      e != -1) {
    if (e) return e;
  } else {
    using Fn = decltype(&arc_bwd_kernel<0>);
    Fn fn = D == 128 ? &arc_bwd_kernel<2> : D == 256 ? &arc_bwd_kernel<4>
          : D == 512 ? &arc_bwd_kernel<8> : D == 640 ? &arc_bwd_kernel<10> : &arc_bwd_kernel<0>;
    if (const int e = set_max_lds((const void*)fn, lds)) return e;
    hipLaunchKernelGGL(fn, dim3((C + CB - 1) / CB, S), dim3(NT), lds, (hipStream_t)stream,
                       dlogits, cosv, label, xn, W, ldw, inv_nw, B, D, C, make_margin(s, m, easy),
                       eps, RB, dW, lddw, dcs, rows_per, ws, FocalSrc{}, ArcBwd2{});
  }
  if (S > 1) {
    using Gn = decltype(&arc_bwd_finish_kernel<0>);
    Gn gn = D == 128 ? &arc_bwd_finish_kernel<2> : D == 256 ? &arc_bwd_finish_kernel<4>
          : D == 512 ? &arc_bwd_finish_kernel<8> : D == 640 ? &arc_bwd_finish_kernel<10>
          : &arc_bwd_finish_kernel<0>;
    hipLaunchKernelGGL(gn, dim3((C + CB - 1) / CB), dim3(NT), 0, (hipStream_t)stream, ws, S, W,
                       ldw, inv_nw, D, C, eps, dW, lddw);
  }
  return (int)hipGetLastError();
}

int tgfr_arc_fwd_heads(const tgfr_arc_head* heads, int n_heads, int B, int D, int C, float m,
                       int easy, float eps, void* stream) {
  if (!heads || n_heads < 1 || n_heads > 2 || B <= 0 || B > 4096 || C <= 0 || D <= 0 || D % 8 ||
      D > 1024)
    return 1001;
  for (int k = 0; k < n_heads; ++k)
    if (!a16(heads[k].x) || !a16(heads[k].W) || !a16(heads[k].xn)) return 1001;
  const tgfr_arc_head& a = heads[0];
  ArcHead2 h2{};
  if (n_heads == 2) {
    const tgfr_arc_head& b = heads[1];
    h2 = ArcHead2{b.x, b.W, b.logits, b.cosv, b.xn, b.inv_nx, b.inv_nw, make_margin(b.s, m, easy)};
  }
  // 128-wide k chunks (~51 KB LDS): several blocks per CU, so both heads'
  // class blocks run in one round
  constexpr int fk = 128;
  const int lds = ((CBF + FRB) * (fk + 4) + CBF + 2 * FRB) * 4;
  auto fn = &arc_fwd_kernel<fk>;
  if (const int e = set_max_lds((const void*)fn, lds)) return e;
  hipLaunchKernelGGL(fn, dim3((C + CBF - 1) / CBF, (B + FRB - 1) / FRB, n_heads), dim3(NT), lds,
                     (hipStream_t)stream, a.x, (long long)D, B, D, a.W, (long long)D, C, a.label,
                     make_margin(a.s, m, easy), eps, a.logits, a.cosv, a.xn, a.inv_nx, a.inv_nw,
                     h2);
  return (int)hipGetLastError();
}

int tgfr_arc_focal_bwd_heads(const tgfr_arc_head* heads, int n_heads, int B, int D, int C,
                             float m, int easy, float eps, float gamma, void* stream) {
  // (B <= 128: one row slice of every batch row per class block -- the
  // focal source needs the whole row -- staged in 16-row x chunks past 64)
  if (!heads || n_heads < 1 || n_heads > 2 || B <= 0 || B > 128 || C <= 0 || D <= 0 || D % 4 ||
      D > 1024)
    return 1001;
  for (int k = 0; k < n_heads; ++k)
    if (!a16(heads[k].W) || !a16(heads[k].dW) || !a16(heads[k].xn) || !heads[k].logits ||
        !heads[k].focal_ws || heads[k].label != heads[0].label)
      return 1001;
  const tgfr_arc_head& a = heads[0];
  ArcBwd2 h2{};
  if (n_heads == 2) {
    const tgfr_arc_head& b = heads[1];
    h2 = ArcBwd2{b.cosv, b.xn, b.W, b.inv_nw, b.dW, b.dcs, FocalSrc{b.logits, b.focal_ws, b.g, gamma},
                 make_margin(b.s, m, easy)};
  }
  const FocalSrc fa{a.logits, a.focal_ws, a.g, gamma};
  if (const int e = launch_arc_bwd_mma(nullptr, a.cosv, a.label, a.xn, a.W, (long long)D,
                                       a.inv_nw, B, D, C, make_margin(a.s, m, easy), eps, a.dW,
                                       (long long)D, a.dcs, 1, B, nullptr, fa, h2, n_heads,
                                       stream);
      e != -1)
    return e;
  // 16-row x chunks (~21 KB LDS at D = 256): both heads' class blocks in one round
  const int RB = std::min(16, B);
  const int lds = (B * CB + RB * (D + 4)) * 4;
  using Fn = decltype(&arc_bwd_kernel<0>);
  Fn fn = D == 128 ? &arc_bwd_kernel<2> : D == 256 ? &arc_bwd_kernel<4>
        : D == 512 ? &arc_bwd_kernel<8> : D == 640 ? &arc_bwd_kernel<10> : &arc_bwd_kernel<0>;
  if (const int e = set_max_lds((const void*)fn, lds)) return e;
  hipLaunchKernelGGL(fn, dim3((C + CB - 1) / CB, 1, n_heads), dim3(NT), lds, (hipStream_t)stream,
                     nullptr, a.cosv, a.label, a.xn, a.W, (long long)D, a.inv_nw, B, D, C,
                     make_margin(a.s, m, easy), eps, RB, a.dW, (long long)D, a.dcs, B, nullptr,
                     fa, h2);
  return (int)hipGetLastError();
}

int tgfr_arc_bwd_ws(int B, int D, int C, long long* floats) {
  if (B <= 0 || C <= 0 || D <= 0 || !floats) return 1001;
  const int S = arc_bwd_slices(B);
  *floats = S > 1 ? (long long)S * C * D : 0;
  return 0;
}

}  // extern "C"
