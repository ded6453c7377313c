// FCFM image branch: relu(Conv2d(256, 36, 3, padding=0)) -> MaxPool2d(2)
// (models/fusion_nets.py:229-237, Working.forward :236-237), forward and
// backward, on v_mfma_f32_16x16x32_bf16 (hi*hi in bf16 mode, the split
// hi/lo triple in fp32 mode, as tgfr_common.h).
//
// Shapes are the module's: x [B, 256, 14, 14] read as channels-last rows
// [B][196][256] (the physical layout ImageHeading produces), output pooled
// [B, 36, 6, 6].  With q = y*14 + x an input row and taps (ty, tx), the conv
// output at (oy, ox) is sum_tap X[(oy+ty)*14 + ox+tx] . W[:, :, ty, tx].
//
// Forward (one workgroup per sample, the whole im2col GEMM M = 144 output
// positions x N = 36 (48) channels x K = 9 taps * 256 channels in LDS):
//   * the sample's rows are staged twice, 128 channels at a time, as bf16
//     (hi, + lo) into an XOR-swizzled LDS image; K is split over the 4 waves
//     (wave w owns the 32-channel block w of each half for all 9 taps), so
//     every packed weight fragment is read once per workgroup;
//   * M rows are in POOL order (row m = 4 * window + element of the 2x2
//     window), so after the cross-wave sum each lane's 4 accumulator rows are
//     exactly one pooling window: bias + ReLU + 2x2 max + argmax in registers.
//   Outputs pooled [B][36][36] fp32 and the argmax code (0..3, or -1 when the
//   max is <= 0 and the ReLU blocks the gradient), the MaxPool2d/ReLU
//   backward state.
// Input gradient (one workgroup per sample): the routed gradient G is
//   scattered to an LDS image indexed by k = oy*14 + ox (columns 12, 13 and
//   the margins zero), so dX[q] = sum_tap G[q - (ty*14 + tx)] W_tap^T is a
//   GEMM whose A rows are plain shifted rows of that image (the zero columns
//   absorb the row wrap-around): M = 196 (208), N = 256, K = 9 taps x 40.
// Weight gradient: dW_tap = G^T X_shift over (sample, position), per
//   (32-channel chunk, sample group) workgroup, X read by transposing LDS
//   reads (ds_read_b64_tr_b16) at the tap's row shift; group partials summed
//   in group order by a second launch, which also sums the bias gradient.
#include "tgfr_common.h"

#include <algorithm>

using namespace tgfr;

namespace {

constexpr int CIN = 256, COUT = 36, NPIN = 196, NWIN = 36, NOUT = COUT * NWIN;
constexpr int FK = 72;                                   // fwd k-steps: 9 taps x 8 blocks
constexpr int FNT = 3;                                   // fwd 16-wide co tiles
constexpr int FWD_ELEMS = FK * FNT * 64 * 8;
constexpr int DK = 12;                                   // dx k-steps: 45 (tap, co8) blocks -> 48
constexpr int DNT = 16;                                  // dx 16-wide channel tiles
constexpr int DX_ELEMS = DK * DNT * 64 * 8;
constexpr int PK_ELEMS = 2 * (FWD_ELEMS + DX_ELEMS);     // [fwd hi|fwd lo|dx hi|dx lo]

__device__ __forceinline__ int tap_off(int tap) { return (tap / 3) * 14 + tap % 3; }

template <int MODE>
__device__ __forceinline__ void mma16(f32x4& acc, const bf16x8& ahi, const bf16x8& alo,
                                      const bf16x8& bhi, const bf16x8& blo) {
  if constexpr (MODE == MODE_SPLIT) {
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(alo, bhi, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ahi, blo, acc, 0, 0, 0);
  }
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ahi, bhi, acc, 0, 0, 0);
}

__device__ __forceinline__ void lds_st2(uint32_t off, uint16_t v) {
  *(LDS_AS uint16_t*)(lds_base() + off) = v;
}
__device__ __forceinline__ void lds_st4(uint32_t off, uint32_t v) {
  *(LDS_AS uint32_t*)(lds_base() + off) = v;
}

// 4 fp32 -> 4 bf16 hi (+ lo) as two dwords each
template <int MODE>
__device__ __forceinline__ void cvt4(const float4& v, uint2& hi, uint2& lo) {
  uint16_t h[4], l[4] = {0, 0, 0, 0};
  const float f[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    if constexpr (MODE == MODE_SPLIT)
      split2(f[i], h[i], l[i]);
    else
      h[i] = bf_bits(f[i]);
  }
  hi = make_uint2(pack2(h[0], h[1]), pack2(h[2], h[3]));
  lo = make_uint2(pack2(l[0], l[1]), pack2(l[2], l[3]));
}

// ------------------------------------------------------------- weight pack ---
// W [36][256][3][3] fp32 (the Conv2d weight) -> MFMA B fragments:
//   fwd (s = tap*8 + cb, n): lane l -> W[16n + l%16][32cb + 8(l/16) + i][tap]
//   dx  (s, n): lane l, KB = 4s + l/16 (tap = KB/5, co8 = KB%5) ->
//       W[8 co8 + i][16n + l%16][tap]
// zero outside 36 output channels / 45 k-blocks; bf16 hi and lo planes.
__global__ __launch_bounds__(256) void fcfm_pack_kernel(const float* __restrict__ W,
                                                        uint16_t* __restrict__ pk) {
  const int f = blockIdx.x * 256 + threadIdx.x;
  constexpr int NF = FWD_ELEMS / 8, ND = DX_ELEMS / 8;
  if (f >= NF + ND) return;
  float v[8];
  uint16_t* hi;
  uint16_t* lo;
  if (f < NF) {
    const int l = f & 63, sn = f >> 6, n = sn % FNT, s = sn / FNT;
    const int tap = s >> 3, cb = s & 7, co = 16 * n + (l & 15), c0 = 32 * cb + 8 * (l >> 4);
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = co < COUT ? W[(co * CIN + c0 + i) * 9 + tap] : 0.f;
    hi = pk + f * 8;
    lo = pk + FWD_ELEMS + f * 8;
  } else {
    const int e = f - NF, l = e & 63, sn = e >> 6, n = sn % DNT, s = sn / DNT;
    const int KB = 4 * s + (l >> 4), c = 16 * n + (l & 15);
    const int tap = KB / 5, co0 = 8 * (KB % 5);
#pragma unroll
    for (int i = 0; i < 8; ++i)
      v[i] = (KB < 45 && co0 + i < COUT) ? W[((co0 + i) * CIN + c) * 9 + tap] : 0.f;
    hi = pk + 2 * FWD_ELEMS + e * 8;
    lo = pk + 2 * FWD_ELEMS + DX_ELEMS + e * 8;
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) split2(v[i], hi[i], lo[i]);
}

// ----------------------------------------------------------------- forward ---
constexpr int FX_ROW = 256;                       // 128 channels bf16 per LDS row
constexpr int FX_IMG = NPIN * FX_ROW;             // one plane (hi or lo)
constexpr int F_PART = 4 * 27 * 64 * 16;          // cross-wave partials
constexpr int F_LDS = F_PART > 2 * FX_IMG ? F_PART : 2 * FX_IMG;

template <int MODE>
__global__ __launch_bounds__(256, 1) void fcfm_fwd_kernel(const float* __restrict__ x,
                                                          long long s_b, long long s_p,
                                                          const uint16_t* __restrict__ pk,
                                                          const float* __restrict__ bias,
                                                          float* __restrict__ pooled,
                                                          int8_t* __restrict__ code) {
  const int b = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l16 = lane & 15, g = lane >> 4;
  const float* xb = x + b * s_b;

  // the lane's output position for each 16-row M tile (pool order)
  int qb[9];
#pragma unroll
  for (int mt = 0; mt < 9; ++mt) {
    const int m = 16 * mt + l16, win = m >> 2, e = m & 3;
    qb[mt] = (2 * (win / 6) + (e >> 1)) * 14 + 2 * (win % 6) + (e & 1);
  }
  f32x4 acc[9][FNT];
#pragma unroll
  for (int mt = 0; mt < 9; ++mt)
#pragma unroll
    for (int n = 0; n < FNT; ++n) acc[mt][n] = (f32x4){0.f, 0.f, 0.f, 0.f};

  const uint16_t* pkh = pk;
  const uint16_t* pkl = pk + FWD_ELEMS;
  const int blk = 4 * w + g;                       // the lane's 16-B block of a row
  // rows 0..195 of one 128-channel half: 196 x 32 float4, 25 per thread,
  // held in registers so that half 1's loads are in flight during half 0's
  // MFMAs
  constexpr int NV = NPIN * 32, NU = (NV + 255) / 256;
  float4 xv[NU];
  auto fetch = [&](int h) {
#pragma unroll
    for (int u = 0; u < NU; ++u) {
      const int i = u * 256 + tid;
      if (i < NV) xv[u] = *(const float4*)(xb + (i >> 5) * s_p + 128 * h + 4 * (i & 31));
    }
  };
  fetch(0);
  for (int h = 0; h < 2; ++h) {
    if (h) __syncthreads();                        // half 0's reads are done
#pragma unroll
    for (int u = 0; u < NU; ++u) {
      const int i = u * 256 + tid;
      if (i < NV) {
        const int q = i >> 5, c4 = i & 31;
        uint2 hi, lo;
        cvt4<MODE>(xv[u], hi, lo);
        const uint32_t off = q * FX_ROW + (((c4 >> 1) ^ (q & 15)) << 4) + (c4 & 1) * 8;
        lds_st8(off, hi);
        if constexpr (MODE == MODE_SPLIT) lds_st8(FX_IMG + off, lo);
      }
    }
    __syncthreads();
    if (h == 0) fetch(1);
    const int cb = 4 * h + w;
    bf16x8 bh[FNT], bl[FNT];
    auto load_b = [&](int tap) {
      const int s = tap * 8 + cb;
#pragma unroll
      for (int n = 0; n < FNT; ++n) {
        const long long o = ((long long)(s * FNT + n) * 64 + lane) * 8;
        bh[n] = as_bf8(*(const uint4*)(pkh + o));
        bl[n] = MODE == MODE_SPLIT ? as_bf8(*(const uint4*)(pkl + o)) : bh[n];
      }
    };
    load_b(0);
#pragma unroll 1
    for (int tap = 0; tap < 9; ++tap) {
      bf16x8 ch[FNT], cl[FNT];
#pragma unroll
      for (int n = 0; n < FNT; ++n) {
        ch[n] = bh[n];
        cl[n] = bl[n];
      }
      if (tap + 1 < 9) load_b(tap + 1);
      const int toff = tap_off(tap);
#pragma unroll
      for (int mt = 0; mt < 9; ++mt) {
        const int q = qb[mt] + toff;
        const uint32_t off = q * FX_ROW + ((blk ^ (q & 15)) << 4);
        const bf16x8 ah = as_bf8(lds_ld16(off));
        const bf16x8 al = MODE == MODE_SPLIT ? as_bf8(lds_ld16(FX_IMG + off)) : ah;
#pragma unroll
        for (int n = 0; n < FNT; ++n) mma16<MODE>(acc[mt][n], ah, al, ch[n], cl[n]);
      }
    }
  }
  __syncthreads();
#pragma unroll
  for (int mt = 0; mt < 9; ++mt)
#pragma unroll
    for (int n = 0; n < FNT; ++n)
      lds_st16(((w * 27 + mt * FNT + n) * 64 + lane) * 16, __builtin_bit_cast(uint4, acc[mt][n]));
  __syncthreads();
  for (int it = tid; it < 27 * 64; it += 256) {
    const int tile = it >> 6, l = it & 63;
    const int mt = tile / FNT, n = tile % FNT, co = 16 * n + (l & 15);
    if (co >= COUT) continue;
    f32x4 v = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ww = 0; ww < 4; ++ww)
      v += __builtin_bit_cast(f32x4, lds_ld16(((ww * 27 + tile) * 64 + l) * 16));
    const float bb = bias[co];
    float best = v[0] + bb;
    int idx = 0;
#pragma unroll
    for (int j = 1; j < 4; ++j) {
      const float val = v[j] + bb;
      if (val > best) {
        best = val;
        idx = j;
      }
    }
    const int o = b * NOUT + co * NWIN + 4 * mt + (l >> 4);
    pooled[o] = fmaxf(best, 0.f);
    code[o] = best > 0.f ? (int8_t)idx : (int8_t)-1;
  }
}

// ----------------------------------------------------------- input gradient ---
constexpr int DG_ROW = 80;                        // 40 channels bf16
constexpr int DG_ROWS = 238;                      // k = -30 .. 207
constexpr int DG_IMG = DG_ROWS * DG_ROW;
constexpr int DX_LDS = 2 * DG_IMG;

// position k = oy*14 + ox of the routed gradient of (window, code)
__device__ __forceinline__ int routed_k(int win, int c) {
  return (2 * (win / 6) + (c >> 1)) * 14 + 2 * (win % 6) + (c & 1);
}

template <int MODE>
__global__ __launch_bounds__(256) void fcfm_dx_kernel(const float* __restrict__ gp,
                                                      const int8_t* __restrict__ code,
                                                      const uint16_t* __restrict__ pk,
                                                      float* __restrict__ dx, long long s_b,
                                                      long long s_p) {
  const int b = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l16 = lane & 15, g = lane >> 4;
  // the sample's routed gradient into registers first (its latency overlaps
  // the zeroing of the image)
  int cv[6];
  float gv[6];
#pragma unroll
  for (int r = 0; r < 6; ++r) {
    const int i = r * 256 + tid;
    cv[r] = i < NOUT ? code[b * NOUT + i] : -1;
    gv[r] = i < NOUT ? gp[b * NOUT + i] : 0.f;
  }
  for (int o = tid * 16; o < DX_LDS; o += 256 * 16) lds_st16(o, make_uint4(0, 0, 0, 0));
  __syncthreads();
#pragma unroll
  for (int r = 0; r < 6; ++r) {
    const int i = r * 256 + tid;
    if (cv[r] >= 0) {
      const int co = i / NWIN, k = routed_k(i % NWIN, cv[r]);
      uint16_t hi, lo;
      split2(gv[r], hi, lo);
      const uint32_t off = (30 + k) * DG_ROW + co * 2;
      lds_st2(off, hi);
      if constexpr (MODE == MODE_SPLIT) lds_st2(DG_IMG + off, lo);
    }
  }
  __syncthreads();
  const uint16_t* pkh = pk + 2 * FWD_ELEMS;
  const uint16_t* pkl = pkh + DX_ELEMS;
#pragma unroll 1
  for (int j = 0; j < 4; ++j) {
    const int n = 4 * w + j;
    f32x4 acc[13];
#pragma unroll
    for (int mt = 0; mt < 13; ++mt) acc[mt] = (f32x4){0.f, 0.f, 0.f, 0.f};
    auto ldb = [&](int s, bf16x8& bh, bf16x8& bl) {
      const long long o = ((long long)(s * DNT + n) * 64 + lane) * 8;
      bh = as_bf8(*(const uint4*)(pkh + o));
      bl = MODE == MODE_SPLIT ? as_bf8(*(const uint4*)(pkl + o)) : bh;
    };
    bf16x8 nh, nl;
    ldb(0, nh, nl);
#pragma unroll 2
    for (int s = 0; s < DK; ++s) {
      const bf16x8 bh = nh, bl = nl;
      if (s + 1 < DK) ldb(s + 1, nh, nl);
      const int KB = 4 * s + g;
      // k-blocks past the 45 real ones have zero weights: read row 0 (zero)
      const int valid = KB < 45;
      const int tap = valid ? KB / 5 : 0;
      const uint32_t kb = valid ? (30 - tap_off(tap)) * DG_ROW + (KB % 5) * 16 : 0;
#pragma unroll
      for (int mt = 0; mt < 13; ++mt) {
        const uint32_t off = kb + (valid ? (16 * mt + l16) * DG_ROW : 0);
        const bf16x8 ah = as_bf8(lds_ld16(off));
        const bf16x8 al = MODE == MODE_SPLIT ? as_bf8(lds_ld16(DG_IMG + off)) : ah;
        mma16<MODE>(acc[mt], ah, al, bh, bl);
      }
    }
    float* out = dx + b * s_b + 16 * n + l16;
#pragma unroll
    for (int mt = 0; mt < 13; ++mt)
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        const int q = 16 * mt + 4 * g + jj;
        if (q < NPIN) out[q * s_p] = acc[mt][jj];
      }
  }
}

// ---------------------------------------------------------- weight gradient ---
constexpr int WG_K = 192;                         // positions per sample (168 used)
constexpr int WG_ROW = WG_K * 2;                  // G^T row: one output channel
constexpr int WG_IMG = 48 * WG_ROW;
constexpr int WX_ROW = 64;                        // 32 channels bf16
constexpr int WX_ROWS = 224;                      // k + tap shift <= 221
constexpr int WX_IMG = WX_ROWS * WX_ROW;
constexpr int DW_LDS = 2 * WG_IMG + 2 * WX_IMG + NOUT * 4;
constexpr int DW_CHUNKS = 8;                      // 32-channel chunks

static int dw_groups(int B) { return std::max(1, std::min(B, 32)); }

template <int MODE>
__global__ __launch_bounds__(256) void fcfm_dw_kernel(const float* __restrict__ x, long long s_b,
                                                      long long s_p, const float* __restrict__ gp,
                                                      const int8_t* __restrict__ code, int B,
                                                      int per, float* __restrict__ part,
                                                      float* __restrict__ dbp) {
  const int chunk = blockIdx.x % DW_CHUNKS, grp = blockIdx.x / DW_CHUNKS;
  const int b0 = grp * per, b1 = min(B, b0 + per);
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l16 = lane & 15, g = lane >> 4, q4 = l16 >> 2, p4 = l16 & 3;
  constexpr int GLO = WG_IMG, XHI = 2 * WG_IMG, XLO = XHI + WX_IMG, GSC = XLO + WX_IMG;
  // zeroed once: G^T entries never written per sample (columns 12, 13, k >=
  // 168, output channels >= 36) and X rows 196..223
  for (int o = tid * 16; o < 2 * WG_IMG; o += 256 * 16) lds_st16(o, make_uint4(0, 0, 0, 0));
  for (int o = NPIN * WX_ROW + tid * 16; o < WX_IMG; o += 256 * 16) {
    lds_st16(XHI + o, make_uint4(0, 0, 0, 0));
    lds_st16(XLO + o, make_uint4(0, 0, 0, 0));
  }
  f32x4 acc[14];
#pragma unroll
  for (int i = 0; i < 14; ++i) acc[i] = (f32x4){0.f, 0.f, 0.f, 0.f};
  float db = 0.f;
  // the next sample's X rows and routed gradient, fetched into registers
  // while the current one computes
  float4 xv[7];
  int cv[6];
  float gv[6];
  auto fetch = [&](int b) {
    const float* xb = x + b * s_b + 32 * chunk;
#pragma unroll
    for (int u = 0; u < 7; ++u) {
      const int i = u * 256 + tid;
      if (i < NPIN * 8) xv[u] = *(const float4*)(xb + (i >> 3) * s_p + 4 * (i & 7));
    }
#pragma unroll
    for (int r = 0; r < 6; ++r) {
      const int i = r * 256 + tid;
      cv[r] = i < NOUT ? code[b * NOUT + i] : -1;
      gv[r] = i < NOUT ? gp[b * NOUT + i] : 0.f;
    }
  };
  if (b0 < b1) fetch(b0);
  for (int b = b0; b < b1; ++b) {
    __syncthreads();                               // previous sample's reads done
#pragma unroll
    for (int u = 0; u < 7; ++u) {
      const int i = u * 256 + tid;
      if (i < NPIN * 8) {
        uint2 hi, lo;
        cvt4<MODE>(xv[u], hi, lo);
        const uint32_t off = (i >> 3) * WX_ROW + (i & 7) * 8;
        lds_st8(XHI + off, hi);
        if constexpr (MODE == MODE_SPLIT) lds_st8(XLO + off, lo);
      }
    }
    // every (channel, window) writes its whole 2x2 window of G^T: the routed
    // value at the argmax, zeros elsewhere (no per-sample zeroing pass)
#pragma unroll
    for (int r = 0; r < 6; ++r) {
      const int i = r * 256 + tid;
      if (i < NOUT) {
        const int co = i / NWIN, win = i % NWIN, c = cv[r];
        const float gvr = c >= 0 ? gv[r] : 0.f;
        const int k0 = 28 * (win / 6) + 2 * (win % 6);
        uint16_t h[4], l[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) split2(e == c ? gvr : 0.f, h[e], l[e]);
        const uint32_t o0 = co * WG_ROW + k0 * 2, o1 = o0 + 14 * 2;
        lds_st4(o0, pack2(h[0], h[1]));
        lds_st4(o1, pack2(h[2], h[3]));
        if constexpr (MODE == MODE_SPLIT) {
          lds_st4(GLO + o0, pack2(l[0], l[1]));
          lds_st4(GLO + o1, pack2(l[2], l[3]));
        }
        if (chunk == 0) lds_stf(GSC + i * 4, gvr);
      }
    }
    __syncthreads();
    if (b + 1 < b1) fetch(b + 1);
    if (chunk == 0 && tid < COUT)                  // bias gradient, window order
      for (int win = 0; win < NWIN; ++win) db += lds_ldf(GSC + (tid * NWIN + win) * 4);
#pragma unroll 1
    for (int s = 0; s < WG_K / 32; ++s) {
#pragma unroll
      for (int i = 0; i < 14; ++i) {
        const int t = w + 4 * i;                   // tile (mt, nt) = (t / 18, t % 18)
        if (t >= 54) continue;
        const int mt = t / 18, nt = t % 18, tap = nt >> 1, c16 = (nt & 1) * 16;
        const uint32_t ao = (16 * mt + l16) * WG_ROW + (32 * s + 8 * g) * 2;
        const bf16x8 ah = as_bf8(lds_ld16(ao));
        const bf16x8 al = MODE == MODE_SPLIT ? as_bf8(lds_ld16(GLO + ao)) : ah;
        const uint32_t xo = (32 * s + 8 * g + q4 + tap_off(tap)) * WX_ROW + (c16 + 4 * p4) * 2;
        const bf16x8 bh = join_tr(lds_tr4(XHI + xo), lds_tr4(XHI + xo + 4 * WX_ROW));
        const bf16x8 bl = MODE == MODE_SPLIT
                              ? join_tr(lds_tr4(XLO + xo), lds_tr4(XLO + xo + 4 * WX_ROW))
                              : bh;
        mma16<MODE>(acc[i], ah, al, bh, bl);
      }
    }
  }
  // partials part[grp][tap][co][c]
#pragma unroll
  for (int i = 0; i < 14; ++i) {
    const int t = w + 4 * i;
    if (t >= 54) continue;
    const int mt = t / 18, nt = t % 18, tap = nt >> 1;
    const int c = 32 * chunk + (nt & 1) * 16 + l16;
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      const int co = 16 * mt + 4 * g + jj;
      if (co < COUT) part[(((long long)grp * 9 + tap) * COUT + co) * CIN + c] = acc[i][jj];
    }
  }
  if (chunk == 0 && tid < COUT) dbp[grp * COUT + tid] = db;
}

// dW [36][256][3][3] = sum over groups (group order) of the partials; db too
__global__ __launch_bounds__(256) void fcfm_dw_reduce_kernel(const float* __restrict__ part,
                                                             const float* __restrict__ dbp,
                                                             int groups, float* __restrict__ dW,
                                                             float* __restrict__ db) {
  const int o = blockIdx.x * 256 + threadIdx.x;
  constexpr int NW = COUT * CIN * 9;
  if (o < NW) {
    // o walks the partials' [tap][co][c] order (coalesced group reads)
    const int c = o % CIN, co = (o / CIN) % COUT, tap = o / (CIN * COUT);
    float s = 0.f;
    for (int gr = 0; gr < groups; ++gr) s += part[(long long)gr * NW + o];
    dW[(co * CIN + c) * 9 + tap] = s;
  } else if (o < NW + COUT) {
    const int co = o - NW;
    float s = 0.f;
    for (int gr = 0; gr < groups; ++gr) s += dbp[gr * COUT + co];
    db[co] = s;
  }
}

// ------------------------------------------------- 2x2 max pool, channels last ---
// Working's second MaxPool2d (fusion_nets.py:252) on the LayerNorm output,
// which the attention leaves channels-last: x [B][H*W][C] -> y [B][C][H/2][W/2]
// (NCHW, the order the following flatten + Linear read, :253-254) and the
// argmax (0..3 = dy*2 + dx, first maximum in scan order as MaxPool2d).  One
// thread per output element, reads coalesced along C.
__global__ __launch_bounds__(256) void maxpool2_cl_kernel(const float* __restrict__ x, int B,
                                                          int H, int W, int C,
                                                          float* __restrict__ y,
                                                          uint8_t* __restrict__ idx) {
  const int ph = H / 2, pw = W / 2;
  const long long n = (long long)B * ph * pw * C;
  const long long o = blockIdx.x * 256LL + threadIdx.x;
  if (o >= n) return;
  const int c = o % C, px = (o / C) % pw, py = (o / ((long long)C * pw)) % ph;
  const int b = o / ((long long)C * pw * ph);
  const float* xb = x + (long long)b * H * W * C + c;
  float best = xb[((2 * py) * W + 2 * px) * C];
  int bi = 0;
#pragma unroll
  for (int e = 1; e < 4; ++e) {
    const float v = xb[((2 * py + (e >> 1)) * W + 2 * px + (e & 1)) * C];
    if (v > best) {
      best = v;
      bi = e;
    }
  }
  const long long oy = (((long long)b * C + c) * ph + py) * pw + px;
  y[oy] = best;
  idx[oy] = (uint8_t)bi;
}

// dx [B][H*W][C] (every element written: the gradient at the argmax, 0 elsewhere)
__global__ __launch_bounds__(256) void maxpool2_cl_bwd_kernel(const float* __restrict__ dy,
                                                              const uint8_t* __restrict__ idx,
                                                              int B, int H, int W, int C,
                                                              float* __restrict__ dx) {
  const int ph = H / 2, pw = W / 2;
  const long long n = (long long)B * ph * pw * C;
  const long long o = blockIdx.x * 256LL + threadIdx.x;
  if (o >= n) return;
  const int c = o % C, px = (o / C) % pw, py = (o / ((long long)C * pw)) % ph;
  const int b = o / ((long long)C * pw * ph);
  const long long oy = (((long long)b * C + c) * ph + py) * pw + px;
  const float g = dy[oy];
  const int bi = idx[oy];
  float* xb = dx + (long long)b * H * W * C + c;
#pragma unroll
  for (int e = 0; e < 4; ++e)
    xb[((2 * py + (e >> 1)) * W + 2 * px + (e & 1)) * C] = e == bi ? g : 0.f;
}

bool rows_ok(const float* x, long long s_b, long long s_p) {
  return x && ((uintptr_t)x & 15) == 0 && s_b % 4 == 0 && s_p % 4 == 0 && s_p >= CIN;
}

}  // namespace

extern "C" {

int tgfr_fcfm_pack_elems(void) { return PK_ELEMS; }

int tgfr_maxpool2_cl(const float* x, int B, int H, int W, int C, float* y, uint8_t* idx,
                     void* stream) {
  if (!x || !y || !idx || B <= 0 || C <= 0 || H < 2 || W < 2 || (H & 1) || (W & 1)) return 1001;
  const long long n = (long long)B * (H / 2) * (W / 2) * C;
  hipLaunchKernelGGL(maxpool2_cl_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, x, B, H, W, C, y, idx);
  return (int)hipGetLastError();
}

int tgfr_maxpool2_cl_bwd(const float* dy, const uint8_t* idx, int B, int H, int W, int C,
                         float* dx, void* stream) {
  if (!dy || !idx || !dx || B <= 0 || C <= 0 || H < 2 || W < 2 || (H & 1) || (W & 1)) return 1001;
  const long long n = (long long)B * (H / 2) * (W / 2) * C;
  hipLaunchKernelGGL(maxpool2_cl_bwd_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, dy, idx, B, H, W, C, dx);
  return (int)hipGetLastError();
}

int tgfr_fcfm_pack(const float* W, uint16_t* pk, void* stream) {
  if (!W || !pk || ((uintptr_t)pk & 15)) return 1001;
  const int n = (FWD_ELEMS + DX_ELEMS) / 8;
  hipLaunchKernelGGL(fcfm_pack_kernel, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream,
                     W, pk);
  return (int)hipGetLastError();
}

int tgfr_fcfm_conv_fwd(const float* x, long long s_b, long long s_p, int B, const uint16_t* pk,
                       const float* bias, float* pooled, int8_t* code, int mode, void* stream) {
  if (B <= 0 || !rows_ok(x, s_b, s_p) || !pk || !bias || !pooled || !code) return 1001;
  auto* s = (hipStream_t)stream;
  if (mode == MODE_SPLIT) {
    if (const int e = set_max_lds((const void*)fcfm_fwd_kernel<MODE_SPLIT>, F_LDS)) return e;
    hipLaunchKernelGGL(fcfm_fwd_kernel<MODE_SPLIT>, dim3(B), dim3(256), F_LDS, s, x, s_b, s_p,
                       pk, bias, pooled, code);
  } else if (mode == MODE_BF16) {
    if (const int e = set_max_lds((const void*)fcfm_fwd_kernel<MODE_BF16>, F_LDS)) return e;
    hipLaunchKernelGGL(fcfm_fwd_kernel<MODE_BF16>, dim3(B), dim3(256), F_LDS, s, x, s_b, s_p,
                       pk, bias, pooled, code);
  } else {
    return 1002;
  }
  return (int)hipGetLastError();
}

int tgfr_fcfm_conv_dx(const float* gpool, const int8_t* code, int B, const uint16_t* pk,
                      float* dx, long long s_b, long long s_p, int mode, void* stream) {
  if (B <= 0 || !gpool || !code || !pk || !dx || s_p < CIN) return 1001;
  auto* s = (hipStream_t)stream;
  if (mode == MODE_SPLIT)
    hipLaunchKernelGGL(fcfm_dx_kernel<MODE_SPLIT>, dim3(B), dim3(256), DX_LDS, s, gpool, code,
                       pk, dx, s_b, s_p);
  else if (mode == MODE_BF16)
    hipLaunchKernelGGL(fcfm_dx_kernel<MODE_BF16>, dim3(B), dim3(256), DX_LDS, s, gpool, code,
                       pk, dx, s_b, s_p);
  else
    return 1002;
  return (int)hipGetLastError();
}

int tgfr_fcfm_conv_dw_ws(int B, long long* floats) {
  if (B <= 0 || !floats) return 1001;
  *floats = (long long)dw_groups(B) * (9 * COUT * CIN + COUT);
  return 0;
}

int tgfr_fcfm_conv_dw(const float* x, long long s_b, long long s_p, const float* gpool,
                      const int8_t* code, int B, float* dW, float* db, float* ws, int mode,
                      void* stream) {
  if (B <= 0 || !rows_ok(x, s_b, s_p) || !gpool || !code || !dW || !db || !ws) return 1001;
  auto* s = (hipStream_t)stream;
  const int groups = dw_groups(B), per = (B + groups - 1) / groups;
  float* part = ws;
  float* dbp = ws + (long long)groups * 9 * COUT * CIN;
  const dim3 grid(DW_CHUNKS * groups);
  if (const int e = set_max_lds((const void*)fcfm_dw_kernel<MODE_SPLIT>, DW_LDS)) return e;
  if (const int e = set_max_lds((const void*)fcfm_dw_kernel<MODE_BF16>, DW_LDS)) return e;
  if (mode == MODE_SPLIT)
    hipLaunchKernelGGL(fcfm_dw_kernel<MODE_SPLIT>, grid, dim3(256), DW_LDS, s, x, s_b, s_p, gpool,
                       code, B, per, part, dbp);
  else if (mode == MODE_BF16)
    hipLaunchKernelGGL(fcfm_dw_kernel<MODE_BF16>, grid, dim3(256), DW_LDS, s, x, s_b, s_p, gpool,
                       code, B, per, part, dbp);
  else
    return 1002;
  const int n = 9 * COUT * CIN + COUT;
  hipLaunchKernelGGL(fcfm_dw_reduce_kernel, dim3((n + 255) / 256), dim3(256), 0, s, part, dbp,
                     groups, dW, db);
  return (int)hipGetLastError();
}

}  // extern "C"
