// Word<->region contrastive kernels for gfx950 (MI355X).
//
// Replaces the per-caption Python loop of models/losses.py:61-135 (words_loss)
// and the func_attention it calls (models/attention.py:10-43).  For every
// (image b, caption i) pair:
//   S[r,t]  = R_b[r] . W_i[t]                         (attention.py:27)
//   A1      = softmax_t(S)                            (attention.py:29)
//   A2      = softmax_r(gamma1 * A1)                  (attention.py:35-36)
//   C[t]    = sum_r A2[t,r] R_b[r]                    (attention.py:41)
//   cos_t   = W_t.C_t / max(|W_t||C_t|, eps)          (losses.py:12-16)
//   logit   = gamma3 * log sum_t exp(gamma2 cos_t)    (losses.py:107-122)
//
// Layouts (HBM): R images as bf16 hi/lo [B_img][224][256] (regions >= 196
// zero), words as bf16 hi/lo [B_cap][32][256] (tokens >= len zero).  The fp32
// sources are split by tgfr_prep_rows.
//
// Kernels:
//   prep_rows   one wave per row: fp32 (any strides) -> bf16 hi/lo + L2 norm.
//   wr_fwd      workgroup = (image, 4 captions), one wave per pair.  The R
//               image is streamed through LDS in chunks shared by the 4
//               waves: 8 d-chunks for S^T = W R^T, then 7 region chunks for
//               C^T = R^T E^T.  Writes logits, per-token stats and C.
//   wr_bwd      workgroup = (image, 4 region tiles, caption chunk), one wave
//               per 32-region tile, all waves on the same caption.  Per
//               caption it stages X = [W; dC] in LDS and computes
//               [S^T; dA2^T] = X R_tile^T, the two softmax backwards in
//               registers, and dR_tile += [dS | A2] X.  Writes partial slabs.
//   wr_reduce   sums the caption-chunk slabs into dR (caller's strides).
#include "tgfr_common.h"

using namespace tgfr;

namespace {

constexpr int D = 256;         // feature dim (aux_feat_dim_per_granularity)
constexpr int RPAD = 224;      // 196 regions padded to 7 tiles of 32
constexpr int NREG = 196;
constexpr int TPAD = 32;       // words per caption padded to one tile
constexpr int NRT = 7;         // region tiles

// ----------------------------------------------------------------- prep ---
__global__ __launch_bounds__(256) void prep_rows_kernel(
    const float* __restrict__ x, long long s_item, long long s_row, long long s_col,
    int n_items, int n_rows, int rows_pad, const int* __restrict__ lens,
    uint16_t* __restrict__ hi, uint16_t* __restrict__ lo, float* __restrict__ norms) {
  const int wave = (blockIdx.x * 256 + threadIdx.x) / WAVE;
  const int lane = threadIdx.x % WAVE;
  if (wave >= n_items * rows_pad) return;
  const int item = wave / rows_pad, row = wave % rows_pad;
  int valid_rows = n_rows;
  if (lens) valid_rows = min(valid_rows, lens[item]);
  const bool valid = row < valid_rows;
  float v[4];
  float ss = 0.f;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int col = lane * 4 + k;
    v[k] = valid ? x[item * s_item + row * s_row + col * s_col] : 0.f;
    ss += v[k] * v[k];
  }
  uint16_t h[4], l[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) split2(v[k], h[k], l[k]);
  const long long o = ((long long)item * rows_pad + row) * D + lane * 4;
  *(uint2*)(hi + o) = make_uint2(pack2(h[0], h[1]), pack2(h[2], h[3]));
  *(uint2*)(lo + o) = make_uint2(pack2(l[0], l[1]), pack2(l[2], l[3]));
  ss = wave_sum(ss);
  if (lane == 0 && norms) norms[(long long)item * rows_pad + row] = sqrtf(ss);
}

// ------------------------------------------------------------------ fwd ---
// LDS map (bytes)
constexpr int F_G1_STRIDE = 80;                     // 32 d * 2 B + 16 pad
constexpr int F_G1_HALF = RPAD * F_G1_STRIDE;       // 17920
constexpr int F_G2_STRIDE = 576;                    // 256 d * 2 B + 64 pad
constexpr int F_G2_HALF = 32 * F_G2_STRIDE;         // 18432
constexpr int F_STAGE = 2 * F_G2_HALF;              // hi+lo, max of the two
constexpr int F_ET = 2 * 32 * 64;                   // per-wave E^T tile hi+lo
constexpr int F_OFF_ET = 2 * F_STAGE;
constexpr int F_OFF_TOK = F_OFF_ET + 4 * F_ET;      // per-wave Z[32], N[32]
constexpr int F_LDS = F_OFF_TOK + 4 * 64 * 4;
constexpr int F_NCHUNK = 8 + NRT;                   // 8 d-chunks + 7 region chunks
constexpr int F_PIECES = 8;                         // 16-B pieces per thread per chunk

struct StageRegs {
  uint4 v[F_PIECES];
};

// Issue the global loads for stream chunk c of image b into registers.
__device__ __forceinline__ void fwd_load_chunk(StageRegs& s, int c, const uint16_t* Rhi,
                                               const uint16_t* Rlo, long long img_off,
                                               int tid) {
#pragma unroll
  for (int k = 0; k < F_PIECES; ++k) {
    const int p = tid + 256 * k;
    if (c < 8) {
      // d-chunk: 224 rows x 4 pieces, hi then lo (1792 pieces, 7 per thread)
      if (p < 2 * RPAD * 4) {
        const int which = p / (RPAD * 4), q = p % (RPAD * 4);
        const int row = q / 4, seg = q % 4;
        const uint16_t* src = (which ? Rlo : Rhi) + img_off + row * D + c * 32 + seg * 8;
        s.v[k] = *(const uint4*)src;
      }
    } else {
      // region chunk: 32 rows x 32 pieces, hi then lo (2048 pieces)
      const int which = p / 1024, q = p % 1024;
      const int row = q / 32, seg = q % 32;
      const uint16_t* src = (which ? Rlo : Rhi) + img_off + ((c - 8) * 32 + row) * D + seg * 8;
      s.v[k] = *(const uint4*)src;
    }
  }
}

__device__ __forceinline__ void fwd_store_chunk(const StageRegs& s, int c, int buf, int tid) {
  const uint32_t base = buf * F_STAGE;
#pragma unroll
  for (int k = 0; k < F_PIECES; ++k) {
    const int p = tid + 256 * k;
    if (c < 8) {
      if (p < 2 * RPAD * 4) {
        const int which = p / (RPAD * 4), q = p % (RPAD * 4);
        const int row = q / 4, seg = q % 4;
        lds_st16(base + which * F_G1_HALF + row * F_G1_STRIDE + seg * 16, s.v[k]);
      }
    } else {
      const int which = p / 1024, q = p % 1024;
      const int row = q / 32, seg = q % 32;
      lds_st16(base + which * F_G2_HALF + row * F_G2_STRIDE + seg * 16, s.v[k]);
    }
  }
}

template <int MODE>
__global__ __launch_bounds__(256, 1) void wr_fwd_kernel(
    const uint16_t* __restrict__ Rhi, const uint16_t* __restrict__ Rlo,
    const uint16_t* __restrict__ Whi, const uint16_t* __restrict__ Wlo,
    const float* __restrict__ Wnorm, const int* __restrict__ lens, int B_img, int B_cap,
    int img_offset, float g1, float g2, float g3, float eps, float* __restrict__ logits,
    int ld_logits, float4* __restrict__ stats, float* __restrict__ Cout,
    float* __restrict__ att, int att_T) {
  const int groups = (B_cap + 3) / 4;
  const int work = xcd_remap(blockIdx.x, groups * B_img);
  const int b = work / groups;
  const int grp = work % groups;
  const int tid = threadIdx.x, wid = tid / WAVE, lane = tid % WAVE;
  const int lr = lane & 31, h = lane >> 5;
  const int i = grp * 4 + wid;
  const bool active = i < B_cap;
  const int ic = active ? i : B_cap - 1;  // clamp for address math
  const int len = lens[ic];
  const long long img_off = (long long)b * RPAD * D;
  const long long cap_off = (long long)ic * TPAD * D;

  f32x16 S[NRT];
#pragma unroll
  for (int j = 0; j < NRT; ++j)
#pragma unroll
    for (int q = 0; q < 16; ++q) S[j][q] = 0.f;
  f32x16 C[8];
#pragma unroll
  for (int j = 0; j < 8; ++j)
#pragma unroll
    for (int q = 0; q < 16; ++q) C[j][q] = 0.f;
  float E[NRT][16];

  const uint32_t et = F_OFF_ET + wid * F_ET;       // this wave's E^T tile
  const uint32_t tok = F_OFF_TOK + wid * 256;      // this wave's Z[32], N[32]

  // W_i as A-operand fragments for all 16 k-steps: lane (t, h) -> d = 16 s + 8 h
  bf16x8 Wh[16], Wl[16];
#pragma unroll
  for (int s = 0; s < 16; ++s) {
    Wh[s] = as_bf8(*(const uint4*)(Whi + cap_off + lr * D + s * 16 + h * 8));
    Wl[s] = MODE == MODE_SPLIT ? as_bf8(*(const uint4*)(Wlo + cap_off + lr * D + s * 16 + h * 8))
                               : Wh[s];
  }

  StageRegs st;
  fwd_load_chunk(st, 0, Rhi, Rlo, img_off, tid);
  fwd_store_chunk(st, 0, 0, tid);
  __syncthreads();

  // ---- GEMM1 over 8 d-chunks: S^T[t][r] += W[t][d] R[r][d]
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    fwd_load_chunk(st, c + 1, Rhi, Rlo, img_off, tid);
    const uint32_t sb = (c & 1) * F_STAGE;
    if (active) {
#pragma unroll
      for (int s = 0; s < 2; ++s) {
#pragma unroll
        for (int j = 0; j < NRT; ++j) {
          const uint32_t o = sb + (j * 32 + lr) * F_G1_STRIDE + s * 32 + h * 16;
          const bf16x8 bhi = as_bf8(lds_ld16(o));
          const bf16x8 blo = MODE == MODE_SPLIT ? as_bf8(lds_ld16(o + F_G1_HALF)) : bhi;
          mma<MODE>(S[j], Wh[2 * c + s], Wl[2 * c + s], bhi, blo);
        }
      }
    }
    fwd_store_chunk(st, c + 1, (c + 1) & 1, tid);
    __syncthreads();
  }

  // ---- softmax over words per region (registers), E = exp(gamma1 A1),
  //      per-token Z = sum_r E and N = sum_r E S (reduce-scatter over lanes)
  if (active) {
    float zp[16], np[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) zp[q] = np[q] = 0.f;
#pragma unroll
    for (int j = 0; j < NRT; ++j) {
      const bool rvalid = j * 32 + lr < NREG;
      float m = -INFINITY;
#pragma unroll
      for (int q = 0; q < 16; ++q)
        if (acc_row(q, h) < len) m = fmaxf(m, S[j][q]);
      m = fmaxf(m, __shfl_xor(m, 32));
      float p[16], sum = 0.f;
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        p[q] = acc_row(q, h) < len ? __expf(S[j][q] - m) : 0.f;
        sum += p[q];
      }
      sum += __shfl_xor(sum, 32);
      const float inv = 1.f / sum;
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const bool ok = rvalid && acc_row(q, h) < len;
        const float e = ok ? __expf(g1 * (p[q] * inv)) : 0.f;
        E[j][q] = e;
        zp[q] += e;
        np[q] += e * S[j][q];
      }
    }
    const float zr = rs16(zp, lr), nr = rs16(np, lr);
    if ((lr & 1) == 0) {
      const int t = acc_row(rs16_index(lr), h);
      lds_stf(tok + t * 4, zr);
      lds_stf(tok + 128 + t * 4, nr);
    }
  }

  // ---- GEMM2 over 7 region chunks: C^T[d][t] += R[r][d] E[t][r]
  const int g16 = lane >> 4, q4 = (lane & 15) >> 2, p4 = lane & 3;
#pragma unroll
  for (int j = 0; j < NRT; ++j) {
    const int c = 8 + j;
    if (c + 1 < F_NCHUNK) fwd_load_chunk(st, c + 1, Rhi, Rlo, img_off, tid);
    const uint32_t sb = (c & 1) * F_STAGE;
    if (active) {
      // transpose E tile j through this wave's LDS scratch: Et[r][t]
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        uint16_t hh[4], ll[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) split2(E[j][4 * g + k], hh[k], ll[k]);
        const uint32_t o = et + lr * 64 + (8 * g + 4 * h) * 2;
        lds_st8(o, make_uint2(pack2(hh[0], hh[1]), pack2(hh[2], hh[3])));
        if (MODE == MODE_SPLIT)
          lds_st8(o + 2048, make_uint2(pack2(ll[0], ll[1]), pack2(ll[2], ll[3])));
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int rb = 16 * s + 8 * h;
        const uint32_t eo = et + (rb + q4) * 64 + (16 * (g16 & 1) + 4 * p4) * 2;
        const bf16x8 bhi = join_tr(lds_tr4(eo), lds_tr4(eo + 4 * 64));
        const bf16x8 blo = MODE == MODE_SPLIT
                               ? join_tr(lds_tr4(eo + 2048), lds_tr4(eo + 2048 + 4 * 64))
                               : bhi;
#pragma unroll
        for (int dt = 0; dt < 8; ++dt) {
          const uint32_t ro =
              sb + (rb + q4) * F_G2_STRIDE + (dt * 32 + 16 * (g16 & 1) + 4 * p4) * 2;
          const bf16x8 ahi = join_tr(lds_tr4(ro), lds_tr4(ro + 4 * F_G2_STRIDE));
          const bf16x8 alo =
              MODE == MODE_SPLIT
                  ? join_tr(lds_tr4(ro + F_G2_HALF), lds_tr4(ro + F_G2_HALF + 4 * F_G2_STRIDE))
                  : ahi;
          mma<MODE>(C[dt], ahi, alo, bhi, blo);
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    if (c + 1 < F_NCHUNK) fwd_store_chunk(st, c + 1, (c + 1) & 1, tid);
    __syncthreads();
  }

  if (!active) return;
  // ---- per-token epilogue: lane (t = lr, h) holds C^T[d][t] for d rows of half h
  const int t = lr;
  float csq = 0.f;
#pragma unroll
  for (int dt = 0; dt < 8; ++dt)
#pragma unroll
    for (int q = 0; q < 16; ++q) csq += C[dt][q] * C[dt][q];
  csq += __shfl_xor(csq, 32);
  const float Z = lds_ldf(tok + t * 4);
  const float nhat = lds_ldf(tok + 128 + t * 4);
  const bool tvalid = t < len;
  const float zinv = 1.f / Z;
  const float cn = sqrtf(csq) * zinv;
  const float n = nhat * zinv;
  const float u = Wnorm[(long long)ic * TPAD + t];
  const float cosv = n / fmaxf(u * cn, eps);
  float ex = tvalid ? __expf(g2 * cosv) : 0.f;
  ex = half_sum(ex);
  const long long pair = (long long)b * B_cap + i;
  if (lane == 0) logits[(long long)b * ld_logits + i] = g3 * __logf(ex);
  if (stats && h == 0)
    stats[pair * TPAD + t] = tvalid ? make_float4(Z, n, cn, cosv) : make_float4(0.f, 0.f, 0.f, 0.f);
  if (Cout) {
    float* dst = Cout + (pair * TPAD + t) * D;
#pragma unroll
    for (int dt = 0; dt < 8; ++dt)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int d = dt * 32 + 8 * g + 4 * h;
        float4 v = make_float4(C[dt][4 * g] * zinv, C[dt][4 * g + 1] * zinv,
                               C[dt][4 * g + 2] * zinv, C[dt][4 * g + 3] * zinv);
        if (!tvalid) v = make_float4(0.f, 0.f, 0.f, 0.f);
        *(float4*)(dst + d) = v;
      }
  }
  if (att && b + img_offset == i) {
    // attention map of the matching pair: A2[t][r] = E[t][r] / Z_t
    float* dst = att + (long long)b * att_T * NREG;
#pragma unroll
    for (int j = 0; j < NRT; ++j)
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int tt = acc_row(q, h), r = j * 32 + lr;
        if (tt < len && tt < att_T && r < NREG)
          dst[tt * NREG + r] = E[j][q] / lds_ldf(tok + tt * 4);
      }
  }
}

// ------------------------------------------------------------------ bwd ---
// X image: 2 halves x [64 rows][128 cols] bf16, 256-B rows, XOR-swizzled
// 16-B chunks so both the row reads (ds_read_b128) and the transposed reads
// (ds_read_b64_tr_b16) are conflict-free.
__device__ __forceinline__ uint32_t xoff(int row, int col) {
  const int sw = ((row & 3) << 2) | ((row >> 2) & 3);
  return (col >> 7) * (64 * 256) + row * 256 + ((((col & 127) >> 3) ^ sw) << 4) + (col & 7) * 2;
}
constexpr int B_XIMG = 64 * 256 * 2;               // one bf16 image [64][256]
constexpr int B_BUF = 2 * B_XIMG + 3 * 32 * 4;     // hi + lo + Zinv, sigma, spare
constexpr int B_LDS = 2 * B_BUF;

// Per-token backward scalars for pair (b, i), one per lane t < 32 of the wave.
struct TokScal {
  float alpha, beta, sigma, zinv;
};
__device__ __forceinline__ TokScal bwd_tok(const float4* stats, const float* Wnorm,
                                           const float* dlogits, int ld, int b, int i,
                                           int B_cap, int len, float g2, float g3, float eps,
                                           int t) {
  TokScal r{0.f, 0.f, 0.f, 0.f};
  const long long pair = (long long)b * B_cap + i;
  const bool valid = t < len;
  float4 st = valid ? stats[pair * TPAD + t] : make_float4(1.f, 0.f, 0.f, 0.f);
  float ex = valid ? __expf(g2 * st.w) : 0.f;
  const float tot = half_sum(ex);
  if (!valid) return r;
  const float G = dlogits[(long long)b * ld + i] * g3;   // d loss / d log-sum
  const float dcos = G * g2 * ex / tot;
  const float u = Wnorm[(long long)i * TPAD + t];
  const float cn = st.z, n = st.y, cosv = st.w;
  if (u * cn >= eps) {
    r.alpha = dcos / (u * cn);
    r.beta = -dcos * cosv / (cn * cn);
  } else {
    r.alpha = dcos / eps;
    r.beta = 0.f;
  }
  r.sigma = r.alpha * n + r.beta * cn * cn;
  r.zinv = 1.f / st.x;
  return r;
}

// Stage caption i of image b into LDS buffer `buf`: rows 0-31 = W_i, rows
// 32-63 = dC = alpha W + beta C; plus Zinv/sigma per token.
__device__ __forceinline__ void bwd_stage(int buf, const uint16_t* Whi, const uint16_t* Wlo,
                                          const float* Cbuf, const float4* stats,
                                          const float* Wnorm, const int* lens,
                                          const float* dlogits, int ld, int b, int i, int B_cap,
                                          float g2, float g3, float eps, int tid) {
  const uint32_t base = buf * B_BUF;
  const int lane = tid % WAVE;
  const int len = lens[i];
  const TokScal ts = bwd_tok(stats, Wnorm, dlogits, ld, b, i, B_cap, len, g2, g3, eps, lane & 31);
  if (tid < 32) {
    lds_stf(base + 2 * B_XIMG + tid * 4, ts.zinv);
    lds_stf(base + 2 * B_XIMG + 128 + tid * 4, ts.sigma);
  }
  const long long cap_off = (long long)i * TPAD * D;
  const long long pair = (long long)b * B_cap + i;
  // 32 tokens x 32 pieces of 8 d; 4 pieces per thread
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int p = tid + 256 * k;
    const int t = p / 32, seg = p % 32;
    const int col = seg * 8;
    const uint4 wh = *(const uint4*)(Whi + cap_off + t * D + col);
    const uint4 wl = *(const uint4*)(Wlo + cap_off + t * D + col);
    lds_st16(base + xoff(t, col), wh);
    lds_st16(base + B_XIMG + xoff(t, col), wl);
    const float a = __shfl(ts.alpha, t), bb = __shfl(ts.beta, t);
    const float* cp = Cbuf + (pair * TPAD + t) * D + col;
    const float4 c0 = *(const float4*)cp, c1 = *(const float4*)(cp + 4);
    const float cv[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
    const uint32_t* whp = &wh.x;
    const uint32_t* wlp = &wl.x;
    uint32_t oh[4], ol[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      uint16_t h0, l0, h1, l1;
      const float w0 = bf_val(whp[e] & 0xffff) + bf_val(wlp[e] & 0xffff);
      const float w1 = bf_val(whp[e] >> 16) + bf_val(wlp[e] >> 16);
      split2(a * w0 + bb * cv[2 * e], h0, l0);
      split2(a * w1 + bb * cv[2 * e + 1], h1, l1);
      oh[e] = pack2(h0, h1);
      ol[e] = pack2(l0, l1);
    }
    lds_st16(base + xoff(32 + t, col), make_uint4(oh[0], oh[1], oh[2], oh[3]));
    lds_st16(base + B_XIMG + xoff(32 + t, col), make_uint4(ol[0], ol[1], ol[2], ol[3]));
  }
}

template <int MODE>
__global__ __launch_bounds__(256, 1) void wr_bwd_kernel(
    const uint16_t* __restrict__ Rhi, const uint16_t* __restrict__ Rlo,
    const uint16_t* __restrict__ Whi, const uint16_t* __restrict__ Wlo,
    const float* __restrict__ Wnorm, const int* __restrict__ lens, int B_img, int B_cap,
    int n_chunks, float g1, float g2, float g3, float eps, const float* __restrict__ dlogits,
    int ld, const float4* __restrict__ stats, const float* __restrict__ Cbuf,
    float* __restrict__ slab) {
  const int total = n_chunks * 2 * B_img;
  const int work = xcd_remap(blockIdx.x, total);
  const int b = work / (2 * n_chunks);
  const int rem = work % (2 * n_chunks);
  const int tg = rem / n_chunks, chunk = rem % n_chunks;
  const int per = (B_cap + n_chunks - 1) / n_chunks;
  const int c0 = chunk * per, c1 = min(B_cap, c0 + per);
  const int tid = threadIdx.x, wid = tid / WAVE, lane = tid % WAVE;
  const int lr = lane & 31, h = lane >> 5;
  const int rt = tg * 4 + wid;
  const bool active = rt < NRT;
  const int r = rt * 32 + lr;

  // R tile as B-operand fragments: lane (r, h), k-step s -> d = 16 s + 8 h
  bf16x8 Rh[16], Rl[16];
  const long long roff = ((long long)b * RPAD + (active ? r : 0)) * D;
#pragma unroll
  for (int s = 0; s < 16; ++s) {
    Rh[s] = as_bf8(*(const uint4*)(Rhi + roff + s * 16 + h * 8));
    Rl[s] = MODE == MODE_SPLIT ? as_bf8(*(const uint4*)(Rlo + roff + s * 16 + h * 8)) : Rh[s];
  }
  f32x16 dR[8];
#pragma unroll
  for (int j = 0; j < 8; ++j)
#pragma unroll
    for (int q = 0; q < 16; ++q) dR[j][q] = 0.f;

  if (c0 < c1)
    bwd_stage(0, Whi, Wlo, Cbuf, stats, Wnorm, lens, dlogits, ld, b, c0, B_cap, g2, g3, eps, tid);
  __syncthreads();

  const int g16 = lane >> 4, q4 = (lane & 15) >> 2, p4 = lane & 3;
  for (int i = c0; i < c1; ++i) {
    const int buf = (i - c0) & 1;
    const uint32_t base = buf * B_BUF;
    if (active) {
      const int len = lens[i];
      // ---- [S^T ; dA2^T] = [W ; dC] R_tile^T  (M = 64 tokens, N = 32 regions)
      f32x16 A0, A1;
#pragma unroll
      for (int q = 0; q < 16; ++q) A0[q] = A1[q] = 0.f;
#pragma unroll
      for (int s = 0; s < 16; ++s) {
        const int col = s * 16 + h * 8;
        const bf16x8 w_hi = as_bf8(lds_ld16(base + xoff(lr, col)));
        const bf16x8 c_hi = as_bf8(lds_ld16(base + xoff(32 + lr, col)));
        bf16x8 w_lo = w_hi, c_lo = c_hi;
        if (MODE == MODE_SPLIT) {
          w_lo = as_bf8(lds_ld16(base + B_XIMG + xoff(lr, col)));
          c_lo = as_bf8(lds_ld16(base + B_XIMG + xoff(32 + lr, col)));
        }
        mma<MODE>(A0, w_hi, w_lo, Rh[s], Rl[s]);
        mma<MODE>(A1, c_hi, c_lo, Rh[s], Rl[s]);
      }
      // ---- softmax forward recompute + both softmax backwards (registers)
      const bool rvalid = r < NREG;
      float m = -INFINITY;
#pragma unroll
      for (int q = 0; q < 16; ++q)
        if (acc_row(q, h) < len) m = fmaxf(m, A0[q]);
      m = fmaxf(m, __shfl_xor(m, 32));
      float a1[16], sum = 0.f;
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        a1[q] = acc_row(q, h) < len ? __expf(A0[q] - m) : 0.f;
        sum += a1[q];
      }
      sum += __shfl_xor(sum, 32);
      const float inv = 1.f / sum;
      float a2[16], da1[16], rho = 0.f;
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int t = acc_row(q, h);
        a1[q] *= inv;
        const bool ok = rvalid && t < len;
        const float zinv = lds_ldf(base + 2 * B_XIMG + t * 4);
        const float sig = lds_ldf(base + 2 * B_XIMG + 128 + t * 4);
        a2[q] = ok ? __expf(g1 * a1[q]) * zinv : 0.f;
        da1[q] = g1 * a2[q] * (A1[q] - sig);
        rho += a1[q] * da1[q];
      }
      rho += __shfl_xor(rho, 32);
      float ds[16];
#pragma unroll
      for (int q = 0; q < 16; ++q) ds[q] = rvalid ? a1[q] * (da1[q] - rho) : 0.f;
      // ---- A fragments of M = [dS | A2] (accumulator-as-operand, k permuted)
      bf16x8 Mh[4], Ml[4];
      frag8<MODE>(ds, Mh[0], Ml[0]);
      frag8<MODE>(ds + 8, Mh[1], Ml[1]);
      frag8<MODE>(a2, Mh[2], Ml[2]);
      frag8<MODE>(a2 + 8, Mh[3], Ml[3]);
      // ---- dR_tile[r][d] += sum_k M[r][k] X[k][d]
#pragma unroll
      for (int dt = 0; dt < 8; ++dt) {
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {
          const int rb = (ks >> 1) * 32 + (ks & 1) * 16 + 4 * h;
          const int col = dt * 32 + 16 * (g16 & 1) + 4 * p4;
          const uint32_t o0 = base + xoff(rb + q4, col), o1 = base + xoff(rb + 8 + q4, col);
          const bf16x8 xh = join_tr(lds_tr4(o0), lds_tr4(o1));
          const bf16x8 xl = MODE == MODE_SPLIT
                                ? join_tr(lds_tr4(o0 + B_XIMG), lds_tr4(o1 + B_XIMG))
                                : xh;
          mma<MODE>(dR[dt], Mh[ks], Ml[ks], xh, xl);
        }
      }
    }
    if (i + 1 < c1)
      bwd_stage(buf ^ 1, Whi, Wlo, Cbuf, stats, Wnorm, lens, dlogits, ld, b, i + 1, B_cap, g2,
                g3, eps, tid);
    __syncthreads();
  }
  if (!active) return;
  float* dst = slab + (((long long)chunk * B_img + b) * RPAD + rt * 32) * D;
#pragma unroll
  for (int dt = 0; dt < 8; ++dt)
#pragma unroll
    for (int q = 0; q < 16; ++q) dst[acc_row(q, h) * D + dt * 32 + lr] = dR[dt][q];
}

__global__ __launch_bounds__(256) void wr_reduce_kernel(const float* __restrict__ slab,
                                                        int n_chunks, int B_img,
                                                        float* __restrict__ out, long long s_b,
                                                        long long s_r, long long s_d,
                                                        int accumulate) {
  const long long n = (long long)B_img * NREG * D;
  for (long long e = blockIdx.x * 256LL + threadIdx.x; e < n; e += (long long)gridDim.x * 256) {
    const int d = e % D;
    const long long br = e / D;
    const int rr = br % NREG, b = br / NREG;
    float acc = 0.f;
    for (int c = 0; c < n_chunks; ++c) acc += slab[(((long long)c * B_img + b) * RPAD + rr) * D + d];
    float* o = out + b * s_b + rr * s_r + d * s_d;
    *o = accumulate ? *o + acc : acc;
  }
}

}  // namespace

template <typename K>
static void allow_lds(K kernel, int bytes) {
  hipFuncSetAttribute((const void*)kernel, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
}

// ============================================================== C ABI ===
extern "C" {

int tgfr_prep_rows(const float* x, long long s_item, long long s_row, long long s_col,
                   int n_items, int n_rows, int n_cols, int rows_pad, const int* lens,
                   uint16_t* hi, uint16_t* lo, float* norms, void* stream) {
  if (n_cols != D || n_rows > rows_pad || n_items <= 0) return 1001;
  const int waves = n_items * rows_pad;
  hipLaunchKernelGGL(prep_rows_kernel, dim3((waves + 3) / 4), dim3(256), 0,
                     (hipStream_t)stream, x, s_item, s_row, s_col, n_items, n_rows, rows_pad,
                     lens, hi, lo, norms);
  return (int)hipGetLastError();
}

int tgfr_wr_fwd(const uint16_t* Rhi, const uint16_t* Rlo, const uint16_t* Whi,
                const uint16_t* Wlo, const float* Wnorm, const int* lens, int B_img, int B_cap,
                int img_offset, float gamma1, float gamma2, float gamma3, float eps,
                float* logits, int ld_logits, float* stats, float* Cout, float* att,
                int att_T, int mode, void* stream) {
  if (B_img <= 0 || B_cap <= 0 || ld_logits < B_cap) return 1001;
  const int grid = ((B_cap + 3) / 4) * B_img;
  auto* s = (hipStream_t)stream;
  static bool once = [] {
    allow_lds(wr_fwd_kernel<MODE_SPLIT>, F_LDS);
    allow_lds(wr_fwd_kernel<MODE_BF16>, F_LDS);
    return true;
  }();
  (void)once;
  if (mode == MODE_SPLIT)
    hipLaunchKernelGGL(wr_fwd_kernel<MODE_SPLIT>, dim3(grid), dim3(256), F_LDS, s, Rhi, Rlo,
                       Whi, Wlo, Wnorm, lens, B_img, B_cap, img_offset, gamma1, gamma2, gamma3,
                       eps, logits, ld_logits, (float4*)stats, Cout, att, att_T);
  else if (mode == MODE_BF16)
    hipLaunchKernelGGL(wr_fwd_kernel<MODE_BF16>, dim3(grid), dim3(256), F_LDS, s, Rhi, Rlo,
                       Whi, Wlo, Wnorm, lens, B_img, B_cap, img_offset, gamma1, gamma2, gamma3,
                       eps, logits, ld_logits, (float4*)stats, Cout, att, att_T);
  else
    return 1002;
  return (int)hipGetLastError();
}

int tgfr_wr_bwd(const uint16_t* Rhi, const uint16_t* Rlo, const uint16_t* Whi,
                const uint16_t* Wlo, const float* Wnorm, const int* lens, int B_img, int B_cap,
                int n_chunks, float gamma1, float gamma2, float gamma3, float eps,
                const float* dlogits, int ld, const float* stats, const float* Cbuf,
                float* slab, int mode, void* stream) {
  if (B_img <= 0 || B_cap <= 0 || n_chunks <= 0 || n_chunks > B_cap) return 1001;
  const int grid = n_chunks * 2 * B_img;
  auto* s = (hipStream_t)stream;
  static bool once = [] {
    allow_lds(wr_bwd_kernel<MODE_SPLIT>, B_LDS);
    allow_lds(wr_bwd_kernel<MODE_BF16>, B_LDS);
    return true;
  }();
  (void)once;
  if (mode == MODE_SPLIT)
    hipLaunchKernelGGL(wr_bwd_kernel<MODE_SPLIT>, dim3(grid), dim3(256), B_LDS, s, Rhi, Rlo,
                       Whi, Wlo, Wnorm, lens, B_img, B_cap, n_chunks, gamma1, gamma2, gamma3,
                       eps, dlogits, ld, (const float4*)stats, Cbuf, slab);
  else if (mode == MODE_BF16)
    hipLaunchKernelGGL(wr_bwd_kernel<MODE_BF16>, dim3(grid), dim3(256), B_LDS, s, Rhi, Rlo,
                       Whi, Wlo, Wnorm, lens, B_img, B_cap, n_chunks, gamma1, gamma2, gamma3,
                       eps, dlogits, ld, (const float4*)stats, Cbuf, slab);
  else
    return 1002;
  return (int)hipGetLastError();
}

int tgfr_wr_reduce(const float* slab, int n_chunks, int B_img, float* out, long long s_b,
                   long long s_r, long long s_d, int accumulate, void* stream) {
  const long long n = (long long)B_img * NREG * D;
  const int grid = (int)min((n + 255) / 256, 4096LL);
  hipLaunchKernelGGL(wr_reduce_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, slab,
                     n_chunks, B_img, out, s_b, s_r, s_d, accumulate);
  return (int)hipGetLastError();
}

int tgfr_wr_lds_bytes(int which) { return which == 0 ? F_LDS : B_LDS; }

int tgfr_version(void) { return 100; }

}  // extern "C"
