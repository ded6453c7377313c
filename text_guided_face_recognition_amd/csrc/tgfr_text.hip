// TextHeading / Bert_Word_Mapping forward (models/models.py:170-232): the
// producer of the words W and sentence codes the contrastive losses consume.
// The reference runs it under no_grad (utils/dataset_utils.py:42-45) as three
// Conv2d(1, 256, (K, 768)) over the BERT hidden states, ReLU, then a Python
// double loop over captions and tokens (:203-209) taking the per-token max of
// the three maps, L2-normalising, and for the sentence the mean over K of the
// per-map max over tokens (:215-220).
//
// Here that is two launches for the whole batch:
//   text_conv  all three convs at once, over ALL captions' tokens as one
//     flattened [B*L1, 768] matrix X:
//       Y_K[m, c] = relu(b_K[c] + sum_{r<K, e} X[m + r, e] W_K[c, r, e])
//     i.e. nine "taps" (K, r), each a [rows, 768] x [768, 256] product of X
//     shifted by r rows.  A block owns a 64-row x 32-channel tile: per 32-wide
//     slice of e it stages X rows m0 .. m0+66 (the 3 halo rows give every
//     shift) and the nine taps' 32 x 32 weight slices in LDS as bf16 (hi/lo
//     pairs in the fp32 mode), then each wave runs 9 MFMAs per 16-wide k step
//     into three accumulators -- the im2col is an LDS row offset, nothing is
//     re-read from HBM per tap.  The slices stream through a multi-stage LDS
//     ring filled by global -> LDS DMA (no staging registers), ~140 KB in
//     flight per CU, because the kernel is bound by L2 latency x bytes in
//     flight, not by its 28 MFLOP per block.  Rows whose window straddles two captions (the
//     last K-1 of each) are computed and never read.  Bias and ReLU in the
//     epilogue.  The weights are packed once into tap-major bf16 planes
//     (text_pack; the caller caches them -- TextHeading gets no gradient, so
//     they only change when the caller loads new ones).  A block is 2 waves on
//     a 64-row x 32-channel tile (>= 1 block per CU at config 2); blocks are
//     ordered so each XCD serves one 32-channel tap slice from its L2.
//   text_pool  one block per caption: per token the max over the maps that
//     cover it, row L2-normalisation (words, [B, T, 256] with T = L1 - 1),
//     and per channel the max over tokens of each map -> mean over K -> L2
//     normalised (sent, [B, 256]).
#include "tgfr_common.h"

using namespace tgfr;

namespace {

constexpr int TH_D = 256;    // aux_feat_dim_per_granularity (cfg/train_bert.yml:28)
constexpr int TH_E = 768;    // BERT hidden size (models/models.py:177)
constexpr int TH_NW = 16;    // waves per caption block (<= 2 tokens each at T = 30)

__device__ __forceinline__ float4 max4(float4 a, float4 b) {
  return make_float4(fmaxf(a.x, b.x), fmaxf(a.y, b.y), fmaxf(a.z, b.z), fmaxf(a.w, b.w));
}
__device__ __forceinline__ float dot4(float4 a) {
  return a.x * a.x + a.y * a.y + a.z * a.z + a.w * a.w;
}
__device__ __forceinline__ float4 div4(float4 a, float d) {
  return make_float4(a.x / d, a.y / d, a.z / d, a.w / d);
}

// Y: [3][B*L1][256] (maps of K = 2, 3, 4, rows of caption b start at b*L1).
// Wave w of caption b handles tokens t = w, w + 16, ...; lane l owns channels
// 4l .. 4l+3, so every row access is one coalesced 1 KB float4 sweep.
__global__ __launch_bounds__(64 * TH_NW) void text_pool_kernel(
    const float* __restrict__ Y, long long map_stride, int L1, float* __restrict__ words,
    long long s_wb, long long s_wt, float* __restrict__ sent, long long s_sb,
    uint16_t* __restrict__ Wrows, float* __restrict__ Wnorm, int t_pad, float scale,
    int rows_f16) {
  __shared__ float4 part[TH_NW][3][64];
  const int b = blockIdx.x, w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const int T = L1 - 1;                               // words per caption (L - 2)
  const float* y2 = Y + (long long)b * L1 * TH_D + 4 * l;
  const float* y3 = y2 + map_stride;
  const float* y4 = y3 + map_stride;
  // ReLU outputs are >= 0 and every map has >= 1 row, so 0 is the max's identity
  float4 m2 = make_float4(0.f, 0.f, 0.f, 0.f), m3 = m2, m4 = m2;
  for (int t = w; t < T; t += TH_NW) {
    float4 v = *(const float4*)(y2 + (long long)t * TH_D);
    m2 = max4(m2, v);
    if (t < T - 1) {                                  // K=3 covers t < L1 - 2
      const float4 v3 = *(const float4*)(y3 + (long long)t * TH_D);
      m3 = max4(m3, v3);
      v = max4(v, v3);
    }
    if (t < T - 2) {                                  // K=4 covers t < L1 - 3
      const float4 v4 = *(const float4*)(y4 + (long long)t * TH_D);
      m4 = max4(m4, v4);
      v = max4(v, v4);
    }
    // F.normalize(p=2, dim=2): x / max(|x|, 1e-12)   (models.py:212)
    const float nraw = sqrtf(wave_sum(dot4(v)));
    const float n = fmaxf(nraw, 1e-12f);
    float* dst = words + b * s_wb + t * s_wt + 4 * l;
    float4 u = div4(v, n);
    // pinned: the operand rows below are formed from exactly the stored words
    // (bit-equal to tgfr_prep_rows of them)
    asm volatile("" : "+v"(u.x), "+v"(u.y), "+v"(u.z), "+v"(u.w));
    *(float4*)dst = u;
    if (Wrows) {
      // the word<->region kernels' operand row: scale * u in bf16 (fp16), and |u|
      float a[4] = {scale * u.x, scale * u.y, scale * u.z, scale * u.w};
      // (pinned fp32 products: the fp16 conversion must not fuse with the
      // multiply into a singly-rounded mixed FMA -- tgfr_prep_rows rounds
      // twice, and the rows must be bit-equal to its)
      asm volatile("" : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]));
      uint16_t h[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) h[k] = rows_f16 ? f16_bits(a[k]) : bf_bits(a[k]);
      *(uint2*)(Wrows + ((long long)b * t_pad + t) * TH_D + 4 * l) =
          make_uint2(pack2(h[0], h[1]), pack2(h[2], h[3]));
      if (l == 0) Wnorm[(long long)b * t_pad + t] = nraw / n;
    }
  }
  if (Wrows)                                          // padding words: zero rows
    for (int t = T + w; t < t_pad; t += TH_NW) {
      *(uint2*)(Wrows + ((long long)b * t_pad + t) * TH_D + 4 * l) = make_uint2(0, 0);
      if (l == 0) Wnorm[(long long)b * t_pad + t] = 0.f;
    }
  part[w][0][l] = m2;
  part[w][1][l] = m3;
  part[w][2][l] = m4;
  __syncthreads();
  if (w == 0) {
    float4 a = part[0][0][l], c = part[0][1][l], d = part[0][2][l];
#pragma unroll
    for (int i = 1; i < TH_NW; ++i) {
      a = max4(a, part[i][0][l]);
      c = max4(c, part[i][1][l]);
      d = max4(d, part[i][2][l]);
    }
    // torch.stack((x0, x1, x2)).mean(dim=0)  (models.py:218)
    float4 s = make_float4((a.x + c.x + d.x) / 3.f, (a.y + c.y + d.y) / 3.f,
                           (a.z + c.z + d.z) / 3.f, (a.w + c.w + d.w) / 3.f);
    const float n = fmaxf(sqrtf(wave_sum(dot4(s))), 1e-12f);
    *(float4*)(sent + b * s_sb + 4 * l) = div4(s, n);
  }
}

constexpr int TC_TM = 64, TC_TN = 32, TC_NT = 512;   // 8 waves (see the kernel)
constexpr int TC_BK = 32;                             // e per ring stage
// Stage images, filled by global -> LDS DMA (1 KB per wave instruction):
//   X  fp32 [X_ROWS][32] (rows m0 .. m0+66 used: 3 halo rows), 128-B rows,
//      16-B chunk q of row r at slot q ^ ((r >> 1) & 7); converted to bf16
//      (hi/lo) at fragment read
//   W  bf16 [9 taps x 32 channels][32] per plane (hi, + lo in the fp32 mode),
//      64-B rows, chunk c of row r at slot c ^ ((r >> 2) & 3)
// Both swizzles make the 16 rows one ds_read_b128 phase touches hit distinct
// bank windows.  X_ROWS pads the piece count to a multiple of the 4 loader
// waves (rows past m0+66 are never read).
constexpr int TC_W_PIECES = 9 * TC_TN * TC_BK * 2 / 1024;        // 18 per plane
constexpr int TC_W_BYTES = TC_W_PIECES * 1024;
constexpr int TC_LOADERS = 4;
template <int MODE> struct TcCfg {
  static constexpr int PLANES = MODE == MODE_SPLIT ? 2 : 1;
  static constexpr int X_PIECES = MODE == MODE_SPLIT ? 12 : 10;  // 96 / 80 rows
  static constexpr int X_BYTES = X_PIECES * 1024;
  static constexpr int PIECES = X_PIECES + PLANES * TC_W_PIECES;
  static constexpr int STG = X_BYTES + PLANES * TC_W_BYTES;
  static constexpr int NS = MODE == MODE_SPLIT ? 3 : 5;          // ~140 KB of ring
  static constexpr int PER = PIECES / TC_LOADERS;                // DMA ops / loader wave / stage
  static constexpr int LDS = NS * STG;
  static_assert(PIECES % TC_LOADERS == 0, "pieces must split evenly over the loader waves");
  static_assert(X_PIECES * 8 >= TC_TM + 3, "X image must hold the halo rows");
};
__device__ __attribute__((aligned(16))) float text_zero16[4] = {0.f, 0.f, 0.f, 0.f};
constexpr long long TC_PLANE = 9ll * TH_D * TH_E;            // packed taps, one bf16 plane

__host__ __device__ constexpr int tap_conv(int p) { return p < 2 ? 0 : p < 5 ? 1 : 2; }
__host__ __device__ constexpr int tap_shift(int p) { return p < 2 ? p : p < 5 ? p - 2 : p - 5; }

// conv weights [256][K*768] (K = 2, 3, 4) -> taps [9][256][768] bf16 (hi plane,
// then the lo plane in the fp32 mode): tap p = (K, r) is W_K[:, r, :].
__global__ __launch_bounds__(256) void text_pack_kernel(const float* __restrict__ w2,
                                                        const float* __restrict__ w3,
                                                        const float* __restrict__ w4,
                                                        uint16_t* __restrict__ out, int split) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;     // float4 index
  if (i >= TC_PLANE / 4) return;
  const int e4 = (int)(i % (TH_E / 4)), c = (int)((i / (TH_E / 4)) % TH_D), p = (int)(i / (TH_E / 4 * TH_D));
  const int k = tap_conv(p), r = tap_shift(p);
  const float* w = k == 0 ? w2 : k == 1 ? w3 : w4;
  const float4 v = *(const float4*)(w + (long long)c * ((k + 2) * TH_E) + r * TH_E + 4 * e4);
  // destination: the (channel tile, e stage) block of 288 rows x 32 e, rows
  // tap * 32 + channel, 16-B chunks pre-swizzled into their LDS slots, so the
  // kernel's stage fill is one contiguous 18 KB copy
  const int row = p * TC_TN + (c & (TC_TN - 1)), e = 4 * e4, ee = e % TC_BK;
  const int slot = (ee / 8) ^ ((row >> 2) & 3);
  const long long o = ((long long)((c / TC_TN) * (TH_E / TC_BK) + e / TC_BK) * (9 * TC_TN) + row) *
                          TC_BK + slot * 8 + ee % 8;
  uint16_t h[4], l[4];
  split2(v.x, h[0], l[0]);
  split2(v.y, h[1], l[1]);
  split2(v.z, h[2], l[2]);
  split2(v.w, h[3], l[3]);
  *(uint2*)(out + o) = make_uint2(pack2(h[0], h[1]), pack2(h[2], h[3]));
  if (split) *(uint2*)(out + TC_PLANE + o) = make_uint2(pack2(l[0], l[1]), pack2(l[2], l[3]));
}

// One launch for the three convs; grid = 8 channel tiles x ceil(rows / 64).
// The block's 64 x 32 output tile is shared by 8 waves so that two waves per
// SIMD hide each other's LDS latency (one wave per SIMD left the chains of
// LDS read -> convert -> MFMA exposed):
//   wave w: wm = w & 1   rows wm*32 .. +31
//           ks = (w >> 1) & 1   k step (16 of the stage's 32 e)
//           tg = w >> 2   tap group: 0 = convs K=2,3 (taps 0-4), 1 = K=4 (5-8)
// Waves 0-3 also issue the stage DMA.  The two k-step halves are summed
// through LDS after the loop (fixed order).
template <int MODE>
__global__ __launch_bounds__(TC_NT) void text_conv_kernel(
    const float* __restrict__ X, int rows, const uint16_t* __restrict__ taps,
    const float* __restrict__ b2, const float* __restrict__ b3, const float* __restrict__ b4,
    float* __restrict__ Y, long long map_stride) {
  using G = TcCfg<MODE>;
  constexpr int NS = G::NS, STG = G::STG, PER = G::PER, XP = G::X_PIECES;
  const int mt_n = gridDim.y;
  const int wid_ = xcd_remap(blockIdx.y * gridDim.x + blockIdx.x, gridDim.x * mt_n);
  // channel-tile major: the 8 channel tiles <-> the 8 XCDs (consecutive work
  // indices share an XCD), so an XCD's taps are one channel tile's 442 KB,
  // resident in its 4 MB L2 for all the row tiles, and only X (6.5 MB, one
  // read per XCD, MALL-resident) streams.  Alone the two mappings time the
  // same (30.2 / 30.6 us); beside the main stream's kernels, whose data
  // shares the L2, row-tile major (every XCD cycling all 3.5 MB of taps)
  // made the step 0.414-0.419 ms against 0.408-0.413 (gpurun_out/r6aa).
  const int tn = wid_ / mt_n;
  const int tm = wid_ % mt_n;
  const int m0 = tm * TC_TM, n0 = tn * TC_TN;
  const int tid = threadIdx.x, wid = tid >> 6, lane = tid & 63, li = lane & 31, lh = lane >> 5;
  const int wm = wid & 1, ks = (wid >> 1) & 1, tg = wid >> 2;
  const bool loader = wid < TC_LOADERS;

  // per-lane DMA sources of this loader wave's pieces (fixed but for e0):
  // piece p < XP is X rows 8p .. 8p+7, then the weight planes' pieces
  const char* src[PER];
  uint32_t dst[PER];
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const int pc = (wid & (TC_LOADERS - 1)) + TC_LOADERS * j;
    if (pc < XP) {
      const int row = 8 * pc + (lane >> 3), q = (lane & 7) ^ ((row >> 1) & 7);
      src[j] = m0 + row < rows ? (const char*)(X + (long long)(m0 + row) * TH_E + 4 * q)
                               : nullptr;
      dst[j] = pc * 1024;
    } else {
      // the packed stage block is already in LDS order (text_pack_kernel)
      const int h = (pc - XP) / TC_W_PIECES, wp = (pc - XP) % TC_W_PIECES;
      src[j] = (const char*)(taps + h * TC_PLANE + (long long)tn * (TH_E / TC_BK) * (9 * TC_TN * TC_BK) +
                             wp * 512 + lane * 8);
      dst[j] = G::X_BYTES + h * TC_W_BYTES + wp * 1024;
    }
  }
  auto issue = [&](int kt) {
    const uint32_t o = (kt % NS) * STG;
    const int e0 = kt * TC_BK;
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int pc = (wid & (TC_LOADERS - 1)) + TC_LOADERS * j;
      const int eb = pc < XP ? e0 * 4 : kt * (9 * TC_TN * TC_BK * 2);   // X columns / tap stage
      glds16(src[j] ? (const void*)(src[j] + eb) : (const void*)text_zero16, o + dst[j]);
    }
  };

  f32x16 acc[2];
#pragma unroll
  for (int k = 0; k < 2; ++k)
#pragma unroll
    for (int q = 0; q < 16; ++q) acc[k][q] = 0.f;

  constexpr int nk = TH_E / TC_BK;
  if (loader) {
#pragma unroll
    for (int st = 0; st < NS - 1; ++st) issue(st);
  }
  for (int kt = 0; kt < nk; ++kt) {
    // a loader's pieces of stage kt have landed once at most NS-2 younger
    // stages are outstanding (the other waves have none); the barrier
    // publishes every piece and retires the reads of stage kt-1, whose slot
    // is refilled next
    if (kt + NS - 2 < nk) ring_barrier<(NS - 2) * PER>();
    else ring_barrier<0>();
    if (loader && kt + NS - 1 < nk) issue(kt + NS - 1);
    const uint32_t o = (kt % NS) * STG;
    bf16x8 ah[4], al[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      if (r == 3 && tg == 0) break;                           // K <= 3: shifts 0-2
      const int row = wm * 32 + li + r, q = 4 * ks + 2 * lh;
      const float4 x0 = __builtin_bit_cast(
          float4, lds_ld16(o + row * 128 + ((q ^ ((row >> 1) & 7)) << 4)));
      const float4 x1 = __builtin_bit_cast(
          float4, lds_ld16(o + row * 128 + (((q + 1) ^ ((row >> 1) & 7)) << 4)));
      const float v[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
      frag8<MODE>(v, ah[r], al[r]);
    }
    auto tap = [&](int p, f32x16& a) {
      const int row = p * TC_TN + li, c = 2 * ks + lh;
      const uint32_t w = o + G::X_BYTES + row * 64 + ((c ^ ((row >> 2) & 3)) << 4);
      const bf16x8 bh = as_bf8(lds_ld16(w));
      const bf16x8 bl = MODE == MODE_SPLIT ? as_bf8(lds_ld16(w + TC_W_BYTES)) : bh;
      mma<MODE>(a, ah[tap_shift(p)], al[tap_shift(p)], bh, bl);
    };
    if (tg == 0) {
#pragma unroll
      for (int p = 0; p < 5; ++p) tap(p, acc[p < 2 ? 0 : 1]);
    } else {
#pragma unroll
      for (int p = 5; p < 9; ++p) tap(p, acc[0]);
    }
  }
  // sum the two k-step halves: ks = 1 waves park their accumulators in LDS
  __syncthreads();
  constexpr int RED = 64 * 16 * 4;                            // one f32x16 per lane
  const uint32_t slot = ((tg * 2 + wm) * 2) * RED + lane * 64;
  if (ks == 1) {
#pragma unroll
    for (int a = 0; a < 2; ++a) {
      if (a == 1 && tg == 1) break;
#pragma unroll
      for (int q = 0; q < 16; q += 4)
        lds_st16(slot + a * RED + q * 4,
                 __builtin_bit_cast(uint4, make_float4(acc[a][q], acc[a][q + 1],
                                                       acc[a][q + 2], acc[a][q + 3])));
    }
  }
  __syncthreads();
  if (ks == 1) return;
  const float* bk[3] = {b2, b3, b4};
  const int col = n0 + li;
#pragma unroll
  for (int a = 0; a < 2; ++a) {
    if (a == 1 && tg == 1) break;
    const int k = tg == 0 ? a : 2;
    const float bias = bk[k][col];
    float* yk = Y + k * map_stride + col;
#pragma unroll
    for (int q = 0; q < 16; q += 4) {
      const float4 o4 = __builtin_bit_cast(float4, lds_ld16(slot + a * RED + q * 4));
      const float part[4] = {o4.x, o4.y, o4.z, o4.w};
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int m = m0 + wm * 32 + acc_row(q + u, lh);
        if (m < rows) yk[(long long)m * TH_D] = fmaxf(acc[a][q + u] + part[u] + bias, 0.f);
      }
    }
  }
}

}  // namespace

extern "C" {

int tgfr_text_pack_bytes(int mode, long long* bytes) {
  if (!bytes) return 1001;
  if (mode != MODE_SPLIT && mode != MODE_BF16) return 1002;
  *bytes = (mode == MODE_SPLIT ? 2 : 1) * TC_PLANE * 2;
  return 0;
}

int tgfr_text_pack(const float* const* conv_w, uint16_t* taps, int mode, void* stream) {
  if (!conv_w || !taps || ((uintptr_t)taps & 15)) return 1001;
  for (int k = 0; k < 3; ++k)
    if (!conv_w[k] || ((uintptr_t)conv_w[k] & 15)) return 1001;
  if (mode != MODE_SPLIT && mode != MODE_BF16) return 1002;
  const int blocks = (int)((TC_PLANE / 4 + 255) / 256);
  hipLaunchKernelGGL(text_pack_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream,
                     conv_w[0], conv_w[1], conv_w[2], taps, mode == MODE_SPLIT);
  return (int)hipGetLastError();
}

int tgfr_text_heading_ws(int B, int L1, long long* floats) {
  if (B <= 0 || L1 < 4 || !floats) return 1001;
  *floats = 3ll * B * L1 * TH_D;
  return 0;
}

int tgfr_text_heading(const float* X, int B, int L1, const uint16_t* taps,
                      const float* const* conv_b, float* ws, float* words, long long s_wb,
                      long long s_wt, float* sent, long long s_sb, uint16_t* Wrows, float* Wnorm,
                      int t_pad, float scale, int rows_f16, int mode, void* stream) {
  if (!X || !taps || !conv_b || !ws || !words || !sent || B <= 0 || L1 < 4) return 1001;
  if (Wrows && (!Wnorm || t_pad < L1 - 1 || ((uintptr_t)Wrows & 7))) return 1001;
  for (int k = 0; k < 3; ++k)
    if (!conv_b[k]) return 1001;
  if (((uintptr_t)X & 15) || ((uintptr_t)taps & 15)) return 1001;
  if (s_wt < TH_D || s_wb < (long long)(L1 - 1) * s_wt || s_sb < TH_D) return 1001;
  if ((s_wb | s_wt | s_sb) & 3) return 1001;
  if (mode != MODE_SPLIT && mode != MODE_BF16) return 1002;
  const long long rows = (long long)B * L1;
  if (rows * TH_E >= (1ll << 31)) return 1001;
  const long long map = rows * TH_D;
  auto* s = (hipStream_t)stream;
  const dim3 grid(TH_D / TC_TN, (unsigned)((rows + TC_TM - 1) / TC_TM));
  if (mode == MODE_SPLIT) {
    if (const int e = set_max_lds((const void*)&text_conv_kernel<MODE_SPLIT>,
                                  TcCfg<MODE_SPLIT>::LDS))
      return e;
  } else if (const int e = set_max_lds((const void*)&text_conv_kernel<MODE_BF16>,
                                       TcCfg<MODE_BF16>::LDS)) {
    return e;
  }
  if (mode == MODE_SPLIT) {
    hipLaunchKernelGGL(text_conv_kernel<MODE_SPLIT>, grid, dim3(TC_NT),
                       TcCfg<MODE_SPLIT>::LDS, s, X, (int)rows, taps, conv_b[0], conv_b[1],
                       conv_b[2], ws, map);
  } else {
    hipLaunchKernelGGL(text_conv_kernel<MODE_BF16>, grid, dim3(TC_NT),
                       TcCfg<MODE_BF16>::LDS, s, X, (int)rows, taps, conv_b[0], conv_b[1],
                       conv_b[2], ws, map);
  }
  hipLaunchKernelGGL(text_pool_kernel, dim3(B), dim3(64 * TH_NW), 0, s, ws, map, L1, words,
                     s_wb, s_wt, sent, s_sb, Wrows, Wnorm, t_pad, scale, rows_f16 ? 1 : 0);
  return (int)hipGetLastError();
}

}  // extern "C"
