// IMIM's input BatchNorm folded into the packed q/k/v projection that follows
// it (models/models.py:386-404 then models/fusion_nets.py:97-99):
//
//   z  = bn_img(img)                    training: batch statistics over (N, H, W)
//   px = z^T [key; query; value]^T + b  (three 1x1 convs on the same map)
//
// is computed as px = xhat W'^T + b' with xhat = (x - mean) rstd (channels
// last) and W' = W diag(gamma), b' = b + W beta, so the normalised map is never
// transposed back and the affine costs nothing.  The backward needs only
// G = dpx^T xhat (the projection's weight-gradient GEMM) and s = colsum(dpx):
//   dW = G diag(gamma) + s beta^T,  dgamma_c = sum_o W[o,c] G[o,c],
//   dbeta_c = sum_o W[o,c] s_o.
//
//   bn_stats      per channel: two-pass mean / biased var over N x HW, rstd;
//                 running_mean/var update with the unbiased var (momentum), and
//                 num_batches_tracked += 1 (nn.BatchNorm2d training semantics)
//   bn_norm_cl    xhat[n][hw][c] = (x[n][c][hw] - mean_c) rstd_c, an LDS-tiled
//                 NCHW -> channels-last transpose
//   bn_fold       W' = W diag(gamma), b' = b + W beta
//   bn_unfold     dW, dgamma, dbeta from G and s (fixed-order column sums)
#include "tgfr_fold.h"

using namespace tgfr;

namespace {

// grid C; 256 threads (bn_stats_block, tgfr_fold.h)
__global__ __launch_bounds__(256) void bn_stats_kernel(
    const float* __restrict__ x, int N, int C, int HW, float eps, float momentum, int training,
    float* __restrict__ running_mean, float* __restrict__ running_var,
    long long* __restrict__ nbt, float* __restrict__ mean_out, float* __restrict__ rstd_out) {
  __shared__ float red[4];
  bn_stats_block(x, N, C, HW, eps, momentum, training, running_mean, running_var, nbt, mean_out,
                 rstd_out, blockIdx.x, red);
}

// grid (ceil(C / BN_CT), N); 256 threads; LDS [BN_CT][HW + 1] floats.  OBF: y is
// bf16 (the bf16-mode consumers -- the q/k/v projection GEMM and its weight
// gradient -- round their xhat operand to bf16 anyway: same values, half the
// bytes written and read).
constexpr int BN_CT = 64;   // channels per normalise workgroup
template <bool OBF>
__global__ __launch_bounds__(256) void bn_norm_cl_kernel(const float* __restrict__ x, int C,
                                                         int HW, const float* __restrict__ mean,
                                                         const float* __restrict__ rstd,
                                                         void* __restrict__ yv) {
  extern __shared__ float tile[];
  const int c0 = blockIdx.x * BN_CT, n = blockIdx.y, tid = threadIdx.x;
  const int cn = min(BN_CT, C - c0), ld = HW + 1;
  const float* xs = x + ((long long)n * C + c0) * HW;
  // loads in batches of 16 per thread, all in flight before their LDS stores;
  // past the end a thread repeats the last element (clamped index: the same
  // value to the same LDS word), so there is no branch -- and no wait -- per load
  const int last = cn * HW - 1;
  for (int i0 = 0; i0 <= last; i0 += 256 * 16) {
    float v[16];
    int cc[16], hw[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int i = min(i0 + 256 * u + tid, last);
      cc[u] = i / HW;
      hw[u] = i - cc[u] * HW;
      v[u] = xs[i];
    }
    float m[16], r[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      m[u] = mean[c0 + cc[u]];
      r[u] = rstd[c0 + cc[u]];
    }
#pragma unroll
    for (int u = 0; u < 16; ++u) tile[cc[u] * ld + hw[u]] = (v[u] - m[u]) * r[u];
  }
  __syncthreads();
  if constexpr (OBF) {
    // 4 channels per 8-byte store (cn % 4 == 0: C % 4 == 0)
    uint16_t* ys = (uint16_t*)yv + (long long)n * HW * C + c0;
    const int cq = cn / 4;
    for (int i = tid; i < cq * HW; i += 256) {
      const int hw = i / cq, c4 = 4 * (i % cq);
      *(uint2*)(ys + (long long)hw * C + c4) =
          make_uint2(pk_bf16(tile[c4 * ld + hw], tile[(c4 + 1) * ld + hw]),
                     pk_bf16(tile[(c4 + 2) * ld + hw], tile[(c4 + 3) * ld + hw]));
    }
  } else {
    float* ys = (float*)yv + (long long)n * HW * C + c0;
    for (int i = tid; i < cn * HW; i += 256) {
      const int hw = i / cn, cc = i % cn;
      ys[(long long)hw * C + cc] = tile[cc * ld + hw];
    }
  }
}

// BatchNorm2d input gradient from the channels-last gradient of xhat:
//   dx[n][c][hw] = rstd_c (dxh - mean(dxh) - xhat mean(dxh xhat))   (batch stats)
//   dx[n][c][hw] = rstd_c dxh                                        (running stats)
// means over (N, HW) of channel c; grid C, 256 threads, fixed-order sums.
__global__ __launch_bounds__(256) void bn_bwd_cl_kernel(const float* __restrict__ dxh,
                                                        const float* __restrict__ xhat,
                                                        const float* __restrict__ rstd, int N,
                                                        int C, int HW, int training,
                                                        float* __restrict__ dx) {
  __shared__ float red[2][4];
  const int c = blockIdx.x, tid = threadIdx.x, wid = tid / WAVE, lane = tid % WAVE;
  const long long cnt = (long long)N * HW;
  float m1 = 0.f, m2 = 0.f;
  if (training) {
    float s1 = 0.f, s2 = 0.f;
    for (long long e = tid; e < cnt; e += 256) {
      const float g = dxh[e * C + c];
      s1 += g;
      s2 += g * xhat[e * C + c];
    }
    s1 = wave_sum(s1);
    s2 = wave_sum(s2);
    if (lane == 0) {
      red[0][wid] = s1;
      red[1][wid] = s2;
    }
    __syncthreads();
    m1 = (red[0][0] + red[0][1] + red[0][2] + red[0][3]) / (float)cnt;
    m2 = (red[1][0] + red[1][1] + red[1][2] + red[1][3]) / (float)cnt;
  }
  const float r = rstd[c];
  for (long long e = tid; e < cnt; e += 256) {
    const long long n = e / HW, hw = e % HW;
    dx[(n * C + c) * HW + hw] = r * (dxh[e * C + c] - m1 - xhat[e * C + c] * m2);
  }
}

// one wave per output row o (bn_fold_row, tgfr_fold.h)
__global__ __launch_bounds__(256) void bn_fold_kernel(Parts P, int O, int C,
                                                      const float* __restrict__ gamma,
                                                      const float* __restrict__ beta,
                                                      float* __restrict__ Wf,
                                                      float* __restrict__ bf) {
  const int o = blockIdx.x * 4 + threadIdx.x / WAVE;
  if (o < O) bn_fold_row(P, o, C, gamma, beta, Wf, bf, threadIdx.x % WAVE);
}

// grid (ceil(C / 64), ceil(O / 16)); block = 64 columns x 4 row lanes over a
// 16-row chunk (192 workgroups at O = 768: the 64-row chunks of round 2 put 48
// on the chip, latency-bound at 13 us for 0.8 MB).  dW is elementwise; the
// dgamma / dbeta column partials of the chunks are combined by the last chunk
// of each column group (chunk order, loads of 8 chunks in flight).
constexpr int UF_ROWS = 16;
__global__ __launch_bounds__(256) void bn_unfold_kernel(
    const float* __restrict__ G, const float* __restrict__ s, Parts W, int O,
    int C, const float* __restrict__ gamma, const float* __restrict__ beta, float* __restrict__ dW,
    float* __restrict__ part, unsigned* __restrict__ counters, float* __restrict__ dgamma,
    float* __restrict__ dbeta) {
  __shared__ float red[2 * 4 * 64 + 1];
  const int tx = threadIdx.x & 63, ry = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + tx;
  const int o0 = blockIdx.y * UF_ROWS, o1 = min(O, o0 + UF_ROWS);
  float ag = 0.f, ab = 0.f;
  if (c < C) {
    const float g = gamma[c], bt = beta[c];
#pragma unroll 4
    for (int o = o0 + ry; o < o1; o += 4) {
      const long long e = (long long)o * C + c;
      const float gv = G[e], w = W.row(o, C)[c], so = s[o];
      dW[e] = gv * g + so * bt;
      ag += w * gv;
      ab += w * so;
    }
  }
  red[ry * 64 + tx] = ag;
  red[256 + ry * 64 + tx] = ab;
  __syncthreads();
  if (ry == 0 && c < C) {
    float* pp = part + ((long long)blockIdx.y * C + c) * 2;
    pp[0] = red[tx] + red[64 + tx] + red[128 + tx] + red[192 + tx];
    pp[1] = red[256 + tx] + red[320 + tx] + red[384 + tx] + red[448 + tx];
  }
  if (!last_arrival(counters + blockIdx.x, gridDim.y, (int*)&red[512])) return;
  // the chunks' partials: row lane ry sums chunks ry, ry + 4, ... (all its
  // loads in flight), then the four lanes' sums combine in lane order
  float a = 0.f, b = 0.f;
  if (c < C) {
    const int nch = (int)gridDim.y;
#pragma unroll 12
    for (int k = ry; k < nch; k += 4) {
      const float2 v = *(const float2*)(part + ((long long)k * C + c) * 2);
      a += v.x;
      b += v.y;
    }
  }
  red[ry * 64 + tx] = a;
  red[256 + ry * 64 + tx] = b;
  __syncthreads();
  if (ry == 0 && c < C) {
    dgamma[c] = (red[tx] + red[64 + tx]) + (red[128 + tx] + red[192 + tx]);
    dbeta[c] = (red[256 + tx] + red[320 + tx]) + (red[384 + tx] + red[448 + tx]);
  }
}

// ------------------------------------------ BN apply + q/k/v projection ---
// IMIM's bf16-mode front end in ONE launch (models/models.py:394 then
// models/fusion_nets.py:97-109): xhat = (x - mean) rstd read straight from
// the NCHW input map x [N][C = 256][HW] and
//   px[n][hw][o] = bf16(sum_c xhat[n][c][hw] W'[o][c] + b'[o])
// with the BN-folded weights W' (bf16, tgfr_imim_prep) / b', plus the
// channels-last bf16 xhat [N][HW][256] the projection's weight gradient
// reads -- no normalised-map pass (bn_norm_cl) and no staging GEMM ring.
// Workgroup = (sample n, 256-column slice of O), 8 waves: wave = one 32-column
// tile over all 7 of the sample's 32-row tiles (192 workgroups at B = 64, one
// round on the chip; 128-column slices over m-halves took 29.8 against this
// layout's fewer map re-reads, tools/qkv_lab.py); the product is
// formed transposed, px^T = W' xhat^T, so the weights are the MFMA's A
// operand (their k-contiguous rows, loaded per chunk with the map and
// converted to bf16 fragments) and xhat^T the B operand, read from an LDS image
// [32 channels][224 positions] (the input's own layout) by
// ds_read_b64_tr_b16.  K runs in 8 chunks of 32 channels: chunk k + 1's
// global loads are in flight while chunk k is normalised into one of two LDS
// images and multiplied (one barrier per chunk; a third chunk in flight
// measured slower).  The output tile goes out through LDS as 512-byte row
// segments (8-byte column quads straight from the accumulators: 10 us more).  The
// slices of one sample run on one XCD (xcd_remap), so the map is read from
// HBM once and from L2 twice more; slice s writes xhat for the chunks
// k = s (mod O / 256).
constexpr int QKV_MP = 224;              // LDS image pitch (positions), 7 x 32
constexpr int QKV_CK = 32;               // channels per chunk
constexpr int QKV_IMG = QKV_CK * QKV_MP * 2;
constexpr int QKV_MS = 2 * QKV_IMG;     // mean / rstd of the 256 channels (LDS)
constexpr int QKV_OUT = QKV_MS + 2 * 256 * 4;   // the output tile, staged for row stores
constexpr int QKV_OP = 256 * 2 + 16;    // its row pitch (bytes): 16-B aligned, 4 banks apart
constexpr int QKV_LDS = QKV_OUT + QKV_MP * QKV_OP;
constexpr int QKV_LOADS = 4;             // float4 loads per thread per chunk (<= 2048 / 512)
constexpr int QKV_COLS = 256;            // output columns per workgroup (8 waves x 32)
constexpr int QKV_MT = QKV_MP / 32;      // 32-row tiles per sample (7)

__global__ __launch_bounds__(512) void bn_qkv_kernel(
    const float* __restrict__ x, int HW, const float* __restrict__ mean,
    const float* __restrict__ rstd, const uint16_t* __restrict__ Wb, const float* __restrict__ bf,
    int O, uint16_t* __restrict__ px, uint16_t* __restrict__ xhat) {
  constexpr int C = 256, NCH = C / QKV_CK;
  const int n_sl = O / QKV_COLS;
  const int work = xcd_remap(blockIdx.x, gridDim.x);
  const int nb = work / n_sl, sl = work % n_sl;
  const int tid = threadIdx.x, lane = tid % WAVE;
  const int wv = __builtin_amdgcn_readfirstlane(tid / WAVE);
  // wave = one 32-column tile, every 32-row tile of the sample
  constexpr int mt0 = 0;
  const int n_mt = (HW + 31) / 32;
  const int n0 = sl * QKV_COLS + wv * 32;
  const int lr = lane & 31, h = lane >> 5;
  const int q4 = HW / 4;                        // float4 per channel row
  const int items = QKV_CK * q4;                // float4 per chunk
  const float* xs = x + (long long)nb * C * HW;

  // chunk loads: item i -> channel i / q4, positions 4 (i % q4) .. + 3
  // (clamped: a thread past the end repeats the last item)
  // per chunk: the map's float4s and this wave's W' fragments for the
  // chunk's two k steps (bf16, 32 rows x 32 channels: L2-resident, shared by
  // the sample workgroups of the slice), both issued two chunks ahead
  const uint16_t* wr = Wb + (long long)(n0 + lr) * C + 8 * h;
  float4 ld[2][QKV_LOADS];
  uint4 wl[2][2];
  auto issue = [&](int ck, float4 (&dst)[QKV_LOADS], uint4 (&wd)[2]) {
#pragma unroll
    for (int j = 0; j < QKV_LOADS; ++j) {
      const int i = min(tid + 512 * j, items - 1);
      const int c = ck * QKV_CK + i / q4, p = i % q4;
      dst[j] = *(const float4*)(xs + (long long)c * HW + 4 * p);
    }
#pragma unroll
    for (int k = 0; k < 2; ++k) wd[k] = *(const uint4*)(wr + 32 * ck + 16 * k);
  };
  // the channels' statistics into LDS once (a global load per chunk would
  // be the youngest memory op there, and its wait would drain the prefetch)
  // (loaded first, stored after the first chunks' loads are issued, so the
  // wait for them does not hold those back)
  const float mu0 = mean[min(tid, C - 1)], rs0 = rstd[min(tid, C - 1)];
  issue(0, ld[0], wl[0]);
  issue(1, ld[1], wl[1]);
  if (tid < C) {
    lds_stf(QKV_MS + tid * 4, mu0);
    lds_stf(QKV_MS + (C + tid) * 4, rs0);
  }

  float bias[16];
#pragma unroll
  for (int q = 0; q < 16; ++q) bias[q] = bf[n0 + acc_row(q, h)];
  f32x16 acc[QKV_MT];
#pragma unroll
  for (int t = 0; t < QKV_MT; ++t)
#pragma unroll
    for (int q = 0; q < 16; ++q) acc[t][q] = 0.f;
  __syncthreads();                     // the statistics in LDS

  // B fragment (xhat^T: column = position, 8 consecutive channels) of k step
  // ksl (0, 1) of the chunk image at img, m tile mt: two transposing reads
  const int g16 = lane >> 4, qq = (lane & 15) >> 2, pp = lane & 3;
  const uint32_t boff = ((8 * (g16 >> 1) + qq) * QKV_MP + 16 * (g16 & 1) + 4 * pp) * 2;
  auto bfrag = [&](uint32_t img, int ksl, int mt) {
    const uint32_t o = img + boff + (16 * ksl * QKV_MP + 32 * mt) * 2;
    return join_tr(lds_tr4(o), lds_tr4(o + 4 * QKV_MP * 2));
  };

#pragma unroll
  for (int ck = 0; ck < NCH; ++ck) {
    const uint32_t img = (ck & 1) * QKV_IMG;
    // normalise chunk ck into its image (rows = channels, 8-byte writes)
    {
      float4 (&src)[QKV_LOADS] = ld[ck & 1];
#pragma unroll
      for (int j = 0; j < QKV_LOADS; ++j) {
        const int i = min(tid + 512 * j, items - 1);
        const int cl = i / q4, p = i % q4, c = ck * QKV_CK + cl;
        const float mu = lds_ldf(QKV_MS + c * 4), rs = lds_ldf(QKV_MS + (C + c) * 4);
        const float4 v = src[j];
        lds_st8(img + (cl * QKV_MP + 4 * p) * 2,
                make_uint2(pk_bf16((v.x - mu) * rs, (v.y - mu) * rs),
                           pk_bf16((v.z - mu) * rs, (v.w - mu) * rs)));
      }
    }
    const bf16x8 wa0 = as_bf8(wl[ck & 1][0]), wa1 = as_bf8(wl[ck & 1][1]);
    __syncthreads();
    if (ck + 2 < NCH) issue(ck + 2, ld[ck & 1], wl[ck & 1]);
    // per k step: every m tile's B fragment read first, then the MFMAs (the
    // reads' latency overlaps instead of one wait per MFMA)
#pragma unroll
    for (int ksl = 0; ksl < 2; ++ksl) {
      bf16x8 bb[QKV_MT];
#pragma unroll
      for (int t = 0; t < QKV_MT; ++t) bb[t] = bfrag(img, ksl, mt0 + min(t, n_mt - 1));
#pragma unroll
      for (int t = 0; t < QKV_MT; ++t)
        if (t < n_mt) acc[t] = mfma_lp<MODE_BF16>(ksl ? wa1 : wa0, bb[t], acc[t]);
    }
    // this slice's share of the channels-last xhat: positions x 8-channel groups
    if (ck % n_sl == sl) {
      for (int it = tid; it < HW * (QKV_CK / 8); it += 512) {
        const int m = it % HW, cg = it / HW;
        uint32_t w[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const uint16_t a = *(LDS_AS uint16_t*)(lds_base() + img + ((8 * cg + 2 * k) * QKV_MP + m) * 2);
          const uint16_t b = *(LDS_AS uint16_t*)(lds_base() + img + ((8 * cg + 2 * k + 1) * QKV_MP + m) * 2);
          w[k] = pack2(a, b);
        }
        *(uint4*)(xhat + ((long long)nb * HW + m) * C + ck * QKV_CK + 8 * cg) =
            make_uint4(w[0], w[1], w[2], w[3]);
      }
    }
  }
  // epilogue: bf16(acc + b') into the LDS tile [m][256 columns] (a lane's
  // quad = 4 consecutive columns of one position: 8-byte writes), then the
  // tile's rows out as 512-byte row segments (16 B per lane, coalesced)
#pragma unroll
  for (int t = 0; t < QKV_MT; ++t) {
    if (t >= n_mt) continue;
    const uint32_t row = QKV_OUT + ((mt0 + t) * 32 + lr) * QKV_OP + (wv * 32 + 4 * h) * 2;
#pragma unroll
    for (int g = 0; g < 4; ++g)
      lds_st8(row + 16 * g,
              make_uint2(pk_bf16(acc[t][4 * g] + bias[4 * g], acc[t][4 * g + 1] + bias[4 * g + 1]),
                         pk_bf16(acc[t][4 * g + 2] + bias[4 * g + 2],
                                 acc[t][4 * g + 3] + bias[4 * g + 3])));
  }
  __syncthreads();
  uint16_t* dst = px + (long long)nb * HW * O + sl * QKV_COLS;
  for (int it = tid; it < HW * 32; it += 512) {
    const int m = it >> 5, j = it & 31;
    *(uint4*)(dst + (long long)m * O + 8 * j) = lds_ld16(QKV_OUT + m * QKV_OP + 16 * j);
  }
}

// BN batch statistics alone (bn_fwd_cl's first launch)
static int bn_stats_launch(const float* x, int N, int C, int HW, float eps, float momentum,
                           int training, float* running_mean, float* running_var,
                           long long* nbt, float* mean, float* rstd, hipStream_t st) {
  if (N <= 0 || C <= 0 || HW <= 0) return 1001;
  if (!training && (!running_mean || !running_var)) return 1001;
  hipLaunchKernelGGL(bn_stats_kernel, dim3(C), dim3(256), 0, st, x, N, C, HW, eps, momentum,
                     training, running_mean, running_var, nbt, mean, rstd);
  return (int)hipGetLastError();
}

}  // namespace

extern "C" {

int tgfr_bn_stats(const float* x, int N, int C, int HW, float eps, float momentum, int training,
                  float* running_mean, float* running_var, long long* nbt, float* mean,
                  float* rstd, void* stream) {
  return bn_stats_launch(x, N, C, HW, eps, momentum, training, running_mean, running_var, nbt,
                         mean, rstd, (hipStream_t)stream);
}

int tgfr_bn_qkv_bf16(const float* x, int N, int C, int HW, const float* mean, const float* rstd,
                     const uint16_t* Wfb, const float* bf, int O, uint16_t* px, uint16_t* xhat,
                     void* stream) {
  const uint16_t* Wf = Wfb;
  if (!x || !mean || !rstd || !Wf || !bf || !px || !xhat || N <= 0) return 1001;
  if (C != 256 || HW <= 128 || HW > QKV_MP || HW % 4 || O % QKV_COLS || O / QKV_COLS > 8 ||
      QKV_CK * (HW / 4) > 512 * QKV_LOADS)
    return 1001;
  if (((uintptr_t)x & 15) || ((uintptr_t)Wf & 15) || ((uintptr_t)px & 7) || ((uintptr_t)xhat & 15))
    return 1001;
  const dim3 grid(N * (O / QKV_COLS));
  if (const int e = set_max_lds((const void*)bn_qkv_kernel, QKV_LDS)) return e;
  hipLaunchKernelGGL(bn_qkv_kernel, grid, dim3(512), QKV_LDS, (hipStream_t)stream, x, HW, mean,
                     rstd, Wf, bf, O, px, xhat);
  return (int)hipGetLastError();
}


int tgfr_bn_bwd_cl(const float* dxh, const float* xhat, const float* rstd, int N, int C, int HW,
                   int training, float* dx, void* stream) {
  if (!dxh || !xhat || !rstd || !dx || N <= 0 || C <= 0 || HW <= 0) return 1001;
  hipLaunchKernelGGL(bn_bwd_cl_kernel, dim3(C), dim3(256), 0, (hipStream_t)stream, dxh, xhat,
                     rstd, N, C, HW, training, dx);
  return (int)hipGetLastError();
}

static int bn_fwd_cl(const float* x, int N, int C, int HW, float eps, float momentum,
                     int training, float* running_mean, float* running_var, long long* nbt,
                     float* mean, float* rstd, void* xhat, bool obf, hipStream_t st) {
  if (N <= 0 || C <= 0 || HW <= 0 || (BN_CT * (HW + 1) * 4 > 160 * 1024)) return 1001;
  if (!training && (!running_mean || !running_var)) return 1001;
  hipLaunchKernelGGL(bn_stats_kernel, dim3(C), dim3(256), 0, st, x, N, C, HW, eps, momentum,
                     training, running_mean, running_var, nbt, mean, rstd);
  const int lds = BN_CT * (HW + 1) * 4;
  const void* fn = obf ? (const void*)bn_norm_cl_kernel<true> : (const void*)bn_norm_cl_kernel<false>;
  if (lds > 64 * 1024)
    if (const int e = set_max_lds(fn, lds)) return e;
  if (obf)
    hipLaunchKernelGGL(bn_norm_cl_kernel<true>, dim3((C + BN_CT - 1) / BN_CT, N), dim3(256), lds, st, x, C,
                       HW, mean, rstd, xhat);
  else
    hipLaunchKernelGGL(bn_norm_cl_kernel<false>, dim3((C + BN_CT - 1) / BN_CT, N), dim3(256), lds, st, x,
                       C, HW, mean, rstd, xhat);
  return (int)hipGetLastError();
}

int tgfr_bn_fwd_cl(const float* x, int N, int C, int HW, float eps, float momentum,
                   int training, float* running_mean, float* running_var, long long* nbt,
                   float* mean, float* rstd, float* xhat, void* stream) {
  return bn_fwd_cl(x, N, C, HW, eps, momentum, training, running_mean, running_var, nbt, mean,
                   rstd, xhat, false, (hipStream_t)stream);
}

int tgfr_bn_fwd_cl_bf16(const float* x, int N, int C, int HW, float eps, float momentum,
                        int training, float* running_mean, float* running_var, long long* nbt,
                        float* mean, float* rstd, uint16_t* xhat, void* stream) {
  if (C % 4 || ((uintptr_t)xhat & 7)) return 1001;
  return bn_fwd_cl(x, N, C, HW, eps, momentum, training, running_mean, running_var, nbt, mean,
                   rstd, xhat, true, (hipStream_t)stream);
}

int tgfr_bn_fold(const float* W, const float* b, int O, int C, const float* gamma,
                 const float* beta, float* Wf, float* bf, void* stream) {
  if (O <= 0 || C <= 0) return 1001;
  hipLaunchKernelGGL(bn_fold_kernel, dim3((O + 3) / 4), dim3(256), 0, (hipStream_t)stream,
                     Parts{W, W, W, b, b, b, O}, O, C, gamma, beta, Wf, bf);
  return (int)hipGetLastError();
}

int tgfr_bn_fold3(const float* const* W, const float* const* b, int rows, int C,
                  const float* gamma, const float* beta, float* Wf, float* bf, void* stream) {
  if (!W || rows <= 0 || C <= 0 || !W[0] || !W[1] || !W[2]) return 1001;
  const Parts P{W[0], W[1], W[2], b ? b[0] : nullptr, b ? b[1] : nullptr, b ? b[2] : nullptr,
                rows};
  hipLaunchKernelGGL(bn_fold_kernel, dim3((3 * rows + 3) / 4), dim3(256), 0, (hipStream_t)stream,
                     P, 3 * rows, C, gamma, beta, Wf, bf);
  return (int)hipGetLastError();
}

// ws: 2 * ceil(O / 16) * C floats; counters: ceil(C / 64) zeroed words.
static int bn_unfold_launch(const float* G, const float* s, const Parts& W, int O, int C,
                            const float* gamma, const float* beta, float* dW, float* dgamma,
                            float* dbeta, float* ws, unsigned* counters, void* stream) {
  if (O <= 0 || C <= 0 || !ws || !counters) return 1001;
  hipLaunchKernelGGL(bn_unfold_kernel, dim3((C + 63) / 64, (O + UF_ROWS - 1) / UF_ROWS),
                     dim3(256), 0, (hipStream_t)stream, G, s, W, O, C, gamma, beta, dW, ws,
                     counters, dgamma, dbeta);
  return (int)hipGetLastError();
}

int tgfr_bn_unfold(const float* G, const float* s, const float* W, int O, int C,
                   const float* gamma, const float* beta, float* dW, float* dgamma, float* dbeta,
                   float* ws, unsigned* counters, void* stream) {
  return bn_unfold_launch(G, s, Parts{W, W, W, nullptr, nullptr, nullptr, O}, O, C, gamma,
                          beta, dW, dgamma, dbeta, ws, counters, stream);
}

int tgfr_bn_unfold3(const float* G, const float* s, const float* const* W, int rows, int C,
                    const float* gamma, const float* beta, float* dW, float* dgamma,
                    float* dbeta, float* ws, unsigned* counters, void* stream) {
  if (!W || !W[0] || !W[1] || !W[2]) return 1001;
  return bn_unfold_launch(G, s, Parts{W[0], W[1], W[2], nullptr, nullptr, nullptr, rows},
                          3 * rows, C, gamma, beta, dW, dgamma, dbeta, ws, counters, stream);
}

}  // extern "C"
