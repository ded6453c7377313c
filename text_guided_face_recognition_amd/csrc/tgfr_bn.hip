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

// grid C; 256 threads.  Up to 256 * BN_REG values per channel (B = 64 at
// 14 x 14: 49 per thread) are loaded once into registers; larger maps take the
// two-pass loop (thread t owns positions hw = t, t+256, ... of every sample).
constexpr int BN_REG = 64;
__global__ __launch_bounds__(256) void bn_stats_kernel(
    const float* __restrict__ x, int N, int C, int HW, float eps, float momentum, int training,
    float* __restrict__ running_mean, float* __restrict__ running_var,
    long long* __restrict__ nbt, float* __restrict__ mean_out, float* __restrict__ rstd_out) {
  __shared__ float red[4];
  const int c = blockIdx.x, tid = threadIdx.x, wid = tid / WAVE, lane = tid % WAVE;
  if (!training) {
    if (tid == 0) {
      mean_out[c] = running_mean[c];
      rstd_out[c] = rsqrtf(running_var[c] + eps);
    }
    return;
  }
  const long long cnt = (long long)N * HW;
  const float* xc = x + (long long)c * HW;
  const long long sn = (long long)C * HW;
  float s = 0.f, m2 = 0.f, mean;
  if (cnt <= 256 * BN_REG) {
    // the channel's N x HW values, flattened over all 256 threads, loaded once
    // with every load in flight (one HBM round trip; clamped indices, so no
    // branch -- and no wait -- per load), both moments from registers
    const int last = (int)cnt - 1;
    float v[BN_REG];
#pragma unroll
    for (int u = 0; u < BN_REG; ++u) {
      const int e = min(tid + 256 * u, last), n = e / HW, hw = e - n * HW;
      v[u] = xc[n * sn + hw];
    }
#pragma unroll
    for (int u = 0; u < BN_REG; ++u) s += tid + 256 * u <= last ? v[u] : 0.f;
    s = wave_sum(s);
    if (lane == 0) red[wid] = s;
    __syncthreads();
    mean = (red[0] + red[1] + red[2] + red[3]) / (float)cnt;
    __syncthreads();
#pragma unroll
    for (int u = 0; u < BN_REG; ++u) {
      const float d = tid + 256 * u < cnt ? v[u] - mean : 0.f;
      m2 += d * d;
    }
  } else {
    for (int hw = tid; hw < HW; hw += 256) {
#pragma unroll 8
      for (int n = 0; n < N; ++n) s += xc[n * sn + hw];
    }
    s = wave_sum(s);
    if (lane == 0) red[wid] = s;
    __syncthreads();
    mean = (red[0] + red[1] + red[2] + red[3]) / (float)cnt;
    __syncthreads();
    for (int hw = tid; hw < HW; hw += 256) {
#pragma unroll 8
      for (int n = 0; n < N; ++n) {
        const float d = xc[n * sn + hw] - mean;
        m2 += d * d;
      }
    }
  }
  m2 = wave_sum(m2);
  if (lane == 0) red[wid] = m2;
  __syncthreads();
  if (tid == 0) {
    const float var = (red[0] + red[1] + red[2] + red[3]) / (float)cnt;
    mean_out[c] = mean;
    rstd_out[c] = rsqrtf(var + eps);
    if (running_mean) {
      const float unbiased = cnt > 1 ? var * (float)cnt / (float)(cnt - 1) : var;
      running_mean[c] = (1.f - momentum) * running_mean[c] + momentum * mean;
      running_var[c] = (1.f - momentum) * running_var[c] + momentum * unbiased;
    }
    if (nbt && c == 0) nbt[0] += 1;
  }
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
  if (ry == 0 && c < C) {
    float a = 0.f, b = 0.f;
#pragma unroll 8
    for (int k = 0; k < (int)gridDim.y; ++k) {
      a += part[((long long)k * C + c) * 2];
      b += part[((long long)k * C + c) * 2 + 1];
    }
    dgamma[c] = a;
    dbeta[c] = b;
  }
}

}  // namespace

extern "C" {

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
