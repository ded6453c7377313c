// BatchNorm folded into the 1x1 projection that follows it (W' = W diag(gamma),
// b' = b + W beta), shared by the BN kernels (tgfr_bn.hip) and the IMIM weight
// preparation launch (tgfr_imim_pack, tgfr_tail.hip).
#pragma once
#include "tgfr_common.h"

namespace {

using namespace tgfr;

// A weight [O][C] given as up to 3 row blocks of `rows` rows each (the
// three 1x1 projections of a self-attention, read in place: no concatenated
// copy), and their biases (each nullable).
// (three named pointers picked behind an empty asm: a select between them
// had been folded into a dynamic index into the kernel argument, which put a
// copy of the struct in scratch)
struct Parts {
  const float *w0, *w1, *w2;
  const float *b0, *b1, *b2;
  int rows;
  // (the pointers pass through an empty asm, so the compiler cannot turn the
  // select back into an index into the argument block)
  static __device__ __forceinline__ const float* pick(const float* a, const float* b,
                                                      const float* c, int p) {
    asm("" : "+v"(a), "+v"(b), "+v"(c));
    return p == 0 ? a : p == 1 ? b : c;
  }
  __device__ __forceinline__ const float* row(int o, int C) const {
    const int p = o / rows;
    return pick(w0, w1, w2, p) + (long long)(o - p * rows) * C;
  }
  __device__ __forceinline__ float bias(int o) const {
    const int p = o / rows;
    const float* bp = pick(b0, b1, b2, p);
    return bp ? bp[o - p * rows] : 0.f;
  }
};

// Row o of the folded weight and its bias, one wave.  The row's loads go out
// in batches of 8 per lane before any store: one memory round trip per 512
// columns, not one per 64.  Indices are clamped, not branched on (a branch per
// access serialises them): past the end a lane loads and stores column C - 1
// again -- the same value to the same word.
// (Wfb, nullable: the folded row also as bf16, the operand tgfr_bn_qkv_bf16 reads)
__device__ __forceinline__ void bn_fold_row(const Parts P, int o, int C,
                                            const float* __restrict__ gamma,
                                            const float* __restrict__ beta,
                                            float* __restrict__ Wf, float* __restrict__ bf,
                                            int lane, uint16_t* __restrict__ Wfb = nullptr) {
  constexpr int U = 8;
  const float* wr = P.row(o, C);
  float acc = 0.f;
  for (int c0 = 0; c0 < C; c0 += U * WAVE) {
    float w[U], g[U], b[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int c = min(c0 + u * WAVE + lane, C - 1);
      w[u] = wr[c];
      g[u] = gamma[c];
      b[u] = beta[c];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int c = c0 + u * WAVE + lane;
      Wf[(long long)o * C + min(c, C - 1)] = w[u] * g[u];
      if (Wfb) Wfb[(long long)o * C + min(c, C - 1)] = bf_bits(w[u] * g[u]);
      acc += c < C ? w[u] * b[u] : 0.f;
    }
  }
  acc = wave_sum(acc);
  if (lane == 0) bf[o] = P.bias(o) + acc;
}

// BatchNorm2d batch statistics of channel c (one 256-thread workgroup; red:
// 4 floats of the caller's LDS): two-pass mean / biased var over N x HW, rstd;
// running_mean/var update with the unbiased var (momentum), and
// num_batches_tracked += 1 (nn.BatchNorm2d training semantics).
// Up to 256 * BN_REG values per channel (B = 64 at
// 14 x 14: 49 per thread) are loaded once into registers; larger maps take the
// two-pass loop (thread t owns positions hw = t, t+256, ... of every sample).
constexpr int BN_REG = 64;
__device__ __forceinline__ void bn_stats_block(
    const float* __restrict__ x, int N, int C, int HW, float eps, float momentum, int training,
    float* __restrict__ running_mean, float* __restrict__ running_var,
    long long* __restrict__ nbt, float* __restrict__ mean_out, float* __restrict__ rstd_out,
    int c, float* red) {
  const int tid = threadIdx.x, wid = tid / WAVE, lane = tid % WAVE;
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

}  // namespace
