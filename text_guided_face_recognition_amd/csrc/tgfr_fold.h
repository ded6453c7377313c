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
__device__ __forceinline__ void bn_fold_row(const Parts P, int o, int C,
                                            const float* __restrict__ gamma,
                                            const float* __restrict__ beta,
                                            float* __restrict__ Wf, float* __restrict__ bf,
                                            int lane) {
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
      acc += c < C ? w[u] * b[u] : 0.f;
    }
  }
  acc = wave_sum(acc);
  if (lane == 0) bf[o] = P.bias(o) + acc;
}

}  // namespace
