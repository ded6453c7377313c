// SelfAttention core (models/fusion_nets.py:82-118) for gfx950.
//
// The reference computes, per sample n, with x the image and y the text side:
//   Qr = key_proj(x)^T [HW, C'],  Kr = query_proj(y)^T [HW, C'],  V = value_proj(x)^T [HW, C]
//   P  = softmax_j(Qr Kr^T / sqrt_dim)                  (:103-106)
//   O  = P V  -> permuted to [C, HW]                      (:115-117)
// The products (QK^T, PV, the 1x1 projections and their backward) run on
// tgfr_bgemm (tgfr_gemm.hip); this file holds the row softmax:
//   attn_softmax   P = softmax(scale * S) per row over the valid keys + row LSE.
//   attn_softmax_bwd  dS = scale * P (dP - rowsum(P dP)).
// The attention matrices are HW x HW per sample (196^2 fp32 = 150 KB for IMIM,
// 36^2 for FCFM), so they are materialised instead of recomputed.
#include "tgfr_common.h"

using namespace tgfr;

namespace {

// one wave per row of [rows][n] (row stride ld)
__global__ __launch_bounds__(256) void attn_softmax_kernel(const float* __restrict__ S,
                                                           float* __restrict__ P, float* lse,
                                                           long long rows, int n, long long ld,
                                                           float scale) {
  const long long row = blockIdx.x * 4LL + threadIdx.x / WAVE;
  const int lane = threadIdx.x % WAVE;
  if (row >= rows) return;
  const float* s = S + row * ld;
  float m = -INFINITY;
  for (int j = lane; j < n; j += WAVE) m = fmaxf(m, s[j] * scale);
  m = wave_max(m);
  float sum = 0.f;
  for (int j = lane; j < n; j += WAVE) sum += __expf(s[j] * scale - m);
  sum = wave_sum(sum);
  const float inv = 1.f / sum;
  float* p = P + row * ld;
  for (int j = lane; j < n; j += WAVE) p[j] = __expf(s[j] * scale - m) * inv;
  if (lse && lane == 0) lse[row] = m + __logf(sum);
}

__global__ __launch_bounds__(256) void attn_softmax_bwd_kernel(const float* __restrict__ P,
                                                               const float* __restrict__ dP,
                                                               float* __restrict__ dS,
                                                               long long rows, int n,
                                                               long long ld, float scale) {
  const long long row = blockIdx.x * 4LL + threadIdx.x / WAVE;
  const int lane = threadIdx.x % WAVE;
  if (row >= rows) return;
  const float* p = P + row * ld;
  const float* dp = dP + row * ld;
  float dot = 0.f;
  for (int j = lane; j < n; j += WAVE) dot += p[j] * dp[j];
  dot = wave_sum(dot);
  float* ds = dS + row * ld;
  for (int j = lane; j < n; j += WAVE) ds[j] = scale * p[j] * (dp[j] - dot);
}

}  // namespace

extern "C" {

int tgfr_attn_softmax(const float* S, float* P, float* lse, long long rows, int n, long long ld,
                      float scale, void* stream) {
  if (rows <= 0 || n <= 0) return 1001;
  hipLaunchKernelGGL(attn_softmax_kernel, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0,
                     (hipStream_t)stream, S, P, lse, rows, n, ld, scale);
  return (int)hipGetLastError();
}

int tgfr_attn_softmax_bwd(const float* P, const float* dP, float* dS, long long rows, int n,
                          long long ld, float scale, void* stream) {
  if (rows <= 0 || n <= 0) return 1001;
  hipLaunchKernelGGL(attn_softmax_bwd_kernel, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0,
                     (hipStream_t)stream, P, dP, dS, rows, n, ld, scale);
  return (int)hipGetLastError();
}

}  // extern "C"
