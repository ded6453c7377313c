// Standalone func_attention (models/attention.py:10-43) for gfx950, fp32:
//
//   S  = ctx^T q                 [R, T]   (:27)
//   A1 = softmax_T(S)            per region  (:28-29)
//   A2 = softmax_R(gamma1 A1^T)  [T, R]   per word (:32-36)
//   C  = ctx A2^T                [D, T]   (:41)
//
// returning (C, A2 as attn) like the reference, and the backward to both
// query and context.  This is the per-call API entry point (matched query /
// context batches, differentiable in both); the trainers reach the same
// arithmetic for all (image, caption) pairs at once through the fused
// word-region kernels (tgfr_wr.hip).  Exact fp32 on the VALU: one workgroup
// per sample, the small matrices (S / A1 [R][T], A2 [T][R], q [D][T]) staged
// in LDS, the large operand (ctx, D x R) streamed from L2 with consecutive
// threads on consecutive regions.  Limits: R <= 256, T <= 64, D <= 256.
#include "tgfr_common.h"

using namespace tgfr;

namespace {

constexpr int FA_R = 256, FA_T = 64, FA_D = 256;
constexpr int FA_BUF = FA_R * FA_T * 4;    // one [R][T] or [T][R] fp32 buffer (64 KiB)

struct FaView {                 // element (b, d, x) at p[b*sb + d*sd + x*sx]
  const float* p;
  long long sb, sd, sx;
  __device__ __forceinline__ float at(int b, int d, int x) const {
    return p[b * sb + d * sd + x * sx];
  }
};

// Forward; LDS: buf0 = q [D][T] then A2 [T][R], buf1 = S / A1 [R][T].
__global__ __launch_bounds__(256) void fa_fwd_kernel(FaView q, FaView ctx, int D, int T, int R,
                                                     float g1, float* __restrict__ C,
                                                     long long Csb, long long Csd, long long Cst,
                                                     float* __restrict__ A1o,
                                                     float* __restrict__ A2o) {
  float* buf0 = (float*)g_smem;
  float* buf1 = buf0 + FA_BUF / 4;
  const int b = blockIdx.x, tid = threadIdx.x, wv = tid / WAVE, lane = tid % WAVE;
  for (int i = tid; i < D * T; i += 256) buf0[i] = q.at(b, i / T, i % T);
  __syncthreads();
  // S[r][t] = sum_d ctx[d][r] q[d][t]
  for (int i = tid; i < R * T; i += 256) {
    const int r = i / T, t = i % T;
    float s = 0.f;
    for (int d = 0; d < D; ++d) s = fmaf(ctx.at(b, d, r), buf0[d * T + t], s);
    buf1[i] = s;
  }
  __syncthreads();
  // A1: softmax over the words of each region (thread per region)
  for (int r = tid; r < R; r += 256) {
    float* row = buf1 + r * T;
    float m = -INFINITY;
    for (int t = 0; t < T; ++t) m = fmaxf(m, row[t]);
    float sum = 0.f;
    for (int t = 0; t < T; ++t) {
      const float e = __expf(row[t] - m);
      row[t] = e;
      sum += e;
    }
    const float inv = 1.f / sum;
    for (int t = 0; t < T; ++t) {
      row[t] *= inv;
      A1o[((long long)b * R + r) * T + t] = row[t];
    }
  }
  __syncthreads();
  // A2: softmax over the regions of gamma1 * A1 for each word (wave per word)
  for (int t = wv; t < T; t += 4) {
    float m = -INFINITY;
    for (int r = lane; r < R; r += WAVE) m = fmaxf(m, g1 * buf1[r * T + t]);
    m = wave_max(m);
    float sum = 0.f;
    for (int r = lane; r < R; r += WAVE) sum += __expf(g1 * buf1[r * T + t] - m);
    sum = wave_sum(sum);
    const float inv = 1.f / sum;
    for (int r = lane; r < R; r += WAVE) {
      const float a = __expf(g1 * buf1[r * T + t] - m) * inv;
      buf0[t * R + r] = a;
      A2o[((long long)b * T + t) * R + r] = a;
    }
  }
  __syncthreads();
  // C[d][t] = sum_r ctx[d][r] A2[t][r]
  for (int i = tid; i < D * T; i += 256) {
    const int d = i / T, t = i % T;
    float s = 0.f;
    for (int r = 0; r < R; ++r) s = fmaf(ctx.at(b, d, r), buf0[t * R + r], s);
    C[b * Csb + d * Csd + t * Cst] = s;
  }
}

// Backward; LDS: buf0 = dA2 -> dX [T][R], buf1 = dS [R][T].
__global__ __launch_bounds__(256) void fa_bwd_kernel(
    FaView q, FaView ctx, FaView dC, const float* __restrict__ dattn, int D, int T, int R,
    float g1, const float* __restrict__ A1, const float* __restrict__ A2, float* __restrict__ dq,
    float* __restrict__ dctx) {
  float* buf0 = (float*)g_smem;
  float* buf1 = buf0 + FA_BUF / 4;
  const int b = blockIdx.x, tid = threadIdx.x, wv = tid / WAVE, lane = tid % WAVE;
  const float* A1b = A1 + (long long)b * R * T;
  const float* A2b = A2 + (long long)b * T * R;
  // dA2[t][r] = sum_d dC[d][t] ctx[d][r] (+ dattn)
  for (int i = tid; i < T * R; i += 256) {
    const int t = i / R, r = i % R;
    float s = dattn ? dattn[(long long)b * T * R + i] : 0.f;
    for (int d = 0; d < D; ++d) s = fmaf(dC.at(b, d, t), ctx.at(b, d, r), s);
    buf0[i] = s;
  }
  __syncthreads();
  // softmax-over-regions backward, in place: dX = A2 (dA2 - <A2, dA2>)
  for (int t = wv; t < T; t += 4) {
    float dot = 0.f;
    for (int r = lane; r < R; r += WAVE) dot += A2b[t * R + r] * buf0[t * R + r];
    dot = wave_sum(dot);
    for (int r = lane; r < R; r += WAVE) buf0[t * R + r] = A2b[t * R + r] * (buf0[t * R + r] - dot);
  }
  __syncthreads();
  // softmax-over-words backward: dS[r][t] = A1 (g1 dX^T - <A1, g1 dX^T>)
  for (int r = tid; r < R; r += 256) {
    float dot = 0.f;
    for (int t = 0; t < T; ++t) dot += A1b[r * T + t] * g1 * buf0[t * R + r];
    for (int t = 0; t < T; ++t)
      buf1[r * T + t] = A1b[r * T + t] * (g1 * buf0[t * R + r] - dot);
  }
  __syncthreads();
  // dctx[d][r] = sum_t dC[d][t] A2[t][r] + sum_t q[d][t] dS[r][t]
  for (int i = tid; i < D * R; i += 256) {
    const int d = i / R, r = i % R;
    float s = 0.f;
    for (int t = 0; t < T; ++t)
      s = fmaf(dC.at(b, d, t), A2b[t * R + r], fmaf(q.at(b, d, t), buf1[r * T + t], s));
    dctx[(long long)b * D * R + i] = s;
  }
  // dq[d][t] = sum_r ctx[d][r] dS[r][t]
  for (int i = tid; i < D * T; i += 256) {
    const int d = i / T, t = i % T;
    float s = 0.f;
    for (int r = 0; r < R; ++r) s = fmaf(ctx.at(b, d, r), buf1[r * T + t], s);
    dq[(long long)b * D * T + i] = s;
  }
}

bool fa_shape_ok(int B, int D, int T, int R) {
  return B > 0 && D > 0 && T > 0 && R > 0 && R <= FA_R && T <= FA_T && D <= FA_D;
}

}  // namespace

extern "C" {

// query element (b, d, t) at q[b*qsb + d*qsd + t*qst]; context (b, d, r) at
// ctx[b*csb + d*csd + r*csr] (r = y*iw + x).  C [B][D][T] at the given
// strides; A1 [B][R][T] (saved for the backward) and attn = A2 [B][T][R]
// dense.
int tgfr_func_attention_fwd(const float* q, long long qsb, long long qsd, long long qst,
                            const float* ctx, long long csb, long long csd, long long csr, int B,
                            int D, int T, int R, float gamma1, float* C, long long Csb,
                            long long Csd, long long Cst, float* A1, float* attn, void* stream) {
  if (!fa_shape_ok(B, D, T, R) || !q || !ctx || !C || !A1 || !attn) return 1001;
  if (const int e = set_max_lds((const void*)fa_fwd_kernel, 2 * FA_BUF)) return e;
  hipLaunchKernelGGL(fa_fwd_kernel, dim3(B), dim3(256), 2 * FA_BUF, (hipStream_t)stream,
                     FaView{q, qsb, qsd, qst}, FaView{ctx, csb, csd, csr}, D, T, R, gamma1, C, Csb,
                     Csd, Cst, A1, attn);
  return (int)hipGetLastError();
}

// dC (b, d, t) at the given strides; dattn [B][T][R] dense or NULL; dq
// [B][D][T] and dctx [B][D][R] dense, overwritten.
int tgfr_func_attention_bwd(const float* q, long long qsb, long long qsd, long long qst,
                            const float* ctx, long long csb, long long csd, long long csr,
                            const float* dC, long long dsb, long long dsd, long long dst,
                            const float* dattn, int B, int D, int T, int R, float gamma1,
                            const float* A1, const float* attn, float* dq, float* dctx,
                            void* stream) {
  if (!fa_shape_ok(B, D, T, R) || !q || !ctx || !dC || !A1 || !attn || !dq || !dctx)
    return 1001;
  if (const int e = set_max_lds((const void*)fa_bwd_kernel, 2 * FA_BUF)) return e;
  hipLaunchKernelGGL(fa_bwd_kernel, dim3(B), dim3(256), 2 * FA_BUF, (hipStream_t)stream,
                     FaView{q, qsb, qsd, qst}, FaView{ctx, csb, csd, csr},
                     FaView{dC, dsb, dsd, dst}, dattn, D, T, R, gamma1, A1, attn, dq, dctx);
  return (int)hipGetLastError();
}

}  // extern "C"
