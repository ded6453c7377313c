// One-launch optimiser step for every trainable tensor of a trainer: Adam
// (torch.optim.Adam, amsgrad off) for the image head, SGD with momentum and
// weight decay (torch.optim.SGD) for the ArcMargin classifiers
// (src/train_encoders_bert.py:212-222, src/fusion_bert.py:119-139).
//
// The reference steps two torch optimisers, i.e. one multi-tensor launch per
// parameter group plus a step-count update; here all tensors go into ONE
// launch whose kernel arguments carry the segment table (parameter, gradient,
// two state buffers, length, group).  Each block works inside one segment
// (segment starts are padded to whole blocks), so the segment lookup is a
// scalar loop.  The step count lives on the device (counters[0]) and is
// bumped by the last block to finish, so a captured graph replays the step
// with the right bias corrections.  Learning rates are the group's lr times a
// per-group factor read from device memory (lr_scale), so a schedule
// (ExponentialLR on the head, the 10x classifier cuts of
// src/train_encoders_bert.py:406-410) changes a captured step's lr between
// replays without re-capturing.
//
// HBM-bound: Adam moves 28 B per element (p, g, m, v in; p, m, v out), SGD
// 20 B (p, g, buf in; p, buf out).
#include "tgfr_common.h"

#include <math.h>

#include "../../include/tgfr.h"

using namespace tgfr;

namespace {

constexpr int MAX_SEG = 48, MAX_GRP = 4, THREADS = 256, VEC_PER_BLOCK = 4 * THREADS;

struct Seg {
  float* p;
  const float* g;
  float* s0;
  float* s1;
  long long n;
  int grp;
  int vec;        // every pointer 16-B aligned and n % 4 == 0
};

struct Args {
  Seg seg[MAX_SEG];
  int bstart[MAX_SEG + 1];     // first block of each segment (prefix sums)
  tgfr_optim_group grp[MAX_GRP];
  int nseg;
};

struct Consts {
  float lr;                    // effective learning rate (G.lr * lr_scale[group])
  float step_size, bc2_sqrt;   // Adam: lr / (1 - b1^t), sqrt(1 - b2^t)
  int first;                   // SGD: momentum buffer starts as d_p at t = 1
};

__device__ __forceinline__ void update(float& p, float g, float& s0, float& s1,
                                       const tgfr_optim_group& G, const Consts& c) {
  // c.lr: G.lr times the group's device-side scale
  if (G.weight_decay != 0.f) g = fmaf(G.weight_decay, p, g);
  if (G.kind == TGFR_OPTIM_ADAM) {
    s0 = G.beta1 * s0 + (1.f - G.beta1) * g;
    s1 = G.beta2 * s1 + (1.f - G.beta2) * g * g;
    const float denom = sqrtf(s1) / c.bc2_sqrt + G.eps;
    p -= c.step_size * s0 / denom;
  } else {
    if (G.momentum != 0.f) {
      s0 = c.first ? g : G.momentum * s0 + (1.f - G.dampening) * g;
      g = s0;
    }
    p -= c.lr * g;
  }
}

__device__ __forceinline__ void update_vec(const Seg& sg, long long e0, bool adam, bool has_s0,
                                           const tgfr_optim_group& G, const Consts& c) {
  if (sg.vec && e0 + 4 <= sg.n) {
    float4 p = *(float4*)(sg.p + e0);
    const float4 g = *(const float4*)(sg.g + e0);
    float4 m = has_s0 ? *(float4*)(sg.s0 + e0) : make_float4(0.f, 0.f, 0.f, 0.f);
    float4 v = adam ? *(float4*)(sg.s1 + e0) : make_float4(0.f, 0.f, 0.f, 0.f);
    update(p.x, g.x, m.x, v.x, G, c);
    update(p.y, g.y, m.y, v.y, G, c);
    update(p.z, g.z, m.z, v.z, G, c);
    update(p.w, g.w, m.w, v.w, G, c);
    *(float4*)(sg.p + e0) = p;
    if (has_s0) *(float4*)(sg.s0 + e0) = m;
    if (adam) *(float4*)(sg.s1 + e0) = v;
  } else {
    for (long long e = e0; e < e0 + 4 && e < sg.n; ++e) {
      float p = sg.p[e], m = has_s0 ? sg.s0[e] : 0.f, v = adam ? sg.s1[e] : 0.f;
      update(p, sg.g[e], m, v, G, c);
      sg.p[e] = p;
      if (has_s0) sg.s0[e] = m;
      if (adam) sg.s1[e] = v;
    }
  }
}

__global__ __launch_bounds__(THREADS) void optim_step_kernel(Args a, const float* lr_scale,
                                                             int* counters) {
  const int b = blockIdx.x;
  int s = 0;
  while (s + 1 < a.nseg && a.bstart[s + 1] <= b) ++s;
  const Seg sg = a.seg[s];
  const tgfr_optim_group G = a.grp[sg.grp];
  const int t = counters[0] + 1;
  Consts c;
  c.first = t == 1;
  c.lr = lr_scale ? G.lr * lr_scale[sg.grp] : G.lr;
  c.step_size = (float)((double)c.lr / (1.0 - pow((double)G.beta1, (double)t)));
  c.bc2_sqrt = (float)sqrt(1.0 - pow((double)G.beta2, (double)t));
  const bool adam = G.kind == TGFR_OPTIM_ADAM;
  const bool has_s0 = adam || G.momentum != 0.f;
  const long long base = (long long)(b - a.bstart[s]) * VEC_PER_BLOCK * 4;
  constexpr int J = VEC_PER_BLOCK / THREADS;
  if (sg.vec && base + 4LL * VEC_PER_BLOCK <= sg.n) {
    // a whole block of float4 items: every load first (the stores to p could
    // alias the next item's loads as far as the compiler knows, which
    // serialised four HBM round trips per block), then update and store
    float4 p[J], g[J], m[J], v[J];
#pragma unroll
    for (int j = 0; j < J; ++j) {
      const long long e0 = base + 4LL * (j * THREADS + threadIdx.x);
      p[j] = *(const float4*)(sg.p + e0);
      g[j] = *(const float4*)(sg.g + e0);
      m[j] = has_s0 ? *(const float4*)(sg.s0 + e0) : make_float4(0.f, 0.f, 0.f, 0.f);
      v[j] = adam ? *(const float4*)(sg.s1 + e0) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int j = 0; j < J; ++j) {
      const long long e0 = base + 4LL * (j * THREADS + threadIdx.x);
      update(p[j].x, g[j].x, m[j].x, v[j].x, G, c);
      update(p[j].y, g[j].y, m[j].y, v[j].y, G, c);
      update(p[j].z, g[j].z, m[j].z, v[j].z, G, c);
      update(p[j].w, g[j].w, m[j].w, v[j].w, G, c);
      *(float4*)(sg.p + e0) = p[j];
      if (has_s0) *(float4*)(sg.s0 + e0) = m[j];
      if (adam) *(float4*)(sg.s1 + e0) = v[j];
    }
  } else {
#pragma unroll
    for (int j = 0; j < J; ++j)
      update_vec(sg, base + 4LL * (j * THREADS + threadIdx.x), adam, has_s0, G, c);
  }
  // The last block to arrive advances the step count.  Every block read it
  // at its start; nothing else is published, so the arrival needs no release
  // fence (an agent-scope release per block would write back L2 each time).
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned n = __hip_atomic_fetch_add((unsigned*)counters + 1, 1u, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT);
    if (n == gridDim.x - 1) {
      __hip_atomic_store((unsigned*)counters + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(counters, t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

bool al16(const void* p) { return ((uintptr_t)p & 15) == 0; }

}  // namespace

extern "C" int tgfr_optim_step(const tgfr_optim_seg* segs, int n_segs,
                               const tgfr_optim_group* groups, int n_groups,
                               const float* lr_scale, int* counters, void* stream) {
  if (n_segs <= 0 || n_segs > MAX_SEG || n_groups <= 0 || n_groups > MAX_GRP || !counters)
    return 1001;
  Args a;
  a.nseg = n_segs;
  for (int i = 0; i < n_groups; ++i) {
    const tgfr_optim_group& g = groups[i];
    if (g.kind != TGFR_OPTIM_ADAM && g.kind != TGFR_OPTIM_SGD) return 1002;
    a.grp[i] = g;
  }
  long long blocks = 0;
  for (int i = 0; i < n_segs; ++i) {
    const tgfr_optim_seg& s = segs[i];
    if (s.n <= 0 || !s.param || !s.grad || s.group < 0 || s.group >= n_groups) return 1001;
    const tgfr_optim_group& g = groups[s.group];
    const bool adam = g.kind == TGFR_OPTIM_ADAM;
    if ((adam || g.momentum != 0.f) && !s.state0) return 1001;
    if (adam && !s.state1) return 1001;
    Seg& d = a.seg[i];
    d.p = s.param;
    d.g = s.grad;
    d.s0 = s.state0;
    d.s1 = s.state1;
    d.n = s.n;
    d.grp = s.group;
    d.vec = (s.n % 4) == 0 && al16(s.param) && al16(s.grad) && (!s.state0 || al16(s.state0)) &&
            (!s.state1 || al16(s.state1));
    a.bstart[i] = (int)blocks;
    blocks += (s.n + 4LL * VEC_PER_BLOCK - 1) / (4LL * VEC_PER_BLOCK);
    if (blocks > (1LL << 30)) return 1001;
  }
  a.bstart[n_segs] = (int)blocks;
  hipLaunchKernelGGL(optim_step_kernel, dim3((unsigned)blocks), dim3(THREADS), 0,
                     (hipStream_t)stream, a, lr_scale, counters);
  return (int)hipGetLastError();
}
