// Shared device helpers for the TGFR gfx950 kernels.
//
// Numerics: every contraction runs on v_mfma_f32_32x32x16_bf16 with fp32
// accumulation.  MODE_SPLIT carries each fp32 operand as a bf16 pair
// (hi = bf16(x), lo = bf16(x - hi)) and issues hi*hi + hi*lo + lo*hi, which
// keeps ~16 mantissa bits per operand (the fp32-parity mode); MODE_BF16 issues
// hi*hi only (the bf16 perf mode).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <map>
#include <mutex>
#include <utility>

#define LDS_AS __attribute__((address_space(3)))

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// MODE_F16: fp16 operands (v_mfma_f32_32x32x16_f16, fp32 accumulation), hi
// only -- the BASELINE config-5 precision for the word-region contraction.
enum { MODE_BF16 = 0, MODE_SPLIT = 1, MODE_F16 = 2 };
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

namespace tgfr {

constexpr int WAVE = 64;

__device__ __forceinline__ uint16_t bf_bits(float x) {
  return __builtin_bit_cast(uint16_t, (__bf16)x);
}
__device__ __forceinline__ float bf_val(uint16_t u) {
  return __uint_as_float(((uint32_t)u) << 16);
}
__device__ __forceinline__ uint16_t f16_bits(float x) {
  return __builtin_bit_cast(uint16_t, (_Float16)x);
}
// the single-operand (non-split) encoding of a mode: bf16 or fp16 bits
template <int MODE>
__device__ __forceinline__ uint16_t lowp_bits(float x) {
  if constexpr (MODE == MODE_F16)
    return f16_bits(x);
  else
    return bf_bits(x);
}
// fp32 -> (hi, lo) bf16 pair with x ~= hi + lo to ~2^-17 relative.
__device__ __forceinline__ void split2(float x, uint16_t& hi, uint16_t& lo) {
  hi = bf_bits(x);
  lo = bf_bits(x - bf_val(hi));
}
__device__ __forceinline__ uint32_t pack2(uint16_t a, uint16_t b) {
  return (uint32_t)a | ((uint32_t)b << 16);
}
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
// Two fp32 -> packed bf16x2 (a in the low half) by one v_cvt_pk_bf16_f32.
__device__ __forceinline__ uint32_t pk_bf16(float a, float b) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2){a, b}, bf16x2));
}
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
// Two fp32 -> the packed single-operand encoding of a mode (bf16x2, or fp16x2
// rounded to nearest)
template <int MODE>
__device__ __forceinline__ uint32_t pk_lowp(float a, float b) {
  if constexpr (MODE == MODE_F16)
    return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2){a, b}, f16x2));
  else
    return pk_bf16(a, b);
}
// One single-operand 32x32x16 MFMA of a mode; the operands are bf16x8
// carriers holding bf16 or fp16 bits
template <int MODE>
__device__ __forceinline__ f32x16 mfma_lp(const bf16x8& a, const bf16x8& b, const f32x16& c) {
  if constexpr (MODE == MODE_F16)
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a),
                                                  __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
  else
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

template <int MODE>
__device__ __forceinline__ void mma(f32x16& acc, const bf16x8& ahi, const bf16x8& alo,
                                    const bf16x8& bhi, const bf16x8& blo) {
  if constexpr (MODE == MODE_F16) {
    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, ahi),
                                                  __builtin_bit_cast(f16x8, bhi), acc, 0, 0, 0);
    return;
  }
  if constexpr (MODE == MODE_SPLIT) {
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(alo, bhi, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ahi, blo, acc, 0, 0, 0);
  }
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ahi, bhi, acc, 0, 0, 0);
}

// mma<MODE> with the accumulator pinned to AGPRs ("+a"): for accumulators
// that live across a loop (the word-region backward's dR), where hipcc would
// otherwise keep them in VGPRs and copy them to / from AGPRs around every
// MFMA chain.  Only MFMAs touch these registers until the caller reads them
// back (after mfma_drain()).
template <int MODE>
__device__ __forceinline__ void mma_agpr(f32x16& acc, const bf16x8& ahi, const bf16x8& alo,
                                         const bf16x8& bhi, const bf16x8& blo) {
  if constexpr (MODE == MODE_F16) {
    asm("v_mfma_f32_32x32x16_f16 %0, %1, %2, %0" : "+a"(acc) : "v"(ahi), "v"(bhi));
    return;
  }
  if constexpr (MODE == MODE_SPLIT) {
    asm("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(alo), "v"(bhi));
    asm("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(ahi), "v"(blo));
  }
  asm("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(ahi), "v"(bhi));
}
// Wait states before anything but an MFMA reads an mma_agpr accumulator
// (a 32x32x16 MFMA's result latency; the hazard recognizer does not see
// through inline asm).
__device__ __forceinline__ void mfma_drain() {
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
}

__device__ __forceinline__ bf16x8 as_bf8(uint4 v) { return __builtin_bit_cast(bf16x8, v); }

// 8 fp32 values -> bf16x8 hi (and lo when split).
template <int MODE>
__device__ __forceinline__ void frag8(const float* v, bf16x8& hi, bf16x8& lo) {
  uint32_t hp[4], lp[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    uint16_t a0, a1, b0 = 0, b1 = 0;
    if constexpr (MODE == MODE_SPLIT) {
      split2(v[2 * k], a0, b0);
      split2(v[2 * k + 1], a1, b1);
    } else {
      a0 = lowp_bits<MODE>(v[2 * k]);
      a1 = lowp_bits<MODE>(v[2 * k + 1]);
    }
    hp[k] = pack2(a0, a1);
    lp[k] = pack2(b0, b1);
  }
  hi = as_bf8(make_uint4(hp[0], hp[1], hp[2], hp[3]));
  lo = as_bf8(make_uint4(lp[0], lp[1], lp[2], lp[3]));
}

// LDS access through explicit address-space-3 pointers (byte offsets).
extern __shared__ __attribute__((aligned(16))) char g_smem[];

__device__ __forceinline__ LDS_AS char* lds_base() { return (LDS_AS char*)g_smem; }

__device__ __forceinline__ uint4 lds_ld16(uint32_t off) {
  return __builtin_bit_cast(uint4, *(LDS_AS u32x4*)(lds_base() + off));
}
__device__ __forceinline__ void lds_st16(uint32_t off, uint4 v) {
  *(LDS_AS u32x4*)(lds_base() + off) = __builtin_bit_cast(u32x4, v);
}
__device__ __forceinline__ void lds_st8(uint32_t off, uint2 v) {
  *(LDS_AS u32x2*)(lds_base() + off) = __builtin_bit_cast(u32x2, v);
}
__device__ __forceinline__ float lds_ldf(uint32_t off) {
  return *(LDS_AS float*)(lds_base() + off);
}
__device__ __forceinline__ void lds_stf(uint32_t off, float v) {
  *(LDS_AS float*)(lds_base() + off) = v;
}
// ds_read_b64_tr_b16: within each 16-lane group, lane 4q+p supplies the
// address of row q (columns 4p..4p+3) of a 4-row block; lane i receives
// column i of the 4 rows, row q in element q.
__device__ __forceinline__ s16x4 lds_tr4(uint32_t off) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS s16x4*)(lds_base() + off));
}
__device__ __forceinline__ bf16x8 join_tr(s16x4 a, s16x4 b) {
  s16x8 v = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
  return __builtin_bit_cast(bf16x8, v);
}

// One 16-B-per-lane global -> LDS DMA (global_load_lds_dwordx4) to LDS byte
// offset lds_off (wave-uniform) + 16 * lane.  Issued from inline asm so that
// hipcc does not see an LDS write pending on the VM counter: with the builtin
// it drains every DMA (vmcnt(0)) before the next ds_read and before each
// barrier, which serialises the ring.  The kernel orders the DMA by counted
// vmcnt waits + raw barriers itself (cdna_hip_programming.md, pipelining
// across barriers).
__device__ __forceinline__ void glds16(const void* src, uint32_t lds_off) {
  const uint32_t m0 = __builtin_amdgcn_readfirstlane(
      (uint32_t)(uintptr_t)(lds_base() + lds_off));
  // s_nop: one wait state between the M0 write and the LDS DMA that reads it
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(src),
               "s"(m0)
               : "memory", "m0");
}

// glds16 with a wave-uniform 64-bit base in SGPRs and a per-lane 32-bit byte
// offset (the saddr form): no 64-bit address arithmetic per piece on the VALU.
__device__ __forceinline__ void glds16s(const void* sbase, uint32_t voff, uint32_t lds_off) {
  const uint32_t m0 = __builtin_amdgcn_readfirstlane(
      (uint32_t)(uintptr_t)(lds_base() + lds_off));
  // (readfirstlane returns int: zero-extend each half, never sign-extend)
  const uint64_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)sbase);
  const uint64_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)((uintptr_t)sbase >> 32));
  const uint64_t sb = lo | (hi << 32);
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1" ::"v"(voff),
               "s"(sb), "s"(m0)
               : "memory", "m0");
}

// 128-bit buffer descriptor over [p, p + bytes) from wave-uniform inputs
// (readfirstlane: provably uniform, so no waterfall loop per memory op).  A
// buffer op then takes only a 32-bit lane offset: no per-lane 64-bit address
// for the compiler to hoist out of a loop and spill.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t uniform_rsrc(const void* p, uint32_t bytes) {
  const uint64_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)p);
  const uint64_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)((uintptr_t)p >> 32));
  return __builtin_amdgcn_make_buffer_rsrc((void*)(lo | (hi << 32)), 0,
                                           (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}

// Retire this wave's DMA down to N outstanding ops and its LDS reads, then
// meet the other waves.  One asm statement: nothing moves across it.
template <int N>
__device__ __forceinline__ void ring_barrier() {
  asm volatile("s_waitcnt vmcnt(%0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::"n"(N) : "memory");
}

// Bijective XCD-aware remap of a 1-D grid: blocks L and L+8 run on one XCD,
// so consecutive work indices returned here share that XCD's L2.
__device__ __forceinline__ int xcd_remap(int L, int total) {
  const int q = total / 8, r = total % 8, x = L % 8, s = L / 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + s;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v = fmaxf(v, __shfl_xor(v, m));
  return v;
}
// v combined with the same register of lane l ^ 32 by v_permlane32_swap (a
// VALU op; no LDS round trip as with ds_bpermute).  After the swap, lanes
// 0-31 hold (own, partner) in (r[0], r[1]) and lanes 32-63 (partner, own), so
// a symmetric op of r[0] and r[1] is the pair's result in every lane.
__device__ __forceinline__ float xhalf_sum(float v) {
  const int u = __float_as_int(v);
  const auto r = __builtin_amdgcn_permlane32_swap(u, u, false, false);
  return __int_as_float(r[0]) + __int_as_float(r[1]);
}
__device__ __forceinline__ float xhalf_max(float v) {
  const int u = __float_as_int(v);
  const auto r = __builtin_amdgcn_permlane32_swap(u, u, false, false);
  return __builtin_fmaxf(__int_as_float(r[0]), __int_as_float(r[1]));
}

// max / sum over the 16 lanes of a DPP row, in every lane: mirror (i <->
// 15 - i), half mirror (i <-> 7 - i), then quad xor 1 and xor 2.
template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
  return __builtin_bit_cast(
      float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float row16_max(float v) {
  v = fmaxf(v, dpp<0x140>(v));
  v = fmaxf(v, dpp<0x141>(v));
  v = fmaxf(v, dpp<0xB1>(v));
  return fmaxf(v, dpp<0x4E>(v));
}
__device__ __forceinline__ float row16_sum(float v) {
  v += dpp<0x140>(v);
  v += dpp<0x141>(v);
  v += dpp<0xB1>(v);
  return v + dpp<0x4E>(v);
}

// v summed with lane l ^ 16 by v_permlane16_swap (VALU, no LDS round trip);
// with row16_sum first: the sum over each 32-lane half, in every lane
__device__ __forceinline__ float x16_sum(float v) {
  const int u = __float_as_int(v);
  const auto r = __builtin_amdgcn_permlane16_swap(u, u, false, false);
  return __int_as_float(r[0]) + __int_as_float(r[1]);
}

__device__ __forceinline__ float half_max(float v) {
#pragma unroll
  for (int m = 16; m >= 1; m >>= 1) v = fmaxf(v, __shfl_xor(v, m));
  return v;
}
// Reduce over the 32 lanes of each wave half (lanes differing in bits 0..4).
__device__ __forceinline__ float half_sum(float v) {
#pragma unroll
  for (int m = 16; m >= 1; m >>= 1) v += __shfl_xor(v, m);
  return v;
}

// Reduce-scatter of 16 per-lane values over the 32 lanes of a wave half.
// On return lane lr holds the half-total of index
//   q(lr) = 8*b4 + 4*b3 + 2*b2 + b1  (bk = bit k of lr)
// in BOTH lanes lr and lr^1.  16 shuffles instead of 80.
__device__ __forceinline__ float rs16(const float (&v)[16], int lr) {
  float w8[8], w4[4], w2[2];
  bool up = lr & 16;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    float send = up ? v[k] : v[k + 8];
    float keep = up ? v[k + 8] : v[k];
    w8[k] = keep + __shfl_xor(send, 16);
  }
  up = lr & 8;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    float send = up ? w8[k] : w8[k + 4];
    float keep = up ? w8[k + 4] : w8[k];
    w4[k] = keep + __shfl_xor(send, 8);
  }
  up = lr & 4;
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    float send = up ? w4[k] : w4[k + 2];
    float keep = up ? w4[k + 2] : w4[k];
    w2[k] = keep + __shfl_xor(send, 4);
  }
  up = lr & 2;
  float send = up ? w2[0] : w2[1];
  float w1 = (up ? w2[1] : w2[0]) + __shfl_xor(send, 2);
  return w1 + __shfl_xor(w1, 1);
}
__device__ __forceinline__ int rs16_index(int lr) {
  return (((lr >> 4) & 1) << 3) | (((lr >> 3) & 1) << 2) | (((lr >> 2) & 1) << 1) |
         ((lr >> 1) & 1);
}

// In-launch "last arriver" hand-off (the split-K counter recipe of
// cdna_hip_programming.md 5 item 2 / 6 Guideline 16): every block stores its
// partials with plain stores, drains, and lane 0 releases at agent scope
// before taking a ticket; the block drawing expected-1 acquires, resets the
// counter for the next launch and returns true in all its threads.  Correct
// for any placement of the blocks over XCDs.  `flag` is an LDS word of the
// kernel's (single) shared array.
typedef __attribute__((address_space(1))) unsigned gu32;

__device__ __forceinline__ bool last_arrival(unsigned* cnt, unsigned expected, int* flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned t =
        __hip_atomic_fetch_add((gu32*)cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = t == expected - 1;
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_store((gu32*)cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    *flag = last;
  }
  __syncthreads();
  return *flag != 0;
}

// Row index inside a 32x32 MFMA accumulator tile for register q of wave half h.
__device__ __forceinline__ constexpr int acc_row(int q, int h) {
  return (q & 3) + 8 * (q >> 2) + 4 * h;
}

// Host: allow `bytes` of dynamic LDS for kernel `fn` on the current device,
// once per (kernel, device) and thread-safe; returns the hipError_t of the
// attribute call (0 when already set).  Every entry point that launches with
// more than 64 KB of dynamic LDS calls this before its launch.
inline int set_max_lds(const void* fn, int bytes) {
  static std::mutex mu;
  static std::map<std::pair<const void*, int>, int> done;
  int dev = 0;
  const hipError_t e0 = hipGetDevice(&dev);
  if (e0 != hipSuccess) return (int)e0;
  std::lock_guard<std::mutex> lock(mu);
  auto it = done.find({fn, dev});
  if (it != done.end() && it->second >= bytes) return 0;
  const hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
  if (e != hipSuccess) return (int)e;
  done[{fn, dev}] = bytes;
  return 0;
}

}  // namespace tgfr
