// Shared device helpers for the gfx950 (MI355X / CDNA4) kernels of deconv_api_amd.
//
// Conventions used by every kernel in this directory:
//   * activations are NHWC, bf16 stored as raw uint16_t bits, fp32 accumulation;
//   * a wavefront is 64 lanes (hard-coded, never warpSize);
//   * launchers are plain C++ functions taking raw pointers + a hipStream_t so the
//     torch binding layer (bindings.cpp) stays out of the device compile.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kernels.h"  // DT_BF16 / DT_F16

// ---- DV_DEBUG device bounds checks (python -m deconv_api_amd._build --debug) ----
// DV_BOUNDS(off, n, extent, what): in a debug build, an access of n elements at element offset
// `off` outside [0, extent) prints the kernel site and the offending numbers and evaluates to
// false, so the caller SKIPS the access instead of faulting (a faulting kernel can reset every
// GPU on the host); in a release build it is the constant true and compiles away.
#if defined(DV_DEBUG) && DV_DEBUG
#define DV_BOUNDS(off, n, extent, what)                                                                    \
  ([&]() -> bool {                                                                                        \
    const long long o_ = (long long)(off), n_ = (long long)(n), e_ = (long long)(extent);                \
    if (o_ < 0 || o_ + n_ > e_) {                                                                         \
      printf("DV_DEBUG %s:%d %s: access [%lld, %lld) outside [0, %lld) (block %d,%d thread %d)\n", __FILE__, \
             __LINE__, what, o_, o_ + n_, e_, (int)blockIdx.x, (int)blockIdx.y, (int)threadIdx.x);        \
      return false;                                                                                       \
    }                                                                                                     \
    return true;                                                                                          \
  }())
#else
#define DV_BOUNDS(off, n, extent, what) true
#endif

namespace dv {

// ReLU of output column gcol of a conv (ConvArgs::relu / relu_cols); a template so it also works
// for argument structs without the field
template <class A>
__device__ __forceinline__ bool relu_at(const A& a, int gcol) {
  return a.relu && (a.relu_cols <= 0 || gcol < a.relu_cols);
}

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;

__device__ __forceinline__ float bf2f(uint32_t bits16) { return __uint_as_float(bits16 << 16); }

__device__ __forceinline__ uint16_t f2bf(float f) {
  // plain cast: hipcc emits v_cvt_pk_bf16_f32 (RNE, NaN preserving) on gfx950
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(uint16_t, b);
}

__device__ __forceinline__ uint32_t pack_bf2(float lo, float hi) {
  return (uint32_t)f2bf(lo) | ((uint32_t)f2bf(hi) << 16);
}

// ---- 16-bit storage dtype trait: DT 0 = bf16, DT 1 = fp16 (IEEE half) ----
typedef __attribute__((ext_vector_type(8))) _Float16 f16x8;

template <int DT>
__device__ __forceinline__ float to_f(uint32_t bits16) {
  if constexpr (DT == DT_BF16) return __uint_as_float(bits16 << 16);
  else return (float)__builtin_bit_cast(_Float16, (uint16_t)bits16);
}
template <int DT>
__device__ __forceinline__ uint16_t from_f(float f) {
  if constexpr (DT == DT_BF16) return __builtin_bit_cast(uint16_t, (__bf16)f);
  else return __builtin_bit_cast(uint16_t, (_Float16)f);
}
template <int DT>
__device__ __forceinline__ uint32_t pack2(float lo, float hi) {
  return (uint32_t)from_f<DT>(lo) | ((uint32_t)from_f<DT>(hi) << 16);
}
template <int DT>
struct Vec8 {
  typedef bf16x8 type;
};
template <>
struct Vec8<DT_F16> {
  typedef f16x8 type;
};
template <int DT>
__device__ __forceinline__ f32x4 mfma16x16x32(const typename Vec8<DT>::type& a, const typename Vec8<DT>::type& b,
                                              const f32x4& c) {
  if constexpr (DT == DT_BF16) return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
  else return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}

// bf16 lane predicates on a packed pair (bits of two bf16 values in one u32)
// (sign-bit / zero tests: valid for fp16 bit patterns too)
__device__ __forceinline__ uint32_t relu_bf2(uint32_t v) {
  uint32_t lo = (v & 0x8000u) ? 0u : (v & 0xFFFFu);
  uint32_t hi = (v & 0x80000000u) ? 0u : (v & 0xFFFF0000u);
  return lo | hi;
}
// keep elements of v where the matching element of m is > 0
__device__ __forceinline__ uint32_t mask_pos_bf2(uint32_t v, uint32_t m) {
  uint32_t mlo = m & 0xFFFFu, mhi = m >> 16;
  uint32_t lo = (mlo != 0u && !(mlo & 0x8000u)) ? (v & 0xFFFFu) : 0u;
  uint32_t hi = (mhi != 0u && !(mhi & 0x8000u)) ? (v & 0xFFFF0000u) : 0u;
  return lo | hi;
}

// keep the 16-bit elements of a where the matching element of m is > 0, 2 per u32, branch-free:
// (m & 0x7FFF) + 0x7FFF sets bit 15 iff |m| != 0 (no carry across halves); & ~m clears negatives
__device__ __forceinline__ uint32_t mask_pos_pk(uint32_t a, uint32_t m) {
  const uint32_t pos = (((m & 0x7FFF7FFFu) + 0x7FFF7FFFu) & ~m) & 0x80008000u;
  return a & __umul24(pos >> 15, 0xFFFFu);
}

// Bijective XCD-aware workgroup remap (MI355X: 8 XCDs, consecutive dispatch ids go to
// different XCDs). After the remap logically-adjacent tiles share an XCD (and its L2).
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int q = nwg >> 3, r = nwg & 7, xcd = bid & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

}  // namespace dv

#define DV_HIP_CHECK(expr)                                                     \
  do {                                                                         \
    hipError_t _e = (expr);                                                    \
    if (_e != hipSuccess) return (int)_e;                                      \
  } while (0)
