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

// two floats -> one packed pair through a 2-vector conversion: ONE v_cvt_pk_bf16_f32 (the scalar casts
// combined with a shift + or compile to two converts and two more VALU)
typedef __attribute__((ext_vector_type(2))) float f32x2_t;
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2_t;
typedef __attribute__((ext_vector_type(2))) _Float16 f16x2_t;
__device__ __forceinline__ uint32_t pack_bf2(float lo, float hi) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2_t{lo, hi}, bf16x2_t));
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
__device__ __forceinline__ uint32_t pack2(float lo, float hi) {  // v_cvt_pk_bf16_f32 / v_cvt_pk_f16_f32
  if constexpr (DT == DT_BF16) return __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2_t{lo, hi}, bf16x2_t));
  else return __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2_t{lo, hi}, f16x2_t));
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
// v_perm_b32 selectors 8 / 9 give 0xFF when bit 15 / 31 of the second source is set: the sign masks of both
// halves in one permute, then one AND-NOT (2 VALU instead of ~6 compare/select)
__device__ __forceinline__ uint32_t relu_bf2(uint32_t v) {
  return v & ~__builtin_amdgcn_perm(0u, v, 0x09090808u);
}
// Max-unpool switch select on one 16-B chunk: v = 8 16-bit channels, codes = their switch codes (byte c =
// channel c's window position, 0..3); channels whose code != pos are zeroed. unpool_spread repeats each code
// byte over its channel's two bytes (once per chunk); then per position ONE v_perm_b32(0, 0xFF << 8 pos, spread)
// per dword maps every byte to 0xFF exactly where the code equals pos (selector bytes 0..3 index the constant)
// and an AND applies it: 8 VALU per chunk and position instead of ~28 for per-byte compare/select (the unpool
// expansions are VALU-bound: round 4 tail launch 4.27 -> 3.93 ms, profiles/bench_c2_r4_unpool_perm_ab.txt).
// Precondition: code bytes are 2x2-window positions 0..3 (every switch-code producer writes those). v_perm_b32
// selector bytes 8..15 would select sign-replicated bytes and >= 13 yield 0xFF, i.e. KEEP the value, where
// the old compare zeroed it; the codes are masked to 2 bits first (one VALU per dword) so an out-of-range
// byte can never select a value.
__device__ __forceinline__ uint4 unpool_spread(uint2 codes) {
  codes.x &= 0x03030303u;
  codes.y &= 0x03030303u;
  return make_uint4(__builtin_amdgcn_perm(0u, codes.x, 0x01010000u), __builtin_amdgcn_perm(0u, codes.x, 0x03030202u),
                    __builtin_amdgcn_perm(0u, codes.y, 0x01010000u), __builtin_amdgcn_perm(0u, codes.y, 0x03030202u));
}
__device__ __forceinline__ uint4 unpool_pick_s(uint4 v, uint4 spread, uint32_t pos) {
  const uint32_t K = 0xFFu << (8u * pos);
  return make_uint4(v.x & __builtin_amdgcn_perm(0u, K, spread.x), v.y & __builtin_amdgcn_perm(0u, K, spread.y),
                    v.z & __builtin_amdgcn_perm(0u, K, spread.z), v.w & __builtin_amdgcn_perm(0u, K, spread.w));
}
__device__ __forceinline__ uint4 unpool_pick(uint4 v, uint2 codes, uint32_t pos) {
  return unpool_pick_s(v, unpool_spread(codes), pos);
}
// keep elements of v where the matching element of m is > 0
// keep the 16-bit elements of a where the matching element of m is > 0, 2 per u32, branch-free:
// (m & 0x7FFF) + 0x7FFF sets bit 15 iff |m| != 0 (no carry across halves); & ~m clears negatives
// (a sign-select v_perm_b32 in place of the multiply raised conv_pw's spills: 8-12 -> 12-17 VGPRs)
__device__ __forceinline__ uint32_t mask_pos_pk(uint32_t a, uint32_t m) {
  const uint32_t pos = (((m & 0x7FFF7FFFu) + 0x7FFF7FFFu) & ~m) & 0x80008000u;
  return a & __umul24(pos >> 15, 0xFFFFu);
}
__device__ __forceinline__ uint32_t mask_pos_bf2(uint32_t v, uint32_t m) { return mask_pos_pk(v, m); }
// 1-bit ReLU masks: bit e of the byte = element e of an 8-element chunk is > 0 (the mask_pos_pk predicate
// on the stored 16-bit value, so masking by the bits equals masking by the values)
__device__ __forceinline__ uint32_t pos_bits2(uint32_t v) {
  const uint32_t pos = (((v & 0x7FFF7FFFu) + 0x7FFF7FFFu) & ~v) & 0x80008000u;
  return ((pos >> 15) & 1u) | (pos >> 30);
}
__device__ __forceinline__ uint32_t pos_bits8(uint4 v) {
  return pos_bits2(v.x) | (pos_bits2(v.y) << 2) | (pos_bits2(v.z) << 4) | (pos_bits2(v.w) << 6);
}
// keep the two 16-bit elements of a whose bits (two: bit 0 low, bit 1 high) are set
__device__ __forceinline__ uint32_t mask_bits_pk(uint32_t a, uint32_t two) {
  return a & (__umul24(two & 1u, 0xFFFFu) | (__umul24(two >> 1, 0xFFFFu) << 16));
}
__device__ __forceinline__ uint4 mask_bits8(uint4 v, uint32_t b) {
  return make_uint4(mask_bits_pk(v.x, b & 3u), mask_bits_pk(v.y, (b >> 2) & 3u), mask_bits_pk(v.z, (b >> 4) & 3u),
                    mask_bits_pk(v.w, b >> 6));
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
