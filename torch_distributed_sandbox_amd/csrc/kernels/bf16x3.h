// bf16x3 split-precision MFMA helpers (gfx950, v_mfma_f32_16x16x32_bf16).
//
// An fp32 operand x is carried as hi = bf16(x), lo = bf16(x - hi); a product is
// formed as hi*hi + hi*lo + lo*hi with fp32 accumulation (the lo*lo term,
// ~2^-16 relative, is dropped).  Per-product relative error ~2^-16 (≈1.5e-5),
// i.e. ~30x tighter than the TF32 (10-bit mantissa) convolutions cuDNN runs by
// default for the reference on Ampere; accumulation and all I/O stay fp32.
// Cost: 3 bf16 MFMAs = 3/16 of the f32-MFMA time (5.3x faster than exact
// v_mfma_f32_16x16x4_f32 at the same FLOPs).
#pragma once

#include "common.h"

namespace tds {

typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

__device__ __forceinline__ f32x4 mfma_bf16(const s16x8& a, const s16x8& b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a), __builtin_bit_cast(bf16x8_t, b), c,
                                                 0, 0, 0);
}

// c += a*b with a = ahi+alo, b = bhi+blo (small terms first)
__device__ __forceinline__ f32x4 mfma_bf16x3(const s16x8& ahi, const s16x8& alo, const s16x8& bhi, const s16x8& blo,
                                             f32x4 c) {
  c = mfma_bf16(alo, bhi, c);
  c = mfma_bf16(ahi, blo, c);
  c = mfma_bf16(ahi, bhi, c);
  return c;
}

// c += (ahi + alo) * b for a b that is exact in bf16 (integer levels <= 256): two products
__device__ __forceinline__ f32x4 mfma_bf16x2a(const s16x8& ahi, const s16x8& alo, const s16x8& b, f32x4 c) {
  c = mfma_bf16(alo, b, c);
  c = mfma_bf16(ahi, b, c);
  return c;
}

__device__ __forceinline__ unsigned short bf16_rne(float f) {
  unsigned int u = __float_as_uint(f);
  if ((u & 0x7f800000u) == 0x7f800000u) return (unsigned short)((u >> 16) | ((u & 0xffff) ? 0x40 : 0));  // inf/nan
  u += 0x7FFFu + ((u >> 16) & 1u);
  return (unsigned short)(u >> 16);
}

__device__ __forceinline__ void split_bf16(float x, unsigned short& hi, unsigned short& lo) {
  hi = bf16_rne(x);
  const float h = __uint_as_float(((unsigned int)hi) << 16);
  lo = bf16_rne(x - h);
}

// Hardware RNE conversion (v_cvt_pk_bf16_f32) of two floats -> packed hi pair and lo pair
// (element 0 in the low half).  NaN stays NaN.
typedef float f32x2_t __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void split2_bf16(float a, float b, uint32_t& hi, uint32_t& lo) {
  const bf16x2_t h = __builtin_convertvector((f32x2_t){a, b}, bf16x2_t);
  const f32x2_t hf = __builtin_convertvector(h, f32x2_t);
  const bf16x2_t l = __builtin_convertvector((f32x2_t){a - hf.x, b - hf.y}, bf16x2_t);
  hi = __builtin_bit_cast(uint32_t, h);
  lo = __builtin_bit_cast(uint32_t, l);
}

// ---------------------------------------------------------------------------- fp16x2
// The conv2 kernels (conv2_fwd2.hip, conv2_bwd.hip) run on v_mfma_f32_16x16x32_f16 with ONE
// operand carried exactly (fp16 hi + fp16 lo, 22 significant bits) and the other rounded once
// to fp16 (11 significant bits): c += a*bhi + a*blo, 2 MFMAs per product instead of bf16x3's 3.
// Per-product relative error <= 2^-11 (the single operand's rounding) -- the unit roundoff of
// the TF32 convolutions cuDNN runs for the reference by default (10 explicit mantissa bits; TF32
// rounds BOTH operands, so its product error is up to 2^-10).  fp16's exponent range is
// narrower than fp32's: activations (p1, O(1)) fit as they are, the conv2 output gradient is
// carried with a power-of-two scale chosen per step from a bound of its magnitude.
typedef _Float16 f16x8_t __attribute__((ext_vector_type(8)));
typedef _Float16 f16x2_t __attribute__((ext_vector_type(2)));

__device__ __forceinline__ f32x4 mfma_f16(const s16x8& a, const s16x8& b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8_t, a), __builtin_bit_cast(f16x8_t, b), c, 0,
                                                0, 0);
}

// c += a * (bhi + blo) (small term first)
__device__ __forceinline__ f32x4 mfma_f16x2(const s16x8& a, const s16x8& bhi, const s16x8& blo, f32x4 c) {
  c = mfma_f16(a, blo, c);
  c = mfma_f16(a, bhi, c);
  return c;
}

// two floats -> packed fp16 pair (v_cvt_pk_f16_f32, round to nearest even; element 0 low)
__device__ __forceinline__ uint32_t cvt2_f16(float a, float b) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2_t){a, b}, f16x2_t));
}

// exact split of two floats: hi = f16(x), lo = f16(x - hi), each as a packed pair
__device__ __forceinline__ void split2_f16(float a, float b, uint32_t& hi, uint32_t& lo) {
  const f16x2_t h = __builtin_convertvector((f32x2_t){a, b}, f16x2_t);
  const f32x2_t hf = __builtin_convertvector(h, f32x2_t);
  const f16x2_t l = __builtin_convertvector((f32x2_t){a - hf.x, b - hf.y}, f16x2_t);
  hi = __builtin_bit_cast(uint32_t, h);
  lo = __builtin_bit_cast(uint32_t, l);
}

// The same split with lo formed by v_fma_mix{lo,hi}_f16: x - hi computed exactly and rounded once
// to fp16 (the value split2_f16 gets from cvt back, sub, cvt), 3 VALU per pair instead of 6.
// Bitwise equal to split2_f16 (tools/micro/f16_split_check.hip).
__device__ __forceinline__ void split2_f16_mix(float a, float b, uint32_t& hi, uint32_t& lo) {
  hi = __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2_t){a, b}, f16x2_t));
  asm("v_fma_mixlo_f16 %0, %1, -1.0, %2 op_sel_hi:[1,0,0]" : "=v"(lo) : "v"(hi), "v"(a));
  asm("v_fma_mixhi_f16 %0, %1, -1.0, %2 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "+v"(lo) : "v"(hi), "v"(b));
}

__device__ __forceinline__ void split_f16(float x, unsigned short& hi, unsigned short& lo) {
  uint32_t h, l;
  split2_f16(x, 0.f, h, l);
  hi = (unsigned short)(h & 0xffffu);
  lo = (unsigned short)(l & 0xffffu);
}

constexpr unsigned short kF16One = 0x3C00;

// lane ^ 1 (within each quad) through DPP quad_perm [1,0,3,2]: no LDS crossbar traffic
__device__ __forceinline__ float dpp_xor1(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0xB1, 0xF, 0xF, false));
}

__device__ __forceinline__ float bf16_to_f32(unsigned short h) { return __uint_as_float(((unsigned int)h) << 16); }

// ds_read_b64_tr_b16: per 16-lane group, lane 4q+p supplies the address of row q,
// columns 4p..4p+3; lane i gets column i of the 4 rows (element q = row q).
__device__ __forceinline__ s16x4 ds_read_tr16(const void* lds_ptr) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(lds_ptr));
}

}  // namespace tds
