// Shared pieces of the conv2 kernels (conv2_fwd2.hip, conv2_bwd.hip): the operand / MFMA
// wrappers, parameterised by a timing-only diagnostic variant that only a -DTDS_DIAG build
// can select (tools/conv2_diag.py, TDS_CONV2_DIAG); production builds instantiate DIAG = 0.
#pragma once

#include "bf16x3.h"

namespace tds {

// Words of the step's magnitude workspace ("mag", fused_ops.cpp) past the 33 bounds: written by
// conv2_pack_weights_kernel, read by the conv2 forward / backward epilogues (powers of two).
constexpr int kMagScales = 40;  // mag[40] = 2^-ew (packed weights' scale), mag[41] = 1 / p1 scale,
                                // mag[42] = 2^k, the y2h store factor (conv2_fwd2.hip),
                                // mag[43] = 2^kd, the dp1h store factor (conv2_bwd.hip),
                                // mag[44] = the dp1h decode (written by the conv2 backward)

// ---------------------------------------------------------------------------- dp1h
// The conv2 data gradient dp1 travels to the layer-1 backward as dp1h [B][P][PG = ceil(P/4)][16 ch]
// [4 px] fp16: h = fp16(acc * 2^kd), acc the dgrad accumulator (dp1 = acc * 2^-e * 2^-ew).  The
// dy2 operand is below 2^15 by its scale e, so |acc| <= 2^15 max_ci sum |w~_ci| and conv2_pack
// picks 2^kd with 1.01 * 2^15 * max_ci sum_{co,tap} |w_co,ci,tap| * 2^ew * 2^kd <= 65504: no
// overflow, 11 significant bits (the TF32 rounding the reference's conv1 weight gradient applies
// to this operand).  The layout is the dgrad MFMA's: a lane's 4 columns of one channel are 8
// contiguous bytes, a wave-instruction 512 contiguous bytes of one row.

// ---------------------------------------------------------------------------- y2h
// The conv2 output travels from the forward to the backward as y2h [B][P][P][32] fp16 (64 B per
// pixel, half of fp32): y2h = fp16(acc * 2^k), acc the bias-free MFMA accumulator (y2 = acc * inv
// + b2), 2^k from conv2_pack: max_c sum |w_c| * 2^ew * 1.01 * 2^k <= 1, so with |p1 operand| <=
// 65504 no value can overflow, and everything above 2^-14 of the fp16 grid keeps 11 significant
// bits (TF32's).  Rounding is to nearest.  The pooling argmax does not come from these values:
// the forward stores it (a2 below), as max_pool2d_with_indices saves its indices for its backward.
//
// a2 [B][Q][Q][2] uint32 (Q = P / 2, the pooled windows): each 2x2 window's argmax in scan order
// (0 = (0,0), 1 = (0,1), 2 = (1,0), 3 = (1,1)) of the forward's fp32 conv2 output -- the first
// extreme, max for gamma2 >= 0 and min for gamma2 < 0 (BN2's affine is monotone in the sign of
// gamma2, so this is the first max of the BN2 output) -- as 2-bit codes of 16 channels per word:
// word h holds channels 16h .. 16h+15, bit c = code bit 0, bit 16 + c = code bit 1 of channel
// 16h + c.  8 B per window (22.5 MB at the bench shape); written by conv2_fwd2, read by the
// conv2 backward's staging.
__device__ __forceinline__ uint32_t f16_bits(float x) {
  return (uint32_t)__builtin_bit_cast(unsigned short, (_Float16)x);
}
__device__ __forceinline__ float f16_val(uint32_t h) {
  return (float)__builtin_bit_cast(_Float16, (unsigned short)(h & 0xFFFFu));
}

// ---------------------------------------------------------------------------- diagnostics
// DIAG = 0: the real kernel.  Timing-only builds (tools/conv2_diag.py, TDS_CONV2_DIAG):
//   1: no MFMAs (operand reads kept alive by one VALU op),  2: no LDS operand reads
//   (register constants), 3: no global tile loads (LDS holds whatever it held).
// conv2 backward, DIAG >= 16: flag sets, per-role barrier clocks always on (conv2_bwd.hip):
//   +1 no staging, +2 no LDS operand reads in the MFMA waves, +4 dgrad waves idle, +8 wgrad
//   waves idle (an idle role only takes part in the per-tile barriers), +32 staging without its
//   global loads, +64 staging without the BN2 / pool backward math
constexpr bool diag_no_lds(int D) { return D == 2 || (D >= 16 && (D & 2)); }
// Operand precision of the three conv2 products (forward, data gradient, weight gradient): ONE
// v_mfma_f32_16x16x32_f16 per product, both operands rounded once to fp16 -- 11 significant bits,
// exactly TF32's significand (10 explicit bits + the implicit one), products exact, fp32
// accumulation: the arithmetic of the reference's cuDNN convolutions under PyTorch's default
// allow_tf32 (Ampere).  fp16's narrower exponent range is covered by exact power-of-two scales:
// the packed weights' (conv2_pack.hip), p1's range guard (convnet_fused.hip) and dy2's
// magnitude-bound scale (conv2_bwd.hip) keep each operand's largest value in [2^14, 2^16), so
// values down to 2^-28 of it are normal fp16.  (Rounds 2-3 carried one operand as fp16 hi + lo,
// two MFMAs per product; that build is in git history.)
template <int DIAG>
__device__ __forceinline__ f32x4 mmaw(const s16x8& a, const s16x8& b, f32x4 c) {
  if constexpr (DIAG == 1) {
    c[0] += (float)((int)(a[0] ^ b[2]) & 1);
    return c;
  } else {
    return mfma_f16(a, b, c);
  }
}
template <int DIAG>
__device__ __forceinline__ s16x8 lds8(const void* p) {
  if constexpr (diag_no_lds(DIAG)) {
    const short v = (short)(threadIdx.x & 7);
    return s16x8{v, v, v, v, v, v, v, v};
  } else {
    return *reinterpret_cast<const s16x8*>(p);
  }
}
template <int DIAG>
__device__ __forceinline__ s16x4 ldtr(const void* p) {
  if constexpr (diag_no_lds(DIAG)) {
    const short v = (short)(threadIdx.x & 7);
    return s16x4{v, v, v, v};
  } else {
    return ds_read_tr16(p);
  }
}

// ---------------------------------------------------------------------------- tile order
// L2-blocked tile order for the persistent conv kernels (built on the host by
// tds_tile_order_fill, conv2_pack.hip; device table from the torch caching allocator, one int
// per work index: b << 24 | tile_row << 12 | tile_col).  xcd_remap hands each XCD a contiguous
// run of 64 work indices per round (grid = 512 = 8 XCDs x 64 workgroups), and t -> t + grid is
// the same workgroup's next tile.  A plain row-major order makes those 64 tiles a 1-D strip,
// so the 2-pixel halo above/below each tile (a third of the staged rows) is fetched again a
// round later, long after it left the XCD's 4 MiB L2.  The table walks, per image, bands of 32
// tile-columns; each band in row groups of 16 tile-rows; each row group in column groups of 4:
// one XCD round = one 16 x 4 block of tiles (its halos fetched once, concurrently, into one
// L2), the 8 XCDs take the 8 blocks of a band row side by side, and the next round is the
// block right below (its top halo still in L2).  A decode is one scalar load instead of six
// runtime integer divisions on the scalar unit.
__device__ __forceinline__ void tile_from_order(const int* __restrict__ order, int t, int& b, int& tr, int& tc) {
  const int v = order[t];
  b = v >> 24;
  tr = (v >> 12) & 4095;
  tc = v & 4095;
}

}  // namespace tds
