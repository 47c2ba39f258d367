// conv2 of the ConvNet (Conv2d(16, 32, 5, stride 1, pad 2), mnist_onegpu.py:20): shared host
// pieces of the fp16 MFMA kernels (conv2_fwd2.hip, conv2_bwd.hip) -- the on-device weight
// packing into MFMA fragment order (w * 2^ew rounded once to fp16: the TF32 class), the
// deterministic fp64 reduction of the per-workgroup weight
// gradient slabs, and the blocked tile order table.  SURVEY.md §2.4 K5 / K19 / K20.
//
// Activation formats (produced/consumed by convnet_fused.hip and the conv2 kernels):
//   p1  [B][P][P][16] fp16                                          (pooled layer-1 output)
//   y2h [B][P][P][32] fp16                        (conv2 output: bias-free, scaled; conv2_common.h)
//   dp1h [B][P][ceil(P/4)][16][4] fp16           (grad wrt p1: scaled, dgrad-MFMA layout; conv2_common.h)
// MFMA mapping (v_mfma_f32_16x16x32_f16, lane l: i = l&15, g = l>>4):
//   A[i][k = 8g+j] (8 consecutive k per lane), B[k = 8g+j][n = i], C row = 4g+r, col = i.
#include <vector>

#include "conv2_common.h"
#include "conv2_pack.h"
#include "launchers.h"

namespace tds {

// ---------------------------------------------------------------------------- weight packing
// fwd : wp[s<13][nt<2][g<4][co16][j8], k = 32s+8g+j, ci = 8(g&1)+j, taps paired so that one
//       input-row A fragment serves every output row:  s < 10: (ky = s>>1, kx = 2(s&1) + (g>>1));
//       s = 10 + kp: (ky = 2kp + (g>>1), kx = 4)  (ky = 5 -> zero)
// dgrad: wd[s<25][g<4][ci16][j8],      k = 32s+8g+j -> tap' = s, co = 8g+j; w = w2[co][ci][24-tap']
// mag (optional, kMagScales + 2 words): the step's magnitude bounds (max |y2| per channel, max
// |g2m|) are reset here, at the start of the conv2 forward they feed (conv2_fwd2.hip, head_pb.hip).
//
// fp16 range of the weights: below fp16's normal range (|w| < 2^-14) the 11-bit rounding breaks,
// so with mag given the packed weights are w * 2^ew with
// max |w| * 2^ew in [2^14, 2^15) (every block finds max |w| itself over the 12 800 weights, by
// float4 loads from L2: no inter-block step), and mag[kMagScales] = 2^-ew, mag[kMagScales + 1] = 1 / p1_scale (the layer-1
// range guard, convnet_fused.hip l1_gram; 1 when not given) are what the conv2 forward and
// backward epilogues multiply their accumulators by (powers of two: exact); mag[kMagScales + 2]
// is the y2h store factor (conv2_common.h).  Without mag the weights are packed unscaled (and
// the forward stores y2h unscaled).
__global__ void conv2_pack_weights_kernel(const float* __restrict__ w2, short* __restrict__ wp,
                                          short* __restrict__ wd, uint32_t* __restrict__ mag,
                                          const float* __restrict__ p1_scale, int write_p1) {
  conv2_pack_block(w2, wp, wd, mag, p1_scale, write_p1, blockIdx.x, gridDim.x);  // (conv2_pack.h)
}

// dw2[co][ci][tap] = sum_wg slab (fixed order, fp64), db2[co] = sum_wg slab[tap 25][co][0].
// A block owns 64 consecutive slab elements; its WGR_WAVES waves sum interleaved shares of the
// workgroup rows (w = WGR_WAVES * j + wave, 16 loads in flight per lane, rows past the end clamped
// and added as 0.0, which keeps the sum), then wave 0 adds the partials in a fixed order: deterministic.  At 4 waves the
// 256 rows take 4 rounds of loads, at 16 one.
constexpr int WGR_WAVES = 16;  // (r5_s47: 4.9 us at 4 waves with clamped loads, 4.8 at 16; guarded loads 20 us at 4)
__global__ __launch_bounds__(64 * WGR_WAVES) void conv2_wgrad_reduce_kernel(const float* __restrict__ slab, int nwg,
                                                                            float* __restrict__ dw,
                                                                            float* __restrict__ db, float scale) {
  constexpr int NW = WGR_WAVES;
  __shared__ double part[NW][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int e = blockIdx.x * 64 + lane;  // over 26*32*16
  double s = 0.0;
  if (e < 26 * 512) {
    for (int w = wv; w < nwg; w += 16 * NW) {
      float v[16];
#pragma unroll
      for (int k = 0; k < 16; ++k) v[k] = slab[(int64_t)min(w + NW * k, nwg - 1) * 26 * 512 + e];  // (clamped:
      // a load under a branch is waited for inside it, which serialises the batch)
#pragma unroll
      for (int k = 0; k < 16; ++k) s += w + NW * k < nwg ? (double)v[k] : 0.0;
    }
  }
  part[wv][lane] = s;
  __syncthreads();
  if (wv != 0 || e >= 26 * 512) return;
  double tot = part[0][lane];
#pragma unroll
  for (int i = 1; i < NW; ++i) tot += part[i][lane];
  const int tap = e / 512, co = (e / 16) & 31, ci = e & 15;
  const float v = (float)tot * scale;
  if (tap < 25) dw[(co * 16 + ci) * 25 + tap] = v;
  else if (db && ci == 0) db[co] = v;
}

}  // namespace tds

using namespace tds;

void tds_conv2_pack_weights(const float* w2, short* wp, short* wd, uint32_t* mag, const float* p1_scale,
                            hipStream_t st, bool write_p1) {
  hipLaunchKernelGGL(conv2_pack_weights_kernel, dim3(64), dim3(256), 0, st, w2, wp, wd, mag, p1_scale,
                     write_p1 ? 1 : 0);
  TDS_LAUNCH_CHECK();
}

int tds_conv2_num_wg() { return tds_device_cus(); }

void tds_conv2_wgrad_reduce(const float* slab, int nwg, float* dw, float* db, float scale, hipStream_t st) {
  hipLaunchKernelGGL(conv2_wgrad_reduce_kernel, dim3(26 * 512 / 64), dim3(64 * WGR_WAVES), 0, st, slab, nwg, dw, db, scale);
  TDS_LAUNCH_CHECK();
}

// Blocked tile order (conv2_common.h) into a host array of B * tiles_r * tiles_c ints:
// b << 24 | tile_row << 12 | tile_col.  Bands of 32 tile columns, row groups of GR tile rows,
// column groups of 4 (one XCD round of the forward's 512 workgroups = one 16 x 4 block).  The
// binding layer copies it to a device tensor from the torch caching allocator and caches it
// per (shape, GR).
int tds_tile_order_fill(int* out, int B, int tiles_r, int tiles_c, int GR) {
  if (B < 1 || B > 255 || tiles_r < 1 || tiles_r > 4095 || tiles_c < 1 || tiles_c > 4095 || GR < 1) return -1;
  constexpr int BC = 32, GC = 4;
  const int per_img = tiles_r * tiles_c, total = per_img * B;
  for (int t = 0; t < total; ++t) {
    const int b = t / per_img;
    int off = t - b * per_img;
    const int band = off / (BC * tiles_r);
    off -= band * BC * tiles_r;
    const int wj = std::min(BC, tiles_c - band * BC);
    const int gr = off / (GR * wj);
    off -= gr * GR * wj;
    const int hg = std::min(GR, tiles_r - gr * GR);
    const int cg = off / (GC * hg);
    off -= cg * GC * hg;
    const int wc = std::min(GC, wj - cg * GC);
    const int r = off / wc;
    out[t] = (b << 24) | ((gr * GR + r) << 12) | (band * BC + cg * GC + (off - r * wc));
  }
  return 0;
}
