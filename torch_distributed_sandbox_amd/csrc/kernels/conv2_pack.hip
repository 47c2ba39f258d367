// conv2 of the ConvNet (Conv2d(16, 32, 5, stride 1, pad 2), mnist_onegpu.py:20): shared host
// pieces of the fp16 MFMA kernels (conv2_fwd2.hip, conv2_bwd.hip) -- the on-device weight
// packing into MFMA fragment order (w * 2^ew rounded once to fp16 in the TF32-class default; fp16
// hi + lo in the -DTDS_CONV2_SPLIT=1 build), the deterministic fp64 reduction of the per-workgroup weight
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
#include "launchers.h"

namespace tds {

// ---------------------------------------------------------------------------- weight packing
// fwd : wp[hl][s<13][nt<2][g<4][co16][j8], k = 32s+8g+j, ci = 8(g&1)+j, taps paired so that one
//       input-row A fragment serves every output row:  s < 10: (ky = s>>1, kx = 2(s&1) + (g>>1));
//       s = 10 + kp: (ky = 2kp + (g>>1), kx = 4)  (ky = 5 -> zero)
// dgrad: wd[hl][s<25][g<4][ci16][j8],      k = 32s+8g+j -> tap' = s, co = 8g+j; w = w2[co][ci][24-tap']
// mag (optional, kMagScales + 2 words): the step's magnitude bounds (max |y2| per channel, max
// |g2m|) are reset here, at the start of the conv2 forward they feed (conv2_fwd2.hip, head_pb.hip).
//
// fp16 range of the exactly carried weights: hi + lo represents w to ~2^-22 relative only while
// lo stays a normal fp16 (|w| >= ~2^-3); below fp16's normal range (|w| < 2^-14) even the
// per-product bound 2^-11 of fp16x2 breaks.  With mag given, the packed weights are w * 2^ew with
// max |w| * 2^ew in [2^14, 2^15) (every block finds max |w| itself over the 12 800 weights, by
// float4 loads from L2: no inter-block step), and mag[kMagScales] = 2^-ew, mag[kMagScales + 1] = 1 / p1_scale (the layer-1
// range guard, convnet_fused.hip l1_gram; 1 when not given) are what the conv2 forward and
// backward epilogues multiply their accumulators by (powers of two: exact); mag[kMagScales + 2]
// is the y2h store factor (conv2_common.h).  Without mag the weights are packed unscaled (and
// the forward stores y2h unscaled).
__global__ void conv2_pack_weights_kernel(const float* __restrict__ w2, short* __restrict__ wp,
                                          short* __restrict__ wd, uint32_t* __restrict__ mag,
                                          const float* __restrict__ p1_scale) {
  const int FW = 13 * 2 * 4 * 16 * 8;  // per hl plane (fwd)
  const int DW = 25 * 4 * 16 * 8;      // per hl plane (dgrad)
  __shared__ float red[16];
  float wsc = 1.f;
  if (mag != nullptr) {
    float m = 0.f;
    const float4* w4 = reinterpret_cast<const float4*>(w2);  // (a contiguous fp32 tensor: 16-B aligned)
    float4 v[13];  // all loads in flight first (3200 float4 over 256 threads)
#pragma unroll
    for (int k = 0; k < 13; ++k) {
      const int e = threadIdx.x + k * 256;
      v[k] = e < 32 * 16 * 25 / 4 ? w4[e] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int k = 0; k < 13; ++k)  // NaN: ignored
      m = fmaxf(m, fmaxf(fmaxf(fabsf(v[k].x), fabsf(v[k].y)), fmaxf(fabsf(v[k].z), fabsf(v[k].w))));
    m = wave_max(m);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
    __syncthreads();
    m = red[0];
    for (int i = 1; i < (int)(blockDim.x >> 6); ++i) m = fmaxf(m, red[i]);
    int ew = 0;
    if (m > 0.f && __builtin_isfinite(m)) {
      int x;
      (void)frexpf(m, &x);  // m < 2^x
      ew = min(100, max(-100, 15 - x));
    }
    wsc = ldexpf(1.f, ew);
    if (blockIdx.x == 0) {
      // the y2h store factor 2^k (conv2_common.h): L = max_c sum |w_c| (channel c = 100 float4,
      // 8 lanes each, summed in a fixed order), 1.01 * L * 2^ew * 2^k <= 1
      const int c = threadIdx.x >> 3, j = threadIdx.x & 7;
      float l1 = 0.f;
      for (int k = j; k < 100; k += 8) {
        const float4 q = w4[c * 100 + k];
        l1 += (fabsf(q.x) + fabsf(q.y)) + (fabsf(q.z) + fabsf(q.w));
      }
      l1 += __shfl_xor(l1, 1, 64);
      l1 += __shfl_xor(l1, 2, 64);
      l1 += __shfl_xor(l1, 4, 64);
      l1 = wave_max(l1);
      if ((threadIdx.x & 63) == 0) red[8 + (threadIdx.x >> 6)] = l1;
      __syncthreads();
      float L = red[8];
      for (int i = 1; i < (int)(blockDim.x >> 6); ++i) L = fmaxf(L, red[8 + i]);
      L *= 1.01f * wsc;
      int ky = 0;
      if (L > 0.f && __builtin_isfinite(L)) {
        int x;
        (void)frexpf(L, &x);  // L < 2^x
        ky = min(100, max(-100, -x));
      }
      // the dp1h store factor 2^kd (conv2_common.h): Ld = max_ci sum_{co,tap} |w| (16 lanes per ci,
      // co = lane and lane + 16, fixed order), 1.01 * 2^15 * Ld * 2^ew * 2^kd <= 65504
      __syncthreads();  // red[8..] read above
      {
        const int ci = threadIdx.x >> 4, j = threadIdx.x & 15;
        float ld = 0.f;
        for (int co = j; co < 32; co += 16)
          for (int tp = 0; tp < 25; ++tp) ld += fabsf(w2[(co * 16 + ci) * 25 + tp]);
        ld += __shfl_xor(ld, 1, 64);
        ld += __shfl_xor(ld, 2, 64);
        ld += __shfl_xor(ld, 4, 64);
        ld += __shfl_xor(ld, 8, 64);
        ld = wave_max(ld);
        if ((threadIdx.x & 63) == 0) red[8 + (threadIdx.x >> 6)] = ld;
      }
      __syncthreads();
      float Ld = red[8];
      for (int i = 1; i < (int)(blockDim.x >> 6); ++i) Ld = fmaxf(Ld, red[8 + i]);
      Ld *= 1.01f * 32768.f / 65504.f * wsc;
      int kd = 0;
      if (Ld > 0.f && __builtin_isfinite(Ld)) {
        int x;
        (void)frexpf(Ld, &x);  // Ld < 2^x
        kd = min(100, max(-100, -x));
      }
      if (threadIdx.x < 33) mag[threadIdx.x] = 0u;
      if (threadIdx.x == 0) {
        mag[kMagScales] = __float_as_uint(ldexpf(1.f, -ew));
        mag[kMagScales + 1] = __float_as_uint(p1_scale != nullptr ? 1.f / p1_scale[0] : 1.f);
        mag[kMagScales + 2] = __float_as_uint(ldexpf(1.f, ky));
        mag[kMagScales + 3] = __float_as_uint(ldexpf(1.f, kd));
      }
    }
  }
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < FW + DW; e += gridDim.x * blockDim.x) {
    if (e < FW) {
      const int j = e & 7, co_in = (e >> 3) & 15, g = (e >> 7) & 3, nt = (e >> 9) & 1, s = e >> 10;
      const int ky = s < 10 ? (s >> 1) : 2 * (s - 10) + (g >> 1);
      const int kx = s < 10 ? 2 * (s & 1) + (g >> 1) : 4;
      const int ci = 8 * (g & 1) + j, co = nt * 16 + co_in;
      const float v = ky < 5 ? w2[(co * 16 + ci) * 25 + ky * 5 + kx] * wsc : 0.f;
      unsigned short hi, lo;
      split_f16(v, hi, lo);
      wp[e] = (short)hi;
      wp[FW + e] = (short)lo;
    } else {
      const int f = e - FW;
      const int j = f & 7, ci = (f >> 3) & 15, g = (f >> 7) & 3, s = f >> 9;
      const int co = 8 * g + j;
      const float v = w2[(co * 16 + ci) * 25 + (24 - s)] * wsc;
      unsigned short hi, lo;
      split_f16(v, hi, lo);
      wd[f] = (short)hi;
      wd[DW + f] = (short)lo;
    }
  }
}

// dw2[co][ci][tap] = sum_wg slab (fixed order, fp64), db2[co] = sum_wg slab[tap 25][co][0].
// A block owns 64 consecutive slab elements; its 4 waves sum interleaved quarters of the
// workgroup rows (w = 4j + wave, 8 loads in flight per lane), then wave 0 adds the four
// partials in a fixed order: deterministic, and 4x the parallelism of one lane per element.
__global__ __launch_bounds__(256) void conv2_wgrad_reduce_kernel(const float* __restrict__ slab, int nwg,
                                                                 float* __restrict__ dw, float* __restrict__ db,
                                                                 float scale) {
  __shared__ double part[4][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int e = blockIdx.x * 64 + lane;  // over 26*32*16
  double s = 0.0;
  if (e < 26 * 512) {
    int w = wv;
    for (; w + 28 < nwg; w += 32) {
      float v[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = slab[(int64_t)(w + 4 * k) * 26 * 512 + e];
#pragma unroll
      for (int k = 0; k < 8; ++k) s += (double)v[k];
    }
    for (; w < nwg; w += 4) s += (double)slab[(int64_t)w * 26 * 512 + e];
  }
  part[wv][lane] = s;
  __syncthreads();
  if (wv != 0 || e >= 26 * 512) return;
  const double tot = ((part[0][lane] + part[1][lane]) + part[2][lane]) + part[3][lane];
  const int tap = e / 512, co = (e / 16) & 31, ci = e & 15;
  const float v = (float)tot * scale;
  if (tap < 25) dw[(co * 16 + ci) * 25 + tap] = v;
  else if (db && ci == 0) db[co] = v;
}

}  // namespace tds

using namespace tds;

void tds_conv2_pack_weights(const float* w2, short* wp, short* wd, uint32_t* mag, const float* p1_scale,
                            hipStream_t st) {
  hipLaunchKernelGGL(conv2_pack_weights_kernel, dim3(64), dim3(256), 0, st, w2, wp, wd, mag, p1_scale);
  TDS_LAUNCH_CHECK();
}

int tds_conv2_num_wg() { return tds_device_cus(); }

int tds_conv2_split() { return kConv2Split ? 1 : 0; }  // the build's conv2 operand precision (conv2_common.h)

void tds_conv2_wgrad_reduce(const float* slab, int nwg, float* dw, float* db, float scale, hipStream_t st) {
  hipLaunchKernelGGL(conv2_wgrad_reduce_kernel, dim3(26 * 512 / 64), dim3(256), 0, st, slab, nwg, dw, db, scale);
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
