// The input op and the x moments in ONE pass: the 28x28 -> HxW bilinear upsample to uint8 levels
// (the bench's and trainer's input pipeline, ops/functional.py upsample_bilinear_u8(levels=True))
// that also forms the autocorrelation partials behind BN1's closed-form statistics
// (x_autocorr.hip x_autocorr_u8_kernel: the same 42 sums, the same exact u32 dot4 arithmetic),
// from the levels while they are in registers -- instead of writing the 45 MB image and reading it
// back in a second, VALU-bound launch (upsample 26 us + autocorrelation 64 us per step, r5_s18).
// Every one of the B*H*W pixels is computed and every product of the 41 offsets formed, exactly
// as the two kernels did; the levels written are bit-identical to upsample_bilinear_u8's
// (ups_common.h: one arithmetic for both).  The border strips come from the reducer's launch
// (xmom_u8.h), which reads the written image.
//
// Work unit = one wave (a 64-thread workgroup: the scheduler balances single waves, and 4095 of
// them fill 4 waves on each of the 1024 SIMDs at the bench shape): UM_RB output rows x up to 62
// 4-pixel quads.  Lane l computes quad q0 + l - 1 of every row; lanes 0 and qpw + 1 compute the
// neighbours' edge quads (halo), which the wave-wide DPP shifts hand to lanes 1 and qpw as the
// columns c-4 .. c-1 / c+4 .. c+7 every offset reaches.  Rows r0 .. r0 + UM_RB + 3 are computed
// (the 4 rows below the band are the partners of its last rows: recomputed, not stored); a 5-row
// ring of each row's 9 byte windows (6 v_alignbyte per row, once) feeds 41 v_dot4_u32_u8 + 1
// plain-sum dot4 per quad and row, ring slots static (the row loop unrolled by 5).  The source
// image (784 floats) sits in LDS; a thread keeps its columns' horizontal taps and the two
// horizontally interpolated source rows of the current vertical tap pair, recomputed when the
// pair changes (about every H/h rows).
#include "common.h"
#include "launchers.h"
#include "ups_common.h"
#include "xmom_u8.h"

namespace tds {

// (isolated op, r5_s35: 32 rows 48.1 - 48.6 us, 40: 47.0 - 48.6, 48: 45.8 - 46.2, 64: 45.3 - 46.7)
constexpr int UM_RB = 48;         // output rows per wave
constexpr int UM_QPW = 62;        // quads per wave at most (lanes 1..62 own them)
// a lane's sums: UM_RB rows x 4 products <= 255^2 each; the wave's: 62 lanes
static_assert((unsigned long long)UM_RB * 4ull * 62ull * 65025ull < (1ull << 32), "u32 wave sums would wrap");

struct UmGeo {
  int nqg, qpw, nband;
};
static UmGeo um_geo(int H, int W) {
  UmGeo g;
  const int nq = W / 4;
  g.nqg = (nq + UM_QPW - 1) / UM_QPW;
  g.qpw = (nq + g.nqg - 1) / g.nqg;
  g.nband = (H + UM_RB - 1) / UM_RB;
  return g;
}

__device__ __forceinline__ uint32_t um_shr1(uint32_t v) {  // lane l <- lane l - 1 (lane 0 <- 0)
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x138, 0xF, 0xF, true);
}
__device__ __forceinline__ uint32_t um_shl1(uint32_t v) {  // lane l <- lane l + 1 (lane 63 <- 0)
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x130, 0xF, 0xF, true);
}

typedef float um_f2 __attribute__((ext_vector_type(2)));

__global__ __launch_bounds__(64) void ups_moments_u8_kernel(const uint8_t* __restrict__ src,
                                                            uint8_t* __restrict__ x, double* __restrict__ partial,
                                                            int h, int w, int H, int W, int nqg, int qpw) {
  extern __shared__ float img[];  // h * w
  const int b = blockIdx.y, unit = blockIdx.x, units = gridDim.x;
  const int lane = threadIdx.x;
  const uint8_t* s = src + (int64_t)b * h * w;
  if (((h * w) & 3) == 0) {  // the source in words, every load issued before the first conversion
    const uint32_t* s4 = reinterpret_cast<const uint32_t*>(s);
    const int n4 = (h * w) >> 2;
    for (int i0 = 0; i0 < n4; i0 += 4 * 64) {
      uint32_t v[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) v[k] = s4[min(i0 + k * 64 + lane, n4 - 1)];  // (clamped: used only in range)
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int i = i0 + k * 64 + lane;
        if (i < n4) {
          img[4 * i] = (float)(v[k] & 0xFF);
          img[4 * i + 1] = (float)((v[k] >> 8) & 0xFF);
          img[4 * i + 2] = (float)((v[k] >> 16) & 0xFF);
          img[4 * i + 3] = (float)(v[k] >> 24);
        }
      }
    }
  } else {
    for (int i = lane; i < h * w; i += 64) img[i] = (float)s[i];
  }
  __syncthreads();
  const int qg = unit % nqg, band = unit / nqg;
  const int q = qg * qpw + lane - 1;
  const bool vq = lane <= qpw + 1 && q >= 0 && q < (W >> 2);
  const bool own = vq && lane >= 1 && lane <= qpw;
  const float sy = (float)h / (float)H, sx = (float)w / (float)W;
  int x0[4], x1[4];
  float ax[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) ups_taps(vq ? 4 * q + k : 0, sx, w, x0[k], x1[k], ax[k]);
  um_f2 top[2], bot[2];  // pixels 0,1 | 2,3
  int ycur = -1;
  uint32_t acc[42];
#pragma unroll
  for (int i = 0; i < 42; ++i) acc[i] = 0u;
  uint32_t ring[5][9];
  const int r0 = band * UM_RB;
  // the vertical taps of the wave's rows r0 .. r0 + UM_RB + 3, lane i holding row r0 + i's (read
  // back per row with v_readlane: one instruction each instead of the tap arithmetic per row)
  static_assert(UM_RB + 4 <= 64, "one lane per row of the band");
  int ty0 = 0, ty1 = 0;
  float tay = 0.f;
  ups_taps(min(r0 + lane, H - 1), sy, h, ty0, ty1, tay);
  uint32_t* xrow = reinterpret_cast<uint32_t*>(x + ((int64_t)b * H + r0) * W) + q;
#pragma unroll 1
  for (int i0 = 0; i0 < UM_RB + 4; i0 += 5) {
#pragma unroll
    for (int j = 0; j < 5; ++j) {
      const int i = i0 + j, r = r0 + i;
      if (i < UM_RB + 4) {
        uint32_t cur = 0u;
        if (r < H) {
          const int y0 = __builtin_amdgcn_readlane(ty0, i), y1 = __builtin_amdgcn_readlane(ty1, i);
          const float ay = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, tay), i));
          if (y0 != ycur) {  // wave-uniform: a new vertical tap pair
            ycur = y0;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
              top[k >> 1][k & 1] = ups_lerp(img[y0 * w + x0[k]], img[y0 * w + x1[k]], ax[k]);
              bot[k >> 1][k & 1] = ups_lerp(img[y1 * w + x0[k]], img[y1 * w + x1[k]], ax[k]);
            }
          }
          // ups_level(ups_lerp(top, bot, ay)) two pixels per packed op: the lerp is ups_lerp's
          // fmaf(ay, bot, (1 - ay) * top) elementwise, and a convex combination of levels lies in
          // [0, 255 + 2^-15], so adding 1.5 * 2^23 rounds it to the nearest integer (ties to even, as
          // rintf) into the low mantissa byte and the clamp never binds: the same level
          const um_f2 ay2 = {ay, ay}, na2 = {1.f - ay, 1.f - ay}, mag = {12582912.f, 12582912.f};
          const um_f2 m01 = __builtin_elementwise_fma(ay2, bot[0], na2 * top[0]) + mag;
          const um_f2 m23 = __builtin_elementwise_fma(ay2, bot[1], na2 * top[1]) + mag;
          // (__float_as_uint of the element VALUE: clang's __builtin_bit_cast of an ext-vector element
          // lvalue read element 0 for every index)
          const uint32_t l0 = __float_as_uint(m01.x) & 0xFFu, l1 = __float_as_uint(m01.y) & 0xFFu;
          const uint32_t l2 = __float_as_uint(m23.x) & 0xFFu, l3 = __float_as_uint(m23.y) & 0xFFu;
          cur = vq ? (l0 | (l1 << 8) | (l2 << 16) | (l3 << 24)) : 0u;
          if (own && i < UM_RB) xrow[(int64_t)i * (W >> 2)] = cur;
        }
        const uint32_t left = um_shr1(cur), right = um_shl1(cur);
#pragma unroll
        for (int s9 = 0; s9 < 9; ++s9) ring[j][s9] = xm_win(left, cur, right, s9);
        if (i >= 4) {  // the band's row i - 4 against rows i - 4 .. i (ring slots j+1 .. j+5 mod 5)
          const uint32_t u = own ? ring[(j + 1) % 5][4] : 0u;
          int k = 0;
#pragma unroll
          for (int dx = 0; dx <= 4; ++dx, ++k) acc[k] = __builtin_amdgcn_udot4(u, ring[(j + 1) % 5][4 + dx], acc[k], false);
#pragma unroll
          for (int dy = 1; dy <= 4; ++dy)
#pragma unroll
            for (int dx = -4; dx <= 4; ++dx, ++k)
              acc[k] = __builtin_amdgcn_udot4(u, ring[(j + 1 + dy) % 5][4 + dx], acc[k], false);
          acc[41] = __builtin_amdgcn_udot4(u, 0x01010101u, acc[41], false);
        }
      }
    }
  }
  // wave sums (exact in u32), one partial row per wave
  double out = 0.0;
#pragma unroll
  for (int k = 0; k < 42; ++k) {
    const uint32_t v = xm_wave_sum(acc[k]);
    if (lane == k) out = (double)v;
  }
  if (lane < 42) partial[((int64_t)b * units + unit) * 42 + lane] = out;
}

}  // namespace tds

using namespace tds;

// partial rows [B * units][42] the fused upsample + moments writes; 0 = shape unsupported
int tds_ups_moments_rows(int B, int h, int w, int H, int W) {
  if (B < 1 || B > 65535 || h < 1 || w < 1 || h * w > kUpsImg || W % 4 != 0 || W < 8 || H < 8) return 0;
  const UmGeo g = um_geo(H, W);
  return B * g.nband * g.nqg;
}

void tds_ups_moments_u8(const uint8_t* src, uint8_t* x, double* partial, int nrows, int B, int h, int w, int H, int W,
                        hipStream_t st) {
  if (nrows < 1 || nrows != tds_ups_moments_rows(B, h, w, H, W)) {
    tds_launch_fail("ups_moments_u8: partial row count does not match the shape");
    return;
  }
  const UmGeo g = um_geo(H, W);
  hipLaunchKernelGGL(ups_moments_u8_kernel, dim3(g.nband * g.nqg, B), dim3(64), (size_t)h * w * sizeof(float), st, src,
                     x, partial, h, w, H, W, g.nqg, g.qpw);
  TDS_LAUNCH_CHECK();
}
