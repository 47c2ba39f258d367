// conv2's weight packing as a workgroup body (conv2_pack.hip conv2_pack_weights_kernel runs it
// on 64 workgroups; the layer-1 reducer's launch runs it on extra workgroups of its own, so the
// packing costs no launch of its own: convnet_fused.hip l1_reduce_gram_kernel).  blk / nblk: this
// workgroup's index among the packing workgroups and their count; every thread must call it.
#pragma once
#include "conv2_common.h"

namespace tds {

__device__ __forceinline__ void conv2_pack_block(const float* __restrict__ w2, short* __restrict__ wp,
                                                 short* __restrict__ wd, uint32_t* __restrict__ mag,
                                                 const float* __restrict__ p1_scale, int write_p1, int blk,
                                                 int nblk) {
  const int FW = 13 * 2 * 4 * 16 * 8;  // fwd fragments
  const int DW = 25 * 4 * 16 * 8;      // dgrad fragments
  __shared__ float red[16];
  float wsc = 1.f;
  if (mag != nullptr) {
    float m = 0.f;
    const float4* w4 = reinterpret_cast<const float4*>(w2);  // (a contiguous fp32 tensor: 16-B aligned)
    float4 v[13];  // all loads in flight first (3200 float4 over 256 threads)
#pragma unroll
    for (int k = 0; k < 13; ++k) {
      // (clamped, not guarded: a guarded load is waited for inside its branch; a repeated element
      // leaves the max unchanged)
      v[k] = w4[min((int)threadIdx.x + k * 256, 32 * 16 * 25 / 4 - 1)];
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
    if (blk == 0) {
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
        if (write_p1) mag[kMagScales + 1] = __float_as_uint(p1_scale != nullptr ? 1.f / p1_scale[0] : 1.f);
        mag[kMagScales + 2] = __float_as_uint(ldexpf(1.f, ky));
        mag[kMagScales + 3] = __float_as_uint(ldexpf(1.f, kd));
      }
    }
  }
  for (int e = blk * blockDim.x + threadIdx.x; e < FW + DW; e += nblk * blockDim.x) {
    if (e < FW) {
      const int j = e & 7, co_in = (e >> 3) & 15, g = (e >> 7) & 3, nt = (e >> 9) & 1, s = e >> 10;
      const int ky = s < 10 ? (s >> 1) : 2 * (s - 10) + (g >> 1);
      const int kx = s < 10 ? 2 * (s & 1) + (g >> 1) : 4;
      const int ci = 8 * (g & 1) + j, co = nt * 16 + co_in;
      const float v = ky < 5 ? w2[(co * 16 + ci) * 25 + ky * 5 + kx] * wsc : 0.f;
      wp[e] = (short)f16_bits(v);  // rounded once (TF32 class, conv2_common.h)
    } else {
      const int f = e - FW;
      const int j = f & 7, ci = (f >> 3) & 15, g = (f >> 7) & 3, s = f >> 9;
      const int co = 8 * g + j;
      const float v = w2[(co * 16 + ci) * 25 + (24 - s)] * wsc;
      wd[f] = (short)f16_bits(v);
    }
  }
}

}  // namespace tds
