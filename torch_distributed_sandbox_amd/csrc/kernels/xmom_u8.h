// Border strips of the uint8 x moments, computed by one 256-thread workgroup per (image, side) inside
// the launch that reduces the autocorrelation partials (convnet_fused.hip l1_reduce_gram_kernel):
// strips[b][L][d] = sum over line L of x(u) x(u + d), d in [-4,4]^2, d index 81 = the plain line sum;
// L 0,1 = rows 0,1, 2,3 = rows H-2,H-1, 4,5 = cols 0,1, 6,7 = cols W-2,W-1 (l1_build_gram's layout),
// summed over the batch.
// A side's six outermost lines (the two strip lines and every partner line a |d| <= 4 reaches
// inside the image) go through LDS in chunks of BSIDE_CH positions, loaded once -- the
// per-(d, line) workgroups of x_autocorr.hip's merged launch re-read every line 82 times, column
// lines one scattered byte per load (16 us of that launch at the bench shape, r5_s22) -- and
// each wave takes (strip line, perpendicular offset) pairs, 9 along-line offsets each with one
// v_dot4_u32_u8 per 4 positions.  The sums are exact integers: N * 255^2 < 2^32 for N <= 66051.
#pragma once
#include "common.h"

namespace tds {

constexpr int BSIDE_CH = 1024;                // positions per chunk
constexpr int BSIDE_LD = BSIDE_CH / 4 + 2;    // words per stored line: one pad word each end
constexpr int BSIDE_LDS_WORDS = 6 * BSIDE_LD;
constexpr int XMOM_MAX_LINE = 66051;          // longest line whose u32 sums cannot wrap

// line chunks per side: one workgroup each (all in flight together)
__host__ __device__ inline int xmom_border_chunks(int H, int W) {
  return ((H > W ? H : W) + BSIDE_CH - 1) / BSIDE_CH;
}

// wave sum of a u32: quad / half-row / row steps as DPP adds, the two cross-row steps as swizzles
__device__ __forceinline__ uint32_t xm_wave_sum(uint32_t v) {
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);   // quad_perm [1,0,3,2]
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false);   // quad_perm [2,3,0,1]
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x141, 0xF, 0xF, false);  // row_half_mirror
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x140, 0xF, 0xF, false);  // row_mirror
  v += __shfl_xor(v, 16, 64);
  v += __shfl_xor(v, 32, 64);
  return v;
}

// bytes s .. s+3 of the 12 bytes (w0 | w1 | w2), s in 0..8
__device__ __forceinline__ uint32_t xm_win(uint32_t w0, uint32_t w1, uint32_t w2, int s) {
  return s == 0 ? w0 : s < 4 ? __builtin_amdgcn_alignbyte(w1, w0, s) : s == 4 ? w1
       : s < 8 ? __builtin_amdgcn_alignbyte(w2, w1, s - 4) : w2;
}

// Chunk ch (of nch) of side 0 top, 1 bottom, 2 left, 3 right of image b: its partial sums added
// into sacc[L][82] (the batch's strips, exact u64 integer sums: any order gives the same value;
// agent-scope atomics, which the reducer sees after tds_arrive's acquire); lines: BSIDE_LDS_WORDS
// words of LDS.  Every thread of the workgroup must call it.
__device__ __forceinline__ void x_border_side_u8(const uint8_t* __restrict__ x, unsigned long long* __restrict__ sacc,
                                                 int b, int side, int ch, int nch, int H, int W, uint32_t* lines) {
  const bool rows = side < 2;
  const int N = rows ? W : H;                                  // positions along a line
  const int first = (side & 1) ? (rows ? H - 6 : W - 6) : 0;   // image row / col of stored line 0
  const int l0 = (side & 1) ? 4 : 0;                           // stored index of the first strip line
  const int tid = (int)threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const __amdgpu_buffer_rsrc_t rx = tds_buffer_rsrc(x + (int64_t)b * H * W, (uint32_t)((int64_t)H * W));
  constexpr uint32_t kOob = 0xFFFFFFF0u;
  uint8_t* lb = reinterpret_cast<uint8_t*>(lines);
  uint32_t acc[5][9];
#pragma unroll
  for (int m = 0; m < 5; ++m)
#pragma unroll
    for (int s = 0; s < 9; ++s) acc[m][s] = 0u;
  uint32_t plain = 0u;
  {
    const int c0 = ch * BSIDE_CH;
    if (rows) {
      // word k of stored line t = image row first + t, positions c0 - 4 + 4k .. +3 (W % 4 == 0:
      // a word lies inside the row or outside it whole); all loads issued before the LDS writes
      constexpr int NIT = (BSIDE_LDS_WORDS + 255) / 256;
      uint32_t v[NIT];
#pragma unroll
      for (int it = 0; it < NIT; ++it) {
        const int e = tid + it * 256, t = e / BSIDE_LD, k = e % BSIDE_LD;
        const int line = first + t, p = c0 - 4 + 4 * k;
        const bool in = e < BSIDE_LDS_WORDS && line >= 0 && line < H && p >= 0 && p < N;
        v[it] = __builtin_amdgcn_raw_buffer_load_b32(rx, in ? (uint32_t)line * (uint32_t)W + (uint32_t)p : kOob, 0, 0);
      }
#pragma unroll
      for (int it = 0; it < NIT; ++it)
        if (tid + it * 256 < BSIDE_LDS_WORDS) lines[tid + it * 256] = v[it];
    } else {
      // image rows c0 - 4 .. c0 + BSIDE_CH + 3: the side's 6 columns from two aligned words
      // (left: cols 0..7, right: cols W-8..W-1), transposed into the 6 stored lines bytewise
      constexpr int NR = BSIDE_CH + 8, NIT = (NR + 255) / 256;
      const int cw = (side & 1) ? W - 8 : 0, sh = (side & 1) ? 2 : 0;  // byte of stored line 0 in the pair
      uint32_t v0[NIT], v1[NIT];
#pragma unroll
      for (int it = 0; it < NIT; ++it) {
        const int i = tid + it * 256, r = c0 - 4 + i;
        const bool in = i < NR && r >= 0 && r < H;
        const uint32_t o = in ? (uint32_t)r * (uint32_t)W + (uint32_t)cw : kOob;
        v0[it] = __builtin_amdgcn_raw_buffer_load_b32(rx, o, 0, 0);
        v1[it] = __builtin_amdgcn_raw_buffer_load_b32(rx, in ? o + 4u : kOob, 0, 0);
      }
#pragma unroll
      for (int it = 0; it < NIT; ++it) {
        const int i = tid + it * 256;
        if (i < NR) {
          const uint64_t pair = ((uint64_t)v1[it] << 32) | v0[it];
#pragma unroll
          for (int t = 0; t < 6; ++t) lb[t * BSIDE_LD * 4 + i] = (uint8_t)(pair >> (8 * (t + sh)));
        }
      }
    }
    __syncthreads();
    // wave wv: pairs pr = 4m + wv (< 18): strip line l0 + pr / 9, perpendicular offset pr % 9 - 4
#pragma unroll
    for (int m = 0; m < 5; ++m) {
      const int pr = 4 * m + wv;
      const int tl = l0 + pr / 9, tp = tl + pr % 9 - 4;
      if (pr < 18 && tp >= 0 && tp < 6) {
        const uint32_t* lu = lines + tl * BSIDE_LD + 1;
        const uint32_t* lp = lines + tp * BSIDE_LD;
#pragma unroll
        for (int j = 0; j < BSIDE_CH / 4 / 64; ++j) {
          const int qi = lane + 64 * j;
          const uint32_t u = lu[qi], w0 = lp[qi], w1 = lp[qi + 1], w2 = lp[qi + 2];
#pragma unroll
          for (int s = 0; s < 9; ++s) acc[m][s] = __builtin_amdgcn_udot4(u, xm_win(w0, w1, w2, s), acc[m][s], false);
        }
      }
    }
    if (wv < 2) {
#pragma unroll
      for (int j = 0; j < BSIDE_CH / 4 / 64; ++j)
        plain = __builtin_amdgcn_udot4(lines[(l0 + wv) * BSIDE_LD + 1 + lane + 64 * j], 0x01010101u, plain, false);
    }
    __syncthreads();
  }
  // (positions past N are zeros in LDS: a chunk's tail past the line adds nothing)
#pragma unroll
  for (int m = 0; m < 5; ++m) {
    const int pr = 4 * m + wv;
    if (pr < 18) {
      const int tl = pr / 9, dd = pr % 9 - 4;
      unsigned long long* out = sacc + (2 * side + tl) * 82;
#pragma unroll
      for (int s = 0; s < 9; ++s) {
        const uint32_t v = xm_wave_sum(acc[m][s]);
        if (lane == 0 && v != 0u)
          __hip_atomic_fetch_add(out + (rows ? (dd + 4) * 9 + s : s * 9 + (dd + 4)), (unsigned long long)v,
                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
  if (wv < 2) {
    const uint32_t v = xm_wave_sum(plain);
    if (lane == 0 && v != 0u)
      __hip_atomic_fetch_add(sacc + (2 * side + wv) * 82 + 81, (unsigned long long)v, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
  }
}

}  // namespace tds
