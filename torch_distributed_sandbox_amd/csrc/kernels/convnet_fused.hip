// Fused ConvNet kernels: layer 1 (forward and backward) and the small reductions around the conv2 /
// head kernels (conv2: conv2_fwd2.hip, conv2_bwd.hip; head: head_pb.hip; the input op with the x
// moments: ups_moments.hip).  Reference model: mnist_onegpu.py:11-31; SURVEY.md §2.4 K1-K4, K6, K22-K25.
// Forward
//   l1_reduce_gram  : one launch after the input op: the x moments' column sums and border strips ->
//                     Gram G = sum xpatch xpatch^T and S = sum xpatch; BN1's statistics in closed form
//                     (sum y1 - b1 = w1.S, sum (y1 - b1)^2 = w1^T G w1), so conv1 runs ONCE; 64 more
//                     workgroups pack conv2's weights (conv2_pack.h).
//   l1_conv_bf3     : conv1 (bf16x2 MFMA on the uint8 levels, bf16x3 on an fp32 image), BN1 affine,
//                     2x2 max-pool, ReLU -> p1 (fp16 NHWC, 32-B records: conv2's single-rounded
//                     operand) and a 1-byte argmax per pooled value; y1 is never written.
// Backward
//   l1_bwd_mfma     : dz1 is non-zero only at the argmax of each pooled window with p1 > 0:
//                     sum dz1 x xpatch as one MFMA product per tile (bf16x3 / bf16x2 split).
//   l1_reduce_finalize : the per-workgroup partials' reduction and
//                     dW1 = a1*sum(dz1 xpatch) + a2*(W1 G + b1 S) + a3*S, db1, dgamma1, dbeta1.
// Separate-launch forms kept as ops (tests/test_fused_gpu.py, tools/micro; not in the default step):
//   l1_gram, bn_finalize_shifted, bn_reduce_finalize, reduce_partials, bn_bwd_finalize2, l1_finalize.
#include <cstdlib>

#include "bf16x3.h"
#include "bn_finalize.h"
#include "launchers.h"
#include "xmom_u8.h"
#include "conv2_pack.h"

namespace tds {

// zero source of the layer-1 kernels' out-of-range prefetch lanes
__device__ __attribute__((aligned(16))) uint4 g_l1b_zero = {0u, 0u, 0u, 0u};

// ============================================================================ layer 1 conv
constexpr int L1_TR = 16;           // conv1 output rows per tile
constexpr int L1_TC = 64;           // conv1 output cols per tile
constexpr int L1_XR = L1_TR + 4;
// LDS row stride (words), odd: the two 16-lane groups of a 32-lane half read taps one row apart
// (l1b_tap: g = 0 / 1 and 2 / 3 differ in ky), and 2*li spans the 16 banks of one parity, so
// an odd stride puts the two groups on opposite parities (conflict-free; 80 = 16 mod 32 put
// them on the same 16 banks -- 2-way on every read, 33 % of LDS cycles in the round-4 PMC)
constexpr int L1_XS = 81;
// uint8 level input: x = L1_LEVEL_SCALE * level, the fp32 constant upsample_bilinear_u8 (elementwise.hip)
// and ToTensor scale by
constexpr float L1_LEVEL_SCALE = 1.f / 255.f;

// 4 words at an odd-stride LDS row (no 16-B alignment)
__device__ __forceinline__ void l1_store4(uint32_t* d, uint4 v) {
  d[0] = v.x;
  d[1] = v.y;
  d[2] = v.z;
  d[3] = v.w;
}

// conv1 on v_mfma_f32_16x16x32_bf16 with the bf16x3 split (bf16x3.h): K = 32 slots per lane
// group g: taps (ky = g, kx = 0..4) and the row-4 taps spread over g = 0 (kx 0..2) and g = 1
// (kx 3, 4); the rest are zero-weight pads.  x is staged in LDS as one word per value
// (bf16 hi << 16 | bf16 lo), so a lane's 8 taps are 8 ds_read_b32 + 8 v_perm; 3 MFMAs per
// 16 px x 16 co replace 7 v_mfma_f32_16x16x4_f32 (4.7x fewer MFMA cycles).
__device__ __forceinline__ int l1b_tap(int g, int j) {
  if (j < 5) return g * 5 + j;
  if (g == 0) return 20 + (j - 5);           // (4, 0..2)
  if (g == 1 && j < 7) return 23 + (j - 5);  // (4, 3..4)
  return -1;
}

// LV K-slot pairs: lane group g's slots 2p, 2p+1 hold horizontally adjacent taps (ky, kx0) and
// (ky, kx0 + 1) of one row, so ONE ds_read_b32 of a pair word (bf16 x[c] | bf16 x[c+1] << 16, the
// LV staging layout) is the B operand's two slots -- 4 reads and no v_perm per 8 slots instead of
// 8 reads + 4 perms.  Rows 0-3: pairs kx (0,1), (2,3), (4,pad) in group g = ky; row 4 spread over
// p = 3 as (4: 0,1) g0, (4: 3,4) g1, (4: 2,pad) g2; g3's p = 3 is a zero-weight pair reading (3,0).
// Pads read column kx0 + 1 = 5 or 3 of the row with weight 0 (levels are finite).  Bank parity:
// the two groups of a 32-lane half read offsets of opposite parity (odd L1_XS, row-4 kx0 0/3 and
// 2/(3,0)), so with 2*li spanning one parity the 32 lanes hit 32 banks.
struct L1Pair {
  int ky, kx0;
  bool second;  // slot 2p+1 carries a real tap
};
__device__ __forceinline__ L1Pair l1_pair(int g, int p) {
  if (p < 3) return L1Pair{g, 2 * p, p < 2};
  if (g == 0) return L1Pair{4, 0, true};
  if (g == 1) return L1Pair{4, 3, true};
  if (g == 2) return L1Pair{4, 2, false};
  return L1Pair{3, 0, false};  // zero weights
}

// LV: x holds uint8 levels (x = L1_LEVEL_SCALE * level).  A level is exact in bf16, so the LDS word
// is the level's fp32 bit pattern (bf16 hi | lo = 0), conv1 takes two MFMAs (w hi, w lo) per
// product instead of three and half the operand perms, and the scale folds into BN1's affine.
template <bool LV>
__global__ __launch_bounds__(256) void l1_conv_bf3_kernel(const void* __restrict__ xv, const float* __restrict__ w1,
                                                      const float* __restrict__ b1, const float* __restrict__ aff,
                                                      uint4* __restrict__ p1, uint8_t* __restrict__ idx1, int B,
                                                      int H, int W) {
  __shared__ __attribute__((aligned(16))) uint32_t xs[L1_XR * L1_XS];  // x as (bf16 hi << 16 | bf16 lo)
  constexpr bool PAIR = LV;  // level input: pair words (l1_pair)
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int li = lane & 15, g = lane >> 4;
  const int P = H / 2, PW = W / 2;
  const int tiles_c = (W + L1_TC - 1) / L1_TC, tiles_r = (H + L1_TR - 1) / L1_TR;
  const int per_img = tiles_c * tiles_r, total = per_img * B;

  // A operand (weights) in registers as bf16 hi / lo: lane -> co = li, k = 8g + j -> tap
  // l1b_tap(g, j) (rows ky = g plus row 4 spread over g = 0, 1; pads carry weight 0)
  s16x8 wah, wal;
  int koff[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    int tp;
    if constexpr (PAIR) {
      const L1Pair pr = l1_pair(g, j >> 1);
      const bool real = (g < 3 || j < 6) && ((j & 1) == 0 || pr.second);
      tp = real ? pr.ky * 5 + pr.kx0 + (j & 1) : -1;
      if ((j & 1) == 0) koff[j >> 1] = pr.ky * L1_XS + pr.kx0;
    } else {
      tp = l1b_tap(g, j);
      koff[j] = tp >= 0 ? (tp / 5) * L1_XS + (tp % 5) : 1;  // pad: tap (0, 1) (odd word: opposite bank parity to g = 0 j = 7)
    }
    // channel li's weights carry the sign of its BN1 scale (below)
    const float wv = tp >= 0 ? (aff[li] < 0.f ? -w1[li * 25 + tp] : w1[li * 25 + tp]) : 0.f;
    unsigned short h, l;
    split_bf16(wv, h, l);
    wah[j] = (short)h;
    wal[j] = (short)l;
  }

  // per-lane epilogue constants for co = 4g + r: z = ea * (acc + b1) + eb = ea * acc + ebb.  The
  // weights of a channel with ea < 0 are negated (exact), so acc holds -acc and z = |ea| * acc + ebb
  // bit for bit: BN1's affine is then increasing in acc, the 2x2 max-pool picks the window's largest
  // ACCUMULATOR and the affine runs once per pooled value instead of once per pixel (the epilogue's
  // VALU bounds this kernel).  A window whose top two pixels round to one z keeps the larger acc
  // (torch: the first in scan order) -- as the conv2 forward's pooling on y2 does.
  float ea[4], ebb[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const float a = aff[4 * g + r];
    ebb[r] = fmaf(a, b1[4 * g + r], aff[16 + 4 * g + r]);
    ea[r] = fabsf(a);
  }
  bool fin = true;
#pragma unroll
  for (int r = 0; r < 4; ++r) fin = fin && __builtin_isfinite(ea[r]) && __builtin_isfinite(ebb[r]) && ea[r] != 0.f;
  const bool fast_ok = __builtin_amdgcn_ballot_w64(!fin) == 0 && __syncthreads_and(fin) != 0;
  if constexpr (LV) {
#pragma unroll
    for (int r = 0; r < 4; ++r) ea[r] *= L1_LEVEL_SCALE;  // z = ea * (scale * acc + b1) + eb
  }
  const float* __restrict__ x = static_cast<const float*>(xv);
  const uint8_t* __restrict__ xl = static_cast<const uint8_t*>(xv);

  // x tile staging: LDS column 0 <-> global column c0-4 (16-B aligned since W % 4 == 0),
  // 20 rows x 18 float4; the next tile's loads are issued before this tile's MFMAs.
  constexpr int NV = L1_XR * 18;
  constexpr int PER = (NV + 255) / 256;
  float4 pre[PER];  // LV: .x = 4 levels, .y = the next 4 (the pair words' right neighbours)
  // unconditional loads (out-of-range lanes read a zero vector): a load under a per-lane branch
  // is waited for before the branches merge (conv2_bwd.hip, l1_bwd_mfma_kernel)
  auto load_tile = [&](int t) {
    const int b = t / per_img, rem = t - b * per_img;
    const int r0 = (rem / tiles_c) * L1_TR, c0 = (rem % tiles_c) * L1_TC;
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int e = tid + 256 * u;
      const int rr = e / 18, cv = e - rr * 18;
      const int gr = r0 - 2 + rr, gc = c0 - 4 + 4 * cv;
      const bool ok = (e < NV) & ((uint32_t)gr < (uint32_t)H) & ((uint32_t)gc < (uint32_t)W);
      const int64_t o = ((int64_t)b * H + gr) * W + gc;
      if constexpr (LV) {  // 4 levels in .x, the next 4 in .y (zero past the image / the tile)
        // (its own range test: at the image's left edge the word at column -1 pairs with x[0])
        const bool okn = (e < NV) & (cv < 17) & ((uint32_t)gr < (uint32_t)H) & ((uint32_t)(gc + 4) < (uint32_t)W);
        const uint32_t* src = ok ? reinterpret_cast<const uint32_t*>(xl + o) : &g_l1b_zero.x;
        const uint32_t* srn = okn ? reinterpret_cast<const uint32_t*>(xl + o + 4) : &g_l1b_zero.x;
        pre[u] = make_float4(__uint_as_float(*src), PAIR ? __uint_as_float(*srn) : 0.f, 0.f, 0.f);
      } else {
        const float4* src = ok ? reinterpret_cast<const float4*>(x + o) : reinterpret_cast<const float4*>(&g_l1b_zero);
        pre[u] = *src;
      }
    }
  };
  int t = xcd_remap(blockIdx.x, gridDim.x);
  if (t < total) load_tile(t);
  for (; t < total; t += gridDim.x) {
    const int b = t / per_img, rem = t - b * per_img;
    const int r0 = (rem / tiles_c) * L1_TR, c0 = (rem % tiles_c) * L1_TC;
    __syncthreads();
    bool nonfinite = false;
#pragma unroll
    for (int u = 0; u < PER; ++u) asm volatile("" ::"v"(pre[u].x), "v"(pre[u].y), "v"(pre[u].z), "v"(pre[u].w));
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int e = tid + 256 * u;
      if (e < NV) {
        const int rr = e / 18, cv = e - rr * 18;
        if constexpr (PAIR) {  // levels are exact in bf16 (the fp32 bits' upper half): pair words
          const uint32_t q = __float_as_uint(pre[u].x);
          const uint32_t f0 = __float_as_uint((float)(q & 0xFFu)), f1 = __float_as_uint((float)((q >> 8) & 0xFFu));
          const uint32_t f2 = __float_as_uint((float)((q >> 16) & 0xFFu)), f3 = __float_as_uint((float)(q >> 24));
          const uint32_t f4 = __float_as_uint((float)(__float_as_uint(pre[u].y) & 0xFFu));
          uint4 v;  // word c = bf16 x[c] | bf16 x[c+1] << 16
          v.x = __builtin_amdgcn_perm(f1, f0, 0x07060302u);
          v.y = __builtin_amdgcn_perm(f2, f1, 0x07060302u);
          v.z = __builtin_amdgcn_perm(f3, f2, 0x07060302u);
          v.w = __builtin_amdgcn_perm(f4, f3, 0x07060302u);
          l1_store4(xs + rr * L1_XS + 4 * cv, v);
          continue;
        }
        nonfinite |= !__builtin_isfinite((pre[u].x + pre[u].y) + (pre[u].z + pre[u].w));
        uint32_t h01, l01, h23, l23;
        split2_bf16(pre[u].x, pre[u].y, h01, l01);
        split2_bf16(pre[u].z, pre[u].w, h23, l23);
        uint4 v;  // per value: hi in the upper half, lo in the lower half
        v.x = __builtin_amdgcn_perm(h01, l01, 0x05040100u);
        v.y = __builtin_amdgcn_perm(h01, l01, 0x07060302u);
        v.z = __builtin_amdgcn_perm(h23, l23, 0x05040100u);
        v.w = __builtin_amdgcn_perm(h23, l23, 0x07060302u);
        l1_store4(xs + rr * L1_XS + 4 * cv, v);
      }
    }
    // a non-finite x anywhere in the tile (or a degenerate BN1 affine) sends the whole tile to
    // the general epilogue (torch's NaN rules); otherwise no window can hold a NaN
    // (wave-uniform in an SGPR: as a per-lane bool the compiler computed both epilogues below
    // and selected, ~40 % more VALU per window)
    const bool slow = __builtin_amdgcn_readfirstlane((__syncthreads_or(nonfinite) != 0 || !fast_ok) ? 1 : 0) != 0;
    if (t + (int)gridDim.x < total) load_tile(t + gridDim.x);
#pragma unroll
    for (int rp = 0; rp < 2; ++rp) {
#pragma unroll
      for (int sp = 0; sp < 2; ++sp) {
        // rows (4wv + 2rp + a), 32-pixel span sp; MFMA c takes the pixels 2*li + c of the
        // span, so a lane's two columns ARE the two columns of pooling window li: the 2x2
        // window is acc[0..1][0..1][r] of one lane (no cross-lane exchange, no duplicate work)
        f32x4 acc[2][2];
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
          for (int c = 0; c < 2; ++c) {
            const int row = 4 * wv + 2 * rp + a;
            const uint32_t* src = xs + row * L1_XS + 2 + 32 * sp + 2 * li + c;  // +2: tile origin is c0-4
            s16x8 bh, bl;
            uint32_t* hp = reinterpret_cast<uint32_t*>(&bh);
            uint32_t* lp = reinterpret_cast<uint32_t*>(&bl);
            if constexpr (PAIR) {  // pair words: the B operand as read (l1_pair)
              // (the c = 1 base laundered: merged with c = 0's reads into ds_read2_b32, each
              // result pair straddled two MFMA operands and cost 3 v_mov per operand)
              // (the word index, not the pointer: a laundered pointer loses the LDS address space
              // and becomes flat loads, whose vmcnt wait also drains the x prefetch)
              int i0 = row * L1_XS + 2 + 32 * sp + 2 * li + c;
              if (c == 1) asm volatile("" : "+v"(i0));
              typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
              bh = __builtin_bit_cast(s16x8, u32x4{xs[i0 + koff[0]], xs[i0 + koff[1]], xs[i0 + koff[2]], xs[i0 + koff[3]]});
            } else {
              uint32_t u[8];
#pragma unroll
              for (int j = 0; j < 8; ++j) u[j] = src[koff[j]];
#pragma unroll
              for (int j = 0; j < 4; ++j) {
                hp[j] = __builtin_amdgcn_perm(u[2 * j + 1], u[2 * j], 0x07060302u);
                if constexpr (!LV) lp[j] = __builtin_amdgcn_perm(u[2 * j + 1], u[2 * j], 0x05040100u);
              }
            }
            if constexpr (LV)
              acc[a][c] = mfma_bf16x2a(wah, wal, bh, f32x4{0.f, 0.f, 0.f, 0.f});
            else
              acc[a][c] = mfma_bf16x3(wah, wal, bh, bl, f32x4{0.f, 0.f, 0.f, 0.f});
          }
        // BN1 affine -> 2x2 max-pool (first max in scan order) -> ReLU -> fp16 record +
        // argmax byte (bit 2 = ReLU passes the gradient) for channels 4g .. 4g+3
        const int prow = (r0 + 4 * wv + 2 * rp) >> 1;
        const int pcol = (c0 >> 1) + 16 * sp + li;
        float pv[4];
        uint32_t ixw = 0;
        // scan order: (row 0, col 0), (row 0, col 1), (row 1, col 0), (row 1, col 1)
        if (!slow) {  // every z finite (tile-uniform)
          float mz[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float a0 = acc[0][0][r], a1 = acc[0][1][r], a2 = acc[1][0][r], a3 = acc[1][1][r];
            const float m = __builtin_elementwise_maximum(__builtin_elementwise_maximum(a0, a1),
                                                          __builtin_elementwise_maximum(a2, a3));
            // first max, branch-free (the ?: chain compiled to exec-mask branches)
            uint32_t am = a2 == m ? 2u : 3u;
            am = a1 == m ? 1u : am;
            am = a0 == m ? 0u : am;
            mz[r] = m;
            ixw |= am << (8 * r);
          }
          // the affine on the pooled values only, in packed fp32 (channel pairs r, r + 1)
#pragma unroll
          for (int r = 0; r < 4; r += 2) {
            const f32x2 zz = __builtin_elementwise_fma(f32x2{mz[r], mz[r + 1]}, f32x2{ea[r], ea[r + 1]},
                                                       f32x2{ebb[r], ebb[r + 1]});
            mz[r] = zz.x;
            mz[r + 1] = zz.y;
          }
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            pv[r] = fmaxf(mz[r], 0.f);
            ixw |= (mz[r] > 0.f ? 4u : 0u) << (8 * r);
          }
        } else {  // torch's rule: update when (v > max || isnan(v)), relu(NaN) = NaN
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float z0 = fmaf(ea[r], acc[0][0][r], ebb[r]), z1 = fmaf(ea[r], acc[0][1][r], ebb[r]);
            const float z2 = fmaf(ea[r], acc[1][0][r], ebb[r]), z3 = fmaf(ea[r], acc[1][1][r], ebb[r]);
            float m = z0;
            uint32_t am = 0;
            if (z1 > m || isnan(z1)) { m = z1; am = 1; }
            if (z2 > m || isnan(z2)) { m = z2; am = 2; }
            if (z3 > m || isnan(z3)) { m = z3; am = 3; }
            pv[r] = m > 0.f ? m : (isnan(m) ? m : 0.f);
            ixw |= (am | (m > 0.f ? 4u : 0u)) << (8 * r);
          }
        }
        // p1 is conv2's single fp16 operand (bf16x3.h, fp16x2): one rounding, 32-B records
        const uint32_t h01 = cvt2_f16(pv[0], pv[1]), h23 = cvt2_f16(pv[2], pv[3]);
        if (prow < P && pcol < PW) {
          const int64_t rec = ((int64_t)b * P + prow) * PW + pcol;
          uint2* dst = reinterpret_cast<uint2*>(p1 + rec * 2);  // 32-B record: fp16[16]
          // (non-temporal: plain, allocating p1 stores cost the layer-1 conv +14 us and the conv2
          // forward +23 us, r5_s44)
          st_stream(dst + g, make_uint2(h01, h23));
          st_stream(reinterpret_cast<uint32_t*>(idx1 + rec * 16) + g, ixw);
        }
      }
    }
  }
}

// BN2: reduce the per-workgroup partials of channel c (partial[c][nchunk][2], fixed order) and
// finalize it -- one workgroup per channel, one launch instead of a reduction + a finalize.
__global__ __launch_bounds__(256) void bn_reduce_finalize_kernel(
    const double* __restrict__ partial, int C, int nchunk, int64_t n, const float* __restrict__ shift, float eps,
    float momentum, const float* __restrict__ gamma, const float* __restrict__ beta, float* __restrict__ stats,
    float* __restrict__ running_mean, float* __restrict__ running_var, int64_t* __restrict__ num_batches,
    float* __restrict__ aff) {
  __shared__ double sh[8];
  const int c = blockIdx.x;
  double s = 0.0, ss = 0.0;
  for (int k = threadIdx.x; k < nchunk; k += blockDim.x) {
    s += partial[((int64_t)c * nchunk + k) * 2];
    ss += partial[((int64_t)c * nchunk + k) * 2 + 1];
  }
  s = block_sum(s, sh);
  ss = block_sum(ss, sh);
  if (threadIdx.x != 0) return;
  if (c == 0 && num_batches) num_batches[0] += 1;
  bn_finalize_channel(c, C, s, ss, n, shift, eps, momentum, gamma, beta, stats, running_mean, running_var, aff);
}

// Shifted BN finalize: statistics were accumulated on (y - shift[c]).
__global__ void bn_finalize_shifted_kernel(const double* __restrict__ partial, int C, int nchunk, int64_t n,
                                           const float* __restrict__ shift, float eps, float momentum,
                                           const float* __restrict__ gamma, const float* __restrict__ beta,
                                           float* __restrict__ stats /* mean[C], invstd[C] */,
                                           float* __restrict__ running_mean, float* __restrict__ running_var,
                                           int64_t* __restrict__ num_batches, float* __restrict__ aff /* a[C], b[C] */) {
  const int c = threadIdx.x;
  if (c == 0 && num_batches) num_batches[0] += 1;
  if (c >= C) return;
  double s = 0.0, ss = 0.0;
  for (int k = 0; k < nchunk; ++k) {
    s += partial[((int64_t)c * nchunk + k) * 2];
    ss += partial[((int64_t)c * nchunk + k) * 2 + 1];
  }
  bn_finalize_channel(c, C, s, ss, n, shift, eps, momentum, gamma, beta, stats, running_mean, running_var, aff);
}

// head kernels: see head_fused.hip

// out[e] = sum_k in[(e / inner) * ostride + (e % inner) + k * kstride]  (one workgroup per output, fp64)
__global__ __launch_bounds__(256) void reduce_partials_kernel(const double* __restrict__ in, double* __restrict__ out,
                                                              int nchunk, int inner, int64_t ostride, int64_t kstride) {
  __shared__ double sh[8];
  const int e = blockIdx.x;
  const int64_t base = (int64_t)(e / inner) * ostride + (e % inner);
  double s = 0.0;
#pragma unroll 8  // (the loads in flight together; the adds keep their order)
  for (int k = threadIdx.x; k < nchunk; k += blockDim.x) s += in[base + (int64_t)k * kstride];
  s = block_sum(s, sh);
  if (threadIdx.x == 0) out[e] = s;
}

// BN backward finalize from (sum dz, sum dz*y) partials (x2: fp32 dz / stored dz, below):
//   dgamma = invstd*(sdzy - mean*sdz), dbeta = sdz,
//   dy = k1*dz + k2*y + k3,  k1 = g*is, k2 = -g*is^3*(sdzy - mean*sdz)/n, k3 = -g*is*sdz/n - k2*mean
// One workgroup per channel (the head backward leaves ~10^3 partials per channel: a serial
// loop per channel took 21 us).
// Block C (the last) also forms the fc bias gradient dbfc[j] = scale * sum_b dl[b][j].
__global__ __launch_bounds__(256) void bn_bwd_finalize2_kernel(const double* __restrict__ partial, int C, int nchunk,
                                                               int64_t n, const float* __restrict__ gamma,
                                                               const float* __restrict__ stats,
                                                               float* __restrict__ dgamma, float* __restrict__ dbeta,
                                                               float* __restrict__ kbuf, double* __restrict__ sums_out,
                                                               const float* __restrict__ dl, int B, int NC,
                                                               float* __restrict__ dbfc, float scale,
                                                               const uint32_t* __restrict__ ypart, int nyp,
                                                               const uint32_t* __restrict__ gpart, int ngp,
                                                               uint32_t* __restrict__ mag) {
  __shared__ double sh[8];
  __shared__ uint32_t shm[8];
  const int c = blockIdx.x;
  // magnitude bounds of the conv2 backward's fp16 scale (conv2_bwd.hip); ypart == nullptr: the
  // conv2 forward reduced its part (mag[0..C)) in its own launch (conv2_fwd2.hip f2_finalize)
  if (mag != nullptr && (c == C || ypart != nullptr)) {
    const uint32_t* src = c == C ? gpart : ypart + (int64_t)c * nyp;
    const int cnt = c == C ? ngp : nyp;
    uint32_t m = 0u;
    for (int k = threadIdx.x; k < cnt; k += blockDim.x) m = max(m, src[k]);
    m = block_max(m, shm);
    if (threadIdx.x == 0) mag[c] = m;
  }
  if (c == C) {
    if (dbfc && (int)threadIdx.x < NC) {
      float v = 0.f;
      for (int b = 0; b < B; ++b) v += dl[b * NC + threadIdx.x];
      dbfc[threadIdx.x] = v * scale;
    }
    return;
  }
  // partial[c][k][4]: (sum dz, sum dz*y) over the fp32 pooled gradient (dgamma, dbeta), then over
  // the values the conv2 backward reads (its fp16 g2m, head_pb.hip: k2, k3)
  double sdz = 0.0, sdzy = 0.0, sdr = 0.0, sdyr = 0.0;
  for (int k = threadIdx.x; k < nchunk; k += blockDim.x) {
    const double2 v = *reinterpret_cast<const double2*>(partial + ((int64_t)c * nchunk + k) * 4);
    const double2 vr = *reinterpret_cast<const double2*>(partial + ((int64_t)c * nchunk + k) * 4 + 2);
    sdz += v.x;
    sdzy += v.y;
    sdr += vr.x;
    sdyr += vr.y;
  }
  sdz = block_sum(sdz, sh);
  sdzy = block_sum(sdzy, sh);
  sdr = block_sum(sdr, sh);
  sdyr = block_sum(sdyr, sh);
  if (threadIdx.x != 0) return;
  const double mean = stats[c], is = stats[C + c];
  const double gm = gamma ? gamma[c] : 1.0;
  const double sdxh = sdzy - mean * sdz;  // sum dz*(y-mean)
  if (dgamma) dgamma[c] = (float)(is * sdxh);
  if (dbeta) dbeta[c] = (float)sdz;
  const double sdxr = sdyr - mean * sdr;
  const double k1 = gm * is;
  const double k2 = -gm * is * is * is * sdxr / (double)n;
  const double k3 = -gm * is * sdr / (double)n - k2 * mean;
  kbuf[c] = (float)k1;
  kbuf[C + c] = (float)k2;
  kbuf[2 * C + c] = (float)k3;
  if (sums_out) {
    sums_out[c * 2] = sdz;
    sums_out[c * 2 + 1] = sdzy;
  }
}


// layer-1 backward tile: 8 pooled rows x 32 pooled columns (x tile 20 rows incl. the halo)
constexpr int LB_PR = 8, LB_PC = 32;
constexpr int LB_XR = 2 * LB_PR + 4;
constexpr int LB_XS = 76;  // LDS x row stride (floats); column 0 <-> global column 2*pc0 - 4
constexpr int LB_NACC = 27;
constexpr int LB_NP = LB_PR * LB_PC;                     // pooled pixels per tile
// dp1h (conv2_common.h: [B][P][ceil(P/4)][16][4] fp16): a tile row is 8 column groups x 128 B
constexpr int LB_V_DP = LB_NP * 2, LB_V_PH = 0, LB_V_ID = LB_NP, LB_V_X = LB_XR * 18;
constexpr int LB_V = LB_V_DP + LB_V_PH + LB_V_ID + LB_V_X;  // 16-B vectors staged per tile
// The argmax byte carries the ReLU mask in bit 2 (set by l1_conv: pooled max > 0), so the
// backward never reads p1 (360 MB of 32-B fp16 records at the bench shape).
constexpr int LB_PER = (LB_V + 255) / 256;
static_assert(LB_V_PH == 0 && LB_V_DP % 256 == 0 && LB_V_ID % 256 == 0, "l1_bwd prefetch classes per vector");
// fp16 bits (low half) -> float
__device__ __forceinline__ float lb_f16(uint32_t h) { return (float)__builtin_bit_cast(_Float16, (unsigned short)(h & 0xFFFFu)); }
__device__ __forceinline__ void lb_store4(uint32_t* p, const uint4& v) {
  p[0] = v.x;
  p[1] = v.y;
  p[2] = v.z;
  p[3] = v.w;
}

// ============================================================================ layer-1 backward (MFMA)
// The sums the sparse kernel above forms with 25 VALU FMAs per active (pooled pixel,
// channel) as one matrix product on v_mfma_f32_16x16x32_bf16 (bf16x3 split):
//   D[co][n] = sum_pixels dz1[co][pix] * X[pix][n],  X[pix][n] = x(pix + tap n) for n < 25,
//   X[pix][25] = 1 (-> sum dz1), n = 26..31 zero pads;
// dz1[co][pix] = dp1 at the pooled window's argmax when the pooled value is > 0, else 0 (the
// dense full-resolution form of the sparse routing).  M = 16 channels, K = 32 pixels (2 rows
// x 16 columns), N = 32 taps in two MFMA blocks.  Tile = 16 x 64 conv1 pixels = 8 x 32 pooled
// (the sparse kernel's tile); 4 waves, wave w = row pairs 2w, 2w+1 x 4 column segments.  The
// dp1 / argmax tile and the x tile (packed bf16 hi|lo words, as l1_conv_bf3 stages it)
// go through LDS; fp32 MFMA accumulation per tile (256 pixels), fp64 across tiles.
// partial[wg][16][27] in the sparse kernel's layout ([0] sum dz, [1] 0, [2+j] taps).
// x tile row stride (words): 20 rows x (72 staged columns + 65 columns of bf16 1.0).  137 = 9 mod 32:
// a K-step's B read (one ds_read_b32 lane half = taps of 3-4 rows x 9 columns) then hits distinct banks
// (80 put rows ky and ky + 2 on the same banks: 2-way on every read).  The sum-dz lanes (n = 25) read
// the ones block at LM_ONES past the K-step base, a bank no data lane of that read touches; the pad
// lanes (n = 26..31, outputs discarded) read tap 24's address (a broadcast).  tools/micro/
// l1b_lds_check.py emulates both layouts' reads.
constexpr int LM_XS = 137;
constexpr int LM_ONES = LM_XS + 80;
static_assert(LM_XS % 32 == 9 && 80 + 3 * 16 + 3 < LM_XS && 1 + 2 * 7 + 1 < LB_XR, "l1_bwd ones block");
constexpr int LM_X_BYTES = LB_XR * LM_XS * 4;
// LV: x holds uint8 levels (see l1_conv_bf3_kernel); the tap sums are scaled by L1_LEVEL_SCALE at
// the end.
// waves per SIMD the register budget is cut for (4: <= 128 VGPRs, 4 workgroups per CU with
// fused_ops.cpp l1b_wg(); 3: <= 168, the measured configuration -- the compiler then keeps the
// default variants at 124-126 VGPRs, so 4 workgroups still fit a CU)
constexpr int L1B_WAVES = 3;
// Level input: dz1 * x on ONE v_mfma_f32_16x16x32_f16 per product instead of
// the bf16 pair (dz hi, dz lo): dz1 is dp1h's fp16 value as stored and a level (0..255) is exact
// in fp16, so every product is exact either way; the A operand is the fp16 bits themselves (no
// conversion, no bf16 split) and the MFMA count halves.  x words are PAIRS: word c = fp16 x[c] |
// fp16 x[c+1] << 16 (the l1_conv layout), so a window row's two B slots (dc = 0, 1) are one
// ds_read_b32 at the dc = 0 address -- 4 reads and no v_perm per operand; the ones block holds
// the pair (1.0, 1.0).  (A conflict-free bf16-pair x tile, two MFMAs per product, timed slower and
// is in git history.)  fp32 images (!LV): bf16x3, the x operand split hi + lo.
template <bool LV>
__global__ __launch_bounds__(256, L1B_WAVES) void l1_bwd_mfma_kernel(const void* __restrict__ xv, const uint4* __restrict__ dp1,
                                                          const uint32_t* __restrict__ dp1_dec,
                                                          const uint4* __restrict__ p1, const uint8_t* __restrict__ idx1,
                                                          double* __restrict__ partial, int B, int H, int W) {
  __shared__ __attribute__((aligned(16))) char lds[LB_NP * 64 + LB_NP * 16 + LM_X_BYTES];
  const uint32_t* dps = reinterpret_cast<const uint32_t*>(lds);  // dp1h tile [row 8][group 8][ch 16][px 4] fp16
  unsigned short* phs = nullptr;
  uint8_t* ids = reinterpret_cast<uint8_t*>(lds + LB_NP * 64);
  uint32_t* xs = reinterpret_cast<uint32_t*>(lds + LB_NP * 80);
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int li = lane & 15, g = lane >> 4;
  const int P = H / 2, PW = W / 2, PG = (PW + 3) >> 2;
  const int tiles_c = (PW + LB_PC - 1) / LB_PC, tiles_r = (P + LB_PR - 1) / LB_PR;
  const int per_img = tiles_c * tiles_r, total = per_img * B;
  const double dec = (double)__uint_as_float(dp1_dec[0]);

  // K ordering of a K-step (2 rows x 16 columns = 8 pooling windows): k = 4*w + 2*dr + dc, so
  // lane group g holds windows 2g, 2g+1 whole -- dz1 of a window is one pooled value placed
  // at its argmax slot (a 64-bit shift), no per-pixel selects.
  // B-operand geometry: x tile word offset (tile origin row r0 - 2, column c0 - 4) of this
  // lane's tap relative to the K-step base 2*rp*XS + 16*s; slot j adds (row dr2, column 2wi + dc).
  // n = 25 reads the ones block (bf16 1.0: the sum-dz column), n = 26..31 tap 24 (discarded).
  int boff[2];
#pragma unroll
  for (int blk = 0; blk < 2; ++blk) {
    const int n = 16 * blk + li, t = n < 25 ? n : 24;
    boff[blk] = n == 25 ? LM_ONES : (t / 5) * LM_XS + t % 5 + 2 + 4 * g;
  }
  constexpr bool H16 = LV;  // level input: fp16 pair words, one MFMA per product
  // the ones block (never overwritten: the x tile uses columns 0..71)
  for (int e = tid; e < LB_XR * (LM_XS - 72); e += 256)  // bf16 1.0 | lo 0, or fp16 1.0 << 16
    xs[(e / (LM_XS - 72)) * LM_XS + 72 + e % (LM_XS - 72)] = H16 ? 0x3C003C00u : 0x3F800000u;
  const float* __restrict__ x = static_cast<const float*>(xv);
  const uint8_t* __restrict__ xl = static_cast<const uint8_t*>(xv);
  uint4 pre[LB_PER];
  // One unconditional load per vector u: the class of vector u (dp1 records, argmax bytes, x
  // words) is a compile-time property of u (LB_V_DP and LB_V_ID are multiples of 256, the block is
  // 256 threads), and lanes out of range read a zero vector.  (Loads under per-lane branches had
  // to land before the branches merged: the compiler waited for each one right after issuing it,
  // which serialised the whole prefetch.)
  auto load_tile = [&](int t) {
    // tiles last-to-first, the reverse of the conv2 backward's dp1 writes: the first tiles read are
    // the most recent writes, still in the Infinity Cache (129.8 -> 128.0 us r5_s44, 132.8 -> 129.8
    // r5_s50)
    t = total - 1 - t;
    const int b = t / per_img, rem = t - b * per_img;
    const int pr0 = (rem / tiles_c) * LB_PR, pc0 = (rem % tiles_c) * LB_PC;
#pragma unroll
    for (int u = 0; u < LB_PER; ++u) {
      const int e = tid + 256 * u;
      if (256 * u < LB_V_DP) {  // dp1h: 64 vectors per tile row (8 column groups x 8)
        const int gpr = pr0 + (e >> 6), cg = (pc0 >> 2) + ((e >> 3) & 7);
        const int64_t rec = ((int64_t)b * P + gpr) * PG + cg;
        const uint4* src = ((gpr < P) & (cg < PG)) ? dp1 + rec * 8 + (e & 7) : &g_l1b_zero;
        pre[u] = *src;
      } else if (256 * u < LB_V_DP + LB_V_ID) {
        const int pp = e - LB_V_DP;
        const int gpr = pr0 + pp / LB_PC, gpc = pc0 + pp % LB_PC;
        const int64_t rec = ((int64_t)b * P + gpr) * PW + gpc;
        const uint4* src = ((gpr < P) & (gpc < PW)) ? reinterpret_cast<const uint4*>(idx1) + rec : &g_l1b_zero;
        pre[u] = *src;
      } else {
        const int ex = e - LB_V_DP - LB_V_ID;
        const int rr = ex / 18, cv = ex - rr * 18;
        const int gr = 2 * pr0 - 2 + rr, gcol = 2 * pc0 - 4 + 4 * cv;
        const bool ok = (ex < LB_V_X) & ((uint32_t)gr < (uint32_t)H) & ((uint32_t)gcol < (uint32_t)W);
        const int64_t o = ((int64_t)b * H + gr) * W + gcol;
        if constexpr (LV) {  // 4 levels in .x; H16: the next 4 in .y (the pair words' right neighbours)
          const uint32_t* src = ok ? reinterpret_cast<const uint32_t*>(xl + o) : &g_l1b_zero.x;
          const bool okn = (ex < LB_V_X) & (cv < 17) & ((uint32_t)gr < (uint32_t)H) & ((uint32_t)(gcol + 4) < (uint32_t)W);
          const uint32_t* srn = okn ? reinterpret_cast<const uint32_t*>(xl + o + 4) : &g_l1b_zero.x;
          pre[u] = make_uint4(*src, H16 ? *srn : 0u, 0u, 0u);
        } else {
          const uint4* src = ok ? reinterpret_cast<const uint4*>(x + o) : &g_l1b_zero;
          pre[u] = *src;
        }
      }
    }
  };
  auto store_tile = [&]() {
    // every prefetch register read here on every path (the stores below are predicated): a
    // result consumed only under a branch stays "pending" for the waitcnt pass, and the next
    // prefetch into it then waits for every load in flight
#pragma unroll
    for (int u = 0; u < LB_PER; ++u) asm volatile("" ::"v"(pre[u].x), "v"(pre[u].y), "v"(pre[u].z), "v"(pre[u].w));
#pragma unroll
    for (int u = 0; u < LB_PER; ++u) {
      int e = tid + 256 * u;
      if (e < LB_V_DP) reinterpret_cast<uint4*>(lds)[e] = pre[u];
      else if (e < LB_V_DP + LB_V_PH) reinterpret_cast<uint4*>(phs)[e - LB_V_DP] = pre[u];
      else if (e < LB_V_DP + LB_V_PH + LB_V_ID) reinterpret_cast<uint4*>(ids)[e - LB_V_DP - LB_V_PH] = pre[u];
      else if (e < LB_V) {
        e -= LB_V_DP + LB_V_PH + LB_V_ID;
        const int rr = e / 18, cv = e - rr * 18;
        if constexpr (H16) {  // pair words: fp16 x[c] | fp16 x[c+1] << 16 (levels are exact)
          const uint32_t q = pre[u].x;
          auto h = [](uint32_t l) { return (uint32_t)__builtin_bit_cast(unsigned short, (_Float16)(float)l); };
          const uint32_t h0 = h(q & 0xFFu), h1 = h((q >> 8) & 0xFFu), h2 = h((q >> 16) & 0xFFu), h3 = h(q >> 24);
          const uint32_t h4 = h(pre[u].y & 0xFFu);
          lb_store4(xs + rr * LM_XS + 4 * cv, make_uint4(h0 | h1 << 16, h1 | h2 << 16, h2 | h3 << 16, h3 | h4 << 16));
          continue;
        }
        const float4 f = __builtin_bit_cast(float4, pre[u]);
        uint32_t h01, l01, h23, l23;
        split2_bf16(f.x, f.y, h01, l01);
        split2_bf16(f.z, f.w, h23, l23);
        uint4 v;  // per value: hi in the upper half, lo in the lower half
        v.x = __builtin_amdgcn_perm(h01, l01, 0x05040100u);
        v.y = __builtin_amdgcn_perm(h01, l01, 0x07060302u);
        v.z = __builtin_amdgcn_perm(h23, l23, 0x05040100u);
        v.w = __builtin_amdgcn_perm(h23, l23, 0x07060302u);
        lb_store4(xs + rr * LM_XS + 4 * cv, v);  // odd row stride: dword stores
      }
    }
  };

  double dacc[2][4];
#pragma unroll
  for (int blk = 0; blk < 2; ++blk)
#pragma unroll
    for (int r = 0; r < 4; ++r) dacc[blk][r] = 0.0;

  int t = xcd_remap(blockIdx.x, gridDim.x);
  if (t < total) load_tile(t);
  for (; t < total; t += gridDim.x) {
    __syncthreads();
    store_tile();
    __syncthreads();
    if (t + (int)gridDim.x < total) load_tile(t + gridDim.x);
    f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int rp = 2 * wv + h;
#pragma unroll
      for (int sg = 0; sg < 4; ++sg) {
        // A = dz1 for (co = li, windows 2g, 2g+1 of the K-step): pooled pp = rp*32 + 8*sg + w
        s16x8 ah, al;
        {
          uint32_t* hp = reinterpret_cast<uint32_t*>(&ah);
          uint32_t* lp = reinterpret_cast<uint32_t*>(&al);
          // pooled columns 8sg + 2g + {0, 1}: column group 2sg + (g >> 1), pixels 2(g & 1) + {0, 1} --
          // one dword (a 32-lane half reads 32 consecutive words: conflict-free)
          const uint32_t dpair = dps[((rp * 8 + 2 * sg + (g >> 1)) * 16 + li) * 2 + (g & 1)];
          if constexpr (H16) {  // fp16 bits at the argmax slot, zero where ReLU blocks the gradient;
            // K order here: dword 2 dr + wi = (window wi, row dr), halves dc = 0, 1 (the B reads'
            // order: ds_read2_b32 pairs (wi 0, 1) of one row land in consecutive registers)
#pragma unroll
            for (int wi = 0; wi < 2; ++wi) {
              const uint32_t ab = ids[(rp * LB_PC + 8 * sg + 2 * g + wi) * 16 + li];
              const uint32_t hb = (ab & 4u) ? ((dpair >> (16 * wi)) & 0xFFFFu) : 0u;
              const uint32_t hs = hb << (16u * (ab & 1u));
              hp[wi] = (ab & 2u) ? 0u : hs;
              hp[2 + wi] = (ab & 2u) ? hs : 0u;
            }
          } else
#pragma unroll
          for (int wi = 0; wi < 2; ++wi) {
            const int pp = rp * LB_PC + 8 * sg + 2 * g + wi;
            const float dp = lb_f16(dpair >> (16 * wi));
            const uint32_t ab = ids[pp * 16 + li];
            const float d = (ab & 4u) ? dp : 0.f;  // ReLU: a pooled value <= 0 blocks the gradient
            uint32_t h, l;
            split2_bf16(d, 0.f, h, l);             // low halves: bf16 hi / lo of d
            const uint32_t sh = 16u * (ab & 3u);  // argmax slot (dr, dc) of the window
            const uint64_t h64 = (uint64_t)(h & 0xFFFFu) << sh, l64 = (uint64_t)(l & 0xFFFFu) << sh;
            hp[2 * wi] = (uint32_t)h64;
            hp[2 * wi + 1] = (uint32_t)(h64 >> 32);
            lp[2 * wi] = (uint32_t)l64;
            lp[2 * wi + 1] = (uint32_t)(l64 >> 32);
          }
        }
        const int base = 2 * rp * LM_XS + 16 * sg;
#pragma unroll
        for (int blk = 0; blk < 2; ++blk) {
          const int bo = base + boff[blk];
          if constexpr (H16) {  // dword 2 dr + wi = (window wi, row dr), cols dc = 0, 1: one pair word
            typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
            const s16x8 bp = __builtin_bit_cast(
                s16x8, u32x4{xs[bo], xs[bo + 2], xs[bo + LM_XS], xs[bo + LM_XS + 2]});
            acc[blk] = mfma_f16(ah, bp, acc[blk]);
            continue;
          }
          uint32_t u[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const int wi = j >> 2, dr2 = (j >> 1) & 1, dc = j & 1;  // slot j = (window wi, row dr2, col dc)
            u[j] = xs[bo + dr2 * LM_XS + 2 * wi + dc];
          }
          s16x8 bh, bl;
          uint32_t* hp = reinterpret_cast<uint32_t*>(&bh);
          uint32_t* lp = reinterpret_cast<uint32_t*>(&bl);
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            hp[j] = __builtin_amdgcn_perm(u[2 * j + 1], u[2 * j], 0x07060302u);
            if constexpr (!LV) lp[j] = __builtin_amdgcn_perm(u[2 * j + 1], u[2 * j], 0x05040100u);
          }
          acc[blk] = mfma_bf16x3(ah, al, bh, bl, acc[blk]);
        }
      }
    }
#pragma unroll
    for (int blk = 0; blk < 2; ++blk)
#pragma unroll
      for (int r = 0; r < 4; ++r) dacc[blk][r] += (double)acc[blk][r];
  }
  // D layout: lane holds column n = 16*blk + li, rows co = 4*g + r.  The 4 waves' sums are
  // added in LDS (fixed order) so the workgroup writes ONE partial row (the cross-workgroup
  // reduction reads a quarter of the rows it did with one row per wave).
  __syncthreads();  // the last tile's LDS reads are done
  double* red = reinterpret_cast<double*>(lds);  // [4 waves][16 co][27]: 13.8 KB of the tile buffers
#pragma unroll
  for (int blk = 0; blk < 2; ++blk) {
    const int n = 16 * blk + li;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      double* o = red + (wv * 16 + 4 * g + r) * LB_NACC;
      // (dec: dp1h's decode, a power of two)
      if (n < 25) o[2 + n] = LV ? dacc[blk][r] * ((double)L1_LEVEL_SCALE * dec) : dacc[blk][r] * dec;
      else if (n == 25) o[0] = dacc[blk][r] * dec;
      else if (n == 26) o[1] = 0.0;
    }
  }
  __syncthreads();
  double* out = partial + (int64_t)blockIdx.x * 16 * LB_NACC;
  for (int e = tid; e < 16 * LB_NACC; e += 256)
    st_agent(out + e, (red[e] + red[16 * LB_NACC + e]) + (red[2 * 16 * LB_NACC + e] + red[3 * 16 * LB_NACC + e]));
}
static_assert(4 * 16 * LB_NACC * 8 <= LB_NP * 64 + LB_NP * 16 + LM_X_BYTES, "l1_bwd LDS reduction scratch");

// Gram of the conv1 patches from the x autocorrelation (one workgroup):
//   G[k][j] = Full(d) - sum_{excluded rows of k} R(d,row) - sum_{excluded cols} C(d,col)
//             + sum corners,  d = o_j - o_k  (see x_autocorr / x_border)
//   S[j]    = sum of x over the pixels tap j sees (total - excluded lines + corners)
// ac_sum: reduced autocorrelation [42] (slot 41 = plain sum).
// The corner terms read x only inside the 6 x 6 pixel block at each image corner (excluded rows /
// columns lie within 2 of the border, their partners within 4 more): those blocks are loaded into
// LDS once, all loads in flight together (read one by one from global memory inside the loops
// below, they made this one-workgroup kernel latency-bound: 19 us per step).  H, W >= 12.
constexpr int L1G_MAXB = 32;
struct L1Corners {
  float v[L1G_MAXB][4][6][6];
  __device__ float at(int b, int r, int c, int H, int W) const {
    const int q = (r >= 6 ? 2 : 0) + (c >= 6 ? 1 : 0);
    return v[b][q][r >= 6 ? r - (H - 6) : r][c >= 6 ? c - (W - 6) : c];
  }
};

// corner products, every (corner row, corner col, offset) triple: e < 16 * 81 -> cp[ri][ci][d] =
// sum_b x(b, r, c) x(b, r + dy, c + dx) for r in rows 0, 1, H-2, H-1 (ri 0..3), c likewise, the
// partner inside the image; e - 16 * 81 < 16 -> cs[ri][ci] = sum_b x(b, r, c).  (Summed per Gram
// entry inside its loops, the B-long LDS chains cost 8 us of the one-workgroup body, r5_s29b.)
__device__ __forceinline__ double l1_corner_term(const L1Corners& cx, int B, int H, int W, int e) {
  const bool sum = e >= 16 * 81;
  const int rc = sum ? e - 16 * 81 : e / 81, d = sum ? 40 : e - rc * 81;
  const int ri = rc >> 2, ci = rc & 3;
  const int r = ri < 2 ? ri : H - 4 + ri, c = ci < 2 ? ci : W - 4 + ci;
  const int r2 = r + d / 9 - 4, c2 = c + d % 9 - 4;
  double v = 0.0;
  if (sum) {
#pragma unroll 8
    for (int b = 0; b < B; ++b) v += cx.at(b, r, c, H, W);
  } else if (r2 >= 0 && r2 < H && c2 >= 0 && c2 < W) {
#pragma unroll 8
    for (int b = 0; b < B; ++b) v += (double)cx.at(b, r, c, H, W) * cx.at(b, r2, c2, H, W);
  }
  return v;
}

// T = uint8_t: x holds levels (x = xs * level); the sums are of the levels and G, S are scaled by
// xs^2, xs at the end (fp64), so the Gram is that of the fp32 image either way.
template <typename T>
__device__ void l1_build_gram(const double* __restrict__ ac_sum, const double* __restrict__ strips_b,
                              const T* __restrict__ x, int B, int H, int W, double (*G)[25], double* S,
                              double* full, double* strips, const L1Corners& cx, double xs, int nch,
                              unsigned long long* __restrict__ sacc, const double* __restrict__ cpg) {
  const int tid = threadIdx.x;
  // the autocorrelation sum this thread places in full[] (load issued with the strips' below)
  double fa = 0.0;
  if (tid < 81) {
    const int dy = tid / 9 - 4, dx = tid % 9 - 4;
    int sy = dy, sx = dx;
    if (dy < 0 || (dy == 0 && dx < 0)) { sy = -dy; sx = -dx; }
    fa = ac_sum[sy == 0 ? sx : 5 + (sy - 1) * 9 + (sx + 4)];
  } else if (tid == 81) {
    fa = ac_sum[41];  // the plain sum (full[81])
  }
  // per-image border strips [B][8][nch][82] (nch line chunks, xmom_u8.h; 1 otherwise) -> batch
  // sums, images then chunks in order
  // (up to 16 values per sum in flight at once: written by other workgroups of the launch, they
  // sit behind a cross-XCD round trip each -- as a dependent chain 15 of them cost ~20 us)
  const int nv = B * nch;
  static_assert(8 * 82 <= 3 * 256, "three strip sums per thread");
  __shared__ double cp[16][81];
  __shared__ double cs[16];
  if (sacc != nullptr) {
    // the batch's strips as exact u64 sums (xmom_u8.h) and the corner table formed before the
    // hand-off by the column workgroups (cpg): one round of loads; the accumulator is zeroed for
    // the stream's next launch
    unsigned long long a[3];
    double c[6];
#pragma unroll
    for (int u = 0; u < 3; ++u) a[u] = sacc[min(tid + 256 * u, 8 * 82 - 1)];  // (clamped: used only in range below)
#pragma unroll
    for (int u = 0; u < 6; ++u) c[u] = cpg[min(tid + 256 * u, 16 * 81 + 15)];  // (clamped, as a[])
#pragma unroll
    for (int u = 0; u < 3; ++u)
      if (tid + 256 * u < 8 * 82) {
        strips[tid + 256 * u] = (double)a[u];
        sacc[tid + 256 * u] = 0ull;
      }
#pragma unroll
    for (int u = 0; u < 6; ++u) {
      const int e = tid + 256 * u;
      if (e < 16 * 81) cp[e / 81][e % 81] = c[u];
      else if (e < 16 * 81 + 16) cs[e - 16 * 81] = c[u];
    }
  } else {
    // every thread's (up to) 3 x 16 loads issued before the first add (r5_s29b: 5.4 us for this
    // phase with the loads issued per sum)
    double t[3][16];
#pragma unroll
    // (loads clamped into range and dropped at the add: guarded ones were waited for one by one)
    for (int u = 0; u < 3; ++u) {
      const int e = min(tid + 256 * u, 8 * 82 - 1), L = e / 82, d = e - L * 82;
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const int kc = min(k, nv - 1), b = kc / nch, ch = kc - b * nch;
        t[u][k] = strips_b[(((int64_t)b * 8 + L) * nch + ch) * 82 + d];
      }
    }
#pragma unroll
    for (int u = 0; u < 3; ++u) {
      const int e = tid + 256 * u, L = e / 82, d = e - L * 82;
      double v = 0.0;
#pragma unroll
      for (int k = 0; k < 16; ++k) v += (e < 8 * 82 && k < nv) ? t[u][k] : 0.0;
      for (int j = 16; j < nv; ++j) {  // (more than 16 image-chunks: the rest one by one)
        const int b = j / nch, ch = j - b * nch;
        v += strips_b[(((int64_t)b * 8 + L) * nch + ch) * 82 + d];
      }
      if (e < 8 * 82) strips[e] = v;
    }
  }
  if (tid < 82) full[tid] = fa;
  if (sacc == nullptr)
    for (int e = tid; e < 16 * 81 + 16; e += blockDim.x) {
      const double v = l1_corner_term(cx, B, H, W, e);
      if (e < 16 * 81) cp[e / 81][e % 81] = v;
      else cs[e - 16 * 81] = v;
    }
  __syncthreads();
  for (int e = tid; e < 625 + 25; e += blockDim.x) {
    const bool isS = e >= 625;
    const int k = isS ? e - 625 : e / 25, j = isS ? e - 625 : e % 25;
    const int oky = k / 5 - 2, okx = k % 5 - 2, ojy = j / 5 - 2, ojx = j % 5 - 2;
    const int dy = ojy - oky, dx = ojx - okx;
    const int di = (dy + 4) * 9 + (dx + 4);
    // excluded rows / cols of U_k (u = px + o_k must map back into the image)
    int er[2], ne = 0, ec[2], nc = 0;
    const int ak = isS ? ojy : oky, bk = isS ? ojx : okx;
    if (ak > 0) { for (int i = 0; i < ak; ++i) er[ne++] = i; }
    if (ak < 0) { for (int i = 0; i < -ak; ++i) er[ne++] = H - 1 - i; }
    if (bk > 0) { for (int i = 0; i < bk; ++i) ec[nc++] = i; }
    if (bk < 0) { for (int i = 0; i < -bk; ++i) ec[nc++] = W - 1 - i; }
    auto line_index_row = [&](int r) { return r < 2 ? r : (r - (H - 4)); };       // 0,1,2,3
    auto line_index_col = [&](int cidx) { return 4 + (cidx < 2 ? cidx : (cidx - (W - 4))); };
    double v;
    if (!isS) {
      v = full[di];
      for (int i = 0; i < ne; ++i) v -= strips[line_index_row(er[i]) * 82 + di];
      for (int i = 0; i < nc; ++i) v -= strips[line_index_col(ec[i]) * 82 + di];
      for (int i = 0; i < ne; ++i)
        for (int q = 0; q < nc; ++q) v += cp[line_index_row(er[i]) * 4 + (line_index_col(ec[q]) - 4)][di];
      G[k][j] = v * (xs * xs);
    } else {
      v = full[81];
      for (int i = 0; i < ne; ++i) v -= strips[line_index_row(er[i]) * 82 + 81];
      for (int i = 0; i < nc; ++i) v -= strips[line_index_col(ec[i]) * 82 + 81];
      for (int i = 0; i < ne; ++i)
        for (int q = 0; q < nc; ++q) v += cs[line_index_row(er[i]) * 4 + (line_index_col(ec[q]) - 4)];
      S[j] = v * xs;
    }
  }
  __syncthreads();
}

// What the Gram body reads besides the sums, staged in LDS by EVERY workgroup of its launch at the
// start (l1_gram_stage): the reducing workgroup only learns it is last after the column sums, and
// these loads issued then were rounds of global latency on the step's critical path (w1, the BN1
// parameters and running statistics, the image corners).
struct L1GramPre {
  float w1s[16 * 25];
  float prm[5][16];  // b1, gamma (1 if absent), beta (0), running mean, running var (0 if absent)
  L1Corners cx;
};

template <typename T>
__device__ __forceinline__ void l1_gram_stage(L1GramPre& pre, const T* __restrict__ x, int B, int H, int W,
                                              const float* __restrict__ w1, const float* __restrict__ b1,
                                              const float* __restrict__ gamma, const float* __restrict__ beta,
                                              const float* __restrict__ running_mean,
                                              const float* __restrict__ running_var) {
  const int tid = threadIdx.x;
  for (int e = tid; e < 16 * 25; e += blockDim.x) pre.w1s[e] = w1[e];
  if (tid < 80) {
    const int k = tid >> 4, c = tid & 15;
    const float* p = k == 0 ? b1 : k == 1 ? gamma : k == 2 ? beta : k == 3 ? running_mean : running_var;
    pre.prm[k][c] = p ? p[c] : (k == 1 ? 1.f : 0.f);
  }
  // corner blocks: x only inside the 6 x 6 pixel block at each image corner
#pragma unroll 4
  for (int e = tid; e < B * 144; e += blockDim.x) {
    const int b = e / 144, q = (e / 36) % 4, i = (e / 6) % 6, j = e % 6;
    const int r = q < 2 ? i : H - 6 + i, c = (q & 1) == 0 ? j : W - 6 + j;
    pre.cx.v[b][q][i][j] = (float)x[(int64_t)b * H * W + (int64_t)r * W + c];
  }
}

// Forward: Gram + patch sums (kept for the backward) and the BN1 statistics they
// imply, so conv1 never runs a separate statistics pass:
//   sum_px (y1 - b1)[c]   = w1[c] . S
//   sum_px (y1 - b1)^2[c] = w1[c]^T G w1[c]
// gram = G[625] | S[25] (fp64); sums = [c][sum, sumsq] in the bn_finalize_shifted layout.
// pre: l1_gram_stage's LDS (staged and synchronized by the caller).
template <typename T>
__device__ __forceinline__ void l1_gram_body(const double* __restrict__ ac_sum,
                                                      const double* __restrict__ strips, const T* __restrict__ x,
                                                      int B, int H, int W, const L1GramPre& pre,
                                                      double* __restrict__ gram, double* __restrict__ sums,
                                                      float eps, float momentum,
                                                      float* __restrict__ stats, float* __restrict__ running_mean,
                                                      float* __restrict__ running_var, int64_t* __restrict__ num_batches,
                                                      float* __restrict__ aff, double xs, int nch = 1,
                                                      uint32_t* __restrict__ p1inv = nullptr,
                                                      unsigned long long* __restrict__ sacc = nullptr,
                                                      const double* __restrict__ cpg = nullptr) {
  __shared__ double full[82];  // autocorrelation at the 81 offsets | the plain sum
  __shared__ double G[25][25];
  __shared__ double S[25];
  __shared__ double Gw[16][25];
  __shared__ double strips_sum[8 * 82];
  const float* w1s = pre.w1s;
  l1_build_gram(ac_sum, strips, x, B, H, W, G, S, full, strips_sum, pre.cx, xs, nch, sacc, cpg);
  const int tid = threadIdx.x;
  for (int e = tid; e < 650; e += blockDim.x) gram[e] = e < 625 ? G[e / 25][e % 25] : S[e - 625];
  for (int e = tid; e < 16 * 25; e += blockDim.x) {
    const int c = e / 25, j = e % 25;
    double h = 0.0;
    for (int k = 0; k < 25; ++k) h += (double)w1s[c * 25 + k] * G[k][j];
    Gw[c][j] = h * (double)w1s[c * 25 + j];
  }
  // p1's fp16 range guard (conv2's single operand, fp16x2): p1 = relu(gamma * xhat + beta) and,
  // for ANY batch, |xhat| <= sqrt(n - 1) (Samuelson's inequality, population variance; eps only
  // shrinks it), so max p1 <= max_c |gamma_c| sqrt(n - 1) + |beta_c| before the data is seen.
  // If that bound (with a 2^-10 margin for the conv's rounding) passes fp16's 65504, the BN1
  // affine -- and with it p1 -- is scaled by the power of two 2^e1 that keeps it in range
  // (ReLU and max-pool commute with it); aff[32] = 2^e1, taken out exactly by the conv2 kernels
  // (conv2_pack.hip records its inverse).  |gamma| <= ~9.7 at beta = 0 leaves e1 = 0, p1 as is.
  float p1_scale = 1.f;
  if (tid < 64) {
    const int c = tid & 15;
    const double sq = sqrt((double)((int64_t)B * H * W - 1));
    double bound = tid < 16 ? fabs((double)pre.prm[1][c]) * sq + fabs((double)pre.prm[2][c]) : 0.0;
    for (int off = 32; off > 0; off >>= 1) bound = fmax(bound, __shfl_xor(bound, off, 64));
    bound *= 1.0 + 1.0 / 1024.0;
    int e1 = 0;
    if (bound > 65504.0 && __builtin_isfinite(bound)) {
      int x;
      (void)frexp(bound / 65504.0, &x);  // bound / 65504 < 2^x
      e1 = -min(x, 120);
    }
    p1_scale = ldexpf(1.f, e1);
    if (tid == 0) aff[32] = p1_scale;
    // the conv2 kernels' copy of its inverse (mag[kMagScales + 1]), when the weight packing ran
    // ahead of this launch (models/convnet_fused.py: conv2_pack on a side stream)
    if (tid == 0 && p1inv != nullptr) *p1inv = __float_as_uint(1.f / p1_scale);
  }
  __syncthreads();
  if (tid < 16) {
    double s = 0.0, q = 0.0;
    for (int j = 0; j < 25; ++j) {
      s += (double)w1s[tid * 25 + j] * S[j];
      q += Gw[tid][j];
    }
    sums[tid * 2] = s;
    sums[tid * 2 + 1] = q;
    // BN1 statistics of (y1 - b1) finalized here (no separate finalize launch)
    if (tid == 0 && num_batches) num_batches[0] += 1;
    // bn_finalize_channel (bn_finalize.h) on the staged parameters
    const int64_t n = (int64_t)B * H * W;
    const double m0 = s / (double)n;
    double var = q / (double)n - m0 * m0;
    if (var < 0.0) var = 0.0;
    const double mean = m0 + (double)pre.prm[0][tid];
    const float invstd = (float)(1.0 / sqrt(var + (double)eps));
    stats[tid] = (float)mean;
    stats[16 + tid] = invstd;
    if (running_mean) {
      const double unb = n > 1 ? var * (double)n / (double)(n - 1) : var;
      running_mean[tid] = (float)((1.0 - momentum) * pre.prm[3][tid] + momentum * mean);
      running_var[tid] = (float)((1.0 - momentum) * pre.prm[4][tid] + momentum * unb);
    }
    const float gm = pre.prm[1][tid], bt = pre.prm[2][tid];
    aff[tid] = gm * invstd * p1_scale;
    aff[16 + tid] = (bt - (float)mean * gm * invstd) * p1_scale;
  }
}


template <typename T>
__global__ __launch_bounds__(256) void l1_gram_kernel(const double* __restrict__ ac_sum,
                                                      const double* __restrict__ strips, const T* __restrict__ x,
                                                      int B, int H, int W, const float* __restrict__ w1,
                                                      double* __restrict__ gram, double* __restrict__ sums,
                                                      const float* __restrict__ b1, float eps, float momentum,
                                                      const float* __restrict__ gamma, const float* __restrict__ beta,
                                                      float* __restrict__ stats, float* __restrict__ running_mean,
                                                      float* __restrict__ running_var, int64_t* __restrict__ num_batches,
                                                      float* __restrict__ aff, double xs, uint32_t* __restrict__ p1inv) {
  __shared__ L1GramPre pre;
  l1_gram_stage(pre, x, B, H, W, w1, b1, gamma, beta, running_mean, running_var);
  __syncthreads();
  l1_gram_body<T>(ac_sum, strips, x, B, H, W, pre, gram, sums, eps, momentum, stats, running_mean, running_var,
                  num_batches, aff, xs, 1, p1inv);
}

// The x autocorrelation partials' reduction and the Gram in ONE launch: workgroup e sums column
// e of the [nchunk][42] partials in reduce_partials_kernel's order (write-through), and the last
// to arrive (common.h tds_arrive) runs l1_gram_body on the sums -- one launch boundary and one
// launch floor fewer on the step's critical path than reduce_partials + l1_gram.
// BORDER (uint8 levels): workgroups 42 .. 42 + 4B*chunks - 1 form the border strips from x
// themselves (xmom_u8.h, one per image side and line chunk) and arrive with the column sums.
// pack.n > 0: the last pack.n workgroups pack conv2's weights (conv2_pack.h; they do not arrive:
// nothing of this launch reads their output, the conv2 kernels after it do), the Gram body storing
// 1 / p1_scale where the packing would have (p1inv).
struct L1Pack {
  const float* w2;
  short* wp;
  short* wd;
  uint32_t* mag;
  int n;
};
template <typename T, bool BORDER>
__global__ __launch_bounds__(256) void l1_reduce_gram_kernel(const double* __restrict__ ac_part, int nchunk,
                                                             double* __restrict__ ac_sum, uint32_t* __restrict__ sync,
                                                             double* __restrict__ strips, const T* __restrict__ x,
                                                             int B, int H, int W, const float* __restrict__ w1,
                                                             double* __restrict__ gram, double* __restrict__ sums,
                                                             const float* __restrict__ b1, float eps, float momentum,
                                                             const float* __restrict__ gamma,
                                                             const float* __restrict__ beta, float* __restrict__ stats,
                                                             float* __restrict__ running_mean,
                                                             float* __restrict__ running_var,
                                                             int64_t* __restrict__ num_batches, float* __restrict__ aff,
                                                             double xs, uint32_t* __restrict__ p1inv, L1Pack pack,
                                                             unsigned long long* __restrict__ sacc,
                                                             double* __restrict__ cpg) {
  __shared__ double sh[8];
  __shared__ int last;
  __shared__ L1GramPre pre;
  const int e = blockIdx.x;
  const int npart = (int)gridDim.x - pack.n;  // the workgroups that arrive
  if (e >= npart) {
    conv2_pack_block(pack.w2, pack.wp, pack.wd, pack.mag, nullptr, 0, e - npart, pack.n);
    return;
  }
  const int nch = BORDER ? xmom_border_chunks(H, W) : 1;
  if constexpr (BORDER) {
    __shared__ uint32_t lines[BSIDE_LDS_WORDS];
    if (e >= 42) {  // (e < npart)
      const int j = e - 42;
      x_border_side_u8(x, sacc, j / (4 * nch), (j / nch) & 3, j % nch, nch, H, W, lines);
    }
  }
  if (e < 42) {
    double s = 0.0;
#pragma unroll 16
    for (int k = threadIdx.x; k < nchunk; k += blockDim.x) s += ac_part[e + (int64_t)k * 42];
    s = block_sum(s, sh);
    if (threadIdx.x == 0) st_agent(ac_sum + e, s);
  }
  // (after the workgroup's own loads: issued first, the stage's loads put a round trip before them)
  l1_gram_stage(pre, x, B, H, W, w1, b1, gamma, beta, running_mean, running_var);  // (synchronized by tds_arrive)
  if constexpr (BORDER) {
    // the column workgroups form the Gram body's corner table meanwhile (32 entries each), handed
    // over with the sums
    if (e < 42) {
      __syncthreads();  // pre.cx staged
      const int i = e * 32 + (int)threadIdx.x;
      if (threadIdx.x < 32 && i < 16 * 81 + 16) st_agent(cpg + i, l1_corner_term(pre.cx, B, H, W, i));
    }
  }
  if (!tds_arrive(sync, (uint32_t)npart, &last)) return;
  l1_gram_body<T>(ac_sum, strips, x, B, H, W, pre, gram, sums, eps, momentum, stats, running_mean, running_var,
                  num_batches, aff, xs, nch, p1inv, BORDER ? sacc : nullptr, BORDER ? cpg : nullptr);
}

// Closed-form layer-1 gradients (one workgroup) from the l1_bwd sums and the Gram:
//   dw1[c][j] = a1 sdzx[c][j] + a2 (sum_k w1[c][k] G[k][j] + b1[c] S[j]) + a3 S[j]
// one thread per (c, j) (400 of 512); every thread of channel c forms its a1..a3 (25 FMAs).
__device__ __forceinline__ void l1_finalize_one(int e, const double* __restrict__ bwd_sum,
                                                const double* __restrict__ gram, int64_t n,
                                                const float* __restrict__ w1, const float* __restrict__ b1,
                                                const float* __restrict__ gamma1, const float* __restrict__ stats1,
                                                float* __restrict__ dw1, float* __restrict__ db1,
                                                float* __restrict__ dgamma1, float* __restrict__ dbeta1, float scale) {
  const int c = e / 25, j = e - 25 * (e / 25);
  const double* acc = bwd_sum + c * LB_NACC;
  const double* G = gram;
  const double* S = gram + 625;
  const double mean = stats1[c], is = stats1[16 + c];
  const double gm = gamma1 ? gamma1[c] : 1.0;
  const double sdz = acc[0];
  // sum dz1 * y1 = w1[c] . sum dz1 xpatch + b1[c] sum dz1  (y1 = w1 . xpatch + b1)
  double sdzy = (double)b1[c] * sdz;
  for (int k = 0; k < 25; ++k) sdzy += (double)w1[c * 25 + k] * acc[2 + k];
  const double sdxh = sdzy - mean * sdz;
  const double a1 = gm * is;
  const double a2 = -gm * is * is * is * sdxh / (double)n;
  const double a3 = -gm * is * sdz / (double)n - a2 * mean;
  if (j == 0) {
    if (dgamma1) dgamma1[c] = (float)(is * sdxh);
    if (dbeta1) dbeta1[c] = (float)sdz;
    // db1 = sum dy1 = a1 sdz + a2 sum y1 + a3 n  (sum y1 = n*mean)
    if (db1) db1[c] = (float)(scale * (a1 * sdz + a2 * (double)n * mean + a3 * (double)n));
  }
  double h = (double)b1[c] * S[j];
  for (int k = 0; k < 25; ++k) h += (double)w1[c * 25 + k] * G[k * 25 + j];
  dw1[c * 25 + j] = (float)(scale * (a1 * acc[2 + j] + a2 * h + a3 * S[j]));
}

// l1_finalize_one over the 400 (c, j) with its inputs staged in LDS by one round of loads (read
// through global memory, each thread's 75 dependent-free loads ran as a chain of latencies)
__device__ __forceinline__ void l1_finalize_body(const double* __restrict__ bwd_sum, const double* __restrict__ gram,
                                                 int64_t n, const float* __restrict__ w1, const float* __restrict__ b1,
                                                 const float* __restrict__ gamma1, const float* __restrict__ stats1,
                                                 float* __restrict__ dw1, float* __restrict__ db1,
                                                 float* __restrict__ dgamma1, float* __restrict__ dbeta1, float scale) {
  __shared__ double sg[650];
  __shared__ double sb[16 * LB_NACC];
  __shared__ float sw[16 * 25];
  const int t = threadIdx.x;
  for (int i = t; i < 650; i += blockDim.x) sg[i] = gram[i];
  for (int i = t; i < 16 * LB_NACC; i += blockDim.x) sb[i] = bwd_sum[i];
  for (int i = t; i < 16 * 25; i += blockDim.x) sw[i] = w1[i];
  __syncthreads();
  for (int e = t; e < 16 * 25; e += blockDim.x)
    l1_finalize_one(e, sb, sg, n, sw, b1, gamma1, stats1, dw1, db1, dgamma1, dbeta1, scale);
}

__global__ __launch_bounds__(512) void l1_finalize_kernel(const double* __restrict__ bwd_sum,
                                                          const double* __restrict__ gram, int64_t n,
                                                          const float* __restrict__ w1, const float* __restrict__ b1,
                                                          const float* __restrict__ gamma1,
                                                          const float* __restrict__ stats1, float* __restrict__ dw1,
                                                          float* __restrict__ db1, float* __restrict__ dgamma1,
                                                          float* __restrict__ dbeta1, float scale) {
  l1_finalize_body(bwd_sum, gram, n, w1, b1, gamma1, stats1, dw1, db1, dgamma1, dbeta1, scale);
}

// The layer-1 backward partials' reduction and the closed-form gradients in ONE launch: workgroup
// e sums columns 8e .. 8e+7 of the [rows][432] partials in a fixed order (write-through), the last
// to arrive runs l1_finalize_body.
constexpr int L1RF_LANES = 128;  // row lanes per column (workgroup = 8 x lanes threads; 32: 11.8 us, 128: 10.3, r5_s47)
static_assert(L1RF_LANES % 8 == 0 && L1RF_LANES >= 8 && L1RF_LANES <= 128, "l1_reduce_finalize lanes");
__global__ __launch_bounds__(8 * L1RF_LANES) void l1_reduce_finalize_kernel(const double* __restrict__ part, int nchunk,
                                                                 double* __restrict__ bwd_sum, uint32_t* __restrict__ sync,
                                                                 const double* __restrict__ gram, int64_t n,
                                                                 const float* __restrict__ w1,
                                                                 const float* __restrict__ b1,
                                                                 const float* __restrict__ gamma1,
                                                                 const float* __restrict__ stats1,
                                                                 float* __restrict__ dw1, float* __restrict__ db1,
                                                                 float* __restrict__ dgamma1,
                                                                 float* __restrict__ dbeta1, float scale) {
  // 8 columns per workgroup (54 workgroups: one arrival each on the counter instead of 432 --
  // same-address atomics serialize), L1RF_LANES row lanes per column; each lane issues 16 loads
  // together (rows past the end clamped and added as 0.0, which keeps the sum), so 1280 rows take one round of loads at
  // 128 lanes and three at 32
  constexpr int RL = L1RF_LANES;
  __shared__ double sh[RL][9];
  __shared__ int last;
  const int col = blockIdx.x * 8 + (threadIdx.x & 7), rl = threadIdx.x >> 3;
  double s = 0.0;
  for (int k = rl; k < nchunk; k += 16 * RL) {
    double v[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) v[j] = part[col + (int64_t)min(k + j * RL, nchunk - 1) * (16 * LB_NACC)];  // (clamped:
    // a load under a branch is waited for inside it, which serialises the batch)
#pragma unroll
    for (int j = 0; j < 16; ++j) s += k + j * RL < nchunk ? v[j] : 0.0;
  }
  sh[rl][threadIdx.x & 7] = s;
  __syncthreads();
  // fold to at most 32 row sums per column (fixed order), then 8 threads sum those in order
  __shared__ double sf[32][9];
  double(*rows)[9] = sh;
  if constexpr (RL > 32) {
    if (threadIdx.x < 256) {
      const int c = threadIdx.x & 7, p = threadIdx.x >> 3;
      double t = 0.0;
#pragma unroll
      for (int i = 0; i < RL / 32; ++i) t += sh[p * (RL / 32) + i][c];
      sf[p][c] = t;
    }
    __syncthreads();
    rows = sf;
  }
  if (threadIdx.x < 8) {
    double t = 0.0;
    for (int i = 0; i < (RL < 32 ? RL : 32); ++i) t += rows[i][threadIdx.x];
    st_agent(bwd_sum + col, t);
  }
  // the body's other inputs staged by every workgroup before the hand-off (the reducer learns it is
  // last only after its sums; loaded then they were a round of latency on the critical path)
  __shared__ double sg[650];
  __shared__ float sw[16 * 25], sp[64];  // w1 | b1[16], gamma1[16] (1 if absent), stats1[32]
  for (int i = threadIdx.x; i < 650; i += blockDim.x) sg[i] = gram[i];
  for (int i = threadIdx.x; i < 16 * 25; i += blockDim.x) sw[i] = w1[i];
  if (threadIdx.x < 64) {
    const int i = threadIdx.x;
    sp[i] = i < 16 ? b1[i] : i < 32 ? (gamma1 ? gamma1[i - 16] : 1.f) : stats1[i - 32];
  }
  if (!tds_arrive(sync, gridDim.x, &last)) return;
  __shared__ double sb[16 * LB_NACC];
  for (int i = threadIdx.x; i < 16 * LB_NACC; i += blockDim.x) sb[i] = bwd_sum[i];
  __syncthreads();
  for (int e = threadIdx.x; e < 16 * 25; e += blockDim.x)
    l1_finalize_one(e, sb, sg, n, sw, sp, sp + 16, sp + 32, dw1, db1, dgamma1, dbeta1, scale);
}

}  // namespace tds

using namespace tds;

int tds_fused_num_wg(int per_cu) { return tds_device_cus() * per_cu; }

void tds_l1_gram(const double* ac_sum, const double* strips, const void* x, bool levels, int B, int H, int W,
                 const float* w1,
                 double* gram, double* sums, const float* b1, float eps, float momentum, const float* gamma,
                 const float* beta, float* stats, float* running_mean, float* running_var, int64_t* num_batches,
                 float* aff, hipStream_t st, uint32_t* p1inv) {
  if (B > L1G_MAXB || H < 12 || W < 12) {
    tds_launch_fail("l1_gram: needs batch <= 32 and H, W >= 12");
    return;
  }
  if (levels)
    hipLaunchKernelGGL(l1_gram_kernel<uint8_t>, dim3(1), dim3(256), 0, st, ac_sum, strips,
                       static_cast<const uint8_t*>(x), B, H, W, w1, gram, sums, b1, eps, momentum, gamma, beta, stats,
                       running_mean, running_var, num_batches, aff, (double)L1_LEVEL_SCALE, p1inv);
  else
    hipLaunchKernelGGL(l1_gram_kernel<float>, dim3(1), dim3(256), 0, st, ac_sum, strips, static_cast<const float*>(x),
                       B, H, W, w1, gram, sums, b1, eps, momentum, gamma, beta, stats, running_mean, running_var,
                       num_batches, aff, 1.0, p1inv);
  TDS_LAUNCH_CHECK();
}

void tds_l1_apply(const void* x, bool levels, const float* w1, const float* b1, const float* aff, void* p1,
                  uint8_t* idx1, int nwg, int B, int H, int W, hipStream_t st) {
  if (levels)
    hipLaunchKernelGGL(l1_conv_bf3_kernel<true>, dim3(nwg), dim3(256), 0, st, x, w1, b1, aff,
                       reinterpret_cast<uint4*>(p1), idx1, B, H, W);
  else
    hipLaunchKernelGGL(l1_conv_bf3_kernel<false>, dim3(nwg), dim3(256), 0, st, x, w1, b1, aff,
                       reinterpret_cast<uint4*>(p1), idx1, B, H, W);
  TDS_LAUNCH_CHECK();
}

void tds_bn_finalize_shifted(const double* partial, int C, int nchunk, int64_t n, const float* shift, float eps,
                             float momentum, const float* gamma, const float* beta, float* stats, float* running_mean,
                             float* running_var, int64_t* num_batches, float* aff, hipStream_t st) {
  hipLaunchKernelGGL(bn_finalize_shifted_kernel, dim3(1), dim3(64), 0, st, partial, C, nchunk, n, shift, eps, momentum,
                     gamma, beta, stats, running_mean, running_var, num_batches, aff);
  TDS_LAUNCH_CHECK();
}

void tds_bn_reduce_finalize(const double* partial, int C, int nchunk, int64_t n, const float* shift, float eps,
                            float momentum, const float* gamma, const float* beta, float* stats, float* running_mean,
                            float* running_var, int64_t* num_batches, float* aff, hipStream_t st) {
  hipLaunchKernelGGL(bn_reduce_finalize_kernel, dim3(C), dim3(256), 0, st, partial, C, nchunk, n, shift, eps, momentum,
                     gamma, beta, stats, running_mean, running_var, num_batches, aff);
  TDS_LAUNCH_CHECK();
}

void tds_reduce_partials(const double* in, double* out, int n, int nchunk, int inner, int64_t ostride, int64_t kstride,
                         hipStream_t st) {
  hipLaunchKernelGGL(reduce_partials_kernel, dim3(n), dim3(256), 0, st, in, out, nchunk, inner, ostride, kstride);
  TDS_LAUNCH_CHECK();
}

void tds_bn_bwd_finalize2(const double* partial, int C, int nchunk, int64_t n, const float* gamma, const float* stats,
                          float* dgamma, float* dbeta, float* kbuf, const float* dl, int B, int NC, float* dbfc,
                          float scale, const uint32_t* ypart, int nyp, const uint32_t* gpart, int ngp, uint32_t* mag,
                          hipStream_t st) {
  if (dbfc && (NC < 1 || NC > 256)) {
    tds_launch_fail("bn_bwd_finalize2: the fc bias gradient needs 1 <= classes <= 256");
    return;
  }
  hipLaunchKernelGGL(bn_bwd_finalize2_kernel, dim3(C + 1), dim3(256), 0, st, partial, C, nchunk, n, gamma, stats, dgamma,
                     dbeta, kbuf, nullptr, dl, B, NC, dbfc, scale, ypart, nyp, gpart, ngp, mag);
  TDS_LAUNCH_CHECK();
}

int tds_l1_bwd_rows(int nwg) { return nwg; }

// workgroups of the chosen layer-1 backward variant that fit one CU (its VGPRs decide: 87-99 for
// the level-input word layout -> 5, the fp32-image path -> 4)
int tds_l1_bwd_max_per_cu(bool levels) {
  int n = 0;
  const hipError_t e = levels ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, l1_bwd_mfma_kernel<true>, 256, 0)
                              : hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, l1_bwd_mfma_kernel<false>, 256, 0);
  return e == hipSuccess && n > 0 ? n : 4;
}

void tds_l1_bwd(const void* x, bool levels, const void* dp1h, const uint32_t* dp1_dec, const void* p1,
                const uint8_t* idx1, double* partial, int nwg, int B, int H, int W, hipStream_t st) {
  const uint4* d = static_cast<const uint4*>(dp1h);
  if (levels)
    hipLaunchKernelGGL((l1_bwd_mfma_kernel<true>), dim3(nwg), dim3(256), 0, st, x, d, dp1_dec,
                       reinterpret_cast<const uint4*>(p1), idx1, partial, B, H, W);
  else
    hipLaunchKernelGGL((l1_bwd_mfma_kernel<false>), dim3(nwg), dim3(256), 0, st, x, d, dp1_dec,
                       reinterpret_cast<const uint4*>(p1), idx1, partial, B, H, W);
  TDS_LAUNCH_CHECK();
}

void tds_l1_finalize(const double* bwd_sum, const double* gram, int64_t n, const float* w1, const float* b1,
                     const float* gamma1, const float* stats1, float* dw1, float* db1, float* dgamma1, float* dbeta1,
                     float scale, hipStream_t st) {
  hipLaunchKernelGGL(l1_finalize_kernel, dim3(1), dim3(512), 0, st, bwd_sum, gram, n, w1, b1, gamma1, stats1, dw1, db1,
                     dgamma1, dbeta1, scale);
  TDS_LAUNCH_CHECK();
}

// the [rows][432] partials' reduction + tds_l1_finalize in one launch (bwd_sum: the 432 sums, written)
bool tds_l1_reduce_finalize(const double* part, int rows, double* bwd_sum, const double* gram, int64_t n,
                            const float* w1, const float* b1, const float* gamma1, const float* stats1, float* dw1,
                            float* db1, float* dgamma1, float* dbeta1, float scale, hipStream_t st) {
  uint32_t* sync = tds_sync_words(kSyncL1Fin, st);
  if (sync == nullptr) return false;
  static_assert((16 * LB_NACC) % 8 == 0, "8 columns per workgroup");
  hipLaunchKernelGGL(l1_reduce_finalize_kernel, dim3(16 * LB_NACC / 8), dim3(8 * L1RF_LANES), 0, st, part, rows, bwd_sum, sync, gram,
                     n, w1, b1, gamma1, stats1, dw1, db1, dgamma1, dbeta1, scale);
  TDS_LAUNCH_CHECK();
  return true;
}

// the x autocorrelation partials' reduction [nchunk][42] -> ac_sum + tds_l1_gram in one launch
int tds_xmom_border_chunks(int H, int W) { return xmom_border_chunks(H, W); }

// border: the strips are formed in this launch (uint8 levels only, lines <= XMOM_MAX_LINE long) into
// strips [B][8][tds_xmom_border_chunks][82]
bool tds_l1_reduce_gram(const double* ac_part, int nchunk, double* ac_sum, double* strips, const void* x,
                        bool levels, int B, int H, int W, const float* w1, double* gram, double* sums, const float* b1,
                        float eps, float momentum, const float* gamma, const float* beta, float* stats,
                        float* running_mean, float* running_var, int64_t* num_batches, float* aff, hipStream_t st,
                        bool border, uint32_t* p1inv, const float* pack_w2, short* pack_wp, short* pack_wd,
                        uint32_t* pack_mag) {
  // conv2's weight packing on extra workgroups of this launch (64, as conv2_pack_weights_kernel)
  const L1Pack pack{pack_w2, pack_wp, pack_wd, pack_mag, pack_w2 != nullptr ? 64 : 0};
  if (pack.n > 0 && p1inv == nullptr) {
    tds_launch_fail("l1_reduce_gram: packing conv2's weights in the launch needs the p1 inverse slot");
    return true;
  }
  if (B > L1G_MAXB || H < 12 || W < 12) {
    tds_launch_fail("l1_gram: needs batch <= 32 and H, W >= 12");
    return true;
  }
  if (border && (!levels || W % 4 != 0 || H > XMOM_MAX_LINE || W > XMOM_MAX_LINE || (int64_t)H * W > 0xFFFFFFF0LL)) {
    tds_launch_fail("l1_reduce_gram: in-launch border strips need uint8 levels, W % 4 == 0 and lines <= 66051");
    return true;
  }
  uint32_t* sync = tds_sync_words(kSyncL1Gram, st);
  if (sync == nullptr) return false;
  // border: the strips accumulate in a zeroed u64 block (8 x 82 words) and the strips buffer (>= 1312
  // doubles: B * 8 * chunks * 82) carries the corner table
  unsigned long long* sacc = nullptr;
  if (border) {
    sacc = tds_zeroed_u64(0, 8 * 82, st);
    if (sacc == nullptr) return false;
  }
  if (levels && border)
    hipLaunchKernelGGL((l1_reduce_gram_kernel<uint8_t, true>), dim3(42 + 4 * B * xmom_border_chunks(H, W) + pack.n),
                       dim3(256),
                       0, st, ac_part, nchunk,
                       ac_sum, sync, strips, static_cast<const uint8_t*>(x), B, H, W, w1, gram, sums, b1, eps, momentum,
                       gamma, beta, stats, running_mean, running_var, num_batches, aff, (double)L1_LEVEL_SCALE, p1inv, pack,
                       sacc, strips);
  else if (levels)
    hipLaunchKernelGGL((l1_reduce_gram_kernel<uint8_t, false>), dim3(42 + pack.n), dim3(256), 0, st, ac_part, nchunk, ac_sum,
                       sync, strips, static_cast<const uint8_t*>(x), B, H, W, w1, gram, sums, b1, eps, momentum, gamma,
                       beta, stats, running_mean, running_var, num_batches, aff, (double)L1_LEVEL_SCALE, p1inv, pack,
                       nullptr, nullptr);
  else
    hipLaunchKernelGGL((l1_reduce_gram_kernel<float, false>), dim3(42 + pack.n), dim3(256), 0, st, ac_part, nchunk, ac_sum, sync,
                       strips, static_cast<const float*>(x), B, H, W, w1, gram, sums, b1, eps, momentum, gamma, beta,
                       stats, running_mean, running_var, num_batches, aff, 1.0, p1inv, pack, nullptr, nullptr);
  TDS_LAUNCH_CHECK();
  return true;
}
