// conv2 forward v2 (Conv2d(16, 32, 5, pad 2), mnist_onegpu.py:20):
// y2 = conv(p1) + b2, stored as y2h (NHWC fp16, bias-free, scaled: conv2_common.h), plus BN2
// batch-statistic partials, on
// v_mfma_f32_16x16x32_f16 in the TF32 class (conv2_common.h): ONE MFMA per product, p1 and the
// weights each rounded once to fp16 (11 significant bits, TF32's significand) at exact
// power-of-two range scales.  Laid out for SEVERAL small
// workgroups per CU (3 at 168 VGPRs, 44 KiB LDS):
//   * 4 waves per workgroup, output tile 8 rows x 16 columns (staged p1: 12 x 20 records of
//     32 B);
//   * weights in REGISTERS: wave w owns co half nt = w & 1 and output rows 4(w>>1) .. +3,
//     all 13 K-steps of its half (13 fp16 fragments), loaded once;
//   * p1 staged by LDS-DMA (global_load_lds_dwordx4, no VGPRs, no VALU), double-buffered:
//     tile t+1 streams in while tile t is on the MFMAs;
//   * the epilogue of tile t (y2h stores + statistics) runs after tile t+1's DMA is issued,
//     from a second accumulator set, so the stores drain under the next MFMAs;
//   * the epilogue also resolves the 2x2 max-pool of the BN2 output: BN2's affine a*y + b is
//     monotone per channel with the sign of gamma (a = gamma * invstd), so the window's
//     argmax value is max(y2) (gamma >= 0) or min(y2) (gamma < 0) -- known before the batch
//     statistics are.  Every lane holds whole windows of its channel, the 4 x 8 pooled block
//     of the tile is staged in LDS and stored as ya (pooled_layout.h) in fp16: the y2h value at
//     the window's argmax (y2 = h d + b2, launchers.h TdsYaDec), one 64-B run per channel.  The
//     head then streams ya (36 MB per image at 3000^2) instead of y2 (288 MB in fp32).
//   * max |y2 - b2| per channel and workgroup goes to ypart (a region of the step's magnitude-bound
//     workspace, fused_ops.cpp "mag"); reduced with the head backward's max |g2m| by the BN2
//     backward finalize, it bounds the conv2 output gradient, whose fp16 scale the backward
//     picks from it.
// K order and input-row sharing as conv2_fwd_bf16x3_kernel: K-step s < 10 pairs taps
// (ky = s>>1, kx = 2(s&1) + (g>>1)) so one staged input row R serves output rows R - ky;
// s = 10 + kp pairs (ky = 2kp + (g>>1), kx = 4) with lane groups 2-3 reading row R+1.
#include <cstdlib>

#include "bn_finalize.h"
#include "conv2_common.h"
#include "launchers.h"
#include "pooled_layout.h"

namespace tds {

constexpr int F2_TH = 8, F2_TC = 16;
constexpr int F2_SR = F2_TH + 4, F2_SC = F2_TC + 4;  // 12 x 20 staged records
constexpr int F2_REC = F2_SR * F2_SC;                  // 240
constexpr int F2_THREADS = 256;
constexpr int F2_PGROUPS = 8;                          // DMA groups of 32 records (1 KiB)
constexpr int F2_PPLANE = F2_PGROUPS * 32 * 32;        // 8192 B (256 records of 32 B, 240 used)
constexpr int F2_PBUF = F2_PPLANE;                     // one fp16 plane
// 3 workgroups per CU: the staged tile holds the y2h halves themselves (channel pairs joined by one
// DPP move), 44 KiB of LDS, 168 VGPRs -- 0.427 -> 0.407 ms isolated against 2 workgroups with one
// dword per value (tools/gpu_sessions/r4_s22.sh)
constexpr int F2_WG = 3;
constexpr int F2_PXREC = 32 * 2 + 16;  // staged pixel record: 32 co fp16 + 16 B pad (banks)
constexpr int F2_STAGE = F2_TH * F2_TC * F2_PXREC;           // a finished tile's padded staging buffer
constexpr int F2_OFF_S = 2 * F2_PBUF;                  // p1 double buffer first (32 KiB)
constexpr int F2_YSTAGE = 32 * 32 * 4 + 32 * 2 * 4;     // pooled block: 32 co x 4 x 8 words (fp16 bits) = 4 KiB, + a2 words
constexpr int F2_OFF_Y = F2_OFF_S + 2 * F2_STAGE;
constexpr int F2_LDS = F2_OFF_Y + 2 * F2_YSTAGE;       // + double-buffered output staging
constexpr int F2_DMA_PER_WAVE = F2_PGROUPS / (F2_THREADS / 64);  // 2
static_assert(F2_LDS % 16 == 0, "LDS carve");
static_assert(F2_WG * F2_LDS <= 160 * 1024, "workgroups per CU");

// 16 zero bytes: the DMA source of staged records outside the image
__device__ __attribute__((aligned(16))) uint32_t g_f2_zero[4] = {0u, 0u, 0u, 0u};

struct F2Tile {
  int b, r0, c0;
};

template <int DIAG, int WV>
__device__ __forceinline__ void f2_dma(const uint4* __restrict__ p1, const F2Tile& x, int P, char* buf, int lane) {
  if constexpr (DIAG == 3) return;
  const char* base = reinterpret_cast<const char*>(p1) + (((int64_t)x.b * P + x.r0 - 2) * P + (x.c0 - 2)) * 32;
#pragma unroll
  for (int j = 0; j < F2_DMA_PER_WAVE; ++j) {
    const int rg = WV * F2_DMA_PER_WAVE + j;
    const int px = rg * 32 + (lane >> 1), half = lane & 1;
    const int rr = px / F2_SC, cc = px - rr * F2_SC;
    const int gr = x.r0 - 2 + rr, gc = x.c0 - 2 + cc;
    const bool ok = px < F2_REC && gr >= 0 && gr < P && gc >= 0 && gc < P;
    const char* src = ok ? base + ((int64_t)rr * P + cc) * 32 + half * 16 : reinterpret_cast<const char*>(g_f2_zero);
    __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)(buf + rg * 1024), 16, 0, 0);
  }
}

// One wave's MFMAs for one tile: rows 4RH .. 4RH+3 of the tile, co half NT (weights in W).
// The 24 A-fragment row loads (3 tap groups x 8 staged rows) form one sequence read through
// a 4-deep register ring, 3 rows ahead of the MFMAs that use them: the rows at a group's
// edges feed only 1-2 MFMA triples, too few to hide an LDS round trip one row ahead.
template <int DIAG>
__device__ __forceinline__ void f2_compute(const char* buf, const f32x4 (&W)[13], f32x4 (&acc)[4], int RH, int lane) {
  constexpr int DEPTH = 4;
  const int li = lane & 15, g = lane >> 4;
  const int boff = (g & 1) * 16;  // ci half of the 32-B record
  const char* ph = buf;
#pragma unroll
  for (int o = 0; o < 4; ++o) acc[o] = f32x4{0.f, 0.f, 0.f, 0.f};
  s16x8 ah[DEPTH];
  // load i: group i / 8 (0, 1: kx pairs 2a + (g>>1); 2: kx = 4 with lane groups 2-3 one row down)
  auto load_a = [&](int i) {
    const int grp = i >> 3, R = i & 7;
    int rec;
    if (grp < 2) {
      rec = (4 * RH + R) * F2_SC + li + 2 * grp + (g >> 1);
    } else {
      int row = 4 * RH + R + (g >> 1);
      if (row > F2_SR - 1) row = F2_SR - 1;  // only reached with a zero weight (ky = 5)
      rec = row * F2_SC + li + 4;
    }
    ah[i % DEPTH] = lds8<DIAG>(ph + rec * 32 + boff);
  };
#pragma unroll
  for (int i = 0; i < DEPTH - 1; ++i) load_a(i);
#pragma unroll
  for (int i = 0; i < 24; ++i) {
    if (i + DEPTH - 1 < 24) load_a(i + DEPTH - 1);
    __builtin_amdgcn_sched_barrier(0);  // keep the ring's loads ahead of this row's MFMAs
    const int grp = i >> 3, R = i & 7, cur = i % DEPTH;
    if (grp < 2) {
#pragma unroll
      for (int ky = 0; ky < 5; ++ky) {
        const int o = R - ky;
        if (o >= 0 && o < 4)
          acc[o] = mmaw<DIAG>(ah[cur], __builtin_bit_cast(s16x8, W[2 * ky + grp]), acc[o]);
      }
    } else {
#pragma unroll
      for (int kp = 0; kp < 3; ++kp) {
        const int o = R - 2 * kp;
        if (o >= 0 && o < 4)
          acc[o] = mmaw<DIAG>(ah[cur], __builtin_bit_cast(s16x8, W[10 + kp]), acc[o]);
      }
    }
  }
}

// A finished tile goes to LDS first ([row][px][32 co] with 144-B pixel records: the 16-B pad
// puts the 4 lane groups' pixels 4g + r on disjoint bank quarters, so the MFMA-layout writes
// are conflict-free AND every lane's 16 writes are one base register plus immediate offsets --
// the XOR swizzle it replaces cost 2-3 VALU per element), then the workgroup stores it as full
// 128-B pixel records, 1 KiB contiguous per wave-instruction.  (Stored straight from the MFMA
// layout, each wave wrote 64-B halves of lines whose other half came from another wave: the y2
// writes then cost ~0.3 ms more, TDS_CONV2_DIAG=4.)
__device__ __forceinline__ int f2_stage_off(int row, int px, int chunk) {  // chunk: 16 B
  return (row * F2_TC + px) * F2_PXREC + chunk * 16;
}

// pooled block staging: channel co's 32 floats [prow 4][pcol 8], float4 chunks XOR-swizzled by co
__device__ __forceinline__ int f2_ystage_off(int co, int e) { return co * 32 + ((((e >> 2) ^ co) & 7) << 2) + (e & 3); }

// window extreme in the direction of BN2's affine; a NaN anywhere wins (torch's max-pool rule):
// v_maximum3_f32 / v_minimum3_f32 (IEEE maximum/minimum, NaN-propagating) on gfx950
__device__ __forceinline__ float f2_ext4(float a, float b, float c, float d, bool neg) {
  const float mx = __builtin_elementwise_maximum(__builtin_elementwise_maximum(a, b), __builtin_elementwise_maximum(c, d));
  const float mn = __builtin_elementwise_minimum(__builtin_elementwise_minimum(a, b), __builtin_elementwise_minimum(c, d));
  return neg ? mn : mx;
}

// stage + shifted statistics of one finished tile: lane holds C[px = 4g + r][co = 16NT + li].
// EDGE: a tile reaching past the image (last tile row / column) masks its statistics; interior
// tiles (all but ~1 %) accumulate unmasked, in packed fp32 (v_pk_add_f32 / v_pk_fma_f32: two
// outputs per instruction), and take max |y2 - b2| as max |acc| with the NaN-propagating
// v_maximum_f32 (|v| as a source modifier; scaled by inv once per workgroup).  A wave64 VALU
// instruction holds its SIMD for 4 cycles, and that issue competes with the same SIMD's MFMAs.
typedef float f2v __attribute__((ext_vector_type(2)));
// PLAIN: every lane of the wave has gamma2 > 0 (wave-uniform, the usual case): the window extreme is
// its maximum, no minimum / select / gamma2 == 0 case
template <bool EDGE, bool PLAIN>
__device__ __forceinline__ void f2_stage(const f32x4 (&acc)[4], const F2Tile& x, char* stage, float* ystage, int P,
                                         int RH, int NT, int lane, float bco, float inv, float ksc, bool neg, bool zg,
                                         f2v& s_acc, f2v& q_acc, uint32_t& ymx, uint32_t* __restrict__ a2) {
  const int li = lane & 15, g = lane >> 4;
  const int co = 16 * NT + li;
  float ymf = 0.f;
  uint32_t h[4][4];  // y2h bits (conv2_common.h)
#pragma unroll
  for (int o = 0; o < 4; ++o)
#pragma unroll
    for (int r = 0; r < 4; ++r) h[o][r] = f16_bits(acc[o][r] * ksc);
  // acc = (y2 - b2) / inv: statistics shifted by the bias, scaled at the end
#pragma unroll
  for (int o = 0; o < 4; ++o) {
    const int row = 4 * RH + o;
    const bool rok = !EDGE || x.r0 + row < P;
    if constexpr (EDGE) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float v = acc[o][r];
        if (rok && x.c0 + 4 * g + r < P) {
          s_acc.x += v;
          q_acc.x += v * v;
          ymx = max(ymx, __float_as_uint(v) & 0x7fffffffu);  // |v| bits (NaN: above every finite)
        }
      }
    } else {
#pragma unroll
      for (int r = 0; r < 4; r += 2) {
        const f2v v = {acc[o][r], acc[o][r + 1]};
        s_acc += v;
        q_acc = __builtin_elementwise_fma(v, v, q_acc);
        ymf = __builtin_elementwise_maximum(ymf, __builtin_elementwise_maximum(fabsf(v.x), fabsf(v.y)));  // NaN wins
      }
    }
  }
  if constexpr (!EDGE) ymx = max(ymx, __float_as_uint(ymf));
  // pooled windows (rows 4RH + 2i + {0,1}, columns 4g + 2j + {0,1}) -> ya block entry
  // (prow 2RH + i, pcol 2g + j): the fp16 bits of the window's extreme as y2h stores it (v -> v *
  // ksc is monotone and rounds monotonically, so this is y2h at the argmax pixel)
  // and the argmax codes (a2, conv2_common.h): the first extreme in scan order, two code bits per
  // channel gathered by ballots (lane = 16 g + li: channel 16NT + li of window column 2g + j)
  uint64_t cb0[4], cb1[4];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    uint32_t e[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const float v0 = acc[2 * i][2 * j], v1 = acc[2 * i][2 * j + 1], v2 = acc[2 * i + 1][2 * j];
      // gamma2 == 0 (zg): every BN2 output of the window is beta2 and torch's max-pool keeps the
      // first position: code 0, and ya holds that position's value (the head backward's dgamma2
      // reads xhat there)
      const float v3 = acc[2 * i + 1][2 * j + 1];
      float m;
      if constexpr (PLAIN)
        m = __builtin_elementwise_maximum(__builtin_elementwise_maximum(v0, v1), __builtin_elementwise_maximum(v2, v3));
      else
        m = zg ? v0 : f2_ext4(v0, v1, v2, v3, neg);
      e[j] = f16_bits(m * ksc);
      // (a NaN window: code 3, unused); the code bits from the three comparisons' ballots by
      // scalar logic (as lane booleans the compiler formed them with ~4 VALU selects a window)
      const uint64_t b0 = __builtin_amdgcn_ballot_w64(v0 == m), b1 = __builtin_amdgcn_ballot_w64(v1 == m),
                     b2 = __builtin_amdgcn_ballot_w64(v2 == m);
      cb0[2 * i + j] = ~b0 & (b1 | ~b2);  // code 1 or 3
      cb1[2 * i + j] = ~b0 & ~b1;         // code 2 or 3
    }
    // pcols 2g, 2g+1 are adjacent words of one swizzled chunk: one ds_write_b64
    *reinterpret_cast<uint2*>(ystage + f2_ystage_off(co, (2 * RH + i) * 8 + 2 * g)) = make_uint2(e[0], e[1]);
  }
  // lane li = 0 of group g stages the 4 windows (2RH + i, 2g + j) in LDS after the pooled block
  // (word = bits 16g .. 16g+15 of each code-bit ballot: channels 16NT + 0..15); f2_store_a2 writes
  // the tile's 32 windows as 4 rows of 64 B
  {
    uint32_t* ab = reinterpret_cast<uint32_t*>(ystage + 32 * 32);
    // group g's 16 bits of each ballot: the 32-bit half (g >= 2: upper), then one byte permute takes
    // bits 16(g & 1) .. +15 of both code-bit words (a 64-bit shift by the per-lane 16g cost ~9 VALU a window)
    const bool upper = g >= 2;
    const uint32_t psel = (g & 1) ? 0x07060302u : 0x05040100u;
    if (li == 0) {
#pragma unroll
      for (int sl = 0; sl < 4; ++sl) {
        const uint32_t w0 = upper ? (uint32_t)(cb0[sl] >> 32) : (uint32_t)cb0[sl];
        const uint32_t w1 = upper ? (uint32_t)(cb1[sl] >> 32) : (uint32_t)cb1[sl];
        ab[((2 * RH + (sl >> 1)) * 8 + 2 * g + (sl & 1)) * 2 + NT] = __builtin_amdgcn_perm(w1, w0, psel);
      }
    }
  }
  // the y2h values: every lane writes its channel's half-word (no cross-lane pairing: the DPP move
  // and the pack cost 2 VALU per value)
#pragma unroll
  for (int o = 0; o < 4; ++o)
#pragma unroll
    for (int r = 0; r < 4; ++r)
      *reinterpret_cast<unsigned short*>(stage + (((4 * RH + o) * F2_TC + 4 * g + r) * F2_PXREC) + co * 2) =
          (unsigned short)h[o][r];
}

// the workgroup stores the staged pooled block: thread e -> channel e / 8, 4 values (8 B) e % 8
__device__ __forceinline__ void f2_store_ya(const float* ystage, const F2Tile& x, unsigned short* __restrict__ ya,
                                            const PBGeom& pg) {
  const int tr = x.r0 / F2_TH, tc = x.c0 / F2_TC;  // = the tile's pooled block
  if (tr >= pg.Q4 || tc >= pg.Q8) return;          // (odd P: a last tile row beyond the pooled image)
  const int e = threadIdx.x, co = e >> 3, part = e & 7;
  const uint4 v = *reinterpret_cast<const uint4*>(ystage + f2_ystage_off(co, part * 4));
  st_stream(reinterpret_cast<uint2*>(ya + ((((int64_t)x.b * 32 + co) * pg.Q4 + tr) * pg.Q8 + tc) * 32 + part * 4),
            make_uint2(__builtin_amdgcn_perm(v.y, v.x, 0x05040100u), __builtin_amdgcn_perm(v.w, v.z, 0x05040100u)));
}

// the tile's 32 pooling windows' argmax words (a2, conv2_common.h): thread e < 32 -> window e
__device__ __forceinline__ void f2_store_a2(const float* ystage, const F2Tile& x, uint32_t* __restrict__ a2, int P) {
  const int e = threadIdx.x, Q = P >> 1;
  const int py = (x.r0 >> 1) + (e >> 3), px = (x.c0 >> 1) + (e & 7);
  if (e < 32 && py < Q && px < Q)  // (non-temporal, as y2h: dirty lines left to the head forward cost it ~5 us)
    st_stream(reinterpret_cast<uint2*>(a2 + (((int64_t)x.b * Q + py) * Q + px) * 2),
              reinterpret_cast<const uint2*>(ystage + 32 * 32)[e]);
}

// the whole workgroup stores a staged tile as y2h: thread e, i -> 8 channels q = e + 256 i of
// [row 8][px 16][c8 4] (two staged 4-channel chunks packed to 16 B): a wave-instruction writes
// 1 KiB, 16 pixels of one row.  H16: lane quad -> pixel through F2_QPX, so each 16-lane bank
// group of ds_read_b128 ({0-3,12-15,20-27}, ...) reads pixels p, p+4, p+8, p+12, whose 80-B
// records start 0, 64, 128, 192 B apart mod 256 -- conflict-free (quad = pixel read 3-way).
constexpr uint64_t F2_QPX = 0xfeab6732dc894510ull;  // nibble quad -> px
template <int DIAG>
__device__ __forceinline__ void f2_store(const char* stage, const F2Tile& x, unsigned short* __restrict__ y2h, int P) {
  if constexpr (DIAG == 4) return;  // timing-only: no y2h
  const int e = threadIdx.x;
  const int qpx = (int)((F2_QPX >> (4 * ((e >> 2) & 15))) & 15u);
#pragma unroll
  for (int i = 0; i < F2_TH * F2_TC * 4 / F2_THREADS; ++i) {
    const int q = e + F2_THREADS * i;
    const int row = q >> 6, px = qpx, c8 = q & 3;
    const int gr = x.r0 + row, gc = x.c0 + px;
    const uint4 v = *reinterpret_cast<const uint4*>(stage + f2_stage_off(row, px, c8));
    if (gr < P && gc < P)
      st_stream(reinterpret_cast<float4*>(y2h + (((int64_t)x.b * P + gr) * P + gc) * 32 + c8 * 8),
                __builtin_bit_cast(float4, v));
  }
}

template <int DIAG, int WV>
__device__ __forceinline__ void f2_run(const uint4* __restrict__ p1, const uint4* __restrict__ wpack,
                                       const float* __restrict__ bias, const float* __restrict__ gamma,
                                       unsigned short* __restrict__ y2, unsigned short* __restrict__ ya,
                                       uint32_t* __restrict__ a2,
                                       double* __restrict__ partial, uint32_t* __restrict__ ypart,
                                       const uint32_t* __restrict__ scales,
                                       const int* __restrict__ order, int sw, int sk, int B, int P, char* smem) {
  constexpr int NT = WV & 1, RH = WV >> 1;
  const int lane = threadIdx.x & 63, li = lane & 15;
  const int tiles_c = (P + F2_TC - 1) / F2_TC, tiles_r = (P + F2_TH - 1) / F2_TH;
  const int per_img = tiles_c * tiles_r, total = per_img * B;
  const int w = xcd_remap(blockIdx.x, gridDim.x);
  // work index t = w + kk * grid at mine[kk * sk]: the table is per workgroup (fused_ops.cpp
  // tile_order, sw = ceil(total / grid), sk = 1), so consecutive tiles share a scalar-cache line
  const int* __restrict__ mine = order + w * sw;
  auto decode = [&](int kk) {
    F2Tile x;
    int tr, tc;
    tile_from_order(mine, kk * sk, x.b, tr, tc);
    x.r0 = tr * F2_TH;
    x.c0 = tc * F2_TC;
    return x;
  };
  // weights: fwd pack wp[s][nt][g][co16][j8] -> uint4 index (s * 2 + nt) * 64 + lane (conv2_pack.hip)
  f32x4 W[13];
#pragma unroll
  for (int s = 0; s < 13; ++s) W[s] = __builtin_bit_cast(f32x4, wpack[(s * 2 + NT) * 64 + lane]);
  const float bco = bias[16 * NT + li];
  // the packed weights' and p1's power-of-two scales (conv2_pack.hip): y2 = acc * inv + b2, exact
  const float inv = scales != nullptr ? __uint_as_float(scales[0]) * __uint_as_float(scales[1]) : 1.f;
  const float ksc = scales != nullptr ? __uint_as_float(scales[2]) : 1.f;  // y2h store factor
  const bool neg = gamma != nullptr && gamma[16 * NT + li] < 0.f;
  const bool zg = gamma != nullptr && gamma[16 * NT + li] == 0.f;
  const bool plain = __builtin_amdgcn_readfirstlane(__builtin_amdgcn_ballot_w64(neg || zg) == 0 ? 1 : 0) != 0;
  const PBGeom pg = pb_geom(P / 2);
  float* ys = reinterpret_cast<float*>(smem + F2_OFF_Y);
  // BN2 partials: each tile's sums in fp32 (<= 16 values per lane), accumulated across the
  // workgroup's tiles in fp64 (one fp32 running sum per lane over ~1.8 K values had rounding that
  // grows with n (1 + mean^2 / var) in var = E[q] - E[s]^2)
  f2v s_acc = {0.f, 0.f}, q_acc = {0.f, 0.f};
  double s_d = 0.0, q_d = 0.0;
  uint32_t ymx = 0u;
  f32x4 acc[4];
  F2Tile prev{0, 0, 0};
  bool have_prev = false;
  int t = w;
  if (t < total) f2_dma<DIAG, WV>(p1, decode(0), P, smem, lane);
  int kk = 0;
  for (; t < total; t += gridDim.x, ++kk) {
    const F2Tile cur = decode(kk);
    // tile t's DMA landed (vmcnt(0) + barrier); p1 buffer (kk+1)&1 is free; the staged
    // tile t-1 (stage (kk+1)&1) is complete
    __syncthreads();
    if (t + (int)gridDim.x < total) f2_dma<DIAG, WV>(p1, decode(kk + 1), P, smem + ((kk + 1) & 1) * F2_PBUF, lane);
    if (have_prev) {
      f2_store<DIAG>(smem + F2_OFF_S + ((kk + 1) & 1) * F2_STAGE, prev, y2, P);
      f2_store_ya(ys + ((kk + 1) & 1) * (F2_YSTAGE / 4), prev, ya, pg);
      f2_store_a2(ys + ((kk + 1) & 1) * (F2_YSTAGE / 4), prev, a2, P);
    }
    f2_compute<DIAG>(smem + (kk & 1) * F2_PBUF, W, acc, RH, lane);
    if (cur.r0 + F2_TH <= P && cur.c0 + F2_TC <= P && plain)  // tile- and wave-uniform
      f2_stage<false, true>(acc, cur, smem + F2_OFF_S + (kk & 1) * F2_STAGE, ys + (kk & 1) * (F2_YSTAGE / 4), P, RH, NT,
                            lane, bco, inv, ksc, neg, zg, s_acc, q_acc, ymx, a2);
    else if (cur.r0 + F2_TH <= P && cur.c0 + F2_TC <= P)
      f2_stage<false, false>(acc, cur, smem + F2_OFF_S + (kk & 1) * F2_STAGE, ys + (kk & 1) * (F2_YSTAGE / 4), P, RH, NT, lane,
                      bco, inv, ksc, neg, zg, s_acc, q_acc, ymx, a2);
    else
      f2_stage<true, false>(acc, cur, smem + F2_OFF_S + (kk & 1) * F2_STAGE, ys + (kk & 1) * (F2_YSTAGE / 4), P, RH, NT, lane,
                     bco, inv, ksc, neg, zg, s_acc, q_acc, ymx, a2);
    s_d += (double)(s_acc.x + s_acc.y);
    q_d += (double)(q_acc.x + q_acc.y);
    s_acc = f2v{0.f, 0.f};
    q_acc = f2v{0.f, 0.f};
    prev = cur;
    have_prev = true;
  }
  __syncthreads();
  if (have_prev) {
    f2_store<DIAG>(smem + F2_OFF_S + ((kk - 1) & 1) * F2_STAGE, prev, y2, P);
    f2_store_ya(ys + ((kk - 1) & 1) * (F2_YSTAGE / 4), prev, ya, pg);
    f2_store_a2(ys + ((kk - 1) & 1) * (F2_YSTAGE / 4), prev, a2, P);
  }
  // max |acc| of channel 16NT + li over the 4 lane groups (then the two waves of this co half)
  ymx = max(ymx, (uint32_t)__shfl_xor((int)ymx, 16, 64));
  ymx = max(ymx, (uint32_t)__shfl_xor((int)ymx, 32, 64));
  // BN2 partials: reduce the 4 lane groups, then the two row-halves of this co half
  double s_sum = s_d, q_sum = q_d;
  s_sum += __shfl_xor(s_sum, 16, 64);
  s_sum += __shfl_xor(s_sum, 32, 64);
  q_sum += __shfl_xor(q_sum, 16, 64);
  q_sum += __shfl_xor(q_sum, 32, 64);
  __syncthreads();  // all operand reads done: reuse the LDS for the reduction
  double* red = reinterpret_cast<double*>(smem);                   // [4 waves][16 co][2]
  uint32_t* yred = reinterpret_cast<uint32_t*>(smem + 4 * 16 * 2 * 8);  // [4 waves][16 co]
  if (lane < 16) {
    red[(WV * 16 + li) * 2 + 0] = s_sum;
    red[(WV * 16 + li) * 2 + 1] = q_sum;
    yred[WV * 16 + li] = ymx;
  }
  __syncthreads();
  if (WV == 0 && lane < 64) {
    const int co = lane >> 1, k = lane & 1, nt = co >> 4, c16 = co & 15;
    // waves with this co half: nt (rows 0-3) and nt + 2 (rows 4-7)
    const double v = (red[(nt * 16 + c16) * 2 + k] + red[((nt + 2) * 16 + c16) * 2 + k]) * (k ? (double)inv * inv : inv);
    st_agent(partial + ((int64_t)co * gridDim.x + blockIdx.x) * 2 + k, v);  // (write-through: f2_finalize)
    // this workgroup's max |y2 - b2| per channel: a plain store per (channel, workgroup), reduced by
    // the BN2-backward finalize (no same-address atomics: 16 K of them cost ~40 us in the head)
    // (max |acc| * inv = max |y2 - b2|: inv is a power of two, the order and the NaN survive)
    if (ypart != nullptr && k == 0)
      st_agent(ypart + co * gridDim.x + blockIdx.x,
               __float_as_uint(__uint_as_float(max(yred[nt * 16 + c16], yred[(nt + 2) * 16 + c16])) * inv));
  }
}

// In-launch BN2 finalize (common.h tds_arrive; replaces bn_reduce_finalize_kernel and the ypart
// max of bn_bwd_finalize2): groups of F2_GROUP workgroups; the last of a group to arrive reduces
// the group's partial rows (fixed order) into gsum[g][co][2] and its max |y2 - b2| into gmax[g][co];
// the last group-reducer sums the groups in order, finalizes BN2 (batch statistics, running
// statistics, the affine aff = [a|b]) and writes mag[co] = max |y2 - b2| for the conv2 backward.
constexpr int F2_GROUP = 32;
struct F2Fin {
  uint32_t* sync;  // [0, ngroups): group counters, [kSyncWordsPerSite - 1]: groups
  double* gsum;    // [ngroups][32][2]
  uint32_t* gmax;  // [ngroups][32]
  int64_t n;       // B * P * P
  const float* beta;
  float eps, momentum;
  float* stats;    // [64]: mean | invstd
  float* running_mean;
  float* running_var;
  int64_t* num_batches;
  float* aff;      // [64]: a | b
  uint32_t* mag;   // [32]: max |y2 - b2| per channel (float bits)
};

__device__ __forceinline__ void f2_finalize(const F2Fin& fin, const double* __restrict__ partial,
                                            const uint32_t* __restrict__ ypart, const float* __restrict__ bias,
                                            const float* __restrict__ gamma, int* flag) {
  const int nwg = (int)gridDim.x, wg = (int)blockIdx.x, tid = (int)threadIdx.x;
  const int ng = (nwg + F2_GROUP - 1) / F2_GROUP, g = wg / F2_GROUP;
  const int w0 = g * F2_GROUP, w1 = min(nwg, w0 + F2_GROUP);
  double* part = reinterpret_cast<double*>(flag + 4);  // (16 B past the flag, inside the kernel's LDS)
  if (!tds_arrive(fin.sync + g, (uint32_t)(w1 - w0), flag)) return;
  // this group's rows (workgroups w0 .. w1-1) of partial[co][w][k], one round of loads each
  const double s = wide_row_sum(partial + (int64_t)w0 * 2, w1 - w0, 64, 2, part, 2 * (int64_t)nwg);
  if (tid < 64) st_agent(fin.gsum + (int64_t)g * 64 + tid, s);
  if (ypart != nullptr && tid < 32) {  // [co][nwg]: channel co's w0 .. w1-1 are contiguous
    uint32_t v[F2_GROUP];
#pragma unroll
    for (int u = 0; u < F2_GROUP; ++u) v[u] = ypart[(int64_t)tid * nwg + min(w0 + u, w1 - 1)];  // (clamped: a repeat
    // leaves the max; a guarded load is waited for inside its branch, common.h wide_row_sum)
    uint32_t m = 0u;
#pragma unroll
    for (int u = 0; u < F2_GROUP; ++u) m = max(m, v[u]);
    st_agent(fin.gmax + g * 32 + tid, m);
  }
  if (!tds_arrive(fin.sync + kSyncWordsPerSite - 1, (uint32_t)ng, flag)) return;
  // the groups' (co, k) sums and max |y2 - b2|: one round of loads each
  const double sk = wide_row_sum(fin.gsum, ng, 64, 64, part);
  const uint32_t mx = wide_row_max(fin.gmax, ng, 32, 32, reinterpret_cast<uint32_t*>(part + 128));
  if (tid < 64) part[tid] = sk;  // (co, k) -> co * 2 + k
  __syncthreads();
  if (tid < 32) {
    const int co = tid;
    if (co == 0 && fin.num_batches) fin.num_batches[0] += 1;
    bn_finalize_channel(co, 32, part[co * 2], part[co * 2 + 1], fin.n, bias, fin.eps, fin.momentum, gamma, fin.beta,
                        fin.stats, fin.running_mean, fin.running_var, fin.aff);
    if (fin.mag != nullptr && ypart != nullptr) fin.mag[co] = mx;
  }
}

template <int DIAG>
__global__ __launch_bounds__(F2_THREADS, F2_WG) void conv2_fwd2_kernel(const uint4* __restrict__ p1,
                                                                   const uint4* __restrict__ wpack,
                                                                   const float* __restrict__ bias,
                                                                   const float* __restrict__ gamma,
                                                                   unsigned short* __restrict__ y2, unsigned short* __restrict__ ya,
                                                                   uint32_t* __restrict__ a2,
                                                                   double* __restrict__ partial,
                                                                   uint32_t* __restrict__ ypart,
                                                                   const uint32_t* __restrict__ scales,
                                                                   const int* __restrict__ order, int sw, int sk,
                                                                   int B, int P, F2Fin fin) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform role
  if (wv == 0) f2_run<DIAG, 0>(p1, wpack, bias, gamma, y2, ya, a2, partial, ypart, scales, order, sw, sk, B, P, smem);
  else if (wv == 1) f2_run<DIAG, 1>(p1, wpack, bias, gamma, y2, ya, a2, partial, ypart, scales, order, sw, sk, B, P, smem);
  else if (wv == 2) f2_run<DIAG, 2>(p1, wpack, bias, gamma, y2, ya, a2, partial, ypart, scales, order, sw, sk, B, P, smem);
  else f2_run<DIAG, 3>(p1, wpack, bias, gamma, y2, ya, a2, partial, ypart, scales, order, sw, sk, B, P, smem);
  if (fin.sync != nullptr) {
    __syncthreads();  // (f2_run's last LDS reads done: smem is reused for the flag)
    f2_finalize(fin, partial, ypart, bias, gamma, reinterpret_cast<int*>(smem));
  }
}

}  // namespace tds

using namespace tds;

// workgroups the forward launches (BN2 partial rows): F2_WG per CU
int tds_conv2_fwd2_num_wg() { return F2_WG * tds_conv2_num_wg(); }

void tds_conv2_fwd2_tiles(int P, int* tiles_r, int* tiles_c) {
  *tiles_r = (P + F2_TH - 1) / F2_TH;
  *tiles_c = (P + F2_TC - 1) / F2_TC;
}

#ifdef TDS_DIAG
// timing-only variants (tools/conv2_diag.py): 1 no MFMAs, 2 no LDS operand reads, 3 no global
// tile loads, 4 no y2h stores.  Compiled only into a -DTDS_DIAG build.
static int f2_diag_env() {
  const char* e = std::getenv("TDS_CONV2_DIAG");
  return e ? std::atoi(e) : 0;
}
#else
static int f2_diag_env() { return 0; }
#endif

// order: the blocked tile order table (tds_tile_order_fill) as per-workgroup lists [nwg][ceil(total / nwg)]
// (fused_ops.cpp tile_order, sw / sk: the strides of workgroup / tile), allocated by the caller
int tds_conv2_fwd2_fin_doubles(int nwg) { return ((nwg + F2_GROUP - 1) / F2_GROUP) * 32 * 2; }
int tds_conv2_fwd2_fin_words(int nwg) { return ((nwg + F2_GROUP - 1) / F2_GROUP) * 32; }

void tds_conv2_fwd2(const void* p1, const short* wp, const float* bias, const float* gamma, void* y2h, unsigned short* ya,
                    uint32_t* a2, double* partial, uint32_t* ypart, const uint32_t* scales, const int* order, int nwg, int sw, int sk,
                    int B, int P, hipStream_t st, const TdsBnFin* bn) {
  const dim3 grid(nwg), block(F2_THREADS);
  F2Fin fin{};
  if (bn != nullptr) {
    fin.sync = tds_sync_words(kSyncConv2Fwd, st);
    if (fin.sync == nullptr || (nwg + F2_GROUP - 1) / F2_GROUP > WRS_MAXL * 4) {
      tds_launch_fail("conv2_fwd2: in-launch BN2 finalize unavailable (sync words / group count)");
      return;
    }
    fin.gsum = bn->dwork;
    fin.gmax = bn->uwork;
    fin.n = (int64_t)B * P * P;
    fin.beta = bn->beta;
    fin.eps = bn->eps;
    fin.momentum = bn->momentum;
    fin.stats = bn->stats;
    fin.running_mean = bn->running_mean;
    fin.running_var = bn->running_var;
    fin.num_batches = bn->num_batches;
    fin.aff = bn->aff;
    fin.mag = bn->mag;
  }
  unsigned short* y2 = static_cast<unsigned short*>(y2h);
  const uint4* pp = reinterpret_cast<const uint4*>(p1);
  const uint4* w = reinterpret_cast<const uint4*>(wp);
  static bool lds_set = false;
  if (!lds_set) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(conv2_fwd2_kernel<0>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, F2_LDS);
#ifdef TDS_DIAG
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(conv2_fwd2_kernel<1>), hipFuncAttributeMaxDynamicSharedMemorySize, F2_LDS);
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(conv2_fwd2_kernel<2>), hipFuncAttributeMaxDynamicSharedMemorySize, F2_LDS);
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(conv2_fwd2_kernel<3>), hipFuncAttributeMaxDynamicSharedMemorySize, F2_LDS);
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(conv2_fwd2_kernel<4>), hipFuncAttributeMaxDynamicSharedMemorySize, F2_LDS);
#endif
    lds_set = true;
  }
  switch (f2_diag_env()) {
#ifdef TDS_DIAG
    case 1: hipLaunchKernelGGL(conv2_fwd2_kernel<1>, grid, block, F2_LDS, st, pp, w, bias, gamma, y2, ya, a2, partial, ypart, scales, order, sw, sk, B, P, fin); break;
    case 2: hipLaunchKernelGGL(conv2_fwd2_kernel<2>, grid, block, F2_LDS, st, pp, w, bias, gamma, y2, ya, a2, partial, ypart, scales, order, sw, sk, B, P, fin); break;
    case 3: hipLaunchKernelGGL(conv2_fwd2_kernel<3>, grid, block, F2_LDS, st, pp, w, bias, gamma, y2, ya, a2, partial, ypart, scales, order, sw, sk, B, P, fin); break;
    case 4: hipLaunchKernelGGL(conv2_fwd2_kernel<4>, grid, block, F2_LDS, st, pp, w, bias, gamma, y2, ya, a2, partial, ypart, scales, order, sw, sk, B, P, fin); break;
#endif
    default: hipLaunchKernelGGL(conv2_fwd2_kernel<0>, grid, block, F2_LDS, st, pp, w, bias, gamma, y2, ya, a2, partial, ypart, scales, order, sw, sk, B, P, fin); break;
  }
  TDS_LAUNCH_CHECK();
}
