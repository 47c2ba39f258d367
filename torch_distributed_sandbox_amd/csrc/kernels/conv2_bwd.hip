// conv2 backward: BN2 / ReLU / max-pool backward fused into conv2 dgrad + wgrad
// (SURVEY.md §2.4 K16-K21), one persistent 8-wave workgroup per CU, on v_mfma_f32_16x16x32_f16
// in the TF32 class (conv2_common.h): ONE MFMA per product, both operands rounded once to fp16 (11
// significant bits, TF32's significand):
//   dgrad: dp1 = convT(dy2, w2)  -- dy2 rounded once (scaled), w2 as packed by conv2_pack (scaled)
//   wgrad: dw2 = sum dy2 (x) p1  -- dy2 rounded once, p1 the forward's fp16 operand as is
// dy2 is carried with a power-of-two scale 2^e: from the step's magnitude bounds (max |y2 - b2|
// per channel from the forward, max |g2m| from the head backward) |dy2| <= |k1| max|g2m| + |k2|
// (max|y2 - b2| + |b2|) + |k3| per channel, and e puts the largest bound in [2^14, 2^15) -- no fp16
// overflow by construction, ~28 binades of full fp16 precision below it.  The products are
// unscaled exactly (power of two) in the dp1 / weight-slab epilogues.
//
// Roles (one per SIMD each):
//   waves 0/1 : dgrad, taps grouped by kx so an input row's A fragment serves up to 5 output
//               rows:  wave 0 = kx {0,1} x ky 0-4  +  kx 4 x ky 0-2
//                      wave 1 = kx {2,3} x ky 0-4  +  kx 4 x ky 3-4
//               weights in registers; each wave makes a partial dp1 of the whole 8 x 16 tile,
//               the halves are exchanged through LDS (double-buffered slots).
//   waves 2/3 : wgrad, taps 0-12 / 13-25 (tap 25 = the bias "ones" column), both co halves, K =
//               32 pixels = two output rows, operands by ds_read_b64_tr_b16; accumulated over the
//               workgroup's tiles; slab[wg][26][32][16] reduced in fixed order afterwards.
//   waves 4-7 : staging: y2h / argmax codes a2 / pooled gradient g2m / p1 -> BN2 / ReLU / pool
//               backward (dy2 = k1*dz + k2*y2 + k3, dz at the window's argmax) -> dy2 fp16 rows
//               (scaled) and p1 fp16 rows in LDS.
//
// ROLLING WINDOW.  A tile of 8 output rows needs dy2 and p1 on 12 rows (2-row halo above and
// below).  Each workgroup walks vertical SEGMENTS of tiles (one tile column of one image, ~48
// tiles top to bottom, host table tds_conv2_bwd_walk): consecutive tiles share 4 of those 12
// rows, so the staging waves load, recompute and store only the 8 NEW rows of each tile; its
// last 4 rows are stored twice, the second time as the TOP rows of the next tile's slot, so
// every tile reads its 12 rows contiguously from one slot (one base address: the consumers'
// LDS offsets are immediates, as with a slot that stages all 12 rows).  A segment's first tile
// gets its 4 top rows from a prologue staged straight into its slot's top.  Against a tile that stages all 12 rows this
// cuts the staging's global loads (y2 + g2m + p1) and BN2-backward work by a third; the loads
// were the kernel's largest cost (timing build without them: 1.05 vs 1.56 ms).
//
// LDS, in ROW BLOCKS (one staged image row of 20 records per block):
//   dy2 row block: 2 planes (co 0-15, co 16-31) x 20 x 32 B = 1280 B
//   p1  row block: 1 plane x 20 x 32 B = 640 B
//   3 ring slots of 12 row blocks (tile k in slot k % 3: 4 top + 8 new rows), 2 dgrad exchange
//   slots, BN2 backward constants + the dy2 scale, 2 pooled-gradient tiles: 96 400 B.
// One bare s_barrier per tile (after lgkmcnt(0)) separates producer and consumers: while the
// consumers read slot k%3, the staging writes slot (k+1)%3's new rows and slot (k+2)%3's top
// (the slot of tile k-1, finished); the register loads for tile k+3 are already in flight.
#include <algorithm>
#include <cstdlib>
#include <vector>

#include "conv2_common.h"
#include "launchers.h"
#include "pooled_layout.h"

namespace tds {

constexpr int BR_TH = 8, BR_TC = 16;       // output tile
constexpr int BR_SC = BR_TC + 4;           // 20 staged columns (2-pixel halo each side)
constexpr int BR_DPL = BR_SC * 32;         // 640 B: one plane of a row block
constexpr int BR_DROW = 2 * BR_DPL;        // 1280 B: dy2 row block
constexpr int BR_PROW = BR_DPL;            // 640 B: p1 row block (one fp16 plane)
constexpr int BR_THREADS = 512;
constexpr int BR_SLOT = 12;                                  // row blocks per ring slot
constexpr int BR_OFF_D = 0;                                  // 3 x 12 dy2 row blocks
constexpr int BR_OFF_P = BR_OFF_D + 3 * BR_SLOT * BR_DROW;   // 3 x 12 p1 row blocks
constexpr int BR_XCHG = 2 * 4 * 64 * 16;                     // 8 KiB exchange slot
constexpr int BR_OFF_X = BR_OFF_P + 3 * BR_SLOT * BR_PROW;   // 2 exchange slots
constexpr int BR_OFF_K = BR_OFF_X + 2 * BR_XCHG;             // 160 floats of constants + 4
constexpr int BR_KINV = 160;  // kc[160] = 2^-e * 2^-ew (dp1), kc[161] = 2^-e / p1 scale (weight taps), kc[162] = 2^-e (bias),
                              // kc[163] = 2^kd (the dp1h store factor)
// the pipelined staging's pooled-gradient tiles (BRStager GB): 2 x [4 pooled rows][10 cols][32 ch] fp32
constexpr int BR_GTILE = 4 * 10 * 32;
constexpr int BR_OFF_G = (BR_OFF_K + (5 * 32 + 4) * 4 + 15) / 16 * 16;
constexpr int BR_LDS = BR_OFF_G + 2 * BR_GTILE * 4;
static_assert(BR_LDS <= 160 * 1024 && BR_OFF_X % 16 == 0 && BR_OFF_K % 16 == 0, "LDS carve");

// walk table entries (tds_conv2_bwd_walk): bit 31 = first tile of a segment, bit 30 = past the
// end of this workgroup's list (the low bits then repeat its last tile), b << 24 | tr << 12 | tc
constexpr uint32_t kWalkStart = 0x80000000u, kWalkEnd = 0x40000000u;
constexpr int BR_STAGE_SETS = 3;  // staging look-ahead register sets (br_stage)
constexpr int BR_WALK_PAD = 8;    // end entries after each list (>= 2 x BR_STAGE_SETS)
static_assert(BR_WALK_PAD >= 2 * BR_STAGE_SETS, "walk padding below the staging look-ahead");
constexpr int BR_MFMA_PRIO = 1;   // wave priority of the dgrad / wgrad waves (above the staging's VALU)
struct BRTile {
  int b, r0, c0;
  bool start, end;
};
__device__ __forceinline__ BRTile br_decode(const int* __restrict__ walk, int k, int sk, int w) {
  // 32-bit index (the table is far below 2^31 entries): with a 64-bit one the compiler keeps
  // copies of the wgrad accumulators across the tile loop and spills them (256 VGPRs + scratch
  // against 189).  walk is already offset to this workgroup's list (w * sw); the device table is
  // per workgroup ([nwg][rows], fused_ops.cpp bwd_walk, sk = 1): 16 consecutive tiles per
  // scalar-cache line.
  (void)w;
  const uint32_t v = (uint32_t)walk[k * sk];
  BRTile x;
  x.start = (v & kWalkStart) != 0;
  x.end = (v & kWalkEnd) != 0;
  x.b = (int)((v >> 24) & 63);
  x.r0 = (int)((v >> 12) & 4095) * BR_TH;
  x.c0 = (int)(v & 4095) * BR_TC;
  return x;
}

struct BRArgs {
  const uint2* __restrict__ y2;  // y2h [B][P][P][32] fp16 (conv2_common.h)
  const uint32_t* __restrict__ a2;  // the forward's pooling argmax codes [B][Q][Q][2] (conv2_common.h)
  const unsigned short* __restrict__ g2m;  // fp16 planar [B][32][Q][Q] (the fc flatten order), scale 2^e_c
  const uint4* __restrict__ p1;
  uint2* __restrict__ dp1;  // dp1h (conv2_common.h)
  float* __restrict__ slab;
  const int* __restrict__ walk;
  int B, P, Q, sk, w;
};

// ---------------------------------------------------------------------------- dgrad
template <int D, int I>
struct DgGroup {
  static constexpr int KX = D == 0 ? (I == 0 ? 0 : I == 1 ? 1 : 4) : (I == 0 ? 2 : I == 1 ? 3 : 4);
  static constexpr int KY0 = I < 2 ? 0 : (D == 0 ? 0 : 3);
  static constexpr int NKY = I < 2 ? 5 : (D == 0 ? 3 : 2);
};

template <int D, int I>
__device__ __forceinline__ void br_load_w_group(const uint4* __restrict__ wd, f32x4 (&R)[13][2], int lane) {
  using G = DgGroup<D, I>;
#pragma unroll
  for (int k = 0; k < G::NKY; ++k) {
    const int s = (G::KY0 + k) * 5 + G::KX;  // flipped-tap index of the dgrad pack
    R[5 * I + k][0] = __builtin_bit_cast(f32x4, wd[s * 64 + lane]);
  }
}

template <int D>
__device__ __forceinline__ void br_load_w(const uint4* __restrict__ wd, f32x4 (&R)[13][2], int lane) {
  br_load_w_group<D, 0>(wd, R, lane);
  br_load_w_group<D, 1>(wd, R, lane);
  br_load_w_group<D, 2>(wd, R, lane);
}

// Wave D hands the partner's rows (4(1-D) .. +3) to the exchange slot 1-D.
template <int D>
__device__ __forceinline__ void br_xchg_put(f32x4* xs, const f32x4 (&acc)[8], int lane) {
#pragma unroll
  for (int i = 0; i < 4; ++i) xs[((1 - D) * 4 + i) * 64 + lane] = acc[4 * (1 - D) + i];
}

// Wave D owns output rows 4D .. 4D+3: its partial + the partner's, then dp1h (conv2_common.h): the
// lane's 4 columns 4g + r of channel li are 8 contiguous bytes, a row's 64 lanes 512 (columns
// past P land in the last column group's padding)
template <int D>
__device__ __forceinline__ void br_xchg_finish(const f32x4* xs, const f32x4 (&acc)[8], uint2* __restrict__ dp1h,
                                               int lane, int b, int r0, int c0, int P, float sd) {
  const int li = lane & 15, g = lane >> 4;
  const int PG = (P + 3) >> 2;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const f32x4 v = (acc[4 * D + i] + xs[(D * 4 + i) * 64 + lane]) * sd;  // 2^kd: exact
    const int row = r0 + 4 * D + i;
    // (a tile past the image's right edge: whole column groups beyond PG are not stored -- they
    // would land in the next row)
    if (row < P && (c0 >> 2) + g < PG)  // plain stores: read next by the layer-1 backward
      dp1h[(((int64_t)b * P + row) * PG + (c0 >> 2) + g) * 16 + li] = make_uint2(cvt2_f16(v[0], v[1]), cvt2_f16(v[2], v[3]));
  }
}

// The 12 staged rows of a tile, contiguous in its slot (r: a compile-time row in the unrolled
// loops, so r * row-block size folds into the LDS instruction's offset)
struct BRRows {
  const char* dl;
  const char* pl;
  __device__ __forceinline__ const char* d(int r) const { return dl + r * BR_DROW; }
  __device__ __forceinline__ const char* p(int r) const { return pl + r * BR_PROW; }
};

template <int D>
struct DgSeq {
  static constexpr int n(int i) { return 8 + (i < 2 ? 5 : (D == 0 ? 3 : 2)) - 1; }  // rows of group i
  static constexpr int S = n(0) + n(1) + n(2);
  static constexpr int grp(int s) { return s < n(0) ? 0 : s < n(0) + n(1) ? 1 : 2; }
  static constexpr int row(int s) { return s < n(0) ? s : s < n(0) + n(1) ? s - n(0) : s - n(0) - n(1); }
  static constexpr int kx(int i) { return D == 0 ? (i == 0 ? 0 : i == 1 ? 1 : 4) : (i == 0 ? 2 : i == 1 ? 3 : 4); }
  static constexpr int ky0(int i) { return i < 2 ? 0 : (D == 0 ? 0 : 3); }
  static constexpr int nky(int i) { return i < 2 ? 5 : (D == 0 ? 3 : 2); }
};

// one flat, fully unrolled sequence of A-fragment rows with operands fetched two steps ahead
// across group boundaries (one MFMA wave per SIMD: nothing else hides a bubble), through a ring
// of DP + 1 registers
template <int D, int DIAG>
__device__ __forceinline__ void br_dgrad(const BRRows& rw, const f32x4 (&R)[13][2], f32x4 (&acc)[8], int hp, int li) {
  using Q = DgSeq<D>;
  constexpr int DP = 2;
#pragma unroll
  for (int o = 0; o < 8; ++o) acc[o] = f32x4{0.f, 0.f, 0.f, 0.f};
  s16x8 ah[DP + 1];
  auto load_a = [&](int s, int buf) {
    const int i = Q::grp(s), r = Q::row(s);
    const char* rb = rw.d(Q::ky0(i) + r) + (Q::kx(i) + li) * 32;
    ah[buf] = lds8<DIAG>(rb + hp);
  };
#pragma unroll
  for (int s = 0; s < DP; ++s) load_a(s, s);
#pragma unroll
  for (int s = 0; s < Q::S; ++s) {
    if (s + DP < Q::S) load_a(s + DP, (s + DP) % (DP + 1));
    __builtin_amdgcn_sched_barrier(0);
    const int i = Q::grp(s), r = Q::row(s);
#pragma unroll
    for (int k = 0; k < 5; ++k) {
      const int o = r - k;
      if (k < Q::nky(i) && o >= 0 && o < 8)
        acc[o] = mmaw<DIAG>(ah[s % (DP + 1)], __builtin_bit_cast(s16x8, R[5 * i + k][0]), acc[o]);
    }
  }
}

// ---------------------------------------------------------------------------- wgrad
// wgrad waves E = 0 / 1: taps 13E .. 13E+12 of both co halves, K = 32 pixels (two output rows) per
// K-step, summed over the workgroup's tiles: one flat, fully unrolled sequence of the 52 (K-step,
// tap) steps with the B operands read DEPTH steps ahead through a ring of DEPTH + 1 register sets,
// and the next K-step's A operands AD steps before it starts.  Timing-only variants (r5_s2, conv2 backward with the wgrad waves
// alone, no staging) put the rolled loop at ~36 cycles per MFMA with its LDS operand reads and ~21
// without them: the reads' latency is what the MFMA stream waits on.
// r5_s4: the wgrad waves alone 0.550 -> 0.347 ms at depth 6 (21.5 cycles per MFMA: their LDS read
// latency hidden), the whole kernel 0.740 -> 0.728 (now bound by the staging); driver command
// 2.282 / 2.284 -> 2.273 / 2.279 ms on the same box
template <int E, int DIAG>
__device__ __forceinline__ void br_wgrad_ring(const BRRows& rw, f32x4 (&wacc)[13][2], int lane, const s16x8& ones) {
  constexpr int NS = 4 * 13, DEPTH = 6, AD = 6;
  const int g = lane >> 4, q4 = (lane >> 2) & 3, p4 = lane & 3;
  s16x8 a[2][2], bv[DEPTH + 1];
  auto load_a = [&](int m, int slot) {
    const char* r0 = rw.d(2 * m + 2) + (2 + 4 * g + q4) * 32 + p4 * 8;
    const char* r1 = rw.d(2 * m + 3) + (2 + 4 * g + q4) * 32 + p4 * 8;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const s16x4 x0 = ldtr<DIAG>(r0 + h * BR_DPL), x1 = ldtr<DIAG>(r1 + h * BR_DPL);
      a[slot][h] = s16x8{x0[0], x0[1], x0[2], x0[3], x1[0], x1[1], x1[2], x1[3]};
    }
  };
  auto load_b = [&](int s, int buf) {
    const int m = s / 13, tap = 13 * E + s % 13;
    if (tap < 25) {
      const int ky = tap / 5, kx = tap - 5 * (tap / 5);
      const int col = (kx + 4 * g + q4) * 32 + p4 * 8;
      const s16x4 x0 = ldtr<DIAG>(rw.p(2 * m + ky) + col), x1 = ldtr<DIAG>(rw.p(2 * m + ky + 1) + col);
      bv[buf] = s16x8{x0[0], x0[1], x0[2], x0[3], x1[0], x1[1], x1[2], x1[3]};
    } else {
      bv[buf] = ones;  // bias gradient column
    }
  };
  load_a(0, 0);
#pragma unroll
  for (int s = 0; s < DEPTH; ++s) load_b(s, s % (DEPTH + 1));
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    const int m = s / 13, k = s % 13;
    if (s + DEPTH < NS) load_b(s + DEPTH, (s + DEPTH) % (DEPTH + 1));
    if (k == 13 - AD && m + 1 < 4) load_a(m + 1, (m + 1) & 1);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int h = 0; h < 2; ++h) wacc[k][h] = mmaw<DIAG>(a[m & 1][h], bv[s % (DEPTH + 1)], wacc[k][h]);
  }
}

__device__ __forceinline__ void br_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// DIAG 13 (timing-only build): shader-clock cycles each wave spends waiting at the per-tile
// barriers vs its whole run, stored per wave in g_br_clk[wg][wave][wait, total] (read back by
// tds_conv2_bwd_clock_read): which role waits for which.  (printf here made the kernel 10^4x
// slower.)
constexpr int kBRClkMaxWg = 1024;
__device__ uint32_t g_br_clk[kBRClkMaxWg * 8 * 2];
constexpr bool br_clocked(int D) { return D == 13 || D >= 16; }
constexpr bool br_no_stage(int D) { return D == 5 || (D >= 16 && (D & 1)); }
constexpr bool br_idle(int D, int role) { return D >= 16 && (role < 2 ? (D & 4) : (D & 8)); }
constexpr bool br_no_gload(int D) { return D == 3 || (D >= 16 && (D & 32)); }  // staging: no global loads
constexpr bool br_no_math(int D) { return D == 9 || (D >= 16 && (D & 64)); }   // staging: no BN2 / pool math
template <int DIAG>
struct BRClock {
  uint64_t wait = 0, t0 = 0;
  __device__ __forceinline__ void start() {
    if constexpr (br_clocked(DIAG)) t0 = __builtin_amdgcn_s_memtime();
  }
  __device__ __forceinline__ void barrier() {
    if constexpr (br_clocked(DIAG)) {
      const uint64_t a = __builtin_amdgcn_s_memtime();
      br_barrier();
      wait += __builtin_amdgcn_s_memtime() - a;
    } else {
      br_barrier();
    }
  }
  __device__ __forceinline__ void report() {
    if constexpr (br_clocked(DIAG)) {
      const uint64_t tot = __builtin_amdgcn_s_memtime() - t0;
      const int i = ((int)blockIdx.x * 8 + (int)(threadIdx.x >> 6)) * 2;
      if ((threadIdx.x & 63) == 0 && blockIdx.x < kBRClkMaxWg) {
        g_br_clk[i] = (uint32_t)wait;
        g_br_clk[i + 1] = (uint32_t)tot;
      }
    }
  }
};

__device__ __forceinline__ BRRows br_rows(char* smem, int k) {
  const int s = __builtin_amdgcn_readfirstlane(k % 3);
  return BRRows{smem + BR_OFF_D + s * BR_SLOT * BR_DROW, smem + BR_OFF_P + s * BR_SLOT * BR_PROW};
}

template <int ROLE, int DIAG>  // ROLE 0/1 = dgrad wave D, 2/3 = wgrad
__device__ __forceinline__ void br_mfma(const BRArgs& a, const uint4* __restrict__ wdpack, char* smem) {
  __builtin_amdgcn_s_setprio(BR_MFMA_PRIO);
  const int lane = threadIdx.x & 63;
  const int li = lane & 15, g = lane >> 4;
  f32x4 R[13][2];
#pragma unroll
  for (int k = 0; k < 13; ++k) R[k][0] = R[k][1] = f32x4{0.f, 0.f, 0.f, 0.f};
  f32x4 acc[8];
#pragma unroll
  for (int o = 0; o < 8; ++o) acc[o] = f32x4{0.f, 0.f, 0.f, 0.f};
  if constexpr (ROLE < 2) br_load_w<ROLE>(wdpack, R, lane);
  s16x8 ones;
#pragma unroll
  for (int j = 0; j < 8; ++j) ones[j] = (short)(li == 0 ? kF16One : 0);
  const int hp = (g >> 1) * BR_DPL + (g & 1) * 16;
  // epilogue scales (powers of two, exact): dp1h is stored at 2^kd (its decode, 2^-e 2^-ew 2^-kd,
  // goes to mag[kMagScales + 4]), the weight-gradient slab takes out the dy2 and p1 scales, the
  // bias tap (dy2 sums) the dy2 scale only
  const float inv = reinterpret_cast<const float*>(smem + BR_OFF_K)[ROLE < 2 ? BR_KINV + 3 : BR_KINV + 1];
  const float inv_b = reinterpret_cast<const float*>(smem + BR_OFF_K)[BR_KINV + 2];
  BRTile prev{0, 0, 0, false, true};
  BRClock<DIAG> clk;
  clk.start();
  int kk = 0;
  for (;; ++kk) {
    const BRTile cur = br_decode(a.walk, kk, a.sk, a.w);
    if (cur.end) break;
    clk.barrier();  // tile kk staged; the partner's exchange slot of tile kk-1 is written
    const BRRows rw = br_rows(smem, kk);
    if constexpr (br_idle(DIAG, ROLE)) {
      // timing-only: this role does nothing but the barriers
    } else if constexpr (ROLE < 2) {
      if (!prev.end)
        br_xchg_finish<ROLE>(reinterpret_cast<const f32x4*>(smem + BR_OFF_X + ((kk + 1) & 1) * BR_XCHG), acc, a.dp1,
                             lane, prev.b, prev.r0, prev.c0, a.P, inv);
      br_dgrad<ROLE, DIAG>(rw, R, acc, hp, li);
      br_xchg_put<ROLE>(reinterpret_cast<f32x4*>(smem + BR_OFF_X + (kk & 1) * BR_XCHG), acc, lane);
    } else {
      br_wgrad_ring<ROLE - 2, DIAG>(rw, R, lane, ones);
    }
    prev = cur;
  }
  clk.barrier();  // the last exchange slot is written
  clk.report();
  if constexpr (ROLE < 2) {
    if (!prev.end)
      br_xchg_finish<ROLE>(reinterpret_cast<const f32x4*>(smem + BR_OFF_X + ((kk - 1) & 1) * BR_XCHG), acc, a.dp1,
                           lane, prev.b, prev.r0, prev.c0, a.P, inv);
  } else {
    float* out = a.slab + (int64_t)blockIdx.x * 26 * 512;
#pragma unroll
    for (int k = 0; k < 13; ++k) {
      const int tap = 13 * (ROLE - 2) + k;
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int r = 0; r < 4; ++r) out[(tap * 32 + 16 * h + 4 * g + r) * 16 + li] = R[k][h][r] * (tap < 25 ? inv : inv_b);
    }
  }
}

// ---------------------------------------------------------------------------- staging
// Out-of-range lanes get this byte offset: the buffer load's range check returns zeros.
constexpr uint32_t kBROob = 0xFFFFFFF0u;

// Staging of NR rows (8: a tile's new rows, 4: a segment prologue) of image rows R0 ..
// R0+NR-1 (R0 even), columns c0-2 .. c0+17, into dy2 / p1 row blocks.  Item = (2x2 pooling
// window, BR_CW-channel chunk): NR/2 x 10 windows x 32/BR_CW chunks.  BIG: the 32 g2m planes of an
// image exceed a 4 GiB buffer-descriptor range (64-bit g2m loads); a template parameter, because
// two load paths under a runtime branch make the compiler wait vmcnt(0) at their merge.
// BR_CW = 8: a pixel's 8 channels of y2h are one 16-B load and one 16-B dy2 store; a tile's 160
// items leave one per lane for waves 4-6 (r5_s14 PMC: the texture data path was busy 81 % of the
// kernel, ~64 cycles per staging load instruction -- fewer, wider loads; r5_s16: 8 vs 4 channels
// isolated 0.696 -> 0.688 ms).
constexpr int BR_CW = 8;
constexpr int BR_NCH = 32 / BR_CW;  // chunks per window
typedef uint4 BRY;                  // one pixel's BR_CW fp16 y2h values

__device__ __forceinline__ uint32_t br_word(const uint4& v, int i) {
  return i == 0 ? v.x : i == 1 ? v.y : i == 2 ? v.z : v.w;
}

// fma(a, channel cc of the fp16 channels in v, c) on v_fma_mix_f32 (op_sel picks the half)
template <class V>
__device__ __forceinline__ float br_fma_y(float a, const V& v, int cc, float c) {
  float d;
  const uint32_t w = br_word(v, cc >> 1);
  if (cc & 1)
    asm("v_fma_mix_f32 %0, %1, %2, %3 op_sel:[0,1,0] op_sel_hi:[0,1,0]" : "=v"(d) : "v"(a), "v"(w), "v"(c));
  else
    asm("v_fma_mix_f32 %0, %1, %2, %3 op_sel_hi:[0,1,0]" : "=v"(d) : "v"(a), "v"(w), "v"(c));
  return d;
}

__device__ __forceinline__ BRY br_load_y(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
}

// GB (the pipelined 8-row sets): the tile's pooled gradient g2m is not gathered per item (BR_CW
// 4-B loads from as many channel planes) but per RUN -- one (channel, pooled row) of the tile's 10
// pooled columns, on staging lanes 128-255: a 4-B load of the left halo column, two 16-B loads of
// the 8 columns of the tile, a 4-B load of the right halo -- and passed to the items through an LDS
// tile ([pooled row][col][channel]: two 16-B reads per item) written one tile ahead (put_runs).
// Per tile 8 load instructions instead of 20 (r5_s14: the texture path, ~64 cycles per staging
// load instruction, is the staging's limiter).  Mid loads past a row's end read the next row or,
// for the tensor's last row, the 64 B of slack every g2m allocation carries (fused_ops.cpp): those
// columns are never pooled.
template <int NR, bool BIG, int DIAG, bool GB = false>
struct BRStager {
  static constexpr int NWIN = (NR / 2) * (BR_SC / 2);
  static constexpr int ITEMS = NWIN * BR_NCH;
  static constexpr int IPER = (ITEMS + 255) / 256;
  static constexpr int PIECES = NR * BR_SC * 2;  // 16-B p1 pieces (32-B fp16 records)
  static constexpr int PPER = (PIECES + 255) / 256;
  BRY yv[IPER][4];      // y2h: BR_CW channels of each pixel of the window
  float gv[IPER][BR_CW];
  uint32_t av[IPER];    // a2: the window's argmax codes, 16 channels
  uint4 pr[PPER];
  uint4 rm;             // GB: this lane's run, columns 1-8 (fp16)
  uint32_t rl, rr;      // GB: its columns 0 and 9 (the halo; fp16 in the low half)

  // the j-th p1 piece of staging lane tid: the set past 256 goes to a wave without an item (waves
  // 4-6 hold the 160 items, the extra pieces go to wave 7)
  __device__ __forceinline__ static int piece(int tid, int j) { return (j == 1 ? ((tid + 64) & 255) : tid) + 256 * j; }

  __device__ __forceinline__ static void item_geom(int it, int& wy, int& wx) {
    const int w = (it < ITEMS ? it : 0) / BR_NCH;
    wy = w / (BR_SC / 2);
    wx = w - wy * (BR_SC / 2);
  }

  // the block is wholly inside the image and every window is pooled (no bounds work)
  __device__ __forceinline__ static bool interior(const BRArgs& a, int R0, int c0) {
    return R0 >= 0 && R0 + NR <= 2 * a.Q && c0 - 2 >= 0 && c0 + BR_TC + 2 <= 2 * a.Q;
  }

  // (bounds as bitwise &, | of unsigned compares: short-circuit && / || compiled to exec-mask
  // branches around every load's address, and the merges cost a vmcnt(0) per load set)
  __device__ __forceinline__ void load(const BRArgs& a, int b, int R0, int c0, int tid) {
    if constexpr (br_no_gload(DIAG)) {
#pragma unroll
      for (int u = 0; u < IPER; ++u) {
#pragma unroll
        for (int k = 0; k < BR_CW; ++k) gv[u][k] = 0.f;
        av[u] = 0u;
#pragma unroll
        for (int q = 0; q < 4; ++q) yv[u][q] = BRY{};
      }
#pragma unroll
      for (int j = 0; j < PPER; ++j) pr[j] = make_uint4(0u, 0u, 0u, 0u);
      return;
    }
    const int P = a.P, Q = a.Q;
    const bool in = interior(a, R0, c0);
    const int64_t img = (int64_t)b * P;
    // y2 / p1: one descriptor per block, based at (R0, c0-2); lanes outside the image -> kBROob
    const __amdgpu_buffer_rsrc_t ry =
        tds_buffer_rsrc(reinterpret_cast<const char*>(a.y2) + ((img + R0) * P + (c0 - 2)) * 64, 0xFFFFFFF0u);
    const __amdgpu_buffer_rsrc_t rp =
        tds_buffer_rsrc(reinterpret_cast<const char*>(a.p1) + ((img + R0) * P + (c0 - 2)) * 32, 0xFFFFFFF0u);
    const int64_t gplane = (int64_t)Q * Q;
    const int py0 = R0 / 2, px0 = c0 / 2 - 1;
    const __amdgpu_buffer_rsrc_t rg =
        tds_buffer_rsrc(a.g2m + (int64_t)b * 32 * gplane + (int64_t)py0 * Q + px0, 0xFFFFFFF0u);
    const __amdgpu_buffer_rsrc_t ra = tds_buffer_rsrc(a.a2 + (((int64_t)b * Q + py0) * Q + px0) * 2, 0xFFFFFFF0u);
    if constexpr (GB) {
      // the runs first: put_runs waits for them one tile before the rest of this set is needed
      const int rt = tid - 128;  // lanes 128-255: channel rt & 31, pooled row rt >> 5
      const int c = rt & 31, wy = (rt >> 5) & 3;
      const bool row = (rt >= 0) & ((uint32_t)(py0 + wy) < (uint32_t)Q);
      const bool lok = row & (px0 >= 0), rok = row & (px0 + 9 < Q);
      const int64_t e0 = (int64_t)c * gplane + (int64_t)wy * Q;  // element of column 0, from rg's base
      if constexpr (!BIG) {
        // fp16: the 8 inner columns in one (2-B aligned) 16-B load, the halo columns in 2-B loads
        const uint32_t o = (uint32_t)(e0 * 2);
        rl = __builtin_amdgcn_raw_buffer_load_b16(rg, lok ? o : kBROob, 0, 0);
        rm = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rg, row ? o + 2 : kBROob, 0, 0));
        rr = __builtin_amdgcn_raw_buffer_load_b16(rg, rok ? o + 18 : kBROob, 0, 0);
      } else {
        const unsigned short* gp = a.g2m + (int64_t)b * 32 * gplane + (int64_t)py0 * Q + px0 + (row ? e0 : 0);
        rl = lok ? gp[0] : 0u;  // (BIG: 64-bit loads; the rare >4 GiB-per-image shapes)
        const unsigned short* mp = gp + 1;
        rm = make_uint4((uint32_t)mp[0] | ((uint32_t)mp[1] << 16), (uint32_t)mp[2] | ((uint32_t)mp[3] << 16),
                        (uint32_t)mp[4] | ((uint32_t)mp[5] << 16), (uint32_t)mp[6] | ((uint32_t)mp[7] << 16));
        rr = rok ? gp[9] : 0u;
      }
    }
    const int cb = (tid % BR_NCH) * BR_CW;  // the chunk's first channel (256 % BR_NCH == 0: every u)
#pragma unroll
    for (int u = 0; u < IPER; ++u) {
      const int it = tid + 256 * u;
      int wy, wx;
      item_geom(it, wy, wx);
      const bool item = it < ITEMS;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int lr = 2 * wy + (q >> 1), lc = 2 * wx + (q & 1);
        const int gr = R0 + lr, gc = c0 - 2 + lc;
        const bool ok = item & (in | (((uint32_t)gr < (uint32_t)P) & ((uint32_t)gc < (uint32_t)P)));
        const uint32_t off = ok ? (uint32_t)((lr * P + lc) * 64 + cb * 2) : kBROob;
        yv[u][q] = br_load_y(ry, off);
      }
      const int py = py0 + wy, px = px0 + wx;
      const bool pooled = item & (in | (((uint32_t)py < (uint32_t)Q) & ((uint32_t)px < (uint32_t)Q)));
      av[u] = __builtin_amdgcn_raw_buffer_load_b32(ra, pooled ? (uint32_t)(((wy * Q + wx) * 2 + (cb >> 4)) * 4) : kBROob, 0, 0);
      if constexpr (GB) {
        // (from the LDS tile in store())
      } else if constexpr (!BIG) {
        const uint32_t og = (uint32_t)(((int64_t)cb * gplane + (int64_t)wy * Q + wx) * 2);
        const uint32_t gstep = (uint32_t)(gplane * 2);
#pragma unroll
        for (int k = 0; k < BR_CW; ++k)
          gv[u][k] = f16_val(__builtin_amdgcn_raw_buffer_load_b16(rg, pooled ? og + k * gstep : kBROob, 0, 0));
      } else {
        const unsigned short* gp =
            a.g2m + ((int64_t)b * 32 + cb) * gplane + (int64_t)(pooled ? py : 0) * Q + (pooled ? px : 0);
#pragma unroll
        for (int k = 0; k < BR_CW; ++k) gv[u][k] = f16_val(gp[k * gplane]);  // masked at use (store: pooled)
      }
    }
#pragma unroll
    for (int j = 0; j < PPER; ++j) {
      const int e = piece(tid, j);
      const int rec = (e < PIECES ? e : 0) >> 1, q = e & 1;
      const int lr = rec / BR_SC, lc = rec - lr * BR_SC;
      const int gr = R0 + lr, gc = c0 - 2 + lc;
      const bool ok = (e < PIECES) & (in | (((uint32_t)gr < (uint32_t)P) & ((uint32_t)gc < (uint32_t)P)));
      const uint32_t off = ok ? (uint32_t)((lr * P + lc) * 32 + q * 16) : kBROob;
      pr[j] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rp, off, 0, 0));
    }
  }

  // GB: this set's runs into the LDS tile gb ([pooled row][col][channel])
  __device__ __forceinline__ void put_runs(float* gb, int tid) const {
    static_assert(GB, "runs only in the pipelined sets");
    const int rt = tid - 128;
    if (rt < 0) return;
    const int c = rt & 31, wy = rt >> 5;
    float* d = gb + wy * 10 * 32 + c;
    d[0] = f16_val(rl);
    d[32] = f16_val(rm.x); d[64] = f16_val(rm.x >> 16); d[96] = f16_val(rm.y); d[128] = f16_val(rm.y >> 16);
    d[160] = f16_val(rm.z); d[192] = f16_val(rm.z >> 16); d[224] = f16_val(rm.w); d[256] = f16_val(rm.w >> 16);
    d[288] = f16_val(rr);
  }

  // BN2 / ReLU / pool backward of the staged windows -> dy2 rows at dbase; p1 -> pbase;
  // MIRROR: rows 4-7 stored a second time at dmir / pmir (the next slot's top rows).
  // dy2 = k1*dz + k2*y2 + k3, dz = pooled gradient at the window's argmax, which the forward
  // stored (a2, conv2_common.h: as max_pool2d's backward scatters to the indices its forward saved;
  // a NaN in y2 makes its channel's BN2 statistics NaN, hence k1..k3 and every dy2 of the channel,
  // wherever dz goes -- as in torch).  Interior blocks take a short path; border blocks the general
  // one (zero padding, unpooled last row / column).
  template <bool MIRROR>
  __device__ __forceinline__ void store(const BRArgs& a, int R0, int c0, int tid, char* dbase, char* pbase,
                                        const float* kc, char* dmir, char* pmir, const float* gb = nullptr) {
    if constexpr (DIAG == 3) {}
    // every register of the set is read here, on every path: the items / pieces past ITEMS /
    // PIECES are skipped below under exec masks, and a load whose result was consumed only
    // under a branch stays "pending" at the merge for the compiler's waitcnt pass -- the next
    // write of that register (the look-ahead loads into this set) then got a vmcnt(0), draining
    // the OTHER set's look-ahead loads too
#pragma unroll
    for (int u = 0; u < IPER; ++u) {
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int i = 0; i < BR_CW / 2; ++i) asm volatile("" ::"v"(br_word(yv[u][q], i)));
      if constexpr (!GB) {
#pragma unroll
        for (int k = 0; k < BR_CW; ++k) asm volatile("" ::"v"(gv[u][k]));
      }
      asm volatile("" ::"v"(av[u]));
    }
#pragma unroll
    for (int j = 0; j < PPER; ++j) asm volatile("" ::"v"(pr[j].x), "v"(pr[j].y), "v"(pr[j].z), "v"(pr[j].w));
    const int cb = (tid % BR_NCH) * BR_CW;
    const int P = a.P, Q = a.Q;
    if constexpr (GB) {  // the items' pooled gradients from the LDS tile (put_runs, a tile earlier)
#pragma unroll
      for (int u = 0; u < IPER; ++u) {
        int wy, wx;
        item_geom(tid + 256 * u, wy, wx);
        const float4* gp = reinterpret_cast<const float4*>(gb + (wy * 10 + wx) * 32 + cb);
#pragma unroll
        for (int h = 0; h < BR_CW / 4; ++h) {
          const float4 v = gp[h];
          gv[u][4 * h] = v.x; gv[u][4 * h + 1] = v.y; gv[u][4 * h + 2] = v.z; gv[u][4 * h + 3] = v.w;
        }
      }
    }
    float k1[BR_CW], k2[BR_CW], k3[BR_CW];
#pragma unroll
    for (int h = 0; h < BR_CW / 4; ++h) {
      const float4 a1 = *reinterpret_cast<const float4*>(&kc[2 * 32 + cb + 4 * h]);
      const float4 a2v = *reinterpret_cast<const float4*>(&kc[3 * 32 + cb + 4 * h]);
      const float4 a3 = *reinterpret_cast<const float4*>(&kc[4 * 32 + cb + 4 * h]);
      k1[4 * h] = a1.x; k1[4 * h + 1] = a1.y; k1[4 * h + 2] = a1.z; k1[4 * h + 3] = a1.w;
      k2[4 * h] = a2v.x; k2[4 * h + 1] = a2v.y; k2[4 * h + 2] = a2v.z; k2[4 * h + 3] = a2v.w;
      k3[4 * h] = a3.x; k3[4 * h + 1] = a3.y; k3[4 * h + 2] = a3.z; k3[4 * h + 3] = a3.w;
    }
    const bool fast = interior(a, R0, c0);
#pragma unroll
    for (int u = 0; u < IPER; ++u) {
      const int it = tid + 256 * u;
      if (it >= ITEMS) continue;
      int wy, wx;
      item_geom(it, wy, wx);
      float y[4][BR_CW];  // the stored values (ka, kb, k2, k3 carry the decode: kernel header)
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int i = 0; i < BR_CW / 2; ++i) {
          const uint32_t w = br_word(yv[u][q], i);
          y[q][2 * i] = f16_val(w);
          y[q][2 * i + 1] = f16_val(w >> 16);
        }
      float d[4][BR_CW];
      // this item's channels' codes: bits (cb & 15) .. +BR_CW-1 and 16 + that of the window's word
      const uint32_t cw = av[u] >> (cb & 15);
      if constexpr (br_no_math(DIAG)) {  // timing only: no BN2 / pool backward math
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
          for (int cc = 0; cc < BR_CW; ++cc) d[q][cc] = y[q][cc] + gv[u][cc];
      } else if (fast) {
#pragma unroll
        for (int cc = 0; cc < BR_CW; ++cc) {
          // y2h values straight into v_fma_mix_f32 (br_fma_y)
          auto fy = [&](float k, int q, float c) { return br_fma_y(k, yv[u][q], cc, c); };
          // the pooled gradient folded into the constant: k3g at the window's argmax, k3 elsewhere
          const float k3g = fmaf(k1[cc], gv[u][cc], k3[cc]);
          // by bit-field selects on the code's two bits sign-extended to masks (bit cc: column, bit
          // 16 + cc: row of the argmax): 2 + 6 VALU a channel instead of the code, 4 compares and
          // 4 selects (and no VALU-written lane masks)
          const uint32_t mx = (uint32_t)__builtin_amdgcn_sbfe((int)cw, cc, 1);
          const uint32_t my = (uint32_t)__builtin_amdgcn_sbfe((int)cw, 16 + cc, 1);
          const uint32_t ug = __float_as_uint(k3g), u3 = __float_as_uint(k3[cc]);
          // v_bitop3_b32 with truth table 0xCA = S0 ? S1 : S2 bitwise (the intrinsic keeps the
          // optimizer from turning the masks back into compares and selects)
          auto mux = [](uint32_t m, uint32_t x, uint32_t y) { return __builtin_amdgcn_bitop3_b32(m, x, y, 0xCA); };
          const uint32_t t0 = mux(mx, u3, ug), t1 = mux(mx, ug, u3);  // row hit: column 0 / 1 is the argmax
          const float c[4] = {__uint_as_float(mux(my, u3, t0)), __uint_as_float(mux(my, u3, t1)),
                              __uint_as_float(mux(my, t0, u3)), __uint_as_float(mux(my, t1, u3))};
#pragma unroll
          for (int q = 0; q < 4; ++q) d[q][cc] = fy(k2[cc], q, c[q]);
        }
      } else {
        const int gy = R0 + 2 * wy, gx = c0 - 2 + 2 * wx;
        const bool pooled = gy >= 0 && gx >= 0 && (gy >> 1) < Q && (gx >> 1) < Q;
#pragma unroll
        for (int cc = 0; cc < BR_CW; ++cc) {
          const int am = pooled ? (int)(((cw >> cc) & 1u) | ((cw >> (15 + cc)) & 2u)) : -1;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int r = gy + (q >> 1), c = gx + (q & 1);
            const bool inb = r >= 0 && r < P && c >= 0 && c < P;  // zero padding outside the image
            const float dz = am == q ? gv[u][cc] : 0.f;
            d[q][cc] = inb ? fmaf(k1[cc], dz, fmaf(k2[cc], y[q][cc], k3[cc])) : 0.f;
          }
        }
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        uint32_t h[BR_CW / 2];  // dy2 rounded once (TF32 class; k1..k3 carry the scale 2^e: d is dy2 * 2^e)
#pragma unroll
        for (int i = 0; i < BR_CW / 2; ++i) h[i] = cvt2_f16(d[q][2 * i], d[q][2 * i + 1]);
        const int lr = 2 * wy + (q >> 1);
        const int ro = (2 * wx + (q & 1)) * 32 + (cb & 15) * 2;
        char* rec = dbase + lr * BR_DROW + ro;
        auto put = [&](char* r) {
          *reinterpret_cast<uint4*>(r + (cb >> 4) * BR_DPL) = make_uint4(h[0], h[1], h[2], h[3]);
        };
        put(rec);
        if (MIRROR && lr >= 4) put(dmir + (lr - 4) * BR_DROW + ro);
      }
    }
#pragma unroll
    for (int j = 0; j < PPER; ++j) {
      const int e = piece(tid, j);
      if (e < PIECES) {
        const int rec = e >> 1, q = e & 1;
        const int lr = rec / BR_SC, lc = rec - lr * BR_SC;
        const int po = lc * 32 + q * 16;
        *reinterpret_cast<uint4*>(pbase + lr * BR_PROW + po) = pr[j];
        if (MIRROR && lr >= 4) *reinterpret_cast<uint4*>(pmir + (lr - 4) * BR_PROW + po) = pr[j];
      }
    }
  }
};

// One code copy for all four staging waves (workgroup waves 4-7; a wave's share of the work
// comes from threadIdx).  Instantiated per wave, the four identical copies (~36 KB each) made the
// kernel 168 KB of code, far beyond the instruction cache its CU shares.
template <int DIAG, bool BIG>
__device__ __forceinline__ void br_stage(const BRArgs& a, char* smem) {
  if constexpr (br_no_stage(DIAG)) {  // timing only: no staging at all (consumers read stale LDS)
    for (int k = 0; !br_decode(a.walk, k, a.sk, a.w).end; ++k) br_barrier();
    br_barrier();
    return;
  }
  const int tid = threadIdx.x - 256;
  const float* kc = reinterpret_cast<const float*>(smem + BR_OFF_K);
  // slot j % 3: rows 0-3 (top) at dtop / ptop, the tile's 8 new rows at +4
  auto dtop = [&](int j) { return smem + BR_OFF_D + (j % 3) * BR_SLOT * BR_DROW; };
  auto ptop = [&](int j) { return smem + BR_OFF_P + (j % 3) * BR_SLOT * BR_PROW; };
  // tile j's new rows, its last 4 mirrored into tile j+1's top (overwritten by a prologue when
  // tile j+1 starts a segment: a later iteration, past a barrier)
  // the pipelined sets take g2m by runs through an LDS tile (BRStager GB)
  typedef BRStager<8, BIG, DIAG, true> Set;
  float* gtile = reinterpret_cast<float*>(smem + BR_OFF_G);
  auto gbuf = [&](int j) { return gtile + (j & 1) * BR_GTILE; };
  auto stage = [&](Set& s, int j, const BRTile& x) {
    s.template store<true>(a, x.r0 + 2, x.c0, tid, dtop(j) + 4 * BR_DROW, ptop(j) + 4 * BR_PROW, kc, dtop(j + 1),
                           ptop(j + 1), gbuf(j));
  };
  // a segment's first tile: its 4 top rows (image rows r0-2 .. r0+1) staged synchronously
  // straight into its slot's top (once per ~48 tiles)
  auto prologue = [&](int j, const BRTile& x) {
    BRStager<4, BIG, DIAG> pro;
    pro.load(a, x.b, x.r0 - 2, x.c0, tid);
    pro.template store<false>(a, x.r0 - 2, x.c0, tid, dtop(j), ptop(j), kc, nullptr, nullptr);
  };
  // BR_STAGE_SETS register sets: tile j's new-row loads are issued that many tiles
  // before they are staged (r5_s6: the staging's global loads, ~20 KB a tile, are latency-bound --
  // the staging alone ran 0.53 ms, 0.26 without its loads; the sets live in VGPRs the MFMA
  // roles' 180 leave free).  Loads are unconditional (past the end: the list's last tile again,
  // never staged): a load under a branch makes the wait for the OLDER set drain the younger one
  // too (vmcnt(0)).
  BRClock<DIAG> clk;
  clk.start();
  auto tile = [&](int j) { return br_decode(a.walk, j, a.sk, a.w); };
  // (the staging waves run at priority 0: with three sets in flight the look-ahead loads no longer
  // need a raised priority, r5_s13: isolated 0.668 -> 0.659 ms without it)
  auto ld = [&](Set& s, int j) {
    const BRTile x = tile(j);
    s.load(a, x.b, x.r0 + 2, x.c0, tid);
  };
  // stage tile j from set s if it exists (a segment start also gets its prologue: after the set is
  // stored and before it is reloaded, so its registers are the set's); false past the list's end
  // nxt (the set holding tile j+1) puts its g2m runs into tile j+1's LDS tile; they are read
  // after the next barrier, and that tile's previous contents (tile j-1) were read before this one
  auto stage_if = [&](Set& s, Set& nxt, int j) {
    const BRTile x = tile(j);
    if (!x.end) {
      stage(s, j, x);
      nxt.put_runs(gbuf(j + 1), tid);
      if (x.start) prologue(j, x);
    }
    return !x.end;
  };
  Set st0, st1, st2;
  {
    const BRTile x0 = tile(0);
    if (!x0.end) {  // tile 0: its own synchronous set, g2m per item (no LDS tile precedes it)
      BRStager<8, BIG, DIAG, false> s0;
      s0.load(a, x0.b, x0.r0 + 2, x0.c0, tid);
      s0.template store<true>(a, x0.r0 + 2, x0.c0, tid, dtop(0) + 4 * BR_DROW, ptop(0) + 4 * BR_PROW, kc, dtop(1),
                              ptop(1));
      prologue(0, x0);
    }
  }
  ld(st1, 1);
  ld(st2, 2);
  ld(st0, 3);
  st1.put_runs(gbuf(1), tid);  // tile 1's, read after the loop's first barrier
  // iteration kk: tile kk+1 from st1 (reload: kk+4), kk+2 from st2 (kk+5), kk+3 from st0 (kk+6);
  // one exit and every set reloaded on every path (the two-set loop's rule, below).  The walk
  // table carries BR_WALK_PAD end entries: the last iteration (kk <= n-1) reads tile kk + 6.
  bool more = !tile(0).end;
  for (int kk = 0; more; kk += 3) {
    clk.barrier();  // consumers start tile kk
    const bool has1 = stage_if(st1, st2, kk + 1);
    ld(st1, kk + 4);
    bool has2 = false;
    if (has1) {
      clk.barrier();  // tile kk + 1
      has2 = stage_if(st2, st0, kk + 2);
    }
    ld(st2, kk + 5);
    bool has3 = false;
    if (has2) {
      clk.barrier();  // tile kk + 2
      has3 = stage_if(st0, st1, kk + 3);
    }
    ld(st0, kk + 6);
    more = has3;
  }
  clk.barrier();
  clk.report();
}

template <int DIAG, bool BIG>
__global__ __launch_bounds__(BR_THREADS, 2) void conv2_bwd_roll_kernel(
    const uint2* __restrict__ y2, const uint32_t* __restrict__ a2, const unsigned short* __restrict__ g2m,
    const float* __restrict__ aff2, const float* __restrict__ kbuf, const float* __restrict__ b2,
    const uint32_t* __restrict__ mag,
    const uint4* __restrict__ p1,
    const uint4* __restrict__ wdpack, uint2* __restrict__ dp1, uint32_t* __restrict__ dp1_dec, float* __restrict__ slab,
    const int* __restrict__ walk, int sw, int sk, int B, int P) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  BRArgs a;
  a.y2 = y2; a.a2 = a2; a.g2m = g2m; a.p1 = p1; a.dp1 = dp1; a.slab = slab; a.walk = walk;
  a.B = B; a.P = P; a.Q = P / 2;
  a.sk = sk;
  a.w = xcd_remap(blockIdx.x, gridDim.x);  // this workgroup's list (XCD-contiguous: neighbouring columns)
  a.walk = walk + a.w * sw;
  float* kc = reinterpret_cast<float*>(smem + BR_OFF_K);
  if (tid < 64) {
    // the dy2 scale 2^e (header): wave 0, lane c < 32 bounds channel c; k1..k3 are scaled in
    // place, kc[BR_KINV] = 2^-e for the epilogues
    const int c = tid & 31;
    const float k1 = kbuf[c], k2 = kbuf[32 + c], k3 = kbuf[64 + c];
    // mag[c] = max |y2 - b2| (conv2_fwd2.hip): |y2| <= mag[c] + |b2|
    const float gmx = __uint_as_float(mag[32]), ymx = __uint_as_float(mag[c]) + fabsf(b2[c]);
    float bound = fabsf(k1) * gmx + fabsf(k2) * ymx + fabsf(k3);
    bound = wave_max(tid < 32 ? bound : 0.f);  // NaN/inf bound: no scaling (e = 0)
    int e = 0;
    if (bound > 0.f && __builtin_isfinite(bound)) {
      int x;
      (void)frexpf(bound, &x);  // bound < 2^x
      e = min(60, max(-60, 15 - x));
    }
    const float sc = ldexpf(1.f, e);
    // the staging reads y2h (conv2_common.h): y2 = h * d + b2, d = inv / 2^k (powers of two), so
    // a*y2 + b = (a d) h + (a b2 + b) and k2*y2 + k3 = (k2 d) h + (k2 b2 + k3)
    const float d = __uint_as_float(mag[kMagScales]) * __uint_as_float(mag[kMagScales + 1]) /
                    __uint_as_float(mag[kMagScales + 2]);
    if (tid < 32) {
      const float ka = aff2[c], kb = aff2[32 + c], bc = b2[c];
      kc[c] = ka * d;
      kc[32 + c] = fmaf(ka, bc, kb);
      kc[64 + c] = k1 * sc * kbuf[96 + c];  // g2m is stored at 2^e_c: kbuf[96 + c] = 2^-e_c (head_pb.hip)
      kc[96 + c] = k2 * d * sc;
      kc[128 + c] = fmaf(k2, bc, k3) * sc;
    }
    if (tid == 0) {
      const float ie = ldexpf(1.f, -e), sd = __uint_as_float(mag[kMagScales + 3]);
      kc[BR_KINV] = ie * __uint_as_float(mag[kMagScales]);          // dy2 and packed-weight scales
      kc[BR_KINV + 1] = ie * __uint_as_float(mag[kMagScales + 1]);  // dy2 and p1 scales
      kc[BR_KINV + 2] = ie;
      kc[BR_KINV + 3] = sd;                                         // the dp1h store factor
      if (blockIdx.x == 0) dp1_dec[0] = __float_as_uint(kc[BR_KINV] / sd);  // exact: powers of two
    }
  }
  __syncthreads();  // kc visible to every role
  switch (wv) {
    case 0: br_mfma<0, DIAG>(a, wdpack, smem); break;
    case 1: br_mfma<1, DIAG>(a, wdpack, smem); break;
    case 2: br_mfma<2, DIAG>(a, wdpack, smem); break;
    case 3: br_mfma<3, DIAG>(a, wdpack, smem); break;
    default: br_stage<DIAG, BIG>(a, smem); break;  // waves 4-7
  }
}

}  // namespace tds

using namespace tds;

int tds_conv2_bwd3_num_wg() { return tds_conv2_num_wg(); }  // one 8-wave workgroup per CU

// DIAG 13 clocks of the last launch: n uint32 (2 per wave, 8 waves per workgroup)
int tds_conv2_bwd_clock_read(uint32_t* host, int n) {
  if (n > kBRClkMaxWg * 16) n = kBRClkMaxWg * 16;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_br_clk), (size_t)n * 4, 0, hipMemcpyDeviceToHost) == hipSuccess ? n : -1;
}

void tds_conv2_bwd3_tiles(int P, int* tiles_r, int* tiles_c) {
  *tiles_r = (P + BR_TH - 1) / BR_TH;
  *tiles_c = (P + BR_TC - 1) / BR_TC;
}

// Walk table of the rolling conv2 backward: segments of ~seg tiles down one tile column of one
// image (segment s: image-major, then row band, then column).  Whole rounds of nwg segments go
// round-robin (segment s to list s % nwg: the workgroups of one XCD, contiguous lists after
// xcd_remap, take neighbouring columns of the same band).  The last, partial round is cut into
// nwg near-equal runs of consecutive tiles instead (a run may start mid-segment or cross into
// the next column: each such start is flagged and re-stages its 4 top rows), so no workgroup
// ends a whole segment after the others (the round-robin tail left a 4.7 % spread at the bench
// shape).  out == nullptr: returns the table length (rows x nwg ints); else fills it (rows =
// longest list + 3, the tail of each list marked kWalkEnd over a copy of its last tile, which
// the staging's look-ahead loads re-read).  Returns -1 on unsupported sizes.
int64_t tds_conv2_bwd_walk(int* out, int B, int tiles_r, int tiles_c, int nwg, int seg) {
  if (B < 1 || B > 63 || tiles_r < 1 || tiles_r > 4095 || tiles_c < 1 || tiles_c > 4095 || nwg < 1 || seg < 2)
    return -1;
  const int nband = (tiles_r + seg - 1) / seg;
  // near-equal bands (lengths differ by at most 1, every band >= 2 tiles when tiles_r >= 2)
  std::vector<int> bstart(nband + 1);
  for (int j = 0; j <= nband; ++j) bstart[j] = (int)((int64_t)j * tiles_r / nband);
  const int64_t nseg = (int64_t)B * nband * tiles_c;
  const int64_t nfull = nseg / nwg * nwg;  // segments dealt in whole rounds
  auto seg_of = [&](int64_t s, int& b, int& j, int& tc) {
    b = (int)(s / ((int64_t)nband * tiles_c));
    j = (int)((s / tiles_c) % nband);
    tc = (int)(s % tiles_c);
  };
  std::vector<int64_t> len(nwg, 0);
  int64_t ntail = 0;
  for (int64_t s = 0; s < nseg; ++s) {
    int b, j, tc;
    seg_of(s, b, j, tc);
    if (s < nfull) len[s % nwg] += bstart[j + 1] - bstart[j];
    else ntail += bstart[j + 1] - bstart[j];
  }
  const int64_t tbase = ntail / nwg, textra = ntail % nwg;
  int64_t maxlen = 0;
  for (int w = 0; w < nwg; ++w) maxlen = std::max(maxlen, len[w] + tbase + (w < textra ? 1 : 0));
  // + BR_WALK_PAD end-marked entries: the staging's look-ahead reads tile k + 2 * sets at the last
  // iteration of a list of length k + 1 (br_stage: every load set is issued on every path; 4 with
  // two sets, 6 with three) -- with too few the longest list's last read ran past its row (the
  // next list, or past the table for the last one)
  const int64_t rows = maxlen + BR_WALK_PAD;
  if (rows * nwg >= ((int64_t)1 << 31)) return -1;  // the kernel indexes it in 32 bits
  if (out == nullptr) return rows * nwg;
  std::vector<int64_t> fill(nwg, 0);
  std::vector<uint32_t> last(nwg, 0u);
  auto put = [&](int w, uint32_t code, bool start) {
    out[fill[w]++ * nwg + w] = (int)(code | (start ? kWalkStart : 0u));
    last[w] = code;
  };
  int tw = 0;                                   // tail: current list
  int64_t tgot = 0, twant = tbase + (0 < textra ? 1 : 0);
  for (int64_t s = 0; s < nseg; ++s) {
    int b, j, tc;
    seg_of(s, b, j, tc);
    for (int tr = bstart[j]; tr < bstart[j + 1]; ++tr) {
      const uint32_t code = ((uint32_t)b << 24) | ((uint32_t)tr << 12) | (uint32_t)tc;
      if (s < nfull) {
        put((int)(s % nwg), code, tr == bstart[j]);
        continue;
      }
      while (twant == 0) {  // lists that get no tail tiles (ntail < nwg)
        ++tw;
        twant = tbase + (tw < textra ? 1 : 0);
      }
      put(tw, code, tr == bstart[j] || tgot == 0);
      if (++tgot == twant) {
        ++tw;
        tgot = 0;
        twant = tw < nwg ? tbase + (tw < textra ? 1 : 0) : 0;
      }
    }
  }
  for (int w = 0; w < nwg; ++w)
    for (int64_t k = fill[w]; k < rows; ++k) out[k * nwg + w] = (int)(last[w] | kWalkEnd);
  return rows * nwg;
}

#ifdef TDS_DIAG
// timing-only variants: 1 no MFMAs, 3 no global tile loads, 5 no staging, 9 no
// BN2 / pool backward math in the staging, 13 the full kernel with per-wave barrier-wait clocks,
// 16..27 the flag sets of conv2_common.h (with clocks).  Compiled only into a -DTDS_DIAG build
// (python -m torch_distributed_sandbox_amd._build --variant diag -D TDS_DIAG; TDS_CONV2_DIAG=N).
static int br_diag_env() {
  const char* e = std::getenv("TDS_CONV2_DIAG");
  return e ? std::atoi(e) : 0;
}
#else
static int br_diag_env() { return 0; }
#endif

// g2m: fp16 planar [B][32][Q][Q] (kbuf[96 + c] = its scale 2^-e_c); walk: tds_conv2_bwd_walk table for nwg workgroups, transposed to
// [nwg][rows] (fused_ops.cpp bwd_walk)
void tds_conv2_bwd3(const void* y2h, const uint32_t* a2, const unsigned short* g2m, const float* aff2, const float* kbuf,
                    const float* b2,
                    uint32_t* mag, const void* p1, const short* wd, void* dp1h, float* slab, const int* walk,
                    int nwg, int sw, int sk, int B, int P, hipStream_t st) {
  const int Q = P / 2;
  const bool big = (int64_t)32 * Q * Q * 2 >= 0xFFFFFF00LL;  // g2m image beyond a 4 GiB descriptor
#define TDS_BR_LAUNCH_B(D, BG)                                                                                         \
  {                                                                                                                    \
    static bool set = false;                                                                                           \
    if (!set) {                                                                                                        \
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(conv2_bwd_roll_kernel<D, BG>),                           \
                                hipFuncAttributeMaxDynamicSharedMemorySize, BR_LDS);                                   \
      set = true;                                                                                                      \
    }                                                                                                                  \
    hipLaunchKernelGGL((conv2_bwd_roll_kernel<D, BG>), dim3(nwg), dim3(BR_THREADS), BR_LDS, st,                        \
                       reinterpret_cast<const uint2*>(y2h), a2, g2m, aff2, kbuf, b2, mag,                                \
                       reinterpret_cast<const uint4*>(p1),                                                            \
                       reinterpret_cast<const uint4*>(wd), static_cast<uint2*>(dp1h), mag + kMagScales + 4, slab, walk, \
                       sw, sk, B, P);                                                                                 \
    TDS_LAUNCH_CHECK();                                                                                                \
  }
#define TDS_BR_LAUNCH(D)           \
  if (big) TDS_BR_LAUNCH_B(D, true) \
  else TDS_BR_LAUNCH_B(D, false)
  switch (br_diag_env()) {
#ifdef TDS_DIAG
    case 1: TDS_BR_LAUNCH(1) break;
    case 3: TDS_BR_LAUNCH(3) break;
    case 5: TDS_BR_LAUNCH(5) break;
    case 9: TDS_BR_LAUNCH(9) break;
    case 13: TDS_BR_LAUNCH(13) break;
    // flag sets (conv2_common.h): 16 = full + clocks; +1 no staging, +2 no LDS operand reads,
    // +4 dgrad idle, +8 wgrad idle
    case 16: TDS_BR_LAUNCH(16) break;
    case 17: TDS_BR_LAUNCH(17) break;
    case 19: TDS_BR_LAUNCH(19) break;
    case 20: TDS_BR_LAUNCH(20) break;
    case 21: TDS_BR_LAUNCH(21) break;
    case 23: TDS_BR_LAUNCH(23) break;
    case 24: TDS_BR_LAUNCH(24) break;
    case 25: TDS_BR_LAUNCH(25) break;
    case 27: TDS_BR_LAUNCH(27) break;
    // +32 staging without global loads, +64 staging without the BN2 / pool math
    case 28: TDS_BR_LAUNCH(28) break;
    case 60: TDS_BR_LAUNCH(60) break;
    case 92: TDS_BR_LAUNCH(92) break;
    case 48: TDS_BR_LAUNCH(48) break;
    case 80: TDS_BR_LAUNCH(80) break;
#endif
    default: TDS_BR_LAUNCH(0) break;
  }
#undef TDS_BR_LAUNCH
#undef TDS_BR_LAUNCH_B
}
