// conv2 backward v2: BN2 / ReLU / max-pool backward fused into conv2 dgrad + wgrad,
// laid out for TWO 4-wave workgroups per CU.
//
// Why a second design (conv2_bwd_fused_kernel in conv2_bf16x3.hip is the first): that
// kernel runs one 8-wave workgroup per CU, so its staging phase (global loads -> BN2
// backward VALU -> LDS stores, between two barriers) and its MFMA phase alternate on
// every SIMD; rocprof showed the MFMA pipe busy 35% of the time and waves parked on
// barriers/waits half of it.  Here each workgroup needs < 80 KiB of LDS and <= 256 VGPRs
// per wave, so two co-reside on a CU and one workgroup's staging runs under the other's
// MFMAs.  What makes it fit:
//   * output tile 8 x 16 (staged 12 x 20 records incl. the 2-pixel halo);
//   * the dgrad weight fragments live in REGISTERS, not LDS: the 25 flipped taps are
//     split over the two dgrad waves (13 + 12 taps, 8 VGPRs each), each wave produces a
//     partial dp1 for the whole tile, and the halves are exchanged through 8 KiB of LDS;
//   * wgrad: two waves, 13 taps each (tap 25 = the bias "ones" column), K = 32 pixels =
//     two output rows, operands by ds_read_b64_tr_b16 transposed reads.
//
// Per tile (4 waves, one per SIMD):
//   wave 0/1 : dgrad, taps grouped by kx so an input row's A fragment serves up to 5
//              output rows:  wave 0 = kx {0,1} x ky 0-4  +  kx 4 x ky 0-2
//                            wave 1 = kx {2,3} x ky 0-4  +  kx 4 x ky 3-4
//   wave 2/3 : wgrad, taps 0-12 / 13-25, both co halves, accumulated over the tiles of
//              the persistent workgroup; slab[wg][26][32][16] reduced in fp64 afterwards.
// LDS (72 448 B): dy2 planes (hi co0-15, hi co16-31, lo co0-15, lo co16-31) | 2 x p1 planes
// (hi, lo; LDS-DMA, double-buffered) | dgrad exchange | BN2 backward constants.
#include <cstdlib>

#include "conv2_common.h"
#include "launchers.h"
#include "pooled_layout.h"

namespace tds {

constexpr int B2_TH = 8, B2_TC = 16;
constexpr int B2_SR = B2_TH + 4, B2_SC = B2_TC + 4;      // 12 x 20 staged records
constexpr int B2_REC = B2_SR * B2_SC;                      // 240
constexpr int B2_THREADS = 256;
constexpr int B2_DPLANE = B2_REC * 32 + 32;                // 7712 B
// p1 planes are filled by LDS-DMA (global_load_lds_dwordx4): one wave-instruction writes
// 32 records x 32 B of one plane, so a plane holds 8 such groups (256 records, 240 used),
// and they are double-buffered (tile t+1's DMA runs under tile t's MFMAs).
constexpr int B2_PGROUPS = 8;
constexpr int B2_PPLANE = B2_PGROUPS * 32 * 32;            // 8192 B
constexpr int B2_PBUF = 2 * B2_PPLANE;                     // hi + lo planes
constexpr int B2_OFF_P = 4 * B2_DPLANE;                    // 30848
constexpr int B2_OFF_X = B2_OFF_P + 2 * B2_PBUF;           // 63616
constexpr int B2_XCHG = 2 * 4 * 64 * 16;                   // 8192
constexpr int B2_OFF_K = B2_OFF_X + B2_XCHG;               // 71808
constexpr int B2_LDS = B2_OFF_K + 5 * 32 * 4;              // 72448
constexpr int B2_NWIN = (B2_SR / 2) * (B2_SC / 2);         // 60 pooling windows
constexpr int B2_ITEMS = B2_NWIN * 8;                      // (window, 4-channel chunk)
constexpr int B2_IPER = (B2_ITEMS + B2_THREADS - 1) / B2_THREADS;   // 2
constexpr int B2_DMA_PER_WAVE = 2 * B2_PGROUPS / (B2_THREADS / 64);  // 4 p1 DMA instructions per wave
static_assert(B2_LDS % 16 == 0 && B2_OFF_P % 16 == 0 && B2_OFF_X % 16 == 0 && B2_OFF_K % 16 == 0, "LDS carve");
static_assert(2 * B2_LDS <= 160 * 1024, "two workgroups per CU");

// dgrad tap groups: group I of wave D covers kx = KX, ky = KY0 .. KY0 + NKY - 1; its
// weights sit in register slots 5I .. 5I + NKY - 1.
template <int D, int I>
struct DgGroup {
  static constexpr int KX = D == 0 ? (I == 0 ? 0 : I == 1 ? 1 : 4) : (I == 0 ? 2 : I == 1 ? 3 : 4);
  static constexpr int KY0 = I < 2 ? 0 : (D == 0 ? 0 : 3);
  static constexpr int NKY = I < 2 ? 5 : (D == 0 ? 3 : 2);
};

template <int D, int I>
__device__ __forceinline__ void b2_load_w_group(const uint4* __restrict__ wd, f32x4 (&R)[13][2], int lane) {
  using G = DgGroup<D, I>;
#pragma unroll
  for (int k = 0; k < G::NKY; ++k) {
    const int s = (G::KY0 + k) * 5 + G::KX;  // flipped-tap index of the dgrad pack
    const uint4 h = wd[s * 64 + lane], l = wd[(25 + s) * 64 + lane];
    R[5 * I + k][0] = __builtin_bit_cast(f32x4, h);
    R[5 * I + k][1] = __builtin_bit_cast(f32x4, l);
  }
}

template <int D>
__device__ __forceinline__ void b2_load_w(const uint4* __restrict__ wd, f32x4 (&R)[13][2], int lane) {
  b2_load_w_group<D, 0>(wd, R, lane);
  b2_load_w_group<D, 1>(wd, R, lane);
  b2_load_w_group<D, 2>(wd, R, lane);
}

// Wave D hands the partner's rows (4(1-D) .. +3) to the exchange slot 1-D.
template <int D>
__device__ __forceinline__ void b2_xchg_put(f32x4* xs, const f32x4 (&acc)[8], int lane) {
#pragma unroll
  for (int i = 0; i < 4; ++i) xs[((1 - D) * 4 + i) * 64 + lane] = acc[4 * (1 - D) + i];
}

// Wave D owns output rows 4D .. 4D+3: its partial + the partner's, then dp1.
template <int D, int DIAG = 0>
__device__ __forceinline__ void b2_xchg_finish(const f32x4* xs, const f32x4 (&acc)[8], float* __restrict__ dp1,
                                               int lane, int b, int r0, int c0, int P) {
  const int li = lane & 15, g = lane >> 4;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const f32x4 v = acc[4 * D + i] + xs[(D * 4 + i) * 64 + lane];
    const int row = r0 + 4 * D + i;
    if (DIAG == 11 ? v[0] == 1234.5f : row < P) {  // DIAG 11 (timing only): no dp1 stores
      float* orow = dp1 + ((int64_t)b * P + row) * P * 16;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int col = c0 + 4 * g + r;
        if (col < P) orow[(int64_t)col * 16 + li] = v[r];
      }
    }
  }
}

// Per-thread staging state: the next tile's y2 windows, pooled gradients and p1 records
// in registers (loaded under the current tile's MFMAs), then BN2 backward -> LDS.
struct B2Args {
  const float4* __restrict__ y2;
  const float* __restrict__ g2m;  // planar [B][32][Q][Q] (the fc flatten order)
  const uint4* __restrict__ p1;
  float* __restrict__ dp1;
  float* __restrict__ slab;
  const int* __restrict__ order;  // blocked tile order (tds_tile_order)
  int B, P, Q, tiles_r, tiles_c, per_img, total;
};

struct B2Tile {
  int b, r0, c0;
  bool interior;  // whole staged region inside the pooled image: no bounds / padding work
};

__device__ __forceinline__ B2Tile b2_decode(const B2Args& a, int t) {
  B2Tile x;
  int tr, tc;
  tile_from_order(a.order, t, x.b, tr, tc);
  x.r0 = tr * B2_TH;
  x.c0 = tc * B2_TC;
  x.interior = x.r0 >= 2 && x.c0 >= 2 && x.r0 + B2_SR - 2 <= 2 * a.Q && x.c0 + B2_SC - 2 <= 2 * a.Q;
  return x;
}

// wave-uniform buffer descriptor over [base, base + 2 GiB): per-lane byte offsets in voffset,
// an invalid lane gets kB2Oob and reads zeros (hardware range check, no exec masking)
constexpr uint32_t kB2Oob = 0xFFFFFFF0u;
__device__ __forceinline__ __amdgpu_buffer_rsrc_t b2_rsrc(const void* base) { return tds_buffer_rsrc(base, 0x7FFFFFF0u); }

// 16 zero bytes: the LDS-DMA source of staged p1 records outside the image
__device__ __attribute__((aligned(16))) uint32_t g_b2_zero[4] = {0u, 0u, 0u, 0u};

// REGP1 (v3): p1 records go global -> registers -> ds_write in store() instead of LDS-DMA.
// The compiler cannot tell an LDS-DMA's destination from later LDS accesses, so every ds_read /
// ds_write after one waits vmcnt(0) -- which drains the register loads issued for LATER
// tiles too and defeats a multi-tile lookahead.
// BIG: 32 g2m planes of an image exceed a 4 GiB buffer-descriptor range (H >= 23170): 64-bit
// g2m loads.  A template parameter, not a runtime flag: two alternative load paths under a
// runtime branch make the compiler's wait-count analysis assume the fewer-loads path at the
// merge and wait for vmcnt(0), draining the loads issued for later tiles.
template <int DIAG, int WV, bool REGP1 = false, bool BIG = false>  // WV: the wave (= role) this staging code runs in
struct B2Stager {
  float4 yv[B2_IPER][4], gv[B2_IPER];
  uint4 pr[REGP1 ? B2_DMA_PER_WAVE : 1];
  // per-thread byte offsets (fixed for the kernel): global, relative to the tile's
  // descriptor bases, and LDS, of each staging item (window x 4 channels); p1 DMA sources
  uint32_t yoff[B2_IPER], goff[B2_IPER], doff[B2_DMA_PER_WAVE];
  int drec[B2_IPER];

  // staging item u of this thread: window (wy, wx)
  __device__ __forceinline__ static void item_geom(int tid, int u, int& wy, int& wx) {
    const int it = tid + u * B2_THREADS;
    const int w = (it < B2_ITEMS ? it : 0) >> 3;
    wy = w / (B2_SC / 2);
    wx = w - wy * (B2_SC / 2);
  }
  // p1 DMA instruction j of wave wv: plane pl, record group rg; lane -> record, 16-B half
  __device__ __forceinline__ static void dma_geom(int wv, int j, int lane, int& pl, int& rg, int& px, int& half) {
    const int k = wv * B2_DMA_PER_WAVE + j;
    pl = k / B2_PGROUPS;
    rg = k - pl * B2_PGROUPS;
    px = rg * 32 + (lane >> 1);
    half = lane & 1;
  }

  __device__ __forceinline__ void init(const B2Args& a, int tid) {
    const int c4 = tid & 7;
#pragma unroll
    for (int u = 0; u < B2_IPER; ++u) {
      int wy, wx;
      item_geom(tid, u, wy, wx);
      yoff[u] = (uint32_t)(((2 * wy) * a.P + 2 * wx) * 128 + c4 * 16);
      goff[u] = BIG ? 0u : (uint32_t)(((int64_t)c4 * 4 * a.Q * a.Q + (int64_t)wy * a.Q + wx) * 4);
      drec[u] = ((2 * wy) * B2_SC + 2 * wx) * 32 + (c4 & 3) * 8;
    }
#pragma unroll
    for (int j = 0; j < B2_DMA_PER_WAVE; ++j) {
      int pl, rg, px, half;
      dma_geom(WV, j, tid & 63, pl, rg, px, half);
      const int pxc = px < B2_REC ? px : 0;
      const int rr = pxc / B2_SC, cc = pxc - rr * B2_SC;
      doff[j] = (uint32_t)((rr * a.P + cc) * 64 + pl * 32 + half * 16);
    }
  }

  // tile x: y2 windows + pooled gradients -> registers; p1 -> LDS buffer pbuf by DMA
  __device__ __forceinline__ void load(const B2Args& a, const B2Tile& x, int tid, char* pbuf) {
    if constexpr (DIAG == 3) {
#pragma unroll
      for (int u = 0; u < B2_IPER; ++u) {
        gv[u] = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int q = 0; q < 4; ++q) yv[u][q] = gv[u];
      }
      return;
    }
    const int P = a.P, Q = a.Q;
    const int64_t img = (int64_t)x.b * P;
    const __amdgpu_buffer_rsrc_t ry =
        b2_rsrc(reinterpret_cast<const char*>(a.y2) + ((img + x.r0 - 2) * P + (x.c0 - 2)) * 128);
    const char* pbase = reinterpret_cast<const char*>(a.p1) + ((img + x.r0 - 2) * P + (x.c0 - 2)) * 64;
    uint32_t oy[B2_IPER][4];
    // pooled gradients: window (wy, wx) is pooled position (r0/2 - 1 + wy, c0/2 - 1 + wx), four
    // channel planes of the planar g2m.  One buffer descriptor per tile (base: the tile's pooled
    // origin in channel 0 of its image) while 32 planes fit a 4 GiB range (H < 23170); beyond
    // that, 64-bit addresses.
    const int64_t gplane = (int64_t)Q * Q;
    const __amdgpu_buffer_rsrc_t rg =
        tds_buffer_rsrc(a.g2m + (int64_t)x.b * 32 * gplane + (int64_t)(x.r0 / 2 - 1) * Q + (x.c0 / 2 - 1), 0xFFFFFFF0u);
    uint32_t og[B2_IPER];
#pragma unroll
    for (int u = 0; u < B2_IPER; ++u) {
#pragma unroll
      for (int q = 0; q < 4; ++q) oy[u][q] = yoff[u] + (uint32_t)(((q >> 1) * P + (q & 1)) * 128);
      og[u] = goff[u];
    }
    if (!x.interior || BIG) {
      // edge tile: pooled windows outside the image read zeros (big: og only flags validity)
#pragma unroll
      for (int u = 0; u < B2_IPER; ++u) {
        int wy, wx;
        item_geom(tid, u, wy, wx);
        const int py = x.r0 / 2 - 1 + wy, px = x.c0 / 2 - 1 + wx;
        const bool ok = tid + u * B2_THREADS < B2_ITEMS && py >= 0 && py < Q && px >= 0 && px < Q;
        if (!ok) og[u] = kB2Oob;
      }
    }
    const char* psrc[B2_DMA_PER_WAVE];
#pragma unroll
    for (int j = 0; j < B2_DMA_PER_WAVE; ++j) psrc[j] = pbase + doff[j];
    if (!x.interior) {
      // edge tile: lanes outside the image (or past the item count) read zeros
      const int lo_r = max(0, 2 - x.r0), hi_r = min(B2_SR, P - x.r0 + 2);
      const int lo_c = max(0, 2 - x.c0), hi_c = min(B2_SC, P - x.c0 + 2);
#pragma unroll
      for (int u = 0; u < B2_IPER; ++u) {
        int wy, wx;
        item_geom(tid, u, wy, wx);
        const bool item = tid + u * B2_THREADS < B2_ITEMS;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int lr = 2 * wy + (q >> 1), lc = 2 * wx + (q & 1);
          if (!(item && lr >= lo_r && lr < hi_r && lc >= lo_c && lc < hi_c)) oy[u][q] = kB2Oob;
        }
      }
#pragma unroll
      for (int j = 0; j < B2_DMA_PER_WAVE; ++j) {
        int pl, rgp, px, half;
        dma_geom(WV, j, tid & 63, pl, rgp, px, half);
        const int rr = px / B2_SC, cc = px - rr * B2_SC;
        if (!(px < B2_REC && rr >= lo_r && rr < hi_r && cc >= lo_c && cc < hi_c))
          psrc[j] = reinterpret_cast<const char*>(g_b2_zero);
      }
    } else {
#pragma unroll
      for (int j = 0; j < B2_DMA_PER_WAVE; ++j) {
        int pl, rgp, px, half;
        dma_geom(WV, j, tid & 63, pl, rgp, px, half);
        if (px >= B2_REC) psrc[j] = reinterpret_cast<const char*>(g_b2_zero);
      }
    }
    const __amdgpu_buffer_rsrc_t rp = b2_rsrc(pbase);
#pragma unroll
    for (int j = 0; j < B2_DMA_PER_WAVE; ++j) {
      if constexpr (REGP1) {
        // buffer loads (not flat: a flat load makes every later wait a full vmcnt(0) drain)
        const uint32_t po = psrc[j] == reinterpret_cast<const char*>(g_b2_zero) ? kB2Oob : doff[j];
        pr[j] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rp, po, 0, 0));
      } else {
        int pl, rgp, px, half;
        dma_geom(WV, j, 0, pl, rgp, px, half);
        __builtin_amdgcn_global_load_lds(psrc[j], (__attribute__((address_space(3))) void*)(pbuf + pl * B2_PPLANE + rgp * 1024),
                                         16, 0, 0);
      }
    }
#pragma unroll
    for (int u = 0; u < B2_IPER; ++u) {
#pragma unroll
      for (int q = 0; q < 4; ++q)
        yv[u][q] = DIAG == 7 ? make_float4(1.f, 0.f, 0.f, 0.f)  // timing only: no y2 loads
                             : __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(ry, oy[u][q], 0, 0));
      float g4[4];
      if constexpr (!BIG) {
        const uint32_t gstep = (uint32_t)(gplane * 4);
#pragma unroll
        for (int k = 0; k < 4; ++k)
          g4[k] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                                rg, og[u] == kB2Oob ? kB2Oob : og[u] + k * gstep, 0, 0));
      } else {
        int wy, wx;
        item_geom(tid, u, wy, wx);
        const float* gp = a.g2m + ((int64_t)x.b * 32 + 4 * (tid & 7)) * gplane +
                          (int64_t)(x.r0 / 2 - 1 + wy) * Q + (x.c0 / 2 - 1 + wx);
#pragma unroll
        for (int k = 0; k < 4; ++k) g4[k] = og[u] == kB2Oob ? 0.f : gp[k * gplane];
      }
      gv[u] = make_float4(g4[0], g4[1], g4[2], g4[3]);
    }
  }

  // BN2 / ReLU / pool backward of the staged windows -> dy2 hi|lo planes.
  // dy2 = k1*dz + k2*y2 + k3, dz = pooled gradient at the window's argmax of a*y2 + b.
  // Interior tiles take a short path: every window pooled, every pixel inside the image,
  // argmax by max3 + first-equal (torch's scan-order tie rule); a NaN anywhere in the
  // thread's windows sends the wave to the general path (torch's NaN-wins rule).
  // REGP1: the tile's p1 records -> plane buffer pbuf (same layout the DMA writes)
  __device__ __forceinline__ void store_p1(char* pbuf, int tid) {
    if constexpr (REGP1) {
#pragma unroll
      for (int j = 0; j < B2_DMA_PER_WAVE; ++j) {
        int pl, rgp, px, half;
        dma_geom(WV, j, tid & 63, pl, rgp, px, half);
        *reinterpret_cast<uint4*>(pbuf + pl * B2_PPLANE + rgp * 1024 + (tid & 63) * 16) = pr[j];
      }
    }
  }

  __device__ __forceinline__ void store(const B2Args& a, const B2Tile& x, int tid, char* d_l, const float* kc) {
    const int c4 = tid & 7;
    const int P = a.P, Q = a.Q;
    const float4 ka4 = *reinterpret_cast<const float4*>(&kc[0 * 32 + 4 * c4]);
    const float4 kb4 = *reinterpret_cast<const float4*>(&kc[1 * 32 + 4 * c4]);
    const float4 k14 = *reinterpret_cast<const float4*>(&kc[2 * 32 + 4 * c4]);
    const float4 k24 = *reinterpret_cast<const float4*>(&kc[3 * 32 + 4 * c4]);
    const float4 k34 = *reinterpret_cast<const float4*>(&kc[4 * 32 + 4 * c4]);
    const float ka[4] = {ka4.x, ka4.y, ka4.z, ka4.w}, kb[4] = {kb4.x, kb4.y, kb4.z, kb4.w};
    const float k1[4] = {k14.x, k14.y, k14.z, k14.w}, k2[4] = {k24.x, k24.y, k24.z, k24.w},
                k3[4] = {k34.x, k34.y, k34.z, k34.w};
    bool fast = x.interior;
    if (fast) {
      float nsum = 0.f;
#pragma unroll
      for (int u = 0; u < B2_IPER; ++u)
#pragma unroll
        for (int q = 0; q < 4; ++q) nsum += (yv[u][q].x + yv[u][q].y) + (yv[u][q].z + yv[u][q].w);
      fast = __builtin_amdgcn_ballot_w64(isnan(nsum)) == 0;  // wave-uniform
    }
#pragma unroll
    for (int u = 0; u < B2_IPER; ++u) {
      const int it = tid + u * B2_THREADS;
      if (it >= B2_ITEMS) continue;
      float y[4][4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        y[q][0] = yv[u][q].x; y[q][1] = yv[u][q].y; y[q][2] = yv[u][q].z; y[q][3] = yv[u][q].w;
      }
      const float gg[4] = {gv[u].x, gv[u].y, gv[u].z, gv[u].w};
      float d[4][4];
      if constexpr (DIAG == 9) {  // timing only: no BN2 / pool backward math (dy2 := y2 + g)
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
          for (int cc = 0; cc < 4; ++cc) d[q][cc] = y[q][cc] + gg[cc];
      } else if (fast) {
#pragma unroll
        for (int cc = 0; cc < 4; ++cc) {
          float z[4];
#pragma unroll
          for (int q = 0; q < 4; ++q) z[q] = fmaf(ka[cc], y[q][cc], kb[cc]);
          const float m = fmaxf(fmaxf(z[0], z[1]), fmaxf(z[2], z[3]));
          const bool e0 = z[0] == m, e1 = !e0 && z[1] == m, e2 = !e0 && !e1 && z[2] == m;
          const bool e3 = !e0 && !e1 && !e2;
          const float base[4] = {fmaf(k2[cc], y[0][cc], k3[cc]), fmaf(k2[cc], y[1][cc], k3[cc]),
                                 fmaf(k2[cc], y[2][cc], k3[cc]), fmaf(k2[cc], y[3][cc], k3[cc])};
          const float kg = k1[cc] * gg[cc];
          d[0][cc] = e0 ? base[0] + kg : base[0];
          d[1][cc] = e1 ? base[1] + kg : base[1];
          d[2][cc] = e2 ? base[2] + kg : base[2];
          d[3][cc] = e3 ? base[3] + kg : base[3];
        }
      } else {
        int wy, wx;
        item_geom(tid, u, wy, wx);
        const int gy = x.r0 - 2 + 2 * wy, gx = x.c0 - 2 + 2 * wx;
        const bool pooled = gy >= 0 && gx >= 0 && (gy >> 1) < Q && (gx >> 1) < Q;
#pragma unroll
        for (int cc = 0; cc < 4; ++cc) {
          float m = ka[cc] * y[0][cc] + kb[cc];
          int ai = 0;
#pragma unroll
          for (int q = 1; q < 4; ++q) {
            const float z = ka[cc] * y[q][cc] + kb[cc];
            if (z > m || isnan(z)) { m = z; ai = q; }  // first max in scan order, NaN wins (torch)
          }
          const int am = pooled ? ai : -1;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int r = gy + (q >> 1), c = gx + (q & 1);
            const bool inb = r >= 0 && r < P && c >= 0 && c < P;  // zero padding outside the image
            const float dz = am == q ? gg[cc] : 0.f;
            d[q][cc] = inb ? fmaf(k1[cc], dz, fmaf(k2[cc], y[q][cc], k3[cc])) : 0.f;
          }
        }
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        uint32_t h01, l01, h23, l23;
        split2_bf16(d[q][0], d[q][1], h01, l01);
        split2_bf16(d[q][2], d[q][3], h23, l23);
        const int off = drec[u] + ((q >> 1) * B2_SC + (q & 1)) * 32;
        *reinterpret_cast<uint2*>(d_l + (c4 >> 2) * B2_DPLANE + off) = make_uint2(h01, h23);
        *reinterpret_cast<uint2*>(d_l + (2 + (c4 >> 2)) * B2_DPLANE + off) = make_uint2(l01, l23);
      }
    }
  }
};

// ============================================================================ v3: producer/consumer waves
// Counters on v2 (rocprofv3 --pmc, docs/KERNELS.md): MFMA busy ~41% of the kernel, ~725 VALU
// instructions per wave per tile against ~312 MFMAs, and every wave alternating staging and
// MFMA phases between two barriers, so with two waves per SIMD the MFMA pipe idles whenever
// both sit in the same phase.  v3 splits the roles: one 8-wave workgroup per CU, waves 0-3 run
// ONLY the dgrad/wgrad MFMA loops of v2 (one per SIMD), waves 4-7 ONLY stage (BN2/ReLU/pool
// backward -> dy2 hi|lo planes; p1 by LDS-DMA).  Staging runs one tile ahead into double-
// buffered dy2 / p1 planes; its y2 / g2m / p1 register loads run three tiles ahead (two
// register sets: staging alone was memory-latency bound; no LDS-DMA, see B2Stager), the dgrad
// exchange slots are double-buffered, so ONE barrier per tile separates producer and
// consumer.  The barrier is a bare s_barrier after lgkmcnt(0): a producer's register loads
// for later tiles stay in flight across it.
constexpr int B3_THREADS = 512;
constexpr int B3_DBUF = 4 * B2_DPLANE;                      // dy2 hi/lo planes of one tile
constexpr int B3_OFF_P = 2 * B3_DBUF;                       // 61696: 3 x p1 buffers
constexpr int B3_NP = 2;                                   // p1 buffers (staged with dy2, one tile ahead)
constexpr int B3_OFF_X = B3_OFF_P + B3_NP * B2_PBUF;        // 127232: 2 x exchange slots
constexpr int B3_OFF_K = B3_OFF_X + 2 * B2_XCHG;            // 143616
constexpr int B3_LDS = B3_OFF_K + 5 * 32 * 4;               // 144256
static_assert(B3_LDS <= 160 * 1024 && B3_OFF_P % 16 == 0 && B3_OFF_X % 16 == 0 && B3_OFF_K % 16 == 0, "v3 LDS carve");

__device__ __forceinline__ void b3_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// v3 MFMA loops: the v2 loops (b2_dgrad, b2_wgrad) prefetch operands one step ahead and
// restart the pipeline at every kx group / K-step; with ONE MFMA wave per SIMD nothing hides
// those bubbles (v3 with staging disabled ran at ~67% MFMA utilisation).  Here each role's
// tile is one flat, fully unrolled sequence with operands fetched two steps ahead across
// group / K-step boundaries.
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

template <int D, int DIAG>
__device__ __forceinline__ void b3_dgrad(const char* d_l, const f32x4 (&R)[13][2], f32x4 (&acc)[8], int hp, int lp,
                                         int li) {
  using Q = DgSeq<D>;
#pragma unroll
  for (int o = 0; o < 8; ++o) acc[o] = f32x4{0.f, 0.f, 0.f, 0.f};
  s16x8 ah[3], al[3];
  auto load_a = [&](int s, int buf) {
    const int i = Q::grp(s), r = Q::row(s);
    const int rec = (Q::ky0(i) + r) * B2_SC + Q::kx(i) + li;
    ah[buf] = lds8<DIAG>(d_l + hp + rec * 32);
    al[buf] = lds8<DIAG>(d_l + lp + rec * 32);
  };
  load_a(0, 0);
  load_a(1, 1);
#pragma unroll
  for (int s = 0; s < Q::S; ++s) {
    if (s + 2 < Q::S) load_a(s + 2, (s + 2) % 3);
    __builtin_amdgcn_sched_barrier(0);
    const int i = Q::grp(s), r = Q::row(s);
#pragma unroll
    for (int k = 0; k < 5; ++k) {
      const int o = r - k;
      if (k < Q::nky(i) && o >= 0 && o < 8)
        acc[o] = mma3<DIAG>(ah[s % 3], al[s % 3], __builtin_bit_cast(s16x8, R[5 * i + k][0]),
                            __builtin_bit_cast(s16x8, R[5 * i + k][1]), acc[o]);
    }
  }
}

template <int E, int DIAG>
__device__ __forceinline__ void b3_wgrad(const char* d_l, const char* p_l, f32x4 (&wacc)[13][2], int lane,
                                         const s16x8& ones_hi, const s16x8& zero8) {
  const int g = lane >> 4, q4 = (lane >> 2) & 3, p4 = lane & 3;
  s16x8 ahi[2][2], alo[2][2], bhi[3], blo[3];
  auto load_a = [&](int m, int slot) {
    const int ra = (2 * m + 2) * B2_SC + 2 + 4 * g + q4;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const s16x4 x0 = ldtr<DIAG>(d_l + h * B2_DPLANE + ra * 32 + p4 * 8);
      const s16x4 x1 = ldtr<DIAG>(d_l + h * B2_DPLANE + (ra + B2_SC) * 32 + p4 * 8);
      const s16x4 y0 = ldtr<DIAG>(d_l + (2 + h) * B2_DPLANE + ra * 32 + p4 * 8);
      const s16x4 y1 = ldtr<DIAG>(d_l + (2 + h) * B2_DPLANE + (ra + B2_SC) * 32 + p4 * 8);
      ahi[slot][h] = s16x8{x0[0], x0[1], x0[2], x0[3], x1[0], x1[1], x1[2], x1[3]};
      alo[slot][h] = s16x8{y0[0], y0[1], y0[2], y0[3], y1[0], y1[1], y1[2], y1[3]};
    }
  };
  auto load_b = [&](int s, int buf) {
    const int m = s / 13, tap = 13 * E + s % 13;
    if (tap < 25) {
      const int ky = tap / 5, kx = tap - 5 * (tap / 5);
      const int rb = (2 * m + ky) * B2_SC + kx + 4 * g + q4;
      const s16x4 x0 = ldtr<DIAG>(p_l + rb * 32 + p4 * 8);
      const s16x4 x1 = ldtr<DIAG>(p_l + (rb + B2_SC) * 32 + p4 * 8);
      const s16x4 y0 = ldtr<DIAG>(p_l + B2_PPLANE + rb * 32 + p4 * 8);
      const s16x4 y1 = ldtr<DIAG>(p_l + B2_PPLANE + (rb + B2_SC) * 32 + p4 * 8);
      bhi[buf] = s16x8{x0[0], x0[1], x0[2], x0[3], x1[0], x1[1], x1[2], x1[3]};
      blo[buf] = s16x8{y0[0], y0[1], y0[2], y0[3], y1[0], y1[1], y1[2], y1[3]};
    } else {
      bhi[buf] = ones_hi;  // bias gradient column
      blo[buf] = zero8;
    }
  };
  // K-steps m in a rolled loop (static buffer indices inside), operands rotated at the end
  load_a(0, 0);
  load_b(0, 0);
  load_b(1, 1);
#pragma unroll 1
  for (int m = 0; m < 4; ++m) {
#pragma unroll
    for (int k = 0; k < 13; ++k) {
      if (k + 2 < 13) load_b(13 * m + k + 2, (k + 2) % 3);
      else if (m + 1 < 4) load_b(13 * (m + 1) + k + 2 - 13, (k + 2) % 3);  // next K-step's first taps
      if (k == 10 && m + 1 < 4) load_a(m + 1, 1);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int h = 0; h < 2; ++h) wacc[k][h] = mma3<DIAG>(ahi[0][h], alo[0][h], bhi[k % 3], blo[k % 3], wacc[k][h]);
    }
    // taps 0, 1 of the next K-step sit in buffers 1, 2 (13 % 3 == 1), its A in slot 1
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      ahi[0][h] = ahi[1][h];
      alo[0][h] = alo[1][h];
    }
    bhi[0] = bhi[1];
    blo[0] = blo[1];
    bhi[1] = bhi[2];
    blo[1] = blo[2];
  }
}

template <int ROLE, int DIAG>  // ROLE 0/1 = dgrad wave D, 2/3 = wgrad
__device__ __forceinline__ void b3_mfma(const B2Args& a, const uint4* __restrict__ wdpack, char* smem, int first_t) {
#ifdef TDS_B3_MFMA_PRIO
  __builtin_amdgcn_s_setprio(TDS_B3_MFMA_PRIO);
#endif
  const int lane = threadIdx.x & 63;
  const int li = lane & 15, g = lane >> 4;
  f32x4 R[13][2];
#pragma unroll
  for (int k = 0; k < 13; ++k) R[k][0] = R[k][1] = f32x4{0.f, 0.f, 0.f, 0.f};
  f32x4 acc[8];
#pragma unroll
  for (int o = 0; o < 8; ++o) acc[o] = f32x4{0.f, 0.f, 0.f, 0.f};
  if constexpr (ROLE < 2) b2_load_w<ROLE>(wdpack, R, lane);
  s16x8 ones_hi, zero8;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    ones_hi[j] = (short)(li == 0 ? 0x3f80 : 0);
    zero8[j] = 0;
  }
  const int hp = (g >> 1) * B2_DPLANE + (g & 1) * 16;
  const int lp = (2 + (g >> 1)) * B2_DPLANE + (g & 1) * 16;
  B2Tile prev{0, 0, 0, false};
  bool have_prev = false;
  int t = first_t;
  for (int kk = 0; t < a.total; t += gridDim.x, ++kk) {
    const B2Tile cur = b2_decode(a, t);
    char* d_cur = smem + (kk & 1) * B3_DBUF;
    char* p_cur = smem + B3_OFF_P + (kk % B3_NP) * B2_PBUF;
    b3_barrier();  // tile t staged; the partner's exchange slot of tile t-1 is written
    if constexpr (ROLE < 2) {
      if (have_prev)
        b2_xchg_finish<ROLE, DIAG>(reinterpret_cast<const f32x4*>(smem + B3_OFF_X + ((kk + 1) & 1) * B2_XCHG), acc, a.dp1,
                             lane, prev.b, prev.r0, prev.c0, a.P);
      b3_dgrad<ROLE, DIAG>(d_cur, R, acc, hp, lp, li);
      b2_xchg_put<ROLE>(reinterpret_cast<f32x4*>(smem + B3_OFF_X + (kk & 1) * B2_XCHG), acc, lane);
    } else {
      b3_wgrad<ROLE - 2, DIAG>(d_cur, p_cur, R, lane, ones_hi, zero8);
    }
    prev = cur;
    have_prev = true;
  }
  // kk == number of tiles here; the last put went to slot (kk - 1) & 1
  int kk_end = 0;
  for (int tt = first_t; tt < a.total; tt += gridDim.x) ++kk_end;
  b3_barrier();
  if constexpr (ROLE < 2) {
    if (have_prev)
      b2_xchg_finish<ROLE, DIAG>(reinterpret_cast<const f32x4*>(smem + B3_OFF_X + ((kk_end - 1) & 1) * B2_XCHG), acc, a.dp1,
                           lane, prev.b, prev.r0, prev.c0, a.P);
  } else {
    float* out = a.slab + (int64_t)blockIdx.x * 26 * 512;
#pragma unroll
    for (int k = 0; k < 13; ++k) {
      const int tap = 13 * (ROLE - 2) + k;
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int r = 0; r < 4; ++r) out[(tap * 32 + 16 * h + 4 * g + r) * 16 + li] = R[k][h][r];
    }
  }
}

template <int WV, int DIAG, bool BIG>  // staging wave WV (0..3) = workgroup wave 4 + WV
__device__ __forceinline__ void b3_stage(const B2Args& a, char* smem, int first_t) {
  if constexpr (DIAG == 5) {  // timing only: no staging at all (consumers read stale LDS)
    for (int t = first_t; t < a.total; t += gridDim.x) b3_barrier();
    b3_barrier();
    return;
  }
#ifdef TDS_B3_STAGE_PRIO
  __builtin_amdgcn_s_setprio(TDS_B3_STAGE_PRIO);
#endif
  const int tid = threadIdx.x - 256;
  const float* kc = reinterpret_cast<const float*>(smem + B3_OFF_K);
  // two register sets: tile j's y2 / g2m registers are loaded two iterations before they are
  // staged (set j & 1), its p1 DMA lands in buffer j % 4
  B2Stager<DIAG, WV, true, BIG> st0, st1;
  st0.init(a, tid);
  st1.init(a, tid);
  const int G = gridDim.x;
  auto tile = [&](int j) { return first_t + j * G; };
  auto pbuf = [&](int j) { return smem + B3_OFF_P + (j % B3_NP) * B2_PBUF; };  // written in store(j)
  auto dbuf = [&](int j) { return smem + (j & 1) * B3_DBUF; };
  if (tile(0) < a.total) {
    st0.load(a, b2_decode(a, tile(0)), tid, nullptr);
    st0.store(a, b2_decode(a, tile(0)), tid, dbuf(0), kc);
    st0.store_p1(pbuf(0), tid);
  }
  // Loads are issued unconditionally (tiles past the end re-read the last tile, never staged):
  // a load under a branch makes the compiler's wait-count analysis assume it was skipped, and
  // the wait for the OLDER register set then drains the younger one too (vmcnt(0)).
  auto ltile = [&](int j) { return b2_decode(a, min(tile(j), a.total - 1)); };
  st1.load(a, ltile(1), tid, nullptr);
  st0.load(a, ltile(2), tid, nullptr);
  // iteration kk stages tile kk+1 and loads tile kk+3 (both in set (kk+1) & 1)
  for (int kk = 0; tile(kk) < a.total; kk += 2) {
    b3_barrier();  // consumers start tile kk
    if (tile(kk + 1) < a.total) {
      st1.store(a, b2_decode(a, tile(kk + 1)), tid, dbuf(kk + 1), kc);
      st1.store_p1(pbuf(kk + 1), tid);
    }
    st1.load(a, ltile(kk + 3), tid, nullptr);
    if (tile(kk + 1) >= a.total) break;
    b3_barrier();  // consumers start tile kk + 1
    if (tile(kk + 2) < a.total) {
      st0.store(a, b2_decode(a, tile(kk + 2)), tid, dbuf(kk + 2), kc);
      st0.store_p1(pbuf(kk + 2), tid);
    }
    st0.load(a, ltile(kk + 4), tid, nullptr);
  }
  b3_barrier();
}

template <int DIAG, bool BIG>
__global__ __launch_bounds__(B3_THREADS, 2) void conv2_bwd3_kernel(
    const float4* __restrict__ y2, const float* __restrict__ g2m, const float* __restrict__ aff2,
    const float* __restrict__ kbuf, const uint4* __restrict__ p1, const uint4* __restrict__ wdpack,
    float* __restrict__ dp1, float* __restrict__ slab, const int* __restrict__ order, int B, int P, int Q) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  B2Args a;
  a.y2 = y2; a.g2m = g2m; a.p1 = p1; a.dp1 = dp1; a.slab = slab; a.order = order;
  a.B = B; a.P = P; a.Q = Q;
  a.tiles_c = (P + B2_TC - 1) / B2_TC;
  a.tiles_r = (P + B2_TH - 1) / B2_TH;
  a.per_img = a.tiles_c * a.tiles_r;
  a.total = a.per_img * B;
  float* kc = reinterpret_cast<float*>(smem + B3_OFF_K);
  if (tid < 160) kc[tid] = (tid < 64) ? aff2[tid] : kbuf[tid - 64];
  __syncthreads();  // kc visible to the staging waves
  const int t0 = xcd_remap(blockIdx.x, gridDim.x);
  switch (wv) {
    case 0: b3_mfma<0, DIAG>(a, wdpack, smem, t0); break;
    case 1: b3_mfma<1, DIAG>(a, wdpack, smem, t0); break;
    case 2: b3_mfma<2, DIAG>(a, wdpack, smem, t0); break;
    case 3: b3_mfma<3, DIAG>(a, wdpack, smem, t0); break;
    case 4: b3_stage<0, DIAG, BIG>(a, smem, t0); break;
    case 5: b3_stage<1, DIAG, BIG>(a, smem, t0); break;
    case 6: b3_stage<2, DIAG, BIG>(a, smem, t0); break;
    default: b3_stage<3, DIAG, BIG>(a, smem, t0); break;
  }
}

}  // namespace tds

using namespace tds;

int tds_conv2_bwd3_num_wg() { return tds_conv2_num_wg(); }  // one 8-wave workgroup per CU

void tds_conv2_bwd3_tiles(int P, int* tiles_r, int* tiles_c) {
  *tiles_r = (P + B2_TH - 1) / B2_TH;
  *tiles_c = (P + B2_TC - 1) / B2_TC;
}

#ifdef TDS_DIAG
// timing-only variants: 1 no MFMAs, 3 no global tile loads, 5 no staging, 7 no y2 loads, 9 no
// BN2 / pool backward math in the staging, 11 no dp1 stores.  Compiled only into a -DTDS_DIAG build
// (python -m torch_distributed_sandbox_amd._build --variant diag -D TDS_DIAG; TDS_CONV2_DIAG=N).
static int b3_diag_env() {
  const char* e = std::getenv("TDS_CONV2_DIAG");
  return e ? std::atoi(e) : 0;
}
#else
static int b3_diag_env() { return 0; }
#endif

// g2m: planar [B][32][Q][Q]; order: the blocked tile order table (tds_tile_order_fill) from the caller
void tds_conv2_bwd3(const float* y2, const float* g2m, const float* aff2, const float* kbuf, const void* p1,
                    const short* wd, float* dp1, float* slab, const int* order, int nwg, int B, int P,
                    hipStream_t st) {
  const int Q = P / 2;
  const bool big = (int64_t)32 * Q * Q * 4 >= 0xFFFFFF00LL;  // g2m image beyond a 4 GiB descriptor
#define TDS_B3_LAUNCH_B(D, BG)                                                                                         \
  {                                                                                                                    \
    static bool set = false;                                                                                           \
    if (!set) {                                                                                                        \
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(conv2_bwd3_kernel<D, BG>),                               \
                                hipFuncAttributeMaxDynamicSharedMemorySize, B3_LDS);                                   \
      set = true;                                                                                                      \
    }                                                                                                                  \
    hipLaunchKernelGGL((conv2_bwd3_kernel<D, BG>), dim3(nwg), dim3(B3_THREADS), B3_LDS, st,                            \
                       reinterpret_cast<const float4*>(y2), g2m, aff2, kbuf, reinterpret_cast<const uint4*>(p1),       \
                       reinterpret_cast<const uint4*>(wd), dp1, slab, order, B, P, Q);                                  \
    TDS_LAUNCH_CHECK();                                                                                                \
  }
#define TDS_B3_LAUNCH(D)           \
  if (big) TDS_B3_LAUNCH_B(D, true) \
  else TDS_B3_LAUNCH_B(D, false)
  switch (b3_diag_env()) {
#ifdef TDS_DIAG
    case 1: TDS_B3_LAUNCH(1) break;
    case 3: TDS_B3_LAUNCH(3) break;
    case 5: TDS_B3_LAUNCH(5) break;
    case 7: TDS_B3_LAUNCH(7) break;
    case 9: TDS_B3_LAUNCH(9) break;
    case 11: TDS_B3_LAUNCH(11) break;
#endif
    default: TDS_B3_LAUNCH(0) break;
  }
#undef TDS_B3_LAUNCH
#undef TDS_B3_LAUNCH_B
}
