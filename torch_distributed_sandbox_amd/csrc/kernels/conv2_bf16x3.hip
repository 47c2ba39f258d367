// conv2 of the ConvNet (Conv2d(16, 32, 5, stride 1, pad 2), mnist_onegpu.py:20) —
// forward, data-gradient and weight-gradient on MFMA with the bf16x3 split
// (bf16x3.h), NHWC activations.  SURVEY.md §2.4 K5 / K19 / K20 (92% of the
// step's FLOPs).
//
// Activation formats (all produced/consumed by convnet_fused.hip):
//   p1  [B][P][P][32] bf16 : ch 0-15 = hi(ci), 16-31 = lo(ci)      (pooled layer-1 output)
//   y2  [B][P][P][32] fp32                                          (conv2 output, incl. bias)
//   dy2 [B][P][P][64] bf16 : ch 0-31 = hi(co), 32-63 = lo(co)       (grad wrt conv2 output)
//   dp1 [B][P][P][16] fp32                                          (grad wrt p1)
// In LDS every operand lives in "planes" of 16 channels x 2 B = 32-byte
// records (one record per pixel).  16 consecutive pixels read with
// ds_read_b128 then hit 16 distinct 16-B bank slots for ANY tap shift, so the
// implicit-GEMM A operand needs no swizzle (see the bank derivation in
// docs/KERNELS.md).  Weights are pre-packed on device in MFMA-fragment order so
// the 64 lanes of a B-fragment read are one contiguous, conflict-free 1 KiB.
//
// MFMA mapping (v_mfma_f32_16x16x32_bf16, lane l: i = l&15, g = l>>4):
//   A[i][k = 8g+j] (8 consecutive k per lane), B[k = 8g+j][n = i], C row = 4g+r, col = i.
//   fwd  : M = 16 pixels of a row, N = 16 output channels, K = (tap, ci): 32 = 2 taps x 16 ci
//   dgrad: M = 16 pixels,          N = 16 input channels,  K = (tap', co): 32 = 1 tap x 32 co
//   wgrad: M = 16 out channels,    N = 16 input channels,  K = 32 pixels (operands via
//          ds_read_b64_tr_b16 transposed reads of the same NHWC records), one
//          accumulator tile per (tap, co-half), taps split across the 8 waves.
//
// All three are persistent (one 512-thread workgroup per CU) and walk the
// tiles in XCD-grouped order; the next tile's global loads are issued into
// registers before the current tile's MFMAs and written to LDS after them.
#include <cstdlib>

#include "conv2_common.h"
#include "launchers.h"

namespace tds {

constexpr int C2_TH = 8;   // tile rows   (one per wave)
constexpr int C2_TC = 32;  // tile cols   (two 16-pixel M tiles per wave)
constexpr int C2_IR = C2_TH + 4;
constexpr int C2_IC = C2_TC + 4;
constexpr int C2_THREADS = 512;

// ---------------------------------------------------------------------------- weight packing
// fwd : wp[hl][s<13][nt<2][g<4][co16][j8], k = 32s+8g+j, ci = 8(g&1)+j, taps paired so that one
//       input-row A fragment serves every output row:  s < 10: (ky = s>>1, kx = 2(s&1) + (g>>1));
//       s = 10 + kp: (ky = 2kp + (g>>1), kx = 4)  (ky = 5 -> zero)
// dgrad: wd[hl][s<25][g<4][ci16][j8],      k = 32s+8g+j -> tap' = s, co = 8g+j; w = w2[co][ci][24-tap']
__global__ void conv2_pack_weights_kernel(const float* __restrict__ w2, short* __restrict__ wp,
                                          short* __restrict__ wd) {
  const int FW = 13 * 2 * 4 * 16 * 8;  // per hl plane (fwd)
  const int DW = 25 * 4 * 16 * 8;      // per hl plane (dgrad)
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < FW + DW; e += gridDim.x * blockDim.x) {
    if (e < FW) {
      const int j = e & 7, co_in = (e >> 3) & 15, g = (e >> 7) & 3, nt = (e >> 9) & 1, s = e >> 10;
      const int ky = s < 10 ? (s >> 1) : 2 * (s - 10) + (g >> 1);
      const int kx = s < 10 ? 2 * (s & 1) + (g >> 1) : 4;
      const int ci = 8 * (g & 1) + j, co = nt * 16 + co_in;
      const float v = ky < 5 ? w2[(co * 16 + ci) * 25 + ky * 5 + kx] : 0.f;
      unsigned short hi, lo;
      split_bf16(v, hi, lo);
      wp[e] = (short)hi;
      wp[FW + e] = (short)lo;
    } else {
      const int f = e - FW;
      const int j = f & 7, ci = (f >> 3) & 15, g = (f >> 7) & 3, s = f >> 9;
      const int co = 8 * g + j;
      const float v = w2[(co * 16 + ci) * 25 + (24 - s)];
      unsigned short hi, lo;
      split_bf16(v, hi, lo);
      wd[f] = (short)hi;
      wd[DW + f] = (short)lo;
    }
  }
}

struct TileIter {
  int tiles_c, tiles_r, per_img, total;
  __device__ TileIter(int B, int P) {
    tiles_c = (P + C2_TC - 1) / C2_TC;
    tiles_r = (P + C2_TH - 1) / C2_TH;
    per_img = tiles_c * tiles_r;
    total = per_img * B;
  }
  __device__ void decode(int t, int& b, int& r0, int& c0) const {
    b = t / per_img;
    const int rem = t - b * per_img;
    r0 = (rem / tiles_c) * C2_TH;
    c0 = (rem % tiles_c) * C2_TC;
  }
};

// ---------------------------------------------------------------------------- forward
// Tile: 8 output rows x 64 output cols.  Wave w owns output rows 4*(w>>2) .. +3 and columns
// 16*(w&3) .. +15 (four M tiles stacked vertically), N = 32 output channels (two N tiles).
// K steps pair taps so that an input row's A fragment serves every output row it reaches:
//   (ky, kx in {2a, 2a+1}) for a = 0, 1  -> A = input row R, output row o = R - ky
//   (ky in {2kp, 2kp+1}, kx = 4)         -> A = input rows R (lane groups 0-1) and R+1 (2-3),
//                                           output row o = R - 2kp
// Per wave-tile: 100 ds_read_b128 for 104 MFMA triples (the row-per-wave layout needed 208).
// LDS: weights (2 x 13 x 2 x 1 KiB) + p1 planes (2 x 12 x 68 x 32 B).
constexpr int FW_TH = 8, FW_TC = 64;
constexpr int FW_IR = FW_TH + 4, FW_IC = FW_TC + 4;
constexpr int F_WBYTES = 2 * 13 * 2 * 1024;
// plane stride padded by 64 B: the hi/lo planes of one staged record land 4 bank-quads
// apart, so the 8-lane groups of the ds_write_b128 staging stores are conflict-free
constexpr int F_PLANE = FW_IR * FW_IC * 32 + 64;                         // 26176 B
constexpr int F_ONE = 2 * F_PLANE;                                       // one staged tile
constexpr int F_LDS = F_WBYTES + 2 * F_ONE;                              // 157696 B, double-buffered
constexpr int F_CHUNKS = FW_IR * FW_IC * 4;                               // 16-byte chunks per staged tile
constexpr int F_PER_THREAD = (F_CHUNKS + C2_THREADS - 1) / C2_THREADS;   // 7

template <int DIAG>
__global__ __launch_bounds__(C2_THREADS) void conv2_fwd_bf16x3_kernel(const uint4* __restrict__ p1,
                                                                      const uint4* __restrict__ wpack,
                                                                      const float* __restrict__ bias,
                                                                      float* __restrict__ y2,
                                                                      double* __restrict__ partial, int B, int P) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* w_l = smem;
  char* in_l = smem + F_WBYTES;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int li = lane & 15, g = lane >> 4;
  const int rg = wv >> 2, cg = wv & 3;
  const int tiles_c = (P + FW_TC - 1) / FW_TC, tiles_r = (P + FW_TH - 1) / FW_TH;
  const int per_img = tiles_c * tiles_r, total = per_img * B;
  const int vid = xcd_remap(blockIdx.x, gridDim.x);

  // weights -> LDS once (persistent workgroup)
  for (int e = tid; e < F_WBYTES / 16; e += C2_THREADS) reinterpret_cast<uint4*>(w_l)[e] = wpack[e];

  float bco[2];
  bco[0] = bias[li];
  bco[1] = bias[16 + li];
  float s_acc[2] = {0.f, 0.f}, q_acc[2] = {0.f, 0.f};

  auto decode = [&](int t, int& b, int& r0, int& c0) {
    b = t / per_img;
    const int rem = t - b * per_img;
    r0 = (rem / tiles_c) * FW_TH;
    c0 = (rem % tiles_c) * FW_TC;
  };
  uint4 pre[F_PER_THREAD];
  auto load_tile = [&](int t) {
    int b, r0, c0;
    decode(t, b, r0, c0);
#pragma unroll
    for (int u = 0; u < F_PER_THREAD; ++u) {
      const int e = tid + u * C2_THREADS;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (DIAG != 3 && e < F_CHUNKS) {
        const int px = e >> 2, q = e & 3;
        const int rr = px / FW_IC, cc = px - rr * FW_IC;
        const int gr = r0 - 2 + rr, gc = c0 - 2 + cc;
        if (gr >= 0 && gr < P && gc >= 0 && gc < P)
          v = p1[(((int64_t)b * P + gr) * P + gc) * 4 + q];
      }
      pre[u] = v;
    }
  };
  auto store_tile = [&](int buf) {
#pragma unroll
    for (int u = 0; u < F_PER_THREAD; ++u) {
      const int e = tid + u * C2_THREADS;
      if (e < F_CHUNKS) {
        const int px = e >> 2, q = e & 3;
        *reinterpret_cast<uint4*>(in_l + buf * F_ONE + (q >> 1) * F_PLANE + px * 32 + (q & 1) * 16) = pre[u];
      }
    }
  };
  auto ldb = [&](int s, int n, int hl) -> s16x8 {
    return lds8<DIAG>(w_l + hl * 13 * 2 * 1024 + ((s * 2 + n) * 64 + lane) * 16);
  };

  const int boff = (g & 1) * 16;  // ci half of the 32-B record
  // Double-buffered staging: tile t is read from buffer t&1; tile t+1 (already in registers)
  // is written into the other buffer at the start of tile t, so its ds_writes drain under
  // this tile's MFMAs; one barrier per tile.
  int t = vid;
  if (t < total) {
    load_tile(t);
    store_tile(0);
    if (t + (int)gridDim.x < total) load_tile(t + gridDim.x);
  }
  __syncthreads();
  for (int kk = 0; t < total; t += gridDim.x, ++kk) {
    const int cb = kk & 1;
    const char* in_c = in_l + cb * F_ONE;
    int b, r0, c0;
    decode(t, b, r0, c0);
    if (t + (int)gridDim.x < total) {
      store_tile(cb ^ 1);
      if (t + 2 * (int)gridDim.x < total) load_tile(t + 2 * (int)gridDim.x);
    }

    f32x4 acc[4][2];
#pragma unroll
    for (int o = 0; o < 4; ++o) acc[o][0] = acc[o][1] = f32x4{0.f, 0.f, 0.f, 0.f};
    s16x8 ah[2], al[2];
    // ---- kx pairs (0,1) and (2,3): A = input row R at column offset 2a + (g>>1)
#pragma unroll
    for (int a = 0; a < 2; ++a) {
      s16x8 bh[5][2], bl[5][2];
#pragma unroll
      for (int ky = 0; ky < 5; ++ky)
#pragma unroll
        for (int n = 0; n < 2; ++n) {
          bh[ky][n] = ldb(2 * ky + a, n, 0);
          bl[ky][n] = ldb(2 * ky + a, n, 1);
        }
      auto load_a = [&](int R, int buf) {
        const int rec = (4 * rg + R) * FW_IC + 16 * cg + li + 2 * a + (g >> 1);
        ah[buf] = lds8<DIAG>(in_c + rec * 32 + boff);
        al[buf] = lds8<DIAG>(in_c + F_PLANE + rec * 32 + boff);
      };
      load_a(0, 0);
#pragma unroll
      for (int R = 0; R < 8; ++R) {
        const int cur = R & 1;
        if (R + 1 < 8) load_a(R + 1, cur ^ 1);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int ky = 0; ky < 5; ++ky) {
          const int o = R - ky;
          if (o >= 0 && o < 4) {
#pragma unroll
            for (int n = 0; n < 2; ++n)
              acc[o][n] = mma3<DIAG>(ah[cur], al[cur], bh[ky][n], bl[ky][n], acc[o][n]);
          }
        }
      }
    }
    // ---- column kx = 4, ky pairs (2kp, 2kp+1): lane groups 2-3 read input row R+1
    {
      s16x8 bh[3][2], bl[3][2];
#pragma unroll
      for (int kp = 0; kp < 3; ++kp)
#pragma unroll
        for (int n = 0; n < 2; ++n) {
          bh[kp][n] = ldb(10 + kp, n, 0);
          bl[kp][n] = ldb(10 + kp, n, 1);
        }
      auto load_a = [&](int R, int buf) {
        int row = 4 * rg + R + (g >> 1);
        if (row > FW_IR - 1) row = FW_IR - 1;  // only reached with a zero weight (ky = 5): any staged row
        const int rec = row * FW_IC + 16 * cg + li + 4;
        ah[buf] = lds8<DIAG>(in_c + rec * 32 + boff);
        al[buf] = lds8<DIAG>(in_c + F_PLANE + rec * 32 + boff);
      };
      load_a(0, 0);
#pragma unroll
      for (int R = 0; R < 8; ++R) {
        const int cur = R & 1;
        if (R + 1 < 8) load_a(R + 1, cur ^ 1);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int kp = 0; kp < 3; ++kp) {
          const int o = R - 2 * kp;
          if (o >= 0 && o < 4) {
#pragma unroll
            for (int n = 0; n < 2; ++n)
              acc[o][n] = mma3<DIAG>(ah[cur], al[cur], bh[kp][n], bl[kp][n], acc[o][n]);
          }
        }
      }
    }
    // epilogue: lane holds co = 16n + li for pixels col = c0 + 16cg + 4g + r of row 4rg + o
#pragma unroll
    for (int o = 0; o < 4; ++o) {
      const int row = r0 + 4 * rg + o;
      if (row < P) {
        float* yrow = y2 + ((int64_t)b * P + row) * P * 32;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int col = c0 + 16 * cg + 4 * g + r;
          if (col < P) {
#pragma unroll
            for (int n = 0; n < 2; ++n) {
              const float v = acc[o][n][r];  // y2 - b2: statistics shifted by the bias
              yrow[(int64_t)col * 32 + 16 * n + li] = v + bco[n];
              s_acc[n] += v;
              q_acc[n] += v * v;
            }
          }
        }
      }
    }
    __syncthreads();  // this buffer's readers are done; the other buffer is complete
  }
  // BN2 batch-stat partials: reduce the 4 lane groups, then the 8 waves
#pragma unroll
  for (int n = 0; n < 2; ++n) {
    s_acc[n] += __shfl_xor(s_acc[n], 16, 64);
    s_acc[n] += __shfl_xor(s_acc[n], 32, 64);
    q_acc[n] += __shfl_xor(q_acc[n], 16, 64);
    q_acc[n] += __shfl_xor(q_acc[n], 32, 64);
  }
  __syncthreads();
  double* red = reinterpret_cast<double*>(smem);  // [8 waves][32 co][2]
  if (g == 0) {
#pragma unroll
    for (int n = 0; n < 2; ++n) {
      red[(wv * 32 + 16 * n + li) * 2 + 0] = (double)s_acc[n];
      red[(wv * 32 + 16 * n + li) * 2 + 1] = (double)q_acc[n];
    }
  }
  __syncthreads();
  if (tid < 64) {
    const int co = tid >> 1, k = tid & 1;
    double a = 0.0;
    for (int w = 0; w < 8; ++w) a += red[(w * 32 + co) * 2 + k];
    partial[((int64_t)co * gridDim.x + blockIdx.x) * 2 + k] = a;
  }
}

// ---------------------------------------------------------------------------- data gradient
// Tile: 8 output rows x 64 output cols.  Wave w owns output rows 4*(w>>2) .. +3 and
// columns 16*(w&3) .. +15: four 16-pixel M tiles stacked vertically, N = 16 input channels,
// K = (flipped tap, 32 output channels).  An input row R of the wave's 8-row window serves
// every output row it reaches (o = R - ky), so per kx the 5 weight fragments (ky = 0..4)
// stay in registers and each input row's A fragment is read from LDS once:
// 26 ds_read_b128 per 20 MFMA triples (the row-per-wave layout needed 60).
constexpr int DG_TH = 8, DG_TC = 64;
constexpr int DG_IR = DG_TH + 4, DG_IC = DG_TC + 4;
constexpr int D_WBYTES = 2 * 25 * 1024;
// plane stride padded by 32 B: the 4 planes of a staged record land on bank-quads 0,2,4,6
// (+ half 0/1), so the 8-lane groups of the ds_write_b128 staging stores are conflict-free
constexpr int D_PLANE = DG_IR * DG_IC * 32 + 32;                       // 26144 B
constexpr int D_LDS = D_WBYTES + 4 * D_PLANE;                          // 155776 B (< 160 KiB)
constexpr int D_CHUNKS = DG_IR * DG_IC * 8;                             // 16-B chunks per staged tile
constexpr int D_PER_THREAD = (D_CHUNKS + C2_THREADS - 1) / C2_THREADS;  // 13

template <int DIAG>
__global__ __launch_bounds__(C2_THREADS) void conv2_dgrad_bf16x3_kernel(const uint4* __restrict__ dy2,
                                                                        const uint4* __restrict__ wdpack,
                                                                        float* __restrict__ dp1, int B, int P) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* w_l = smem;
  char* in_l = smem + D_WBYTES;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int li = lane & 15, g = lane >> 4;
  const int rg = wv >> 2, cg = wv & 3;
  const int tiles_c = (P + DG_TC - 1) / DG_TC, tiles_r = (P + DG_TH - 1) / DG_TH;
  const int per_img = tiles_c * tiles_r, total = per_img * B;
  const int vid = xcd_remap(blockIdx.x, gridDim.x);
  for (int e = tid; e < D_WBYTES / 16; e += C2_THREADS) reinterpret_cast<uint4*>(w_l)[e] = wdpack[e];

  auto decode = [&](int t, int& b, int& r0, int& c0) {
    b = t / per_img;
    const int rem = t - b * per_img;
    r0 = (rem / tiles_c) * DG_TH;
    c0 = (rem % tiles_c) * DG_TC;
  };
  uint4 pre[D_PER_THREAD];
  auto load_tile = [&](int t) {
    int b, r0, c0;
    decode(t, b, r0, c0);
#pragma unroll
    for (int u = 0; u < D_PER_THREAD; ++u) {
      const int e = tid + u * C2_THREADS;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (DIAG != 3 && e < D_CHUNKS) {
        const int px = e >> 3, q = e & 7;
        const int rr = px / DG_IC, cc = px - rr * DG_IC;
        const int gr = r0 - 2 + rr, gc = c0 - 2 + cc;
        if (gr >= 0 && gr < P && gc >= 0 && gc < P)
          v = dy2[(((int64_t)b * P + gr) * P + gc) * 8 + q];
      }
      pre[u] = v;
    }
  };
  auto store_tile = [&]() {
#pragma unroll
    for (int u = 0; u < D_PER_THREAD; ++u) {
      const int e = tid + u * C2_THREADS;
      if (e < D_CHUNKS) {
        const int px = e >> 3, q = e & 7;
        const int plane = (q >> 2) * 2 + ((q >> 1) & 1);
        *reinterpret_cast<uint4*>(in_l + plane * D_PLANE + px * 32 + (q & 1) * 16) = pre[u];
      }
    }
  };

  // lane group g -> output channels 8g..8g+7: plane g>>1 (+16 B if g odd), hi planes 0-1, lo 2-3
  const int hp = (g >> 1) * D_PLANE + (g & 1) * 16;
  const int lp = (2 + (g >> 1)) * D_PLANE + (g & 1) * 16;
  int t = vid;
  if (t < total) load_tile(t);
  for (; t < total; t += gridDim.x) {
    __syncthreads();
    store_tile();
    __syncthreads();
    int b, r0, c0;
    decode(t, b, r0, c0);
    if (t + (int)gridDim.x < total) load_tile(t + gridDim.x);

    f32x4 acc[4];
#pragma unroll
    for (int o = 0; o < 4; ++o) acc[o] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kx = 0; kx < 5; ++kx) {
      s16x8 bh[5], bl[5];
#pragma unroll
      for (int ky = 0; ky < 5; ++ky) {
        const int s = ky * 5 + kx;
        bh[ky] = lds8<DIAG>(w_l + (s * 64 + lane) * 16);
        bl[ky] = lds8<DIAG>(w_l + 25 * 1024 + (s * 64 + lane) * 16);
      }
      s16x8 ah[2], al[2];
      auto load_a = [&](int R, int buf) {
        const int rec = (4 * rg + R) * DG_IC + 16 * cg + kx + li;
        ah[buf] = lds8<DIAG>(in_l + hp + rec * 32);
        al[buf] = lds8<DIAG>(in_l + lp + rec * 32);
      };
      load_a(0, 0);
#pragma unroll
      for (int R = 0; R < 8; ++R) {
        const int cur = R & 1;
        if (R + 1 < 8) load_a(R + 1, cur ^ 1);
        __builtin_amdgcn_sched_barrier(0);  // next input row's reads ahead of this row's MFMAs
#pragma unroll
        for (int ky = 0; ky < 5; ++ky) {
          const int o = R - ky;
          if (o >= 0 && o < 4) acc[o] = mma3<DIAG>(ah[cur], al[cur], bh[ky], bl[ky], acc[o]);
        }
      }
    }
    // lane holds C[px = 4g + r][ci = li] of output row 4rg + o
#pragma unroll
    for (int o = 0; o < 4; ++o) {
      const int row = r0 + 4 * rg + o;
      if (row < P) {
        float* orow = dp1 + ((int64_t)b * P + row) * P * 16;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int col = c0 + 16 * cg + 4 * g + r;
          if (col < P) orow[(int64_t)col * 16 + li] = acc[o][r];
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------- weight gradient
// Per tile (8 rows x 32 cols of output pixels): dy2 planes 4 x (8 x 32) records,
// p1 planes 2 x (12 x 36) records (halo).  Record r is stored at r ^ (bit3(r) << 2)
// so the two 16-lane groups of a transposed read (rows r..r+3 and r+8..r+11)
// land on disjoint banks.  Wave w owns "taps" {w, w+8, w+16, w+24} (tap 25 =
// ones column -> bias gradient) x 2 co halves.
constexpr int W_DPLANE = C2_TH * C2_TC * 32 + 32;  // 8224 B (+32: conflict-free staging stores)
constexpr int W_PPLANE = C2_IR * C2_IC * 32 + 64;  // 13888 B (+64: conflict-free staging stores)
constexpr int W_ONE = 4 * W_DPLANE + 2 * W_PPLANE;  // one staged tile (60416 B)
constexpr int W_LDS = 2 * W_ONE;                     // double-buffered (120832 B)
constexpr int W_DCHUNKS = C2_TH * C2_TC * 8;
constexpr int W_PCHUNKS = C2_IR * C2_IC * 4;
constexpr int W_DPER = (W_DCHUNKS + C2_THREADS - 1) / C2_THREADS;
constexpr int W_PPER = (W_PCHUNKS + C2_THREADS - 1) / C2_THREADS;

__device__ __forceinline__ int wswz(int r) { return r ^ (((r >> 3) & 1) << 2); }

template <int DIAG>
__global__ __launch_bounds__(C2_THREADS) void conv2_wgrad_bf16x3_kernel(const uint4* __restrict__ dy2,
                                                                        const uint4* __restrict__ p1,
                                                                        float* __restrict__ slab, int B, int P) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  // buffer k: dy2 planes (hi co0-15, hi co16-31, lo co0-15, lo co16-31) then p1 planes (hi, lo).
  // Tile t is read from buffer t&1 while tile t+1 is written into the other one, so the LDS
  // stores overlap MFMAs and there is one barrier per tile.
  char* d_l = smem;
  char* p_l = smem + 4 * W_DPLANE;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int g = lane >> 4;
  const int q4 = (lane >> 2) & 3, p4 = lane & 3;  // tr-read row / column-chunk of this lane
  const TileIter it(B, P);
  const int vid = xcd_remap(blockIdx.x, gridDim.x);

  f32x4 acc[4][2];
#pragma unroll
  for (int k = 0; k < 4; ++k) acc[k][0] = acc[k][1] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int ntap = (wv + 24 <= 25) ? 4 : 3;

  uint4 dpre[W_DPER], ppre[W_PPER];
  auto load_tile = [&](int t) {
    int b, r0, c0;
    it.decode(t, b, r0, c0);
#pragma unroll
    for (int u = 0; u < W_DPER; ++u) {
      const int e = tid + u * C2_THREADS;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (DIAG != 3 && e < W_DCHUNKS) {
        const int px = e >> 3, q = e & 7;
        const int rr = px / C2_TC, cc = px - rr * C2_TC;
        const int gr = r0 + rr, gc = c0 + cc;
        if (gr < P && gc < P) v = dy2[(((int64_t)b * P + gr) * P + gc) * 8 + q];
      }
      dpre[u] = v;
    }
#pragma unroll
    for (int u = 0; u < W_PPER; ++u) {
      const int e = tid + u * C2_THREADS;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (DIAG != 3 && e < W_PCHUNKS) {
        const int px = e >> 2, q = e & 3;
        const int rr = px / C2_IC, cc = px - rr * C2_IC;
        const int gr = r0 - 2 + rr, gc = c0 - 2 + cc;
        if (gr >= 0 && gr < P && gc >= 0 && gc < P) v = p1[(((int64_t)b * P + gr) * P + gc) * 4 + q];
      }
      ppre[u] = v;
    }
  };
  auto store_tile = [&](int buf) {
    char* dd = d_l + buf * W_ONE;
    char* pp = p_l + buf * W_ONE;
#pragma unroll
    for (int u = 0; u < W_DPER; ++u) {
      const int e = tid + u * C2_THREADS;
      if (e < W_DCHUNKS) {
        const int px = e >> 3, q = e & 7;
        const int plane = (q >> 2) * 2 + ((q >> 1) & 1);
        *reinterpret_cast<uint4*>(dd + plane * W_DPLANE + wswz(px) * 32 + (q & 1) * 16) = dpre[u];
      }
    }
#pragma unroll
    for (int u = 0; u < W_PPER; ++u) {
      const int e = tid + u * C2_THREADS;
      if (e < W_PCHUNKS) {
        const int px = e >> 2, q = e & 3;
        *reinterpret_cast<uint4*>(pp + (q >> 1) * W_PPLANE + wswz(px) * 32 + (q & 1) * 16) = ppre[u];
      }
    }
  };

  // ones fragment for the bias column: B[k][n] = 1 for n == 0 (hi = 1.0 bf16 = 0x3f80)
  s16x8 ones_hi, zero8;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    ones_hi[j] = (short)((lane & 15) == 0 ? 0x3f80 : 0);
    zero8[j] = 0;
  }

  int t = vid;
  if (t < it.total) {
    load_tile(t);
    store_tile(0);
    if (t + (int)gridDim.x < it.total) load_tile(t + gridDim.x);
  }
  __syncthreads();
  for (int k = 0; t < it.total; t += gridDim.x, ++k) {
    const int cb = k & 1;
    const char* d_c = d_l + cb * W_ONE;
    const char* p_c = p_l + cb * W_ONE;
    if (t + (int)gridDim.x < it.total) {
      // the next tile (already in registers) -> the other buffer; its ds_writes drain while
      // this tile's MFMAs run (no barrier in between), then prefetch the tile after it
      store_tile(cb ^ 1);
      if (t + 2 * (int)gridDim.x < it.total) load_tile(t + 2 * (int)gridDim.x);
    }

    // transposed operand reads of row+1 are issued while row's MFMAs run
    s16x8 ahi[2][2], alo[2][2], bhi[2][4], blo[2][4];  // [buffer][co half | tap slot]
    auto load_row = [&](int row, int buf) {
      // A = dy2[px = 8g+j of this row][co]: two transposed reads (4 px each) per plane
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int r_a = row * C2_TC + 8 * g + q4;
        const s16x4 x0 = ldtr<DIAG>(d_c + h * W_DPLANE + wswz(r_a) * 32 + p4 * 8);
        const s16x4 x1 = ldtr<DIAG>(d_c + h * W_DPLANE + wswz(r_a + 4) * 32 + p4 * 8);
        const s16x4 y0 = ldtr<DIAG>(d_c + (2 + h) * W_DPLANE + wswz(r_a) * 32 + p4 * 8);
        const s16x4 y1 = ldtr<DIAG>(d_c + (2 + h) * W_DPLANE + wswz(r_a + 4) * 32 + p4 * 8);
        ahi[buf][h] = s16x8{x0[0], x0[1], x0[2], x0[3], x1[0], x1[1], x1[2], x1[3]};
        alo[buf][h] = s16x8{y0[0], y0[1], y0[2], y0[3], y1[0], y1[1], y1[2], y1[3]};
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int tap = wv + 8 * k;
        if (k < ntap && tap < 25) {
          const int ky = tap / 5, kx = tap - 5 * (tap / 5);
          const int r_b = (row + ky) * C2_IC + kx + 8 * g + q4;
          const s16x4 x0 = ldtr<DIAG>(p_c + wswz(r_b) * 32 + p4 * 8);
          const s16x4 x1 = ldtr<DIAG>(p_c + wswz(r_b + 4) * 32 + p4 * 8);
          const s16x4 y0 = ldtr<DIAG>(p_c + W_PPLANE + wswz(r_b) * 32 + p4 * 8);
          const s16x4 y1 = ldtr<DIAG>(p_c + W_PPLANE + wswz(r_b + 4) * 32 + p4 * 8);
          bhi[buf][k] = s16x8{x0[0], x0[1], x0[2], x0[3], x1[0], x1[1], x1[2], x1[3]};
          blo[buf][k] = s16x8{y0[0], y0[1], y0[2], y0[3], y1[0], y1[1], y1[2], y1[3]};
        } else {
          bhi[buf][k] = ones_hi;  // tap 25: ones column -> bias gradient
          blo[buf][k] = zero8;
        }
      }
    };
    auto mma_row = [&](int cur) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        if (k < ntap) {
#pragma unroll
          for (int h = 0; h < 2; ++h)
            acc[k][h] = mma3<DIAG>(ahi[cur][h], alo[cur][h], bhi[cur][k], blo[cur][k], acc[k][h]);
        }
      }
    };
    load_row(0, 0);
#pragma unroll 1
    for (int row = 0; row < C2_TH; row += 2) {
      load_row(row + 1, 1);
      __builtin_amdgcn_sched_barrier(0);  // keep the prefetch ahead of this row's MFMAs
      mma_row(0);
      if (row + 2 < C2_TH) load_row(row + 2, 0);
      __builtin_amdgcn_sched_barrier(0);
      mma_row(1);
    }
    __syncthreads();  // this buffer's readers are done; the other buffer is complete
  }
  // slab[wg][tap(26)][co(32)][ci(16)]: lane holds C[row = co 4g+r][col = ci li] for co half h
  float* out = slab + (int64_t)blockIdx.x * 26 * 512;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    if (k < ntap) {
      const int tap = wv + 8 * k;
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int r = 0; r < 4; ++r) out[(tap * 32 + 16 * h + 4 * g + r) * 16 + (lane & 15)] = acc[k][h][r];
    }
  }
}

// ---------------------------------------------------------------------------- fused backward
// conv2 backward fused with the BN2 / ReLU / max-pool backward that produces its input.
// Per 8 x 32 tile the workgroup builds
//     dy2 = k1*dz + k2*y2 + k3      (dz = pooled gradient g2m at the 2x2 argmax, 0 elsewhere)
// in LDS (bf16 hi|lo planes, 12 x 36 records incl. the 2-pixel halo) straight from y2 and
// g2m, stages p1 (12 x 36), then
//   waves 0-3: data gradient  (4 output rows x 16 columns each, input-row sharing as in
//              conv2_dgrad_bf16x3_kernel), dp1 written per tile;
//   waves 4-7: weight gradient (taps w-4, w, w+4, ... incl. the bias "ones" tap 25, both
//              co halves), accumulated across the persistent workgroup's tiles.
// One dgrad and one wgrad wave share each SIMD.  dy2 never exists in HBM: this replaces
// dy2_build + dgrad + wgrad (3 passes over 1.44 GB) with one pass over y2.
// Transposed reads use the K order k = 8g+j <-> px = (j < 4 ? 4g+j : 16+4g+j-4), so the
// two 16-lane groups of a 32-lane bank group read 8 consecutive records: conflict-free
// for any (unaligned) row start, no swizzle.
constexpr int BW_TH = 8, BW_TC = 32;
constexpr int BW_IR = BW_TH + 4, BW_IC = BW_TC + 4;
constexpr int BW_REC = BW_IR * BW_IC;                                   // 432 records
constexpr int BW_DPLANE = BW_REC * 32 + 32;                             // dy2: hi co0-15, hi co16-31, lo 0-15, lo 16-31
constexpr int BW_PPLANE = BW_REC * 32 + 64;                             // p1: hi, lo
constexpr int BW_WBYTES = 2 * 25 * 1024;                                // dgrad weight fragments
constexpr int BW_LDS = BW_WBYTES + 4 * BW_DPLANE + 2 * BW_PPLANE;       // 134784 B
constexpr int BW_NWIN = (BW_IR / 2) * (BW_IC / 2);                      // 108 windows per tile
constexpr int BW_ITEMS = BW_NWIN * 8;                                   // (window, 4-channel chunk)
constexpr int BW_IPER = (BW_ITEMS + C2_THREADS - 1) / C2_THREADS;       // 2
constexpr int BW_PCHUNKS = BW_REC * 4;
constexpr int BW_PPER = (BW_PCHUNKS + C2_THREADS - 1) / C2_THREADS;     // 4

template <int DIAG>
__global__ __launch_bounds__(C2_THREADS) void conv2_bwd_fused_kernel(
    const float4* __restrict__ y2, const float* __restrict__ g2m, const float* __restrict__ aff2,
    const float* __restrict__ kbuf, const uint4* __restrict__ p1, const uint4* __restrict__ wdpack,
    float* __restrict__ dp1, float* __restrict__ slab, int B, int P, int Q) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* w_l = smem;
  char* d_l = smem + BW_WBYTES;
  char* p_l = d_l + 4 * BW_DPLANE;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int li = lane & 15, g = lane >> 4;
  const int tiles_c = (P + BW_TC - 1) / BW_TC, tiles_r = (P + BW_TH - 1) / BW_TH;
  const int per_img = tiles_c * tiles_r, total = per_img * B;
  const int vid = xcd_remap(blockIdx.x, gridDim.x);
  for (int e = tid; e < BW_WBYTES / 16; e += C2_THREADS) reinterpret_cast<uint4*>(w_l)[e] = wdpack[e];

  // this thread's staging items all use channel chunk c4 = tid & 7 (items tid, tid + 512);
  // the BN2 affine and backward constants live in LDS (registers go to the MFMA operands)
  const int c4 = tid & 7;
  __shared__ float kc[5][32];  // a | b | k1 | k2 | k3
  if (tid < 160) kc[tid >> 5][tid & 31] = (tid < 64) ? aff2[tid] : kbuf[tid - 64];
  auto decode = [&](int t, int& b, int& r0, int& c0) {
    b = t / per_img;
    const int rem = t - b * per_img;
    r0 = (rem / tiles_c) * BW_TH;
    c0 = (rem % tiles_c) * BW_TC;
  };
  float4 yv[BW_IPER][4], gv[BW_IPER];
  uint4 ppre[BW_PPER];
  auto load_tile = [&](int t) {
    int b, r0, c0;
    decode(t, b, r0, c0);
#pragma unroll
    for (int u = 0; u < BW_IPER; ++u) {
      const int it = tid + u * C2_THREADS;
      const int w = it >> 3, wy = w / (BW_IC / 2), wx = w - wy * (BW_IC / 2);
      const int gy = r0 - 2 + 2 * wy, gx = c0 - 2 + 2 * wx;  // window origin (even)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int r = gy + (q >> 1), c = gx + (q & 1);
        yv[u][q] = (DIAG != 3 && it < BW_ITEMS && r >= 0 && r < P && c >= 0 && c < P)
                       ? y2[(((int64_t)b * P + r) * P + c) * 8 + c4]
                       : make_float4(0.f, 0.f, 0.f, 0.f);
      }
      const int py = gy >> 1, px = gx >> 1;  // pooled coordinates (arithmetic shift: -1 for gy = -2)
      gv[u] = (DIAG != 3 && it < BW_ITEMS && gy >= 0 && gx >= 0 && py < Q && px < Q)
                  ? g2m_planar4(g2m, b, c4, py, px, Q)
                  : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int u = 0; u < BW_PPER; ++u) {
      const int e = tid + u * C2_THREADS;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (DIAG != 3 && e < BW_PCHUNKS) {
        const int px = e >> 2, q = e & 3;
        const int rr = px / BW_IC, cc = px - rr * BW_IC;
        const int gr = r0 - 2 + rr, gc = c0 - 2 + cc;
        if (gr >= 0 && gr < P && gc >= 0 && gc < P) v = p1[(((int64_t)b * P + gr) * P + gc) * 4 + q];
      }
      ppre[u] = v;
    }
  };
  // BN2 / ReLU / pool backward of the staged windows -> dy2 hi|lo planes; p1 -> planes
  auto store_tile = [&](int t) {
    int b, r0, c0;
    decode(t, b, r0, c0);
#pragma unroll
    for (int u = 0; u < BW_IPER; ++u) {
      const int it = tid + u * C2_THREADS;
      if (it >= BW_ITEMS) continue;
      const int w = it >> 3, wy = w / (BW_IC / 2), wx = w - wy * (BW_IC / 2);
      const int gy = r0 - 2 + 2 * wy, gx = c0 - 2 + 2 * wx;
      const bool pooled = gy >= 0 && gx >= 0 && (gy >> 1) < Q && (gx >> 1) < Q;
      float y[4][4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        y[q][0] = yv[u][q].x; y[q][1] = yv[u][q].y; y[q][2] = yv[u][q].z; y[q][3] = yv[u][q].w;
      }
      const float gg[4] = {gv[u].x, gv[u].y, gv[u].z, gv[u].w};
      const float4 ka4 = *reinterpret_cast<const float4*>(&kc[0][4 * c4]);
      const float4 kb4 = *reinterpret_cast<const float4*>(&kc[1][4 * c4]);
      const float ka[4] = {ka4.x, ka4.y, ka4.z, ka4.w}, kb[4] = {kb4.x, kb4.y, kb4.z, kb4.w};
      int am[4];
#pragma unroll
      for (int cc = 0; cc < 4; ++cc) {
        float m = ka[cc] * y[0][cc] + kb[cc];
        int ai = 0;
#pragma unroll
        for (int q = 1; q < 4; ++q) {
          const float z = ka[cc] * y[q][cc] + kb[cc];
          if (z > m || isnan(z)) { m = z; ai = q; }  // first max in scan order, NaN wins (torch)
        }
        am[cc] = pooled ? ai : -1;
      }
      const float4 k14 = *reinterpret_cast<const float4*>(&kc[2][4 * c4]);
      const float4 k24 = *reinterpret_cast<const float4*>(&kc[3][4 * c4]);
      const float4 k34 = *reinterpret_cast<const float4*>(&kc[4][4 * c4]);
      const float k1[4] = {k14.x, k14.y, k14.z, k14.w}, k2[4] = {k24.x, k24.y, k24.z, k24.w},
                  k3[4] = {k34.x, k34.y, k34.z, k34.w};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int r = gy + (q >> 1), c = gx + (q & 1);
        const bool inb = r >= 0 && r < P && c >= 0 && c < P;  // zero padding outside the image
        float d[4];
#pragma unroll
        for (int cc = 0; cc < 4; ++cc) {
          const float dz = am[cc] == q ? gg[cc] : 0.f;
          d[cc] = inb ? fmaf(k1[cc], dz, fmaf(k2[cc], y[q][cc], k3[cc])) : 0.f;
        }
        uint32_t h01, l01, h23, l23;
        split2_bf16(d[0], d[1], h01, l01);
        split2_bf16(d[2], d[3], h23, l23);
        const int rec = (2 * wy + (q >> 1)) * BW_IC + 2 * wx + (q & 1);
        const int off = rec * 32 + (c4 & 3) * 8;
        *reinterpret_cast<uint2*>(d_l + (c4 >> 2) * BW_DPLANE + off) = make_uint2(h01, h23);
        *reinterpret_cast<uint2*>(d_l + (2 + (c4 >> 2)) * BW_DPLANE + off) = make_uint2(l01, l23);
      }
    }
#pragma unroll
    for (int u = 0; u < BW_PPER; ++u) {
      const int e = tid + u * C2_THREADS;
      if (e < BW_PCHUNKS) {
        const int px = e >> 2, q = e & 3;
        *reinterpret_cast<uint4*>(p_l + (q >> 1) * BW_PPLANE + px * 32 + (q & 1) * 16) = ppre[u];
      }
    }
  };

  // ---- role-specific state
  const bool is_dgrad = wv < 4;
  const int rg = (wv & 3) >> 1, cg = wv & 1;             // dgrad: rows 4rg.., cols 16cg..
  const int ww = wv & 3;                                  // wgrad: taps ww, ww+4, ...
  const int q4 = (lane >> 2) & 3, p4 = lane & 3;          // transposed-read row / column chunk
  f32x4 wacc[7][2];
#pragma unroll
  for (int k = 0; k < 7; ++k) wacc[k][0] = wacc[k][1] = f32x4{0.f, 0.f, 0.f, 0.f};
  s16x8 ones_hi, zero8;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    ones_hi[j] = (short)((lane & 15) == 0 ? 0x3f80 : 0);
    zero8[j] = 0;
  }
  const int hp = (g >> 1) * BW_DPLANE + (g & 1) * 16;     // dgrad A: co 8g..8g+7 (hi)
  const int lp = (2 + (g >> 1)) * BW_DPLANE + (g & 1) * 16;

  int t = vid;
  if (t < total) load_tile(t);
  for (; t < total; t += gridDim.x) {
    __syncthreads();
    store_tile(t);
    __syncthreads();
    int b, r0, c0;
    decode(t, b, r0, c0);
    if (t + (int)gridDim.x < total) load_tile(t + gridDim.x);

    if (is_dgrad) {
      f32x4 acc[4];
#pragma unroll
      for (int o = 0; o < 4; ++o) acc[o] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
      for (int kx = 0; kx < 5; ++kx) {
        s16x8 bh[5], bl[5];
#pragma unroll
        for (int ky = 0; ky < 5; ++ky) {
          const int s = ky * 5 + kx;
          bh[ky] = lds8<DIAG>(w_l + (s * 64 + lane) * 16);
          bl[ky] = lds8<DIAG>(w_l + 25 * 1024 + (s * 64 + lane) * 16);
        }
        s16x8 ah[2], al[2];
        auto load_a = [&](int R, int buf) {
          const int rec = (4 * rg + R) * BW_IC + 16 * cg + kx + li;
          ah[buf] = lds8<DIAG>(d_l + hp + rec * 32);
          al[buf] = lds8<DIAG>(d_l + lp + rec * 32);
        };
        load_a(0, 0);
#pragma unroll
        for (int R = 0; R < 8; ++R) {
          const int cur = R & 1;
          if (R + 1 < 8) load_a(R + 1, cur ^ 1);
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int ky = 0; ky < 5; ++ky) {
            const int o = R - ky;
            if (o >= 0 && o < 4) acc[o] = mma3<DIAG>(ah[cur], al[cur], bh[ky], bl[ky], acc[o]);
          }
        }
      }
#pragma unroll
      for (int o = 0; o < 4; ++o) {
        const int row = r0 + 4 * rg + o;
        if (row < P) {
          float* orow = dp1 + ((int64_t)b * P + row) * P * 16;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int col = c0 + 16 * cg + 4 * g + r;
            if (col < P) orow[(int64_t)col * 16 + li] = acc[o][r];
          }
        }
      }
    } else {
      // weight gradient: per output row, K = the row's 32 pixels (permuted, see header)
      const int xo = 4 * g + q4;  // x0 pixel; x1 = xo + 16
#pragma unroll 1
      for (int row = 0; row < BW_TH; ++row) {
        const int ra = (row + 2) * BW_IC + 2 + xo;
        s16x8 ahi[2], alo[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const s16x4 x0 = ldtr<DIAG>(d_l + h * BW_DPLANE + ra * 32 + p4 * 8);
          const s16x4 x1 = ldtr<DIAG>(d_l + h * BW_DPLANE + (ra + 16) * 32 + p4 * 8);
          const s16x4 y0 = ldtr<DIAG>(d_l + (2 + h) * BW_DPLANE + ra * 32 + p4 * 8);
          const s16x4 y1 = ldtr<DIAG>(d_l + (2 + h) * BW_DPLANE + (ra + 16) * 32 + p4 * 8);
          ahi[h] = s16x8{x0[0], x0[1], x0[2], x0[3], x1[0], x1[1], x1[2], x1[3]};
          alo[h] = s16x8{y0[0], y0[1], y0[2], y0[3], y1[0], y1[1], y1[2], y1[3]};
        }
#pragma unroll
        for (int k = 0; k < 7; ++k) {
          const int tap = ww + 4 * k;
          if (tap < 26) {
            s16x8 bhi, blo;
            if (tap < 25) {
              const int ky = tap / 5, kx = tap - 5 * (tap / 5);
              const int rb = (row + ky) * BW_IC + kx + xo;
              const s16x4 x0 = ldtr<DIAG>(p_l + rb * 32 + p4 * 8);
              const s16x4 x1 = ldtr<DIAG>(p_l + (rb + 16) * 32 + p4 * 8);
              const s16x4 y0 = ldtr<DIAG>(p_l + BW_PPLANE + rb * 32 + p4 * 8);
              const s16x4 y1 = ldtr<DIAG>(p_l + BW_PPLANE + (rb + 16) * 32 + p4 * 8);
              bhi = s16x8{x0[0], x0[1], x0[2], x0[3], x1[0], x1[1], x1[2], x1[3]};
              blo = s16x8{y0[0], y0[1], y0[2], y0[3], y1[0], y1[1], y1[2], y1[3]};
            } else {
              bhi = ones_hi;  // bias gradient column
              blo = zero8;
            }
#pragma unroll
            for (int h = 0; h < 2; ++h) wacc[k][h] = mma3<DIAG>(ahi[h], alo[h], bhi, blo, wacc[k][h]);
          }
        }
      }
    }
  }
  if (!is_dgrad) {
    // slab[wg][tap(26)][co(32)][ci(16)]: lane holds C[co = 16h + 4g + r][ci = li]
    float* out = slab + (int64_t)blockIdx.x * 26 * 512;
#pragma unroll
    for (int k = 0; k < 7; ++k) {
      const int tap = ww + 4 * k;
      if (tap < 26) {
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
          for (int r = 0; r < 4; ++r) out[(tap * 32 + 16 * h + 4 * g + r) * 16 + li] = wacc[k][h][r];
      }
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

void tds_conv2_pack_weights(const float* w2, short* wp, short* wd, hipStream_t st) {
  hipLaunchKernelGGL(conv2_pack_weights_kernel, dim3(64), dim3(256), 0, st, w2, wp, wd);
}

int tds_conv2_num_wg() {
  int dev = 0, n = 256;
  if (hipGetDevice(&dev) == hipSuccess) {
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, dev) == hipSuccess) n = prop.multiProcessorCount;
  }
  return n;
}

template <int DIAG>
static void set_lds_limits_t() {
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(conv2_fwd_bf16x3_kernel<DIAG>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, F_LDS);
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(conv2_dgrad_bf16x3_kernel<DIAG>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, D_LDS);
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(conv2_wgrad_bf16x3_kernel<DIAG>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, W_LDS);
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(conv2_bwd_fused_kernel<DIAG>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, BW_LDS);
}

static void set_lds_limits() {
  static bool done = false;
  if (done) return;
  set_lds_limits_t<0>();
  set_lds_limits_t<1>();
  set_lds_limits_t<2>();
  set_lds_limits_t<3>();
  done = true;
}

// timing-only variant selector (tools/conv2_diag.py); 0 = the real kernels
static int conv2_diag() {
  const char* e = std::getenv("TDS_CONV2_DIAG");
  return e ? std::atoi(e) : 0;
}

#define TDS_C2_DISPATCH(KERNEL, ...)                                                   \
  switch (conv2_diag()) {                                                             \
    case 1: hipLaunchKernelGGL(KERNEL<1>, __VA_ARGS__); break;                        \
    case 2: hipLaunchKernelGGL(KERNEL<2>, __VA_ARGS__); break;                        \
    case 3: hipLaunchKernelGGL(KERNEL<3>, __VA_ARGS__); break;                        \
    default: hipLaunchKernelGGL(KERNEL<0>, __VA_ARGS__); break;                       \
  }

// Which conv2 forward runs: 2 = conv2_fwd2_kernel (several 4-wave workgroups per CU, weights in
// registers, LDS-DMA staging; conv2_fwd2.hip; default), 1 = conv2_fwd_bf16x3_kernel below.
int tds_conv2_fwd_version() {
  const char* e = std::getenv("TDS_CONV2_FWD");
  return (e && std::atoi(e) == 1) ? 1 : 2;
}
int tds_conv2_fwd_num_wg() { return tds_conv2_fwd_version() == 2 ? tds_conv2_fwd2_num_wg() : tds_conv2_num_wg(); }

void tds_conv2_fwd_bf16x3(const void* p1, const short* wp, const float* bias, float* y2, double* partial, int nwg,
                          int B, int P, hipStream_t st) {
  if (tds_conv2_fwd_version() == 2) {
    tds_conv2_fwd2(p1, wp, bias, y2, partial, nwg, B, P, st);
    return;
  }
  set_lds_limits();
  TDS_C2_DISPATCH(conv2_fwd_bf16x3_kernel, dim3(nwg), dim3(C2_THREADS), F_LDS, st,
                  reinterpret_cast<const uint4*>(p1), reinterpret_cast<const uint4*>(wp), bias, y2, partial, B, P);
}

void tds_conv2_dgrad_bf16x3(const void* dy2, const short* wd, float* dp1, int nwg, int B, int P, hipStream_t st) {
  set_lds_limits();
  TDS_C2_DISPATCH(conv2_dgrad_bf16x3_kernel, dim3(nwg), dim3(C2_THREADS), D_LDS, st,
                  reinterpret_cast<const uint4*>(dy2), reinterpret_cast<const uint4*>(wd), dp1, B, P);
}

void tds_conv2_wgrad_bf16x3(const void* dy2, const void* p1, float* slab, float* dw, float* db, float scale, int nwg,
                            int B, int P, hipStream_t st) {
  set_lds_limits();
  TDS_C2_DISPATCH(conv2_wgrad_bf16x3_kernel, dim3(nwg), dim3(C2_THREADS), W_LDS, st,
                  reinterpret_cast<const uint4*>(dy2), reinterpret_cast<const uint4*>(p1), slab, B, P);
  hipLaunchKernelGGL(conv2_wgrad_reduce_kernel, dim3(26 * 512 / 64), dim3(256), 0, st, slab, nwg, dw, db,
                     scale);
}

int tds_conv2_lds_bytes(int which) { return which == 0 ? F_LDS : (which == 1 ? D_LDS : W_LDS); }

// Which fused backward kernel runs: 2 = conv2_bwd2_kernel (two 4-wave workgroups per CU,
// conv2_bwd2.hip; default), 1 = conv2_bwd_fused_kernel (one 8-wave workgroup per CU).
// TDS_CONV2_BWD selects (A/B timing, tools/conv2_diag.py).
int tds_conv2_bwd_version() {  // TDS_CONV2_BWD = 1 / 2 / 3 (default 3: producer/consumer waves)
  const char* e = std::getenv("TDS_CONV2_BWD");
  const int v = e ? std::atoi(e) : 3;
  return (v == 1 || v == 2) ? v : 3;
}
int tds_conv2_bwd_fused_num_wg() {
  const int v = tds_conv2_bwd_version();
  return v == 2 ? tds_conv2_bwd2_num_wg() : v == 3 ? tds_conv2_bwd3_num_wg() : tds_conv2_num_wg();
}

// fused BN2/pool backward + conv2 dgrad + wgrad: y2 [B,P,P,32] f32, g2m [B,32,Q,Q] f32 (planar),
// aff2 [a32|b32], kbuf [k1|k2|k3]; dp1 [B,P,P,16] f32; slab [nwg][26][512]
void tds_conv2_bwd_fused(const float* y2, const float* g2m, const float* aff2, const float* kbuf, const void* p1,
                         const short* wd, float* dp1, float* slab, float* dw, float* db, float scale, int nwg, int B,
                         int P, hipStream_t st) {
  const int ver = tds_conv2_bwd_version();
  if (ver == 2 || ver == 3) {
    if (ver == 3) tds_conv2_bwd3(y2, g2m, aff2, kbuf, p1, wd, dp1, slab, nwg, B, P, st);
    else tds_conv2_bwd2(y2, g2m, aff2, kbuf, p1, wd, dp1, slab, nwg, B, P, st);
    hipLaunchKernelGGL(conv2_wgrad_reduce_kernel, dim3(26 * 512 / 64), dim3(256), 0, st, slab, nwg, dw, db,
                       scale);
    return;
  }
  set_lds_limits();
  const int Q = P / 2;
  TDS_C2_DISPATCH(conv2_bwd_fused_kernel, dim3(nwg), dim3(C2_THREADS), BW_LDS, st,
                  reinterpret_cast<const float4*>(y2), g2m, aff2, kbuf,
                  reinterpret_cast<const uint4*>(p1), reinterpret_cast<const uint4*>(wd), dp1, slab, B, P, Q);
  hipLaunchKernelGGL(conv2_wgrad_reduce_kernel, dim3(26 * 512 / 64), dim3(256), 0, st, slab, nwg, dw, db,
                     scale);
}
