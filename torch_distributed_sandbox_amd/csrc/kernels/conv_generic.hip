// Generic stride-1 "same-style" 2-D convolution for NCHW fp32 on gfx950 MFMA.
//
// Reference op: nn.Conv2d(Cin, Cout, kernel_size=5, stride=1, padding=2)
// (mnist_onegpu.py:15,20 -> cudnn_convolution / convolution_backward, SURVEY.md
// §2.4 K1, K5, K19, K20, K25).  This file is the exact-fp32 generic path
// (v_mfma_f32_16x16x4_f32: one fp32 per lane per operand, bit-exact fmaf
// chains); the model's fast path lives in convnet_fused.hip.
//
//  fwd   : out[b,co,y,x] = bias[co] + sum_{ci,ky,kx} w[co,ci,ky,kx] * in[b,ci,y+ky-P,x+kx-P]
//          implicit GEMM, M = co (16/32 per workgroup), N = x positions, K = (ci,tap).
//  dgrad : the same kernel on the flipped/transposed weights (pad' = KS-1-P).
//  wgrad : M = co, N = (tap,ci) (+1 "ones" column that yields the bias grad),
//          K = positions; split over workgroups into an fp32 slab, then a
//          deterministic second-stage reduce (no float atomics).
#include "common.h"
#include "launchers.h"

namespace tds {

__device__ __forceinline__ f32x4 mfma16x4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// ----------------------------------------------------------------------------
// Forward (also used for dgrad).  Workgroup = 4 waves, output tile
// (16*MT) co x 8 rows x 64 cols.  Wave w owns rows 2w, 2w+1 and 4 column
// tiles of 16 -> 2*4*MT accumulators of 16x16.
// LDS: input chunk [CIC][8+KS-1][64+KS-1] (channel stride = 16 mod 32 so the
// two 16-lane channel groups of a ds_read_b32 half never share a bank), and
// weight chunk [CIC][KS*KS][16*MT] (ci stride = 16 mod 32).
// ----------------------------------------------------------------------------
constexpr int FWD_TH = 8;
constexpr int FWD_TW = 64;

__host__ __device__ constexpr int pad16mod32(int v) { return ((v + 31 - 16) / 32) * 32 + 16; }

template <int KS, int CIC, int MT>
struct FwdCfg {
  static constexpr int IH = FWD_TH + KS - 1;
  static constexpr int IW = FWD_TW + KS - 1;
  static constexpr int SC = pad16mod32(IH * IW);
  static constexpr int KK = KS * KS;
  static constexpr int COB = 16 * MT;
  static constexpr int SW = pad16mod32(KK * COB);
  static constexpr int LDS_FLOATS = CIC * SC + CIC * SW;
};

template <int KS, int CIC, int MT>
__global__ __launch_bounds__(256) void conv_fwd_f32_kernel(const float* __restrict__ in, const float* __restrict__ w,
                                                           const float* __restrict__ bias, float* __restrict__ out,
                                                           int Cin, int Cout, int H, int W, int P) {
  using C = FwdCfg<KS, CIC, MT>;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* in_l = smem;
  float* w_l = smem + CIC * C::SC;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wv = tid >> 6;
  const int x0 = blockIdx.x * FWD_TW;
  const int y0 = blockIdx.y * FWD_TH;
  const int n_cot = (Cout + C::COB - 1) / C::COB;
  const int b = blockIdx.z / n_cot;
  const int co0 = (blockIdx.z % n_cot) * C::COB;
  const int64_t HW = (int64_t)H * W;
  const float* in_b = in + (int64_t)b * Cin * HW;

  f32x4 acc[MT][2][4];
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int r = 0; r < 2; ++r)
#pragma unroll
      for (int t = 0; t < 4; ++t) acc[m][r][t] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int kq = lane >> 4;   // k index within a 4-deep MFMA step
  const int li = lane & 15;

  for (int ci0 = 0; ci0 < Cin; ci0 += CIC) {
    __syncthreads();
    // stage input halo tile
    for (int e = tid; e < CIC * C::IH * C::IW; e += 256) {
      const int ci = e / (C::IH * C::IW);
      const int rem = e - ci * (C::IH * C::IW);
      const int r = rem / C::IW;
      const int c = rem - r * C::IW;
      const int gy = y0 - P + r, gx = x0 - P + c;
      float v = 0.f;
      if (ci0 + ci < Cin && gy >= 0 && gy < H && gx >= 0 && gx < W) v = in_b[(int64_t)(ci0 + ci) * HW + (int64_t)gy * W + gx];
      in_l[ci * C::SC + r * C::IW + c] = v;
    }
    // stage weights [ci][tap][co]
    for (int e = tid; e < CIC * C::KK * C::COB; e += 256) {
      const int co = e % C::COB;
      const int t = e / C::COB;
      const int tap = t % C::KK;
      const int ci = t / C::KK;
      float v = 0.f;
      if (co0 + co < Cout && ci0 + ci < Cin) v = w[((int64_t)(co0 + co) * Cin + ci0 + ci) * C::KK + tap];
      w_l[ci * C::SW + tap * C::COB + co] = v;
    }
    __syncthreads();
#pragma unroll 1
    for (int cq = 0; cq < CIC / 4; ++cq) {
      const float* wrow = w_l + (cq * 4 + kq) * C::SW + li;
      const float* irow = in_l + (cq * 4 + kq) * C::SC + (2 * wv) * C::IW + li;
#pragma unroll
      for (int ky = 0; ky < KS; ++ky) {
#pragma unroll
        for (int kx = 0; kx < KS; ++kx) {
          const int tap = ky * KS + kx;
          float a[MT];
#pragma unroll
          for (int m = 0; m < MT; ++m) a[m] = wrow[tap * C::COB + m * 16];
#pragma unroll
          for (int r = 0; r < 2; ++r) {
#pragma unroll
            for (int t = 0; t < 4; ++t) {
              const float bv = irow[(r + ky) * C::IW + t * 16 + kx];
#pragma unroll
              for (int m = 0; m < MT; ++m) acc[m][r][t] = mfma16x4(a[m], bv, acc[m][r][t]);
            }
          }
        }
      }
    }
  }
  // epilogue: D row = co (lane>>4)*4+j, col = x (lane&15)
#pragma unroll
  for (int m = 0; m < MT; ++m) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int co = co0 + m * 16 + kq * 4 + j;
      if (co >= Cout) continue;
      const float bb = bias ? bias[co] : 0.f;
      float* orow = out + ((int64_t)b * Cout + co) * HW;
#pragma unroll
      for (int r = 0; r < 2; ++r) {
        const int y = y0 + 2 * wv + r;
        if (y >= H) continue;
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const int x = x0 + t * 16 + li;
          if (x < W) orow[(int64_t)y * W + x] = acc[m][r][t][j] + bb;
        }
      }
    }
  }
}

// wt[ci][co][KS-1-ky][KS-1-kx] = w[co][ci][ky][kx]
__global__ void conv_flip_weights_kernel(const float* __restrict__ w, float* __restrict__ wt, int Cout, int Cin, int KS) {
  const int KK = KS * KS;
  const int total = Cout * Cin * KK;
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < total; e += gridDim.x * blockDim.x) {
    const int tap = e % KK;
    const int ci = (e / KK) % Cin;
    const int co = e / (KK * Cin);
    const int ky = tap / KS, kx = tap % KS;
    wt[((int64_t)ci * Cout + co) * KK + (KS - 1 - ky) * KS + (KS - 1 - kx)] = w[e];
  }
}

// ----------------------------------------------------------------------------
// Weight gradient.  MFMA 16x16x4: A[i=co][k=pos] = g, B[k=pos][j=n] = im2col(in).
// n = tap*Cin + ci for n < Cin*KK, n == Cin*KK is the bias "ones" column.
// Workgroup = 4 waves = one spatial tile (WG_TH x WG_TW) per iteration of a
// grid-stride loop over (b, tile); waves split the tile's positions (k), each
// wave keeps MT x NT accumulators for its n-range [nt0*16, (nt0+NT)*16),
// and the 4 wave partials are folded through LDS before one slab store.
// ----------------------------------------------------------------------------
constexpr int WG_TH = 4;
constexpr int WG_TW = 64;

template <int KS, int CINP>
struct WgCfg {
  static constexpr int KK = KS * KS;
  static constexpr int IH = WG_TH + KS - 1;
  static constexpr int IW = (WG_TW + KS - 1) | 1;          // odd row stride
  // B reads: 16 lanes = 16 channels of one tap, the next 16 lanes the next x
  // position (+1 dword) -> channel stride 2 mod 32 keeps a 32-lane half on 32 banks.
  static constexpr int SC = ((IH * IW + 31 - 2) / 32) * 32 + 2;
  // A reads: 16 lanes = 16 output channels, next 16 lanes +1 position -> 2 mod 32.
  static constexpr int SG = WG_TH * WG_TW + 2;
};

template <int KS, int CINP, int MT, int NT>
__global__ __launch_bounds__(256) void conv_wgrad_f32_kernel(const float* __restrict__ in, const float* __restrict__ g,
                                                             float* __restrict__ slab, int B, int Cin, int Cout, int H,
                                                             int W, int P, int ncols /* Cin*KK+1 */, int n_tiles_total) {
  using C = WgCfg<KS, CINP>;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int COB = 16 * MT;
  float* g_l = smem;                       // [COB][SG]
  float* in_l = smem + COB * C::SG;        // [CINP][SC]

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wv = tid >> 6;
  const int kq = lane >> 4;
  const int li = lane & 15;
  const int co0 = blockIdx.y * COB;
  const int nt_base = blockIdx.z * NT;      // n-tile group (16 columns each)
  const int64_t HW = (int64_t)H * W;
  const int tiles_x = (W + WG_TW - 1) / WG_TW;
  const int tiles_y = (H + WG_TH - 1) / WG_TH;
  const int tiles_per_img = tiles_x * tiles_y;

  // Precompute this lane's B-operand offset for each n tile: n = (nt_base+t)*16 + li
  int boff[NT];
  bool bone[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    int n = (nt_base + t) * 16 + li;
    bone[t] = (n == ncols - 1);
    if (n >= ncols - 1) n = 0;  // bias column / padding -> any valid address
    const int tap = n / Cin, ci = n - (n / Cin) * Cin;
    const int ky = tap / KS, kx = tap - (tap / KS) * KS;
    boff[t] = ci * C::SC + ky * C::IW + kx;
  }

  f32x4 acc[MT][NT];
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[m][t] = f32x4{0.f, 0.f, 0.f, 0.f};

  for (int tile = blockIdx.x; tile < B * tiles_per_img; tile += gridDim.x) {
    const int b = tile / tiles_per_img;
    const int tr = tile - b * tiles_per_img;
    const int y0 = (tr / tiles_x) * WG_TH;
    const int x0 = (tr % tiles_x) * WG_TW;
    __syncthreads();
    for (int e = tid; e < COB * WG_TH * WG_TW; e += 256) {
      const int c = e % WG_TW;
      const int r = (e / WG_TW) % WG_TH;
      const int co = e / (WG_TW * WG_TH);
      const int y = y0 + r, x = x0 + c;
      float v = 0.f;
      if (co0 + co < Cout && y < H && x < W) v = g[((int64_t)b * Cout + co0 + co) * HW + (int64_t)y * W + x];
      g_l[co * C::SG + r * WG_TW + c] = v;
    }
    for (int e = tid; e < CINP * C::IH * C::IW; e += 256) {
      const int c = e % C::IW;
      const int r = (e / C::IW) % C::IH;
      const int ci = e / (C::IW * C::IH);
      const int gy = y0 - P + r, gx = x0 - P + c;
      float v = 0.f;
      if (ci < Cin && gy >= 0 && gy < H && gx >= 0 && gx < W) v = in[((int64_t)b * Cin + ci) * HW + (int64_t)gy * W + gx];
      in_l[ci * C::SC + r * C::IW + c] = v;
    }
    __syncthreads();
    // wave wv takes row wv of the tile; k-steps of 4 consecutive x positions
    const int r = wv;
#pragma unroll 2
    for (int xs = 0; xs < WG_TW; xs += 4) {
      const int px = xs + kq;                   // this lane's k position
      float a[MT];
#pragma unroll
      for (int m = 0; m < MT; ++m) a[m] = g_l[(m * 16 + li) * C::SG + r * WG_TW + px];
      const float* ib = in_l + r * C::IW + px;
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const float bv = bone[t] ? 1.f : ib[boff[t]];
#pragma unroll
        for (int m = 0; m < MT; ++m) acc[m][t] = mfma16x4(a[m], bv, acc[m][t]);
      }
    }
  }
  // fold the 4 wave partials through LDS, then one slab row per workgroup
  __syncthreads();
  float* red = smem;  // [COB][NT*16]
  const int RW = NT * 16;
  for (int wsel = 0; wsel < 4; ++wsel) {
    if (wv == wsel) {
#pragma unroll
      for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int row = m * 16 + kq * 4 + j;
            const int col = t * 16 + li;
            float* p = red + row * RW + col;
            *p = (wsel == 0 ? 0.f : *p) + acc[m][t][j];
          }
    }
    __syncthreads();
  }
  float* out = slab + ((int64_t)blockIdx.x * gridDim.y * gridDim.z + blockIdx.y * gridDim.z + blockIdx.z) * (COB * RW);
  for (int e = tid; e < COB * RW; e += 256) out[e] = red[e];
}

// dw[co][ci][tap] = sum_wg slab, db[co] = sum_wg slab[.., bias column]
__global__ void conv_wgrad_reduce_kernel(const float* __restrict__ slab, float* __restrict__ dw, float* __restrict__ db,
                                         int nwg, int ny, int nz, int COB, int RW, int Cin, int Cout, int KK,
                                         float scale, int accumulate) {
  const int ncols = Cin * KK + 1;
  const int total = Cout * ncols;
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < total; e += gridDim.x * blockDim.x) {
    const int co = e / ncols, n = e - (e / ncols) * ncols;
    const int yb = co / COB, row = co - yb * COB;
    const int zb = n / RW, col = n - zb * RW;
    double s = 0.0;
    for (int i = 0; i < nwg; ++i) s += slab[((int64_t)(i * ny + yb) * nz + zb) * (COB * RW) + row * RW + col];
    const float v = (float)s * scale;
    if (n == ncols - 1) {
      if (db) db[co] = accumulate ? db[co] + v : v;
    } else {
      const int tap = n / Cin, ci = n - (n / Cin) * Cin;
      float* d = dw + ((int64_t)co * Cin + ci) * KK + tap;
      *d = accumulate ? *d + v : v;
    }
  }
}

// ----------------------------------------------------------------------------
template <int KS, int CIC, int MT>
static void launch_fwd(const float* in, const float* w, const float* bias, float* out, int B, int Cin, int Cout, int H,
                       int W, int P, hipStream_t st) {
  using C = FwdCfg<KS, CIC, MT>;
  dim3 grid((W + FWD_TW - 1) / FWD_TW, (H + FWD_TH - 1) / FWD_TH, B * ((Cout + C::COB - 1) / C::COB));
  const size_t lds = sizeof(float) * C::LDS_FLOATS;
  hipLaunchKernelGGL((conv_fwd_f32_kernel<KS, CIC, MT>), grid, dim3(256), lds, st, in, w, bias, out, Cin, Cout, H, W, P);
  TDS_LAUNCH_CHECK();
}

template <int KS>
static int dispatch_fwd(const float* in, const float* w, const float* bias, float* out, int B, int Cin, int Cout, int H,
                        int W, int P, hipStream_t st) {
  const bool small_cin = Cin <= 4;
  const bool mt1 = Cout <= 16;
  if (small_cin) {
    if (mt1) launch_fwd<KS, 4, 1>(in, w, bias, out, B, Cin, Cout, H, W, P, st);
    else launch_fwd<KS, 4, 2>(in, w, bias, out, B, Cin, Cout, H, W, P, st);
  } else {
    if (mt1) launch_fwd<KS, 8, 1>(in, w, bias, out, B, Cin, Cout, H, W, P, st);
    else launch_fwd<KS, 8, 2>(in, w, bias, out, B, Cin, Cout, H, W, P, st);
  }
  return 0;
}

template <int KS, int CINP, int MT, int NT>
static void launch_wgrad(const float* in, const float* g, float* slab, int nwg, int ny, int nz, int B, int Cin,
                         int Cout, int H, int W, int P, int ncols, hipStream_t st) {
  using C = WgCfg<KS, CINP>;
  const int COB = 16 * MT;
  size_t lds = sizeof(float) * (COB * C::SG + CINP * C::SC);
  const size_t red = sizeof(float) * COB * NT * 16;
  if (red > lds) lds = red;
  hipLaunchKernelGGL((conv_wgrad_f32_kernel<KS, CINP, MT, NT>), dim3(nwg, ny, nz), dim3(256), lds, st, in, g, slab, B,
                     Cin, Cout, H, W, P, ncols, 0);
  TDS_LAUNCH_CHECK();
}

}  // namespace tds

using namespace tds;

int tds_conv2d_fwd_f32(const float* in, const float* w, const float* bias, float* out, int B, int Cin, int Cout, int H,
                       int W, int KS, int P, hipStream_t st) {
  if (Cin > 64 || Cout > 4096) return -1;
  switch (KS) {
    case 1: return dispatch_fwd<1>(in, w, bias, out, B, Cin, Cout, H, W, P, st);
    case 3: return dispatch_fwd<3>(in, w, bias, out, B, Cin, Cout, H, W, P, st);
    case 5: return dispatch_fwd<5>(in, w, bias, out, B, Cin, Cout, H, W, P, st);
    default: return -2;
  }
}

void tds_conv2d_flip_weights(const float* w, float* wt, int Cout, int Cin, int KS, hipStream_t st) {
  const int total = Cout * Cin * KS * KS;
  hipLaunchKernelGGL(conv_flip_weights_kernel, dim3((total + 255) / 256), dim3(256), 0, st, w, wt, Cout, Cin, KS);
  TDS_LAUNCH_CHECK();
}

// Returns the slab size (floats) needed, or launches when slab != nullptr.
int64_t tds_conv2d_wgrad_f32(const float* in, const float* g, float* dw, float* db, float* slab, int B, int Cin, int Cout,
                             int H, int W, int KS, int P, float scale, int accumulate, int num_wg, hipStream_t st) {
  const int KK = KS * KS;
  const int ncols = Cin * KK + 1;
  const int MT = Cout > 16 ? 2 : 1;
  const int COB = 16 * MT;
  const int ny = (Cout + COB - 1) / COB;
  // n tiles of 16: group into NT-sized z groups
  const int ntiles = (ncols + 15) / 16;
  int NT;
  if (ntiles <= 2) NT = 2; else if (ntiles <= 4) NT = 4; else if (ntiles <= 8) NT = 8; else NT = 13;
  const int nz = (ntiles + NT - 1) / NT;
  const int CINP = Cin <= 1 ? 1 : (Cin <= 4 ? 4 : (Cin <= 16 ? 16 : 32));
  if (Cin > 32 || (KS != 5 && KS != 3 && KS != 1)) return -1;
  const int64_t slab_floats = (int64_t)num_wg * ny * nz * COB * NT * 16;
  if (!slab) return slab_floats;
#define TDS_WG_CASE(KS_, CINP_, MT_, NT_)                                                                      \
  if (KS == KS_ && CINP == CINP_ && MT == MT_ && NT == NT_) {                                                  \
    launch_wgrad<KS_, CINP_, MT_, NT_>(in, g, slab, num_wg, ny, nz, B, Cin, Cout, H, W, P, ncols, st);        \
    launched = true;                                                                                           \
  }
  bool launched = false;
#define TDS_WG_NT(KS_, CINP_, MT_) \
  TDS_WG_CASE(KS_, CINP_, MT_, 2) TDS_WG_CASE(KS_, CINP_, MT_, 4) TDS_WG_CASE(KS_, CINP_, MT_, 8) TDS_WG_CASE(KS_, CINP_, MT_, 13)
#define TDS_WG_MT(KS_, CINP_) TDS_WG_NT(KS_, CINP_, 1) TDS_WG_NT(KS_, CINP_, 2)
#define TDS_WG_CINP(KS_) TDS_WG_MT(KS_, 1) TDS_WG_MT(KS_, 4) TDS_WG_MT(KS_, 16) TDS_WG_MT(KS_, 32)
  TDS_WG_CINP(5)
  TDS_WG_CINP(3)
  TDS_WG_CINP(1)
#undef TDS_WG_CINP
#undef TDS_WG_MT
#undef TDS_WG_NT
#undef TDS_WG_CASE
  if (!launched) return -3;
  const int RW = NT * 16;
  const int total = Cout * ncols;
  hipLaunchKernelGGL(conv_wgrad_reduce_kernel, dim3((total + 255) / 256), dim3(256), 0, st, slab, dw, db, num_wg, ny, nz,
                     COB, RW, Cin, Cout, KK, scale, accumulate);
  TDS_LAUNCH_CHECK();
  return 0;
}
