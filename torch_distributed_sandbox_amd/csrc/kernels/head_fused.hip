// Fused ConvNet head: BN2 affine + ReLU + 2x2 max-pool + fc, forward and backward
// (reference: mnist_onegpu.py:21-24,29-30 -> native_batch_norm, clamp_min,
// max_pool2d_with_indices, addmm and their backward ops; SURVEY.md §2.4 K6-K9,
// K12-K18).  p2 (the pooled activation, 360 MB at 3000^2) is never stored:
// both directions recompute it from y2 while streaming the fc weight once.
//
// Workgroup = one pooled row py x 64 pooled columns, every image, every channel:
// 8 waves, wave w owns channels 4w..4w+3, lane = pooled column.  The tile's fc
// weights W[j][c][py][px0..px0+63] (coalesced over lanes) stay in registers for
// all images; per image the two y2 rows (2 x 128 NHWC records of 128 B) are
// staged through LDS with coalesced 16-B loads, the next image's loads issued
// into registers before the current image is processed.
#include <cstdlib>

#include "common.h"
#include "launchers.h"

namespace tds {

constexpr int HD_PX = 64;
constexpr int HD_MAXB = 32;  // images per rank (per-image partial sums live in LDS)
constexpr int HD_MAXB_YA = 8;  // images per rank on the ya backward path (per-lane registers)
constexpr int HD_REC = 144;  // padded LDS record stride (bytes): 128 B of y2 + 16 B
constexpr int HD_LDS = 2 * 2 * HD_PX * HD_REC;

template <int NW>  // waves per workgroup; wave w owns channels CPW*w .. CPW*w+CPW-1
struct HeadTile {
  static constexpr int THREADS = 64 * NW;
  static constexpr int PER = (2 * 2 * HD_PX * 8) / THREADS;  // float4 per thread per image
  const float4* y2;
  int P, Q, py, px0;
  __device__ void load(int b, float4 (&pre)[PER]) const {
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int e = threadIdx.x + u * THREADS;
      const int chunk = e & 7, rec = (e >> 3) & 127, row = e >> 10;
      const int col = 2 * px0 + rec;
      pre[u] = col < 2 * Q ? y2[(((int64_t)b * P + 2 * py + row) * P + col) * 8 + chunk] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
  __device__ static void store(char* lds, const float4 (&pre)[PER]) {
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int e = threadIdx.x + u * THREADS;
      const int chunk = e & 7, rec = (e >> 3) & 127, row = e >> 10;
      *reinterpret_cast<float4*>(lds + (row * 2 * HD_PX + rec) * HD_REC + chunk * 16) = pre[u];
    }
  }
};

// BN2 affine + max-pool over this lane's 2x2 window for its CPW channels.
template <int CPW>
__device__ __forceinline__ void head_window(const char* lds, int lane, int wv, const float (&a)[CPW],
                                            const float (&bb)[CPW], float (&p)[CPW], float (&yarg)[CPW],
                                            bool (&pos)[CPW]) {
  float y[4][CPW];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int row = q >> 1, rec = 2 * lane + (q & 1);
    const char* src = lds + (row * 2 * HD_PX + rec) * HD_REC + wv * CPW * 4;
    if constexpr (CPW == 4) {
      const float4 u = *reinterpret_cast<const float4*>(src);
      y[q][0] = u.x; y[q][1] = u.y; y[q][2] = u.z; y[q][3] = u.w;
    } else {
      const float2 u = *reinterpret_cast<const float2*>(src);
      y[q][0] = u.x; y[q][1] = u.y;
    }
  }
#pragma unroll
  for (int c = 0; c < CPW; ++c) {
    float m = fmaf(a[c], y[0][c], bb[c]), ya = y[0][c];
#pragma unroll
    for (int q = 1; q < 4; ++q) {
      const float z = fmaf(a[c], y[q][c], bb[c]);
      if (z > m || isnan(z)) { m = z; ya = y[q][c]; }  // first max in scan order, NaN wins
    }
    pos[c] = m > 0.f;
    p[c] = m > 0.f ? m : (isnan(m) ? m : 0.f);
    yarg[c] = ya;
  }
}

// partial[blk][b*NC + j] (fp64) = sum over the tile of p2[b][c][pos] * W[j][c][pos]
// xout (optional): p2 itself, [B][32*Q*Q] in torch's flatten order (c, py, px) — the fc
// input rows that DDP's activation exchange all-gathers (parallel/factored.py).
template <int NW>
__global__ __launch_bounds__(64 * NW) void head_fwd_kernel(const float4* __restrict__ y2, const float* __restrict__ Wfc,
                                                           const float* __restrict__ aff2,
                                                           double* __restrict__ partial, float* __restrict__ xout,
                                                           float* __restrict__ yaout, int B, int P, int Q, int NC) {
  constexpr int CPW = 32 / NW;
  using Tile = HeadTile<NW>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  __shared__ float red[NW][HD_MAXB * 10];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const Tile tile{y2, P, Q, (int)blockIdx.y, (int)blockIdx.x * HD_PX};
  const int px = tile.px0 + lane;
  const bool valid = px < Q;
  const int64_t QQ = (int64_t)Q * Q, pos = (int64_t)tile.py * Q + px;
  float w[10][CPW], a[CPW], bb[CPW];
#pragma unroll
  for (int c = 0; c < CPW; ++c) {
    a[c] = aff2[CPW * wv + c];
    bb[c] = aff2[32 + CPW * wv + c];
#pragma unroll
    for (int j = 0; j < 10; ++j) w[j][c] = (valid && j < NC) ? Wfc[((int64_t)j * 32 + CPW * wv + c) * QQ + pos] : 0.f;
  }
  float4 pre[Tile::PER];
  tile.load(0, pre);
#pragma unroll 1
  for (int b = 0; b < B; ++b) {
    __syncthreads();
    Tile::store(smem, pre);
    __syncthreads();
    if (b + 1 < B) tile.load(b + 1, pre);
    float p[CPW], ya[CPW];
    bool ps[CPW];
    head_window<CPW>(smem, lane, wv, a, bb, p, ya, ps);
    if (xout != nullptr && valid) {
#pragma unroll
      for (int c = 0; c < CPW; ++c) xout[((int64_t)b * 32 + CPW * wv + c) * QQ + pos] = p[c];
    }
    if (yaout != nullptr && valid) {
#pragma unroll
      for (int c = 0; c < CPW; ++c) yaout[((int64_t)b * 32 + CPW * wv + c) * QQ + pos] = ya[c];
    }
#pragma unroll
    for (int j = 0; j < 10; ++j) {
      float s = 0.f;
#pragma unroll
      for (int c = 0; c < CPW; ++c) s += p[c] * w[j][c];
      s = wave_sum(s);
      if (lane == 0) red[wv][b * 10 + j] = s;
    }
  }
  __syncthreads();
  const int blk = blockIdx.y * gridDim.x + blockIdx.x;
  for (int i = threadIdx.x; i < B * NC; i += blockDim.x) {
    const int b = i / NC, j = i % NC;
    double s = 0.0;
#pragma unroll
    for (int w8 = 0; w8 < NW; ++w8) s += (double)red[w8][b * 10 + j];
    partial[(int64_t)blk * B * NC + i] = s;
  }
}

// logits[i] = sums[i] + bias[i % NC]
__global__ void head_logits_kernel(const double* __restrict__ sums, const float* __restrict__ bias,
                                   float* __restrict__ logits, int BN, int NC) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < BN) logits[i] = (float)sums[i] + (bias ? bias[i % NC] : 0.f);
}

// Backward.  dl = dlogits [B][NC].
//   dW[j][c][pos]  = scale * sum_b dl[b][j] p2[b][c][pos]      (e.g. straight into the DDP bucket)
//   g2m[b][c][pos] = (sum_j dl[b][j] W[j][c][pos]) * [p2 > 0]   (planar pooled gradient, fp32)
//   partial[c][blk][2] = { sum g2m (= sum dz2), sum g2m * y2(argmax) }   (BN2 backward reductions)
template <int NW, bool WITH_DW>
__global__ __launch_bounds__(64 * NW) void head_bwd_kernel(const float4* __restrict__ y2, const float* __restrict__ Wfc,
                                                           const float* __restrict__ aff2, const float* __restrict__ dl,
                                                           float* __restrict__ dW, float* __restrict__ g2m,
                                                           double* __restrict__ partial, int B, int P, int Q, int NC,
                                                           float scale) {
  constexpr int CPW = 32 / NW;
  using Tile = HeadTile<NW>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  __shared__ float dls[HD_MAXB * 10];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const Tile tile{y2, P, Q, (int)blockIdx.y, (int)blockIdx.x * HD_PX};
  const int px = tile.px0 + lane;
  const bool valid = px < Q;
  const int64_t QQ = (int64_t)Q * Q, pos = (int64_t)tile.py * Q + px;
  for (int i = threadIdx.x; i < HD_MAXB * 10; i += blockDim.x) {
    const int b = i / 10, j = i % 10;
    dls[i] = (b < B && j < NC) ? dl[b * NC + j] : 0.f;
  }
  float w[10][CPW], dwa[10][CPW], a[CPW], bb[CPW], sdz[CPW], sdy[CPW];
#pragma unroll
  for (int c = 0; c < CPW; ++c) {
    a[c] = aff2[CPW * wv + c];
    bb[c] = aff2[32 + CPW * wv + c];
    sdz[c] = sdy[c] = 0.f;
#pragma unroll
    for (int j = 0; j < 10; ++j) {
      w[j][c] = (valid && j < NC) ? Wfc[((int64_t)j * 32 + CPW * wv + c) * QQ + pos] : 0.f;
      dwa[j][c] = 0.f;
    }
  }
  float4 pre[Tile::PER];
  tile.load(0, pre);
#pragma unroll 1
  for (int b = 0; b < B; ++b) {
    __syncthreads();
    Tile::store(smem, pre);
    __syncthreads();
    if (b + 1 < B) tile.load(b + 1, pre);
    float p[CPW], ya[CPW];
    bool ps[CPW];
    head_window<CPW>(smem, lane, wv, a, bb, p, ya, ps);
    float gm[CPW];
#pragma unroll
    for (int c = 0; c < CPW; ++c) {
      float g = 0.f;
#pragma unroll
      for (int j = 0; j < 10; ++j) {
        const float d = dls[b * 10 + j];
        g += d * w[j][c];
        if constexpr (WITH_DW) dwa[j][c] += d * p[c];
      }
      gm[c] = ps[c] ? g : 0.f;
      sdz[c] += valid ? gm[c] : 0.f;
      sdy[c] += valid ? gm[c] * ya[c] : 0.f;
    }
    if (valid) {
#pragma unroll
      for (int c = 0; c < CPW; ++c) g2m[((int64_t)b * 32 + CPW * wv + c) * QQ + pos] = gm[c];  // planar
    }
  }
  if (WITH_DW && valid) {
    float* dst = dW + (int64_t)(CPW * wv) * QQ + pos;
#pragma unroll
    for (int j = 0; j < 10; ++j)
      if (j < NC)
#pragma unroll
        for (int c = 0; c < CPW; ++c) __builtin_nontemporal_store(scale * dwa[j][c], dst + ((int64_t)j * 32 + c) * QQ);
  }
  const int nblk = gridDim.x * gridDim.y, blk = blockIdx.y * gridDim.x + blockIdx.x;
#pragma unroll
  for (int c = 0; c < CPW; ++c) {
    const float s0 = wave_sum(sdz[c]);
    const float s1 = wave_sum(sdy[c]);
    if (lane == 0) {
      partial[((int64_t)(CPW * wv + c) * nblk + blk) * 2 + 0] = s0;
      partial[((int64_t)(CPW * wv + c) * nblk + blk) * 2 + 1] = s1;
    }
  }
}

// Backward from the saved argmax values ya = y2 at each pooled window's argmax, [B][32][Q][Q]
// in the fc's flatten order (written by head_fwd).  p2 = relu(a*ya + b) is recomputed
// bit-exactly (same fmaf as head_window), so the kernel streams only ya (360 MB at 3000^2)
// and W instead of y2 (1.44 GB) through an LDS transpose.  Tile: one pooled row py x 64
// columns (lane = column), wave w owns channels 4w..4w+3; every load of a lane is issued
// before any use (60 x 4 B in flight per lane).
// (A persistent two-register-set pipelined variant ran out of SGPRs for its 100 plane
// offsets and was slower; see docs/KERNELS.md.)  Outputs as head_bwd_kernel.
// With UPD (optimizer step fused into the backward, world size 1 only: ops/fused_update.py)
// the kernel also writes W - lr * dW over W (each element read and written by one lane).
// NW = 8: one workgroup per tile and all 32 channels; NW = 4: two workgroups per tile (channel
// halves, consecutive block ids) so up to three fit a CU and one's loads overlap another's
// stores (TDS_HEAD_BWD_NW selects).
template <bool WITH_DW, int NB, bool UPD, int NW = 8>  // NB = images per rank (compile-time: exact register footprint)
__global__ __launch_bounds__(64 * NW, 2) void head_bwd_ya_kernel(const float* __restrict__ ya, const float* Wfc,
                                                             const float* __restrict__ aff2, const float* __restrict__ dl,
                                                             float* __restrict__ dW, float* __restrict__ g2m,
                                                             double* __restrict__ partial, int Q, int NC, float scale,
                                                             float* Wupd, float lr) {
  constexpr int CPW = 4;
  __shared__ float dls[NB * 10];  // dlogits: broadcast LDS reads (as scalars they cost ~50 SGPRs and spill)
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (threadIdx.x < NB * 10) dls[threadIdx.x] = (int)threadIdx.x % 10 < NC ? dl[(threadIdx.x / 10) * NC + threadIdx.x % 10] : 0.f;
  const int half = NW == 8 ? 0 : (int)(blockIdx.x & 1);
  const int pxb = NW == 8 ? (int)blockIdx.x : (int)(blockIdx.x >> 1);
  const int px = pxb * HD_PX + lane;
  const bool valid = px < Q;
  const int64_t QQ = (int64_t)Q * Q, pos = (int64_t)blockIdx.y * Q + (valid ? px : 0);
  const int c0 = 16 * half + CPW * wv;
  float w[10][CPW], y[NB][CPW];
#pragma unroll
  for (int j = 0; j < 10; ++j)
#pragma unroll
    for (int c = 0; c < CPW; ++c) w[j][c] = (valid && j < NC) ? Wfc[((int64_t)j * 32 + c0 + c) * QQ + pos] : 0.f;
#pragma unroll
  for (int b = 0; b < NB; ++b)
#pragma unroll
    for (int c = 0; c < CPW; ++c) y[b][c] = valid ? ya[((int64_t)b * 32 + c0 + c) * QQ + pos] : 0.f;
  float a[CPW], bb[CPW], sdz[CPW], sdy[CPW], dwa[10][CPW];
  __syncthreads();
#pragma unroll
  for (int c = 0; c < CPW; ++c) {
    a[c] = aff2[c0 + c];
    bb[c] = aff2[32 + c0 + c];
    sdz[c] = sdy[c] = 0.f;
#pragma unroll
    for (int j = 0; j < 10; ++j) dwa[j][c] = 0.f;
  }
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    float gm[CPW];
#pragma unroll
    for (int c = 0; c < CPW; ++c) {
      const float m = fmaf(a[c], y[b][c], bb[c]);  // == head_window's max of the window
      const bool ps = m > 0.f;
      const float p = ps ? m : (isnan(m) ? m : 0.f);
      float g = 0.f;
#pragma unroll
      for (int j = 0; j < 10; ++j) {
        const float d = dls[b * 10 + j];
        g += d * w[j][c];
        if constexpr (WITH_DW) dwa[j][c] += d * p;
      }
      gm[c] = ps ? g : 0.f;
      sdz[c] += valid ? gm[c] : 0.f;
      sdy[c] += valid ? gm[c] * y[b][c] : 0.f;
    }
    if (valid) {
#pragma unroll
      for (int c = 0; c < CPW; ++c) g2m[((int64_t)b * 32 + c0 + c) * QQ + pos] = gm[c];  // planar
    }
  }
  if (WITH_DW && valid) {
    float* dst = dW + (int64_t)c0 * QQ + pos;
#pragma unroll
    for (int j = 0; j < 10; ++j)
      if (j < NC)
#pragma unroll
        for (int c = 0; c < CPW; ++c) {
          const float gd = scale * dwa[j][c];
          __builtin_nontemporal_store(gd, dst + ((int64_t)j * 32 + c) * QQ);
          if constexpr (UPD) Wupd[((int64_t)j * 32 + c0 + c) * QQ + pos] = w[j][c] - lr * gd;  // torch SGD: p -= lr*g
        }
  }
  const int tiles_c = NW == 8 ? (int)gridDim.x : (int)(gridDim.x >> 1);
  const int nblk = tiles_c * gridDim.y, blk = blockIdx.y * tiles_c + pxb;
#pragma unroll
  for (int c = 0; c < CPW; ++c) {
    const float s0 = wave_sum(sdz[c]);
    const float s1 = wave_sum(sdy[c]);
    if (lane == 0) {
      partial[((int64_t)(c0 + c) * nblk + blk) * 2 + 0] = s0;
      partial[((int64_t)(c0 + c) * nblk + blk) * 2 + 1] = s1;
    }
  }
}

// Streaming form of the ya backward (the default).  Workgroup = one channel c x HS_RUN
// consecutive pooled positions; thread = 4 positions (dwordx4).  Every plane it touches
// (ya[b][c], W[j][c] in; dW[j][c], the updated W[j][c], g2m[b][c] out) is read or written as
// one contiguous 4 KB run: tools/micro/runlen_bw.hip measured this plane mix at 4.5-5 TB/s
// with >= 1 KB runs against 2-2.4 TB/s for the 128 B runs of a 32-channel x 32-position
// block, and plain stores beat nontemporal ones.  That is why g2m is planar (an NHWC g2m
// needs all 32 channels of a position in one workgroup; a channel-quad layout with a 1 KB-run
// LDS transpose measured 0.67 ms against 0.52 ms for this kernel).  Per-channel BN2 sums: one
// (sum dz, sum dz*y) pair per workgroup, partial[c][run][2].  Planes are addressed through one
// buffer descriptor per tensor (plane base = scalar soffset, lane offset = voffset).
// Requires QQ % 4 == 0 and every tensor < 2 GiB (tds_head_bwd_ya falls back otherwise).
constexpr int HS_RUN = 1024;
typedef unsigned int hs_u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t hs_rsrc(const void* base) { return tds_buffer_rsrc(base, 0x7FFFFFF0u); }

__device__ __forceinline__ float4 hs_ld(__amdgpu_buffer_rsrc_t r, uint32_t vo, uint32_t so) {
  return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, vo, so, 0));
}

__device__ __forceinline__ void hs_st(float4 v, __amdgpu_buffer_rsrc_t r, uint32_t vo, uint32_t so) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(hs_u32x4, v), r, vo, so, 0);
}

__device__ __forceinline__ float hs_relu(float m) { return m > 0.f ? m : (isnan(m) ? m : 0.f); }

template <bool WITH_DW, int NB, bool UPD>
__global__ __launch_bounds__(256) void head_bwd_stream_kernel(
    const float* __restrict__ ya, const float* Wfc, const float* __restrict__ aff2, const float* __restrict__ dl,
    float* __restrict__ dW, float* __restrict__ g2m, double* __restrict__ partial, int64_t QQ, int NC, float scale,
    float* Wupd, float lr) {
  __shared__ float dls[NB * 10];
  __shared__ float red[2][4];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int nrun = (int)((QQ + HS_RUN - 1) / HS_RUN);
  const int c = (int)blockIdx.x / nrun, run = (int)blockIdx.x - c * nrun;  // channel-major: neighbours share planes
  if (t < NB * 10) dls[t] = t % 10 < NC ? dl[(t / 10) * NC + t % 10] : 0.f;
  const float a = aff2[c], bb = aff2[32 + c];
  const __amdgpu_buffer_rsrc_t ry = hs_rsrc(ya), rw = hs_rsrc(Wfc), rd = hs_rsrc(dW), ru = hs_rsrc(Wupd),
                               rg = hs_rsrc(g2m);
  const uint32_t plane = (uint32_t)(32 * QQ * 4);  // bytes between consecutive b (ya, g2m) / j (W, dW)
  const int64_t pos = (int64_t)run * HS_RUN + 4 * t;
  const bool valid = pos < QQ;  // QQ % 4 == 0: a thread's 4 positions are all in or all out
  const uint32_t vo = valid ? (uint32_t)(((int64_t)c * QQ + pos) * 4) : 0u;
  float4 y[NB], w[10];
#pragma unroll
  for (int b = 0; b < NB; ++b) y[b] = hs_ld(ry, vo, b * plane);
#pragma unroll
  for (int j = 0; j < 10; ++j) w[j] = hs_ld(rw, vo, (j < NC ? j : 0) * plane);  // rows >= NC: reload row 0
#pragma unroll
  for (int b = 0; b < NB; ++b) y[b] = valid ? y[b] : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int j = 0; j < 10; ++j) w[j] = (valid && j < NC) ? w[j] : make_float4(0.f, 0.f, 0.f, 0.f);
  __syncthreads();  // dls
  float sdz = 0.f, sdy = 0.f;
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    float4 g = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int j = 0; j < 10; ++j) {
      const float d = dls[b * 10 + j];
      g.x += d * w[j].x;
      g.y += d * w[j].y;
      g.z += d * w[j].z;
      g.w += d * w[j].w;
    }
    // same fmaf as head_window: bit-exact recomputation of the pooled pre-activation
    float4 gm;
    gm.x = fmaf(a, y[b].x, bb) > 0.f ? g.x : 0.f;
    gm.y = fmaf(a, y[b].y, bb) > 0.f ? g.y : 0.f;
    gm.z = fmaf(a, y[b].z, bb) > 0.f ? g.z : 0.f;
    gm.w = fmaf(a, y[b].w, bb) > 0.f ? g.w : 0.f;
    // invalid positions hold zeros: w = 0 -> gm = 0, y = 0 -> no contribution
    sdz += (gm.x + gm.y) + (gm.z + gm.w);
    sdy += (gm.x * y[b].x + gm.y * y[b].y) + (gm.z * y[b].z + gm.w * y[b].w);
    if (valid) hs_st(gm, rg, vo, b * plane);
  }
  if constexpr (WITH_DW) {
#pragma unroll
    for (int j = 0; j < 10; ++j) {
      float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int b = 0; b < NB; ++b) {
        const float d = dls[b * 10 + j];
        s.x += d * hs_relu(fmaf(a, y[b].x, bb));
        s.y += d * hs_relu(fmaf(a, y[b].y, bb));
        s.z += d * hs_relu(fmaf(a, y[b].z, bb));
        s.w += d * hs_relu(fmaf(a, y[b].w, bb));
      }
      s = make_float4(scale * s.x, scale * s.y, scale * s.z, scale * s.w);
      if (valid && j < NC) {
        hs_st(s, rd, vo, j * plane);
        if constexpr (UPD)  // torch SGD: p -= lr * g
          hs_st(make_float4(w[j].x - lr * s.x, w[j].y - lr * s.y, w[j].z - lr * s.z, w[j].w - lr * s.w), ru, vo,
                j * plane);
      }
    }
  }
  sdz = wave_sum(sdz);
  sdy = wave_sum(sdy);
  if (lane == 0) {
    red[0][wv] = sdz;
    red[1][wv] = sdy;
  }
  __syncthreads();
  if (t < 2) {
    const double s = ((double)red[t][0] + (double)red[t][1]) + ((double)red[t][2] + (double)red[t][3]);
    partial[((int64_t)c * nrun + run) * 2 + t] = s;
  }
}

// Forward, wide tiles (the default; TDS_HEAD_FWD=1 selects head_fwd_kernel): workgroup = one
// pooled row x 128 pooled columns, 16 waves x 2 channels, lane = columns l and l + 64.  A wave's
// fc-weight loads and ya stores for a channel are two back-to-back 256 B runs (512 B
// contiguous) instead of one: tools/micro/runlen_bw.hip puts 256 B runs at ~2.9 TB/s and
// 512 B runs at ~3.8 TB/s for this plane mix.  The y2 rows are staged as in head_fwd_kernel
// (2 rows x 256 NHWC records, 72 KB LDS, one workgroup per CU); the next image's records are
// prefetched into registers while the current one is reduced.
template <int NW, int PXL>
struct HeadTile2 {
  static constexpr int THREADS = 64 * NW;
  static constexpr int PX = 64 * PXL;                        // pooled columns per tile
  static constexpr int PER = (2 * 2 * PX * 8) / THREADS;     // float4 per thread per image
  static constexpr int LDS = 2 * 2 * PX * HD_REC;
  const float4* y2;
  int P, Q, py, px0;
  __device__ void load(int b, float4 (&pre)[PER]) const {
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int e = threadIdx.x + u * THREADS;
      const int chunk = e & 7, rec = (e >> 3) % (2 * PX), row = (e >> 3) / (2 * PX);
      const int col = 2 * px0 + rec;
      pre[u] = col < 2 * Q ? y2[(((int64_t)b * P + 2 * py + row) * P + col) * 8 + chunk] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
  __device__ static void store(char* lds, const float4 (&pre)[PER]) {
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int e = threadIdx.x + u * THREADS;
      const int chunk = e & 7, rec = (e >> 3) % (2 * PX), row = (e >> 3) / (2 * PX);
      *reinterpret_cast<float4*>(lds + (row * 2 * PX + rec) * HD_REC + chunk * 16) = pre[u];
    }
  }
};

template <int NW, int PXL>
__global__ __launch_bounds__(64 * NW) void head_fwd2_kernel(const float4* __restrict__ y2, const float* __restrict__ Wfc,
                                                            const float* __restrict__ aff2, double* __restrict__ partial,
                                                            float* __restrict__ xout, float* __restrict__ yaout, int B,
                                                            int P, int Q, int NC) {
  constexpr int CPW = 32 / NW;
  using Tile = HeadTile2<NW, PXL>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  // per-image wave sums, reduced (fixed order) by threads < NC after the next barrier: 640 B
  // of static LDS instead of NW x HD_MAXB x 10 floats, so two workgroups share a CU
  // (2 x 73 KB) and one's weight prologue / tail overlaps the other's streaming
  __shared__ float red[NW][10];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int blk = blockIdx.y * gridDim.x + blockIdx.x;
  auto flush = [&](int b) {  // after a barrier that follows image b's red[] writes
    if ((int)threadIdx.x < NC) {
      double t = 0.0;
#pragma unroll
      for (int w8 = 0; w8 < NW; ++w8) t += (double)red[w8][threadIdx.x];
      partial[((int64_t)blk * B + b) * NC + threadIdx.x] = t;
    }
  };
  const Tile tile{y2, P, Q, (int)blockIdx.y, (int)blockIdx.x * Tile::PX};
  const int64_t QQ = (int64_t)Q * Q;
  bool valid[PXL];
  int64_t pos[PXL];
#pragma unroll
  for (int k = 0; k < PXL; ++k) {
    const int px = tile.px0 + lane + 64 * k;
    valid[k] = px < Q;
    pos[k] = (int64_t)tile.py * Q + px;
  }
  float w[10][PXL][CPW], a[CPW], bb[CPW];
#pragma unroll
  for (int c = 0; c < CPW; ++c) {
    a[c] = aff2[CPW * wv + c];
    bb[c] = aff2[32 + CPW * wv + c];
#pragma unroll
    for (int j = 0; j < 10; ++j)
#pragma unroll
      for (int k = 0; k < PXL; ++k)
        w[j][k][c] = (valid[k] && j < NC) ? Wfc[((int64_t)j * 32 + CPW * wv + c) * QQ + pos[k]] : 0.f;
  }
  float4 pre[Tile::PER];
  tile.load(0, pre);
#pragma unroll 1
  for (int b = 0; b < B; ++b) {
    __syncthreads();
    if (b > 0) flush(b - 1);
    Tile::store(smem, pre);
    __syncthreads();
    if (b + 1 < B) tile.load(b + 1, pre);
    float s[10];
#pragma unroll
    for (int j = 0; j < 10; ++j) s[j] = 0.f;
#pragma unroll
    for (int k = 0; k < PXL; ++k) {
      // BN2 affine + max-pool over the 2x2 window of column lane + 64k (same fmaf / scan
      // order / NaN rule as head_window)
      float y[4][CPW];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int row = q >> 1, rec = 2 * (lane + 64 * k) + (q & 1);
        const char* src = smem + (row * 2 * Tile::PX + rec) * HD_REC + wv * CPW * 4;
        if constexpr (CPW == 2) {
          const float2 u = *reinterpret_cast<const float2*>(src);
          y[q][0] = u.x; y[q][1] = u.y;
        } else {
          const float4 u = *reinterpret_cast<const float4*>(src);
          y[q][0] = u.x; y[q][1] = u.y; y[q][2] = u.z; y[q][3] = u.w;
        }
      }
      float p[CPW], ya[CPW];
#pragma unroll
      for (int c = 0; c < CPW; ++c) {
        float m = fmaf(a[c], y[0][c], bb[c]), yv = y[0][c];
#pragma unroll
        for (int q = 1; q < 4; ++q) {
          const float z = fmaf(a[c], y[q][c], bb[c]);
          if (z > m || isnan(z)) { m = z; yv = y[q][c]; }
        }
        p[c] = m > 0.f ? m : (isnan(m) ? m : 0.f);
        ya[c] = yv;
      }
      if (valid[k]) {
#pragma unroll
        for (int c = 0; c < CPW; ++c) {
          const int64_t o = ((int64_t)b * 32 + CPW * wv + c) * QQ + pos[k];
          if (xout != nullptr) xout[o] = p[c];
          if (yaout != nullptr) yaout[o] = ya[c];
        }
      }
#pragma unroll
      for (int j = 0; j < 10; ++j)
#pragma unroll
        for (int c = 0; c < CPW; ++c) s[j] += p[c] * w[j][k][c];
    }
#pragma unroll
    for (int j = 0; j < 10; ++j) {
      const float t = wave_sum(s[j]);
      if (lane == 0) red[wv][j] = t;
    }
  }
  __syncthreads();
  flush(B - 1);
}

constexpr int HF2_NW = 16, HF2_PXL = 2;
using HF2Tile = HeadTile2<HF2_NW, HF2_PXL>;

// TDS_HEAD_FWD (read per call: in-process A/B): 1 = head_fwd_kernel (64 columns), otherwise
// head_fwd2_kernel<16, 2> (128 columns).  <16, 4> (256 columns, 1 KB plane runs, 144 KB LDS)
// measured 1.26 ms against 0.66 (tools/head_diag.py): 80 weight registers per lane.
static int head_fwd_mode() {
  const char* e = std::getenv("TDS_HEAD_FWD");
  return (e && std::atoi(e) == 1) ? 1 : 2;
}
static int head_fwd_px(int mode) { return mode == 1 ? HD_PX : 64 * mode; }

constexpr int HD_FWD_NW = 8;
constexpr int HD_BWD_NW = 16;

static void head_lds_limits() {
  static bool done = false;
  if (done) return;
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(head_fwd_kernel<HD_FWD_NW>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, HD_LDS);
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(head_fwd2_kernel<HF2_NW, HF2_PXL>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, HF2Tile::LDS);
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(head_bwd_kernel<HD_BWD_NW, true>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, HD_LDS);
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(head_bwd_kernel<HD_BWD_NW, false>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, HD_LDS);
  done = true;
}

}  // namespace tds

using namespace tds;

int tds_head_bwd_nblk(int Q) { return ((Q + HD_PX - 1) / HD_PX) * Q; }  // head_bwd_kernel (y2 path)

int tds_head_fwd_nblk(int Q) {
  const int px = head_fwd_px(head_fwd_mode());
  return ((Q + px - 1) / px) * Q;
}

// partial: double [nblk][B*NC]; sums: double [B*NC] workspace
int tds_head_fwd(const float* y2, const float* Wfc, const float* bias, const float* aff2, double* partial, double* sums,
                 float* logits, float* xout, float* yaout, int B, int P, int NC, hipStream_t st) {
  const int Q = P / 2;
  if (B > HD_MAXB || NC > 10 || Q < 1) return -1;
  head_lds_limits();
  const int mode = head_fwd_mode();
  const int px = head_fwd_px(mode);
  const dim3 grid((Q + px - 1) / px, Q);
  if (mode == 2)
    hipLaunchKernelGGL((head_fwd2_kernel<HF2_NW, HF2_PXL>), grid, dim3(64 * HF2_NW), HF2Tile::LDS, st,
                       reinterpret_cast<const float4*>(y2), Wfc, aff2, partial, xout, yaout, B, P, Q, NC);
  else
    hipLaunchKernelGGL(head_fwd_kernel<HD_FWD_NW>, grid, dim3(64 * HD_FWD_NW), HD_LDS, st,
                       reinterpret_cast<const float4*>(y2), Wfc, aff2, partial, xout, yaout, B, P, Q, NC);
  const int nblk = grid.x * grid.y, BN = B * NC;
  tds_reduce_partials(partial, sums, BN, nblk, BN, 0, BN, st);
  hipLaunchKernelGGL(head_logits_kernel, dim3((BN + 63) / 64), dim3(64), 0, st, sums, bias, logits, BN, NC);
  return 0;
}

// partial: double [32][nblk][2]
int tds_head_bwd(const float* y2, const float* Wfc, const float* aff2, const float* dlogits, float* dW, float* g2m,
                 double* partial, int B, int P, int NC, float scale, hipStream_t st) {
  const int Q = P / 2;
  if (B > HD_MAXB || NC > 10 || Q < 1) return -1;
  head_lds_limits();
  const dim3 grid((Q + HD_PX - 1) / HD_PX, Q);
  // dW == nullptr: the fc weight gradient is formed elsewhere (activation exchange)
  if (dW)
    hipLaunchKernelGGL((head_bwd_kernel<HD_BWD_NW, true>), grid, dim3(64 * HD_BWD_NW), HD_LDS, st,
                       reinterpret_cast<const float4*>(y2), Wfc, aff2, dlogits, dW, g2m, partial, B, P, Q, NC, scale);
  else
    hipLaunchKernelGGL((head_bwd_kernel<HD_BWD_NW, false>), grid, dim3(64 * HD_BWD_NW), HD_LDS, st,
                       reinterpret_cast<const float4*>(y2), Wfc, aff2, dlogits, dW, g2m, partial, B, P, Q, NC, scale);
  return 0;
}

int tds_head_bwd_ya_max_batch() { return HD_MAXB_YA; }

// backward from saved argmax values (head_bwd_ya_kernel); partial: double [32][nblk][2]
// TDS_HEAD_BWD_NW = 4 / 8 select the lane-per-column head_bwd_ya_kernel (A/B); default: streaming
static int head_bwd_ya_form() {
  const char* e = std::getenv("TDS_HEAD_BWD_NW");  // read per call: in-process A/B (tools/head_diag.py)
  const int v = e ? std::atoi(e) : 0;
  return (v == 4 || v == 8) ? v : 0;
}

static int head_bwd_stream_nrun(int Q) { return (int)(((int64_t)Q * Q + HS_RUN - 1) / HS_RUN); }

// the streaming kernel's buffer descriptors cover 2 GiB and its dwordx4 plane accesses need QQ % 4 == 0
static bool head_bwd_use_stream(int B, int P, int NC) {
  const int64_t QQ = (int64_t)(P / 2) * (P / 2);
  const int64_t big = (int64_t)(B > NC ? B : NC) * 32 * QQ * 4;
  return head_bwd_ya_form() == 0 && QQ % 4 == 0 && big < 0x7FFFFFF0LL;
}

int tds_head_bwd_ya_nblk(int B, int P, int NC) {
  const int Q = P / 2;
  if (head_bwd_use_stream(B, P, NC)) return head_bwd_stream_nrun(Q);
  return ((Q + HD_PX - 1) / HD_PX) * Q;
}

bool tds_head_bwd_ya_supported(int B, int P, int NC) { return B >= 1 && B <= HD_MAXB_YA && NC <= 10 && P >= 2; }

int tds_head_bwd_ya(const float* ya, const float* Wfc, const float* aff2, const float* dlogits, float* dW, float* g2m,
                    double* partial, int B, int P, int NC, float scale, float* Wupd, float lr, hipStream_t st) {
  const int Q = P / 2;
  if (!tds_head_bwd_ya_supported(B, P, NC)) return -1;
  if (Wupd && !dW) return -1;
  if (head_bwd_use_stream(B, P, NC)) {
    const dim3 grid(32 * head_bwd_stream_nrun(Q));
    const int64_t QQ = (int64_t)Q * Q;
#define TDS_HBS(NB)                                                                                                    \
  case NB:                                                                                                             \
    if (Wupd)                                                                                                          \
      hipLaunchKernelGGL((head_bwd_stream_kernel<true, NB, true>), grid, dim3(256), 0, st, ya, Wfc, aff2, dlogits, dW, \
                         g2m, partial, QQ, NC, scale, Wupd, lr);                                                       \
    else if (dW)                                                                                                       \
      hipLaunchKernelGGL((head_bwd_stream_kernel<true, NB, false>), grid, dim3(256), 0, st, ya, Wfc, aff2, dlogits,    \
                         dW, g2m, partial, QQ, NC, scale, Wupd, lr);                                                   \
    else                                                                                                               \
      hipLaunchKernelGGL((head_bwd_stream_kernel<false, NB, false>), grid, dim3(256), 0, st, ya, Wfc, aff2, dlogits,   \
                         dW, g2m, partial, QQ, NC, scale, Wupd, lr);                                                   \
    return 0;
    switch (B) { TDS_HBS(1) TDS_HBS(2) TDS_HBS(3) TDS_HBS(4) TDS_HBS(5) TDS_HBS(6) TDS_HBS(7) TDS_HBS(8) default: break; }
#undef TDS_HBS
    return -1;
  }
  const bool half = head_bwd_ya_form() != 8;
  const dim3 grid(((Q + HD_PX - 1) / HD_PX) * (half ? 2 : 1), Q);
#define TDS_HBY_NW(NB, NW)                                                                                              \
  if (Wupd)                                                                                                            \
    hipLaunchKernelGGL((head_bwd_ya_kernel<true, NB, true, NW>), grid, dim3(64 * NW), 0, st, ya, Wfc, aff2, dlogits,   \
                       dW, g2m, partial, Q, NC, scale, Wupd, lr);                                                      \
  else if (dW)                                                                                                         \
    hipLaunchKernelGGL((head_bwd_ya_kernel<true, NB, false, NW>), grid, dim3(64 * NW), 0, st, ya, Wfc, aff2, dlogits,  \
                       dW, g2m, partial, Q, NC, scale, Wupd, lr);                                                      \
  else                                                                                                                 \
    hipLaunchKernelGGL((head_bwd_ya_kernel<false, NB, false, NW>), grid, dim3(64 * NW), 0, st, ya, Wfc, aff2, dlogits, \
                       dW, g2m, partial, Q, NC, scale, Wupd, lr);
#define TDS_HBY(NB)            \
  case NB:                     \
    if (half) {                \
      TDS_HBY_NW(NB, 4)        \
    } else {                   \
      TDS_HBY_NW(NB, 8)        \
    }                          \
    return 0;
  switch (B) { TDS_HBY(1) TDS_HBY(2) TDS_HBY(3) TDS_HBY(4) TDS_HBY(5) TDS_HBY(6) TDS_HBY(7) TDS_HBY(8) default: break; }
#undef TDS_HBY_NW
#undef TDS_HBY
  return -1;
}
