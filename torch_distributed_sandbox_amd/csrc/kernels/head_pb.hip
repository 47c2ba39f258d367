// Fused ConvNet head on the pooled-blocked ya / g2m layout (pooled_layout.h): BN2 affine + ReLU
// + fc forward, and the fc / ReLU backward up to the pooled gradient g2m with the BN2 backward
// sums (reference: mnist_onegpu.py:21-24,29-30 -> native_batch_norm, clamp_min,
// max_pool2d_with_indices, addmm and their backward ops).
//
// The max-pool itself is resolved by the conv2 forward: it writes ya = y2 at each window's
// argmax (conv2_fwd2.hip), so the head streams ya (B x 36 MB in fp16 at 3000^2) instead of y2 (B x
// 288 MB) and both directions are pure streams over the fc weight (720 MB):
//
//   forward : X = relu(a*ya + b);  logits[b][j] = sum X[b][k] W[j][k]           (+ X rows for
//             DDP's activation exchange when asked)
//             ya is fp16: the y2h value at each window's argmax, y2 = h d + b2 (launchers.h TdsYaDec);
//             a*ya + b = (a d) h + (a b2 + b), one v_fma_mix_f32 per value (hp_fma_h)
//   backward: g = dl W, g2m = g [z > 0] (planar, for the conv2 backward), BN2 sums
//             (sum g2m, sum g2m*ya) per channel, dW = scale dl^T X and/or W -= lr dW (SGD
//             step fused into the backward at world size 1)
//
// Workgroup: one channel c and a band of HP_BAND block rows (4 pooled rows each) over the FULL
// pooled width: the fc weight of (class j, channel c, 4 pooled rows) is then one contiguous run
// of 4Q floats (12 KiB at 3000^2) and ya of (image, channel, block row) one run of Q8 blocks
// (12 KiB), walked front to back (256-column spans with 1 KiB weight runs streamed at 2.7 TB/s).
// 256 threads sweep a block row in chunks of 32 blocks (256 pooled columns): wave w takes
// pooled row w of the block row, lane l block l/2 of the chunk, columns 4*(l%2) .. +3.  Per chunk
// and thread:
//   ya  : 4 fp16 values (8 B) per image (the 4 waves together read one 2 KiB run per image),
//   W   : one 4-float group per class from the fc's own (c, h, w) layout at the same row and
//         columns -- a wave-instruction covers one 1 KiB row run.  A row starts at a 16-B boundary
//         only when (c*Q*Q + y*Q) % 4 == 0 (for Q = 750 every odd row is 8 B off).  Loads are
//         dwordx4 at any dword alignment (split loads cost the forward ~50%: 0.27 vs 0.18 ms for
//         the same bytes); stores of a misaligned group are moved as two float2 (or four floats),
//         picked per wave, so no store straddles a 16-B granule -- misaligned dwordx4 stores of
//         the weight update cost 14% of the backward,
//   g2m : 4 fp16 values per image (planar), dW / updated W: one 4-float group per class.
// No LDS and no barriers in the stream.  One load set per thread: a chunk's loads are issued right
// before their use and the latency is left to occupancy -- two sets in alternation (the next chunk's
// loads in flight while the current one is reduced) held 236 / 202 VGPRs in the forward / backward,
// 2 waves per SIMD; one set holds 140 / 149, 3 waves, and measured 10 / 4 us faster in the step
// (r6_s36, r6_s37).  64-bit indexing throughout (no buffer descriptors).
#include "bf16x3.h"
#include "common.h"
#include "ce_small.h"
#include "launchers.h"
#include "pooled_layout.h"

namespace tds {

constexpr int HP_THREADS = 256;
constexpr int HP_BAND = 4;                  // block rows per workgroup (forward)
// the backward's band: 2 block rows (r4_s43: 2 / 4 / 8 -> backward 0.448 / 0.457 / 0.505 ms,
// forward 0.227 / 0.212 / 0.232 -- each direction takes its best)
constexpr int HP_BAND_B = 2;
constexpr int HP_MAXB = 8;                  // images per pass (larger batches run in passes)

struct HPGrid {
  int nband;
  __host__ __device__ int per_channel() const { return nband; }
};

__host__ __device__ inline HPGrid hp_grid(const PBGeom& g) { return HPGrid{(g.Q4 + HP_BAND - 1) / HP_BAND}; }
__host__ __device__ inline HPGrid hp_grid_b(const PBGeom& g) { return HPGrid{(g.Q4 + HP_BAND_B - 1) / HP_BAND_B}; }

__device__ __forceinline__ float hp_relu(float z) { return z > 0.f ? z : (isnan(z) ? z : 0.f); }

// fma(a, the fp16 value in half HI of w, c): one v_fma_mix_f32 (the fp16 operand converted exactly,
// one rounding)
template <int HI>
__device__ __forceinline__ float hp_fma_h(float a, uint32_t w, float c) {
  float d;
  if constexpr (HI != 0)
    asm("v_fma_mix_f32 %0, %1, %2, %3 op_sel:[0,1,0] op_sel_hi:[0,1,0]" : "=v"(d) : "v"(a), "v"(w), "v"(c));
  else
    asm("v_fma_mix_f32 %0, %1, %2, %3 op_sel_hi:[0,1,0]" : "=v"(d) : "v"(a), "v"(w), "v"(c));
  return d;
}

// the 4 values a * h_k + c of a loaded ya group (h_0 .. h_3 in y.x lo, y.x hi, y.y lo, y.y hi)
__device__ __forceinline__ void hp_fma4(float a, uint2 y, float c, float (&o)[4]) {
  o[0] = hp_fma_h<0>(a, y.x, c);
  o[1] = hp_fma_h<1>(a, y.x, c);
  o[2] = hp_fma_h<0>(a, y.y, c);
  o[3] = hp_fma_h<1>(a, y.y, c);
}

// ya's decode factor d (launchers.h TdsYaDec; the conv2 backward forms it the same way)
__device__ __forceinline__ float hp_ydec(const uint32_t* ysc) {
  return ysc != nullptr ? __uint_as_float(ysc[0]) * __uint_as_float(ysc[1]) / __uint_as_float(ysc[2]) : 1.f;
}

struct HPThread {
  int blk, prow, half, part;  // block, pooled row in the block (= wave), column half, float4 in the block
  __device__ HPThread(int chunk) {
    const int lane = threadIdx.x & 63;
    prow = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
    blk = chunk * 32 + (lane >> 1);
    half = lane & 1;
    part = prow * 2 + half;
  }
};

template <class T>
__device__ __forceinline__ void hp_st(T* p, T v, bool nt) {
  if (nt) st_stream(p, v); else *p = v;
}

// 4 consecutive floats of a weight row at p; al = (element index of p) % 4, wave-uniform;
// nt: non-temporal (common.h st_stream)
__device__ __forceinline__ void hp_st4(float* p, int al, float4 v, bool nt = true) {
  if (al == 0) {
    hp_st(reinterpret_cast<float4*>(p), v, nt);
  } else if (al == 2) {
    hp_st(reinterpret_cast<float2*>(p), make_float2(v.x, v.y), nt);
    hp_st(reinterpret_cast<float2*>(p + 2), make_float2(v.z, v.w), nt);
  } else {
    hp_st(p, v.x, nt);
    hp_st(p + 1, v.y, nt);
    hp_st(p + 2, v.z, nt);
    hp_st(p + 3, v.w, nt);
  }
}

// this thread's weight-row geometry for block row R: element offset of column px0 of row py in
// plane (j = 0, c) and its wave-uniform alignment class; nvalid = columns px0 .. px0+nvalid-1
// inside the image.  Loads never branch per lane: a group crossing the row end is read at the
// row's last 4 columns (shifted by sh, values re-aligned with selects), rows past the image at
// row Q-1 (masked), so every lane of a wave issues the same access form.
struct HPRow {
  int64_t off, ldoff;
  int al, nvalid, sh;
  __device__ HPRow(const PBGeom& g, const HPThread& th, int c, int R) {
    const int Q = g.Q;
    const int py = 4 * R + th.prow, px0 = th.blk * 8 + th.half * 4;
    const int64_t rowbase = (int64_t)c * Q * Q + (int64_t)(py < Q ? py : Q - 1) * Q;
    nvalid = (py < Q && th.blk < g.Q8) ? max(0, min(4, Q - px0)) : 0;
    al = __builtin_amdgcn_readfirstlane((int)(rowbase & 3));  // j*32*Q*Q % 4 == 0 for every class
    off = rowbase + px0;
    const int pxl = min(px0, max(0, Q - 4));  // Q >= 4 (supported(): H >= 16)
    sh = px0 - pxl;
    ldoff = rowbase + pxl;
  }
};

// 4 consecutive floats at any dword alignment (one global_load_dwordx4)
__device__ __forceinline__ float4 hp_ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }

// loads of one chunk: ya 4 fp16 values per image, weight 4-groups per class (zeros outside the image)
template <int NB>
struct HPLoad {
  uint2 y[NB];
  float4 w[10];
  int sh, nvalid;  // this lane's edge geometry for fix()
  // the loads only (fix() and the reduction consume them)
  __device__ __forceinline__ void issue(const unsigned short* __restrict__ ya, const float* W, const PBGeom& g, const HPThread& th,
                                        int c, int R, int b0, int NC) {
    const int64_t plane = g.plane(), QQ = (int64_t)g.Q * g.Q;
    const int bc = th.blk < g.Q8 ? th.blk : g.Q8 - 1;  // idle lanes of the last chunk: a valid block
    const int64_t yi = (((int64_t)c * g.Q4 + R) * g.Q8 + bc) * 32 + th.part * 4;
#pragma unroll
    for (int b = 0; b < NB; ++b) y[b] = *reinterpret_cast<const uint2*>(ya + (int64_t)(b0 + b) * 32 * plane + yi);
    const HPRow rw(g, th, c, R);
    sh = rw.sh;
    nvalid = rw.nvalid;
    // one dwordx4 per group at any dword alignment (global loads need only 4-B alignment;
    // tools/micro/head_stream_bw.hip streams this exact pattern with 8-B-misaligned odd rows at
    // 6.1 TB/s).  Only the STORES split misaligned groups (hp_st4).  Classes >= NC read class 0.
#pragma unroll
    for (int j = 0; j < 10; ++j) w[j] = hp_ld4(W + (int64_t)(j < NC ? j : 0) * 32 * QQ + rw.ldoff);
  }
  // re-align the shifted edge groups, zero what lies outside the image and classes >= NC;
  // wave-uniformly skipped for interior chunks with all classes present
  __device__ __forceinline__ void fix(int NC) {
    if (NC == 10 && __builtin_amdgcn_ballot_w64(sh != 0 || nvalid != 4) == 0) return;
#pragma unroll
    for (int j = 0; j < 10; ++j) {
      const float e[4] = {w[j].x, w[j].y, w[j].z, w[j].w};
      float o[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        float v = e[k];
        if (sh > 0) v = (k + sh < 4) ? e[(k + sh) & 3] : 0.f;
        o[k] = (j < NC && k < nvalid) ? v : 0.f;
      }
      w[j] = make_float4(o[0], o[1], o[2], o[3]);
    }
  }
};

// store a 4-group of class j of the weight layout at this thread's (row, 4 columns), inside the image only
__device__ __forceinline__ void hp_store4(float* out, const PBGeom& g, const HPRow& rw, int j, float4 v,
                                          bool nt = true) {
  if (rw.nvalid == 0) return;
  float* p = out + (int64_t)j * 32 * g.Q * (int64_t)g.Q + rw.off;
  if (rw.nvalid == 4) {
    hp_st4(p, rw.al, v, nt);
  } else {
    const float e[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (k < rw.nvalid) hp_st(p + k, e[k], nt);
  }
}

__device__ __forceinline__ float hp_f16(uint32_t h) {  // the low 16 bits as fp16
  return (float)__builtin_bit_cast(_Float16, (unsigned short)(h & 0xFFFFu));
}

// 4 pooled-gradient values as fp16 bits (two packed pairs, element 0 low) at this thread's (row, 4
// columns) of plane j: 8-B, 2 x 4-B or 2-B stores by the row's alignment class
__device__ __forceinline__ void hp_store4h(unsigned short* out, const PBGeom& g, const HPRow& rw, int j, uint32_t lo,
                                           uint32_t hi) {
  if (rw.nvalid == 0) return;
  unsigned short* p = out + (int64_t)j * 32 * g.Q * (int64_t)g.Q + rw.off;
  if (rw.nvalid == 4 && rw.al == 0) {
    st_stream(reinterpret_cast<uint2*>(p), make_uint2(lo, hi));
  } else if (rw.nvalid == 4 && rw.al == 2) {
    st_stream(reinterpret_cast<uint32_t*>(p), lo);
    st_stream(reinterpret_cast<uint32_t*>(p + 2), hi);
  } else {
    const unsigned short e[4] = {(unsigned short)lo, (unsigned short)(lo >> 16), (unsigned short)hi,
                                 (unsigned short)(hi >> 16)};
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (k < rw.nvalid) p[k] = e[k];
  }
}

// Forward.  partial[blk][B*NC] (fp64): this workgroup's share of logits[b][j] for images
// b0 .. b0+NB-1; xout (optional): X in the fc's flatten order, [B][32*Q*Q] -- or, for a launch over
// channels [c0, c1) (the activation exchange's column groups, parallel/factored.py), that range's
// columns as their own [B][(c1-c0)*Q*Q] rows (x_rs = (c1-c0)*Q*Q).
// fin (optional, one pass: B <= HP_MAXB): the logits are finished in this launch -- the last
// workgroup of channel c to arrive sums the channel's rows into fin.cpart[c] (fixed order), the last
// channel to finish sums the 32 channel rows and adds the bias (common.h tds_arrive; replaces
// head_logits_kernel and its launch).
struct HPFin {
  uint32_t* sync;        // 33 counters: [c] per channel, [32] channels
  double* cpart;         // [32][B*NC]
  double* sums;          // [B*NC]
  const float* bias;     // [NC] or nullptr
  float* logits;         // [B*NC]
  // optional: the batch's labels [B] -> the cross-entropy loss (mean, torch's defaults) and dlogits
  // [B*NC] formed by the same workgroup right after the logits (ce_small.h; no separate CE launch)
  const int64_t* labels = nullptr;
  float* dlogits = nullptr;
  float* loss = nullptr;
  float* inv_count = nullptr;
};
template <int NB>
__global__ __launch_bounds__(HP_THREADS) void head_fwd_pb_kernel(const unsigned short* __restrict__ ya,
                                                                 TdsYaDec yd, const float* __restrict__ W,
                                                                 const float* __restrict__ aff2,
                                                                 double* __restrict__ partial,
                                                                 float* __restrict__ xout, PBGeom g, int Btot, int b0,
                                                                 int NC, HPFin fin, int c0, int64_t x_rs,
                                                                 uint32_t* __restrict__ wmaxp) {
  __shared__ float red[HP_THREADS / 64][HP_MAXB * 10];
  __shared__ uint32_t wred[HP_THREADS / 64][10];
  __shared__ int last_flag;
  __shared__ double wpart[256];
  const HPGrid hg = hp_grid(g);
  const int c = c0 + (int)blockIdx.x / hg.per_channel(), band = (int)blockIdx.x - (c - c0) * hg.per_channel();
  const int wg = c * hg.per_channel() + band;  // this workgroup's partial row (all 32 channels' numbering)
  // z = a y + b on the stored h: (a d) h + (a b2 + b)
  const float a = aff2[c], ad = a * hp_ydec(yd.ysc), bd = fmaf(a, yd.b2[c], aff2[32 + c]);
  const int Q = g.Q;
  const int64_t QQ = (int64_t)Q * Q;
  float acc[NB][10];
  float wmx[10];  // max |W[j]| over this workgroup's weights (the backward's fp16 g2m scale)
#pragma unroll
  for (int j = 0; j < 10; ++j) wmx[j] = 0.f;
#pragma unroll
  for (int b = 0; b < NB; ++b)
#pragma unroll
    for (int j = 0; j < 10; ++j) acc[b][j] = 0.f;
  // iteration i: block row R0 + i / nch, chunk (32 blocks) i % nch of the row
  const int nch = (g.Q8 + 31) / 32;
  const int R0 = band * HP_BAND, nit = (min(g.Q4, R0 + HP_BAND) - R0) * nch;
  HPLoad<NB> ld;  // one load set (file header)
  auto issue = [&](HPLoad<NB>& L, int i) { L.issue(ya, W, g, HPThread(i % nch), c, R0 + i / nch, b0, NC); };
  auto body = [&](HPLoad<NB>& cur, int i) {
    const int R = R0 + i / nch;
    const HPThread th(i % nch);
    cur.fix(NC);
    const int py = 4 * R + th.prow, px0 = th.blk * 8 + th.half * 4;
    const bool rok = th.blk < g.Q8 && py < Q;
    const bool xfull = __builtin_amdgcn_ballot_w64(!(rok && px0 + 3 < Q)) == 0;  // wave-uniform
    float x[NB][4];
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      float zz[4];
      hp_fma4(ad, cur.y[b], bd, zz);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float v = hp_relu(zz[k]);
        x[b][k] = (xfull || (rok && px0 + k < Q)) ? v : 0.f;
      }
    }
    if (xout != nullptr) {
      // X rows in the fc's flatten order, an image's row offset (b K + c Q^2 + py Q) has the weight
      // row's alignment (K = 32 Q^2): 16-B stores or float2 pairs as for the weight (hp_store4; 4-B
      // stores per element cost the forward 0.14 ms at the bench shape, r5_s9)
      // (a channel range's own rows start at its first channel: offsets shift by c0 Q^2, a multiple
      // of 4 floats whenever x_rs is -- the host checks -- so the alignment classes are unchanged)
      HPRow rwx(g, th, c, R);
      rwx.off -= (int64_t)c0 * QQ;
#pragma unroll
      for (int b = 0; b < NB; ++b)
        hp_store4(xout + (int64_t)(b0 + b) * x_rs, g, rwx, 0, make_float4(x[b][0], x[b][1], x[b][2], x[b][3]), false);
    }
#pragma unroll
    for (int j = 0; j < 10; ++j) {
      const float4 w4 = cur.w[j];
#pragma unroll
      for (int b = 0; b < NB; ++b)
        acc[b][j] = fmaf(x[b][0], w4.x, fmaf(x[b][1], w4.y, fmaf(x[b][2], w4.z, fmaf(x[b][3], w4.w, acc[b][j]))));
      // (fix() zeroed the lanes outside the image and the classes >= NC)
      wmx[j] = fmaxf(fmaxf(wmx[j], fmaxf(fabsf(w4.x), fabsf(w4.y))), fmaxf(fabsf(w4.z), fabsf(w4.w)));
    }
  };
#pragma unroll 1
  for (int i = 0; i < nit; ++i) {
    issue(ld, i);
    body(ld, i);
  }
  // deterministic workgroup reduction: waves (DPP), then 4 wave partials in fixed order
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int b = 0; b < NB; ++b)
#pragma unroll
    for (int j = 0; j < 10; ++j) {
      if (j < NC) {
        const float s = wave_sum(acc[b][j]);
        if (lane == 0) red[wv][b * 10 + j] = s;
      }
    }
#pragma unroll
  for (int j = 0; j < 10; ++j) {
    const uint32_t m = wave_max(__float_as_uint(wmx[j]));  // (non-negative: bits order as values)
    if (lane == 0) wred[wv][j] = m;
  }
  __syncthreads();
  if (wmaxp != nullptr && (int)threadIdx.x < 10) {
    const int j = threadIdx.x;
    wmaxp[(int64_t)wg * 10 + j] = max(max(wred[0][j], wred[1][j]), max(wred[2][j], wred[3][j]));
  }
  for (int i = threadIdx.x; i < NB * NC; i += HP_THREADS) {
    const int b = i / NC, j = i - b * NC;
    const double s = (((double)red[0][b * 10 + j] + (double)red[1][b * 10 + j]) + (double)red[2][b * 10 + j]) +
                     (double)red[3][b * 10 + j];
    st_agent(partial + (int64_t)wg * Btot * NC + (b0 + b) * NC + j, s);  // (write-through: tds_arrive)
  }
  if (fin.sync == nullptr) return;
  const int BN = Btot * NC, nb = hg.per_channel();
  if (!tds_arrive(fin.sync + c, (uint32_t)nb, &last_flag)) return;
  // this channel's rows (one round of loads behind tds_arrive's acquire; host: BN <= 80, nb <= 48)
  {
    const double s = wide_row_sum(partial + (int64_t)c * nb * BN, nb, BN, BN, wpart);
    if ((int)threadIdx.x < BN) st_agent(fin.cpart + (int64_t)c * BN + threadIdx.x, s);
  }
  if (!tds_arrive(fin.sync + 32, 32u, &last_flag)) return;
  const double s = wide_row_sum(fin.cpart, 32, BN, BN, wpart);
  __shared__ float lg[HP_MAXB * 10];
  if ((int)threadIdx.x < BN) {
    const float z = (float)s + (fin.bias ? fin.bias[threadIdx.x % NC] : 0.f);
    fin.sums[threadIdx.x] = s;
    fin.logits[threadIdx.x] = z;
    lg[threadIdx.x] = z;
  }
  if (fin.labels == nullptr) return;
  __syncthreads();
  ce_small_block(lg, fin.labels, fin.dlogits, fin.loss, fin.inv_count, Btot, NC, -100, 0.f);
}

// sums[i] = sum_k partial[k][i] (fixed order), logits[i] = sums[i] + bias[i % NC]: one workgroup
// per logit, the cross-workgroup reduction and the bias in one launch
__global__ __launch_bounds__(256) void head_logits_kernel(const double* __restrict__ partial, int nwg,
                                                          double* __restrict__ sums, const float* __restrict__ bias,
                                                          float* __restrict__ logits, int BN, int NC) {
  __shared__ double sh[8];
  const int i = blockIdx.x;
  double s = 0.0;
  for (int k = threadIdx.x; k < nwg; k += blockDim.x) s += partial[(int64_t)k * BN + i];
  s = block_sum(s, sh);
  if (threadIdx.x == 0) {
    sums[i] = s;
    logits[i] = (float)s + (bias ? bias[i % NC] : 0.f);
  }
}

// Backward for images b0 .. b0+NB-1.
//   g2m[b][c][py][px] = (sum_j dl[b][j] W[j][c][py][px]) * [a*ya + b > 0]   (planar [B][32][Q][Q])
//   partial[c][pass*nblk + blk][4] = { sum g2m, sum g2m * ya } over the fp32 values (dgamma2,
//                                    dbeta2), then the same over the stored fp16 values (k2, k3)
//   dW[j][c][pos] (= or +=) scale * sum_b dl[b][j] X[b][c][pos]      (WITH_DW; ACC adds)
//   Wupd = W - lr * dW                                               (UPD: SGD step fused)
//   gpart (optional): this workgroup's max |g2m| as float bits (NaN-propagating as an unsigned
//   max), at [(c*npass + pass)*nblk + band] -- reduced by the BN2-backward finalize into the
//   magnitude bound behind the conv2 backward's fp16 scale (conv2_bwd.hip).  Plain stores: one
//   same-address atomic per wave cost ~40 us per step (12.8 K of them at 3000^2).
// KEEP: dW is also stored (UPD without KEEP: the update only -- optimizer-in-backward semantics,
// the gradient itself is never materialised, 720 MB less written at 3000^2).
// fin (optional; one pass over all 32 channels): the BN2 backward finalize in this launch (replaces
// bn_bwd_finalize2_kernel): the last workgroup of channel c to arrive sums the channel's BN2 partials
// (band order) into dgamma / dbeta / the dy2 constants k1..k3 and its max |g2m|; the last channel
// to finish writes mag[32] (the max over channels) and the fc bias gradient.
struct HBFin {
  uint32_t* sync;          // 33 counters
  uint32_t* cmax;          // [32] per-channel max |g2m| bits
  const float* stats;      // [64] mean | invstd of BN2
  const float* gamma;      // [32] or nullptr
  float* dgamma;           // [32] or nullptr
  float* dbeta;            // [32] or nullptr
  float* kbuf;             // [96] k1 | k2 | k3
  int64_t n;               // B * P * P
  int B;
  float* dbfc;             // [NC] or nullptr
  float scale;
  uint32_t* mag;           // mag[32] <- max |g2m| (nullptr: no magnitude bound)
};

template <int NB, bool WITH_DW, bool ACC, bool UPD, bool KEEP = true>
__global__ __launch_bounds__(HP_THREADS) void head_bwd_pb_kernel(
    const unsigned short* __restrict__ ya, TdsYaDec yd, const float* W, const float* __restrict__ aff2,
    const float* __restrict__ dl,
    unsigned short* __restrict__ g2h, double* __restrict__ partial, float* dW, float* Wupd, PBGeom g, int b0, int pass,
    int npass, int NC, float scale, float lr, int c0, uint32_t* __restrict__ gpart, HBFin fin,
    const uint32_t* __restrict__ wmaxp, int wrows, int Btot, float* __restrict__ g2inv) {
  __shared__ float red[4][HP_THREADS / 64];
  __shared__ uint32_t wms[10];
  __shared__ float g2sc;
  __shared__ uint32_t gred[HP_THREADS / 64];
  __shared__ double dred[4][HP_THREADS / 64];
  __shared__ int last_flag;
  const HPGrid hg = hp_grid_b(g);
  // workgroups in the reverse of the forward's order: the backward starts on the channels the
  // forward streamed last, whose ya / weight lines are still in the 256 MB Infinity Cache
  const int wg = (int)gridDim.x - 1 - (int)blockIdx.x;
  const int c = c0 + wg / hg.per_channel(), band = wg - (c - c0) * hg.per_channel();
  float dls[NB * 10];  // dlogits of this pass: wave-uniform, scalar loads
#pragma unroll
  for (int b = 0; b < NB; ++b)
#pragma unroll
    for (int j = 0; j < 10; ++j) dls[b * 10 + j] = j < NC ? dl[(b0 + b) * NC + j] : 0.f;
  // g2m's fp16 scale for channel c: |g2m[b][c][.]| <= sum_j |dl[b][j]| max |W[j][c][.]| (the forward
  // measured the maxima, wmaxp: wrows rows per channel); the power of two 2^e puts that bound below
  // 2^14 (fp16 holds to 65504; ~28 binades of full precision below the bound).  Every workgroup of
  // the channel forms the same e from the same data; the consumers get 2^-e (g2inv[c]).
  if (threadIdx.x < 10) wms[threadIdx.x] = 0u;
  __syncthreads();
  for (int i = threadIdx.x; i < wrows * 10; i += HP_THREADS)
    atomicMax(&wms[i % 10], wmaxp[((int64_t)c * wrows + i / 10) * 10 + i % 10]);
  __syncthreads();
  if (threadIdx.x < 64) {
    float s = 0.f;
    if ((int)threadIdx.x < Btot)
      for (int j = 0; j < NC; ++j) s = fmaf(fabsf(dl[threadIdx.x * NC + j]), __uint_as_float(wms[j]), s);
    const float bound = __uint_as_float(wave_max(__float_as_uint(s)));  // (NaN: bits above inf -> no scale)
    if (threadIdx.x == 0) {
      int e = 0;
      if (bound > 0.f && __builtin_isfinite(bound)) {
        int x;
        (void)frexpf(bound, &x);  // bound < 2^x
        e = min(100, max(-100, 14 - x));
      }
      g2sc = ldexpf(1.f, e);
      if (g2inv != nullptr && band == 0 && pass == 0) g2inv[c] = ldexpf(1.f, -e);
    }
  }
  __syncthreads();
  const float gsc = g2sc, ginv = 1.f / g2sc;  // (powers of two: exact)
  // z = a y + b on the stored h as in the forward; y = h d + b2 itself for the BN2 sums
  const float a = aff2[c], yds = hp_ydec(yd.ysc), ad = a * yds, b2c = yd.b2[c], bd = fmaf(a, b2c, aff2[32 + c]);
  const int Q = g.Q;
  const int64_t plane = g.plane();
  float sdz = 0.f, sdy = 0.f, sdzr = 0.f, sdyr = 0.f;  // (r: the stored values)
  uint32_t gmx = 0u;  // max |g2m| bits
  const int nch = (g.Q8 + 31) / 32;
  const int R0 = band * HP_BAND_B, nit = (min(g.Q4, R0 + HP_BAND_B) - R0) * nch;
  HPLoad<NB> ld;  // one load set, as in the forward
  auto issue = [&](HPLoad<NB>& L, int i) { L.issue(ya, W, g, HPThread(i % nch), c, R0 + i / nch, b0, NC); };
  auto body = [&](HPLoad<NB>& cur, int i) {
    const int R = R0 + i / nch;
    const HPThread th(i % nch);
    cur.fix(NC);
    const bool bok = th.blk < g.Q8;
    const int py = 4 * R + th.prow, px0 = th.blk * 8 + th.half * 4;
    const bool rok = bok && py < Q;
    const HPRow rwg(g, th, c, R);
    float x[NB][4];
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      float zz[4], yy[4];
      hp_fma4(ad, cur.y[b], bd, zz);
      hp_fma4(yds, cur.y[b], b2c, yy);
      float gm[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const bool ok = rok && px0 + k < Q;
        const float z = zz[k];
        float gs = 0.f;
#pragma unroll
        for (int j = 0; j < 10; ++j) {
          const float wk = k == 0 ? cur.w[j].x : k == 1 ? cur.w[j].y : k == 2 ? cur.w[j].z : cur.w[j].w;
          gs = fmaf(dls[b * 10 + j], wk, gs);
        }
        gm[k] = (ok && z > 0.f) ? gs : 0.f;
        x[b][k] = ok ? hp_relu(z) : 0.f;
        sdz += gm[k];
        sdy = fmaf(gm[k], ok ? yy[k] : 0.f, sdy);
      }
      // planar, like a weight plane, in fp16 at 2^e_c.  dy2's constants k2, k3 and the magnitude bound
      // take the sums over the values as stored (the conv2 backward's dz): sum dy2 over the channel
      // stays 0 in exact arithmetic, as torch's, instead of carrying k1 times the sum of g2m's rounding
      // errors; dgamma2 / dbeta2 keep the fp32 values' sums
      const uint32_t lo = cvt2_f16(gm[0] * gsc, gm[1] * gsc), hi = cvt2_f16(gm[2] * gsc, gm[3] * gsc);
      hp_store4h(g2h, g, rwg, b0 + b, lo, hi);
      const float gr[4] = {hp_f16(lo) * ginv, hp_f16(lo >> 16) * ginv, hp_f16(hi) * ginv, hp_f16(hi >> 16) * ginv};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        gmx = max(gmx, __float_as_uint(gr[k]) & 0x7fffffffu);
        sdzr += gr[k];
        sdyr = fmaf(gr[k], (rok && px0 + k < Q) ? yy[k] : 0.f, sdyr);
      }
    }
    if constexpr (WITH_DW) {
      const HPRow& rw = rwg;
#pragma unroll
      for (int j = 0; j < 10; ++j) {
        if (j < NC) {
          float s[4];
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            float v = 0.f;
#pragma unroll
            for (int b = 0; b < NB; ++b) v = fmaf(dls[b * 10 + j], x[b][k], v);
            s[k] = scale * v;
          }
          float4 d = make_float4(s[0], s[1], s[2], s[3]);
          if constexpr (ACC) {  // later image passes add to the stored dW
            if (rw.nvalid > 0) {
              float* p = dW + (int64_t)j * 32 * Q * (int64_t)Q + rw.off;
#pragma unroll
              for (int k = 0; k < 4; ++k)
                if (k < rw.nvalid) p[k] += s[k];
            }
          } else {
            if constexpr (KEEP) hp_store4(dW, g, rw, j, d);
            if constexpr (UPD) {  // torch SGD: p -= lr * g
              const float4 w = cur.w[j];
              hp_store4(Wupd, g, rw, j, make_float4(w.x - lr * d.x, w.y - lr * d.y, w.z - lr * d.z, w.w - lr * d.w));
            }
          }
        }
      }
    }
  };
#pragma unroll 1
  for (int i = 0; i < nit; ++i) {
    issue(ld, i);
    body(ld, i);
  }
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  gmx = wave_max(gmx);
  sdz = wave_sum(sdz);
  sdy = wave_sum(sdy);
  sdzr = wave_sum(sdzr);
  sdyr = wave_sum(sdyr);
  if (lane == 0) {
    red[0][wv] = sdz;
    red[1][wv] = sdy;
    red[2][wv] = sdzr;
    red[3][wv] = sdyr;
    gred[wv] = gmx;
  }
  __syncthreads();
  if (gpart != nullptr && threadIdx.x == 0) {
    uint32_t m = gred[0];
#pragma unroll
    for (int i = 1; i < HP_THREADS / 64; ++i) m = max(m, gred[i]);
    st_agent(gpart + ((int64_t)c * npass + pass) * hg.per_channel() + band, m);  // (write-through: tds_arrive)
  }
  if (threadIdx.x < 4) {
    const int k = threadIdx.x;
    const double s = (((double)red[k][0] + (double)red[k][1]) + (double)red[k][2]) + (double)red[k][3];
    const int64_t nblk = (int64_t)hg.per_channel();
    st_agent(partial + (((int64_t)c * npass + pass) * nblk + band) * 4 + k, s);
  }
  if (fin.sync == nullptr) return;
  const int nb = hg.per_channel();
  if (!tds_arrive(fin.sync + c, (uint32_t)nb, &last_flag)) return;
  {  // channel c: its bands in order (one pass: partial row = c * nb + band)
    double sd[4] = {0.0, 0.0, 0.0, 0.0};
    uint32_t m = 0u;
    for (int k = lane + 64 * wv; k < nb; k += HP_THREADS) {  // (nb <= 256 at Q <= 2044: one load each)
      const double2 v = *reinterpret_cast<const double2*>(partial + ((int64_t)c * nb + k) * 4);
      const double2 vr = *reinterpret_cast<const double2*>(partial + ((int64_t)c * nb + k) * 4 + 2);
      sd[0] += v.x;
      sd[1] += v.y;
      sd[2] += vr.x;
      sd[3] += vr.y;
      if (gpart != nullptr) m = max(m, gpart[(int64_t)c * nb + k]);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) sd[i] = wave_sum(sd[i]);
    m = wave_max(m);
    if (lane == 0) {
#pragma unroll
      for (int i = 0; i < 4; ++i) dred[i][wv] = sd[i];
      gred[wv] = m;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
#pragma unroll
      for (int i = 0; i < 4; ++i) sd[i] = ((dred[i][0] + dred[i][1]) + dred[i][2]) + dred[i][3];
      m = max(max(gred[0], gred[1]), max(gred[2], gred[3]));
      st_agent(fin.cmax + c, m);
      const double mean = fin.stats[c], is = fin.stats[32 + c];
      const double gm = fin.gamma ? fin.gamma[c] : 1.0;
      const double sdxh = sd[1] - mean * sd[0];  // sum dz*(y-mean), fp32 dz
      if (fin.dgamma) fin.dgamma[c] = (float)(is * sdxh);
      if (fin.dbeta) fin.dbeta[c] = (float)sd[0];
      const double sdxr = sd[3] - mean * sd[2];  // the same over the stored dz
      const double k1 = gm * is;
      const double k2 = -gm * is * is * is * sdxr / (double)fin.n;
      const double k3 = -gm * is * sd[2] / (double)fin.n - k2 * mean;
      fin.kbuf[c] = (float)k1;
      fin.kbuf[32 + c] = (float)k2;
      fin.kbuf[64 + c] = (float)k3;
    }
  }
  if (!tds_arrive(fin.sync + 32, 32u, &last_flag)) return;
  if (threadIdx.x < 64) {
    const uint32_t m = wave_max(threadIdx.x < 32 ? fin.cmax[threadIdx.x] : 0u);
    if (threadIdx.x == 0 && fin.mag != nullptr) fin.mag[32] = m;
  } else if (fin.dbfc != nullptr && (int)threadIdx.x - 64 < NC) {
    const int j = (int)threadIdx.x - 64;
    float v = 0.f;
    for (int b = 0; b < fin.B; ++b) v += dl[b * NC + j];
    fin.dbfc[j] = v * fin.scale;
  }
}

// The activation exchange's fc step from every rank's POOLED input (parallel/factored.py, source
// "pooled"): the ranks all-gather ya (fp16, 36 MB per image at 3000^2, half of X in fp32 and no
// encode) and a 128-float record of the head constants their forward used; every rank then forms
//   MODE 0: W -= lr * scale * sum_m dl[m] (x) X_m        (update only, the SGD step)
//   MODE 1: out = scale * sum_m dl[m] (x) X_m             (dW)
//   MODE 2: out += scale * sum_m dl[m] (x) X_m
// with X_m recomputed from rank r's ya as its head forward did (m = r * NB + b; rec[r]: aff2 [64] |
// ya scale words [3] | pad | b2 [32] | pad): the same v_fma_mix arithmetic on the same values, so
// X is bitwise the rows that forward multiplied by the weight.  Workgroup = (channel, band of the
// backward's HP_BAND_B block rows), 4 columns of one pooled row per thread as the head kernels;
// per chunk the weight 4-groups are loaded once and every rank's images stream past them.
constexpr int HP_REC = 128;  // floats per rank record

template <int NB, int MODE>
__global__ __launch_bounds__(HP_THREADS) void head_upd_pb_kernel(const unsigned short* __restrict__ ya_all,
                                                                 int64_t ya_rs, const float* __restrict__ rec,
                                                                 int nranks, const float* __restrict__ dl,
                                                                 const float* W, float* out, PBGeom g, int NC,
                                                                 float scale, float lr) {
  const HPGrid hg = hp_grid_b(g);
  const int c = (int)blockIdx.x / hg.per_channel(), band = (int)blockIdx.x - c * hg.per_channel();
  const int Q = g.Q;
  const int64_t plane = g.plane();
  const int nch = (g.Q8 + 31) / 32;
  const int R0 = band * HP_BAND_B, nit = (min(g.Q4, R0 + HP_BAND_B) - R0) * nch;
#pragma unroll 1
  for (int i = 0; i < nit; ++i) {
    const int R = R0 + i / nch;
    const HPThread th(i % nch);
    HPLoad<NB> cur;  // the weight 4-groups and rank 0's images
    cur.issue(ya_all, W, g, th, c, R, 0, NC);
    cur.fix(NC);
    const int py = 4 * R + th.prow, px0 = th.blk * 8 + th.half * 4;
    const bool rok = th.blk < g.Q8 && py < Q;
    const int64_t yi = (((int64_t)c * g.Q4 + R) * g.Q8 + (th.blk < g.Q8 ? th.blk : g.Q8 - 1)) * 32 + th.part * 4;
    float acc[10][4];
#pragma unroll
    for (int j = 0; j < 10; ++j)
#pragma unroll
      for (int k = 0; k < 4; ++k) acc[j][k] = 0.f;
#pragma unroll 1
    for (int r = 0; r < nranks; ++r) {
      uint2 y[NB];
      if (r == 0) {
#pragma unroll
        for (int b = 0; b < NB; ++b) y[b] = cur.y[b];
      } else {
#pragma unroll
        for (int b = 0; b < NB; ++b)
          y[b] = *reinterpret_cast<const uint2*>(ya_all + r * ya_rs + (int64_t)b * 32 * plane + yi);
      }
      // rank r's head constants, formed as its head kernels formed them (head_fwd_pb_kernel)
      const float* rr = rec + (int64_t)r * HP_REC;
      const TdsYaDec yd{rr + 68, reinterpret_cast<const uint32_t*>(rr + 64)};
      const float a = rr[c], ad = a * hp_ydec(yd.ysc), bd = fmaf(a, yd.b2[c], rr[32 + c]);
#pragma unroll
      for (int b = 0; b < NB; ++b) {
        float zz[4];
        hp_fma4(ad, y[b], bd, zz);
        float x[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) x[k] = (rok && px0 + k < Q) ? hp_relu(zz[k]) : 0.f;
#pragma unroll
        for (int j = 0; j < 10; ++j) {
          if (j < NC) {
            const float dv = dl[(r * NB + b) * NC + j];
#pragma unroll
            for (int k = 0; k < 4; ++k) acc[j][k] = fmaf(dv, x[k], acc[j][k]);
          }
        }
      }
    }
    const HPRow rw(g, th, c, R);
#pragma unroll
    for (int j = 0; j < 10; ++j) {
      if (j < NC) {
        const float4 d = make_float4(scale * acc[j][0], scale * acc[j][1], scale * acc[j][2], scale * acc[j][3]);
        if constexpr (MODE == 0) {
          const float4 w = cur.w[j];
          hp_store4(out, g, rw, j, make_float4(w.x - lr * d.x, w.y - lr * d.y, w.z - lr * d.z, w.w - lr * d.w));
        } else if constexpr (MODE == 1) {
          hp_store4(out, g, rw, j, d);
        } else if (rw.nvalid > 0) {
          float* p = out + (int64_t)j * 32 * Q * (int64_t)Q + rw.off;
          const float e[4] = {d.x, d.y, d.z, d.w};
#pragma unroll
          for (int k = 0; k < 4; ++k)
            if (k < rw.nvalid) p[k] += e[k];
        }
      }
    }
  }
}

// one rank's record (HP_REC floats): aff2 [64] | the ya scale words [3] (1, 1, 1 without) | 0 | b2 [32] | 0
__global__ __launch_bounds__(HP_REC) void hp_record_kernel(const float* __restrict__ aff2, const float* __restrict__ b2,
                                                          const uint32_t* __restrict__ ysc, float* __restrict__ rec) {
  const int t = threadIdx.x;
  float v = 0.f;
  if (t < 64) v = aff2[t];
  else if (t < 67) v = ysc != nullptr ? __uint_as_float(ysc[t - 64]) : 1.f;
  else if (t >= 68 && t < 100) v = b2[t - 68];
  rec[t] = v;
}

}  // namespace tds

using namespace tds;

void tds_head_pooled_record(const float* aff2, const float* b2, const uint32_t* ysc, float* rec, hipStream_t st) {
  hipLaunchKernelGGL(hp_record_kernel, dim3(1), dim3(HP_REC), 0, st, aff2, b2, ysc, rec);
  TDS_LAUNCH_CHECK();
}

int tds_head_upd_pb(const unsigned short* ya_all, int64_t ya_rs, const float* rec, int nranks, const float* dl,
                    const float* W, float* out, int B, int Q, int NC, float scale, float lr, int mode, hipStream_t st) {
  if (B < 1 || B > HP_MAXB || NC < 1 || NC > 10 || Q < 4 || nranks < 1 || mode < 0 || mode > 2) return -1;
  const PBGeom g = pb_geom(Q);
  const int nwg = 32 * hp_grid_b(g).per_channel();
#define TDS_HPU_M(NBV, MD)                                                                                        \
  hipLaunchKernelGGL((head_upd_pb_kernel<NBV, MD>), dim3(nwg), dim3(HP_THREADS), 0, st, ya_all, ya_rs, rec, nranks, \
                     dl, W, out, g, NC, scale, lr);
#define TDS_HPU(NBV)                                    \
  case NBV:                                             \
    if (mode == 0) {                                    \
      TDS_HPU_M(NBV, 0)                                 \
    } else if (mode == 1) {                             \
      TDS_HPU_M(NBV, 1)                                 \
    } else {                                            \
      TDS_HPU_M(NBV, 2)                                 \
    }                                                   \
    break;
  switch (B) {
    TDS_HPU(1) TDS_HPU(2) TDS_HPU(3) TDS_HPU(4) TDS_HPU(5) TDS_HPU(6) TDS_HPU(7) TDS_HPU(8)
    default: return -1;
  }
#undef TDS_HPU
#undef TDS_HPU_M
  TDS_LAUNCH_CHECK();
  return 0;
}

// The forward's per-workgroup max |W[j]| ([32 * nblk][10] float bits), read by the next head backward
// on the same stream for g2m's fp16 scale: one buffer per (device, stream), the forward and the
// backward of one step see the same weight (the fused SGD step runs inside the backward, the
// exchange's update before the forward)
static uint32_t* hp_wmax_buf(int Q, hipStream_t st) {
  const size_t n = (size_t)32 * hp_grid(pb_geom(Q)).per_channel() * 10;
  return reinterpret_cast<uint32_t*>(tds_zeroed_u64(1, (n + 1) / 2, st));
}

int tds_head_pb_nblk(int Q) { return hp_grid(pb_geom(Q)).per_channel(); }  // forward workgroups per channel
int tds_head_bwd_pb_nblk(int Q) { return hp_grid_b(pb_geom(Q)).per_channel(); }  // backward workgroups per channel
int64_t tds_pb_plane(int Q) { return pb_geom(Q).plane(); }

// partial: double [32 * nblk + 32][B*NC] (the last 32 rows: the in-launch finalizer's channel sums);
// sums: double [B*NC].  fused_fin = false: the separate head_logits launch (the A/B reference).
// [c0, c1) != [0, 32): this launch covers those channels only (in-launch finalize required: the
// logits are finished by the launch that completes the 32nd channel, so a step's range launches
// share partial / sums / logits and run on one stream); xout then holds the range's own rows.
int tds_head_fwd_pb(const unsigned short* ya, TdsYaDec yd, const float* Wfc, const float* bias, const float* aff2, double* partial,
                    double* sums, float* logits, float* xout, int B, int Q, int NC, hipStream_t st, bool fused_fin,
                    const int64_t* labels, float* dlogits, float* loss, float* inv_count, int c0, int c1) {
  if (B < 1 || NC < 1 || NC > 10 || Q < 1 || c0 < 0 || c1 > 32 || c0 >= c1) return -1;
  const PBGeom g = pb_geom(Q);
  const bool range = c0 != 0 || c1 != 32;
  const int64_t QQ = (int64_t)Q * Q, x_rs = (int64_t)(c1 - c0) * QQ;
  if (range && (x_rs % 4 != 0 || ((int64_t)c0 * QQ) % 4 != 0)) return -1;  // (X alignment classes, above)
  const int nwg = (c1 - c0) * hp_grid(g).per_channel();
  // one pass: the logits are finished inside the launch (HPFin; partial then holds nwg + 32 rows)
  HPFin fin{nullptr, nullptr, nullptr, nullptr, nullptr};
  const int BN = B * NC, nbc = hp_grid(g).per_channel();
  const bool wide_ok = BN <= 256 && nbc <= WRS_MAXL * (256 / BN) && 32 <= WRS_MAXL * (256 / BN);
  if (B <= HP_MAXB && fused_fin && wide_ok && tds_fused_fin_enabled()) {
    fin.sync = tds_sync_words(kSyncHeadFwd, st);
    fin.cpart = partial + (int64_t)32 * nbc * B * NC;
    fin.sums = sums;
    fin.bias = bias;
    fin.logits = logits;
    fin.labels = labels;
    fin.dlogits = dlogits;
    fin.loss = loss;
    fin.inv_count = inv_count;
  }
  if (range && fin.sync == nullptr) return -1;
  uint32_t* wmaxp = hp_wmax_buf(Q, st);
  if (wmaxp == nullptr) return -2;
  for (int b0 = 0; b0 < B; b0 += HP_MAXB) {
    const int nb = B - b0 < HP_MAXB ? B - b0 : HP_MAXB;
#define TDS_HPF(NBV)                                                                                                   \
  case NBV:                                                                                                            \
    hipLaunchKernelGGL((head_fwd_pb_kernel<NBV>), dim3(nwg), dim3(HP_THREADS), 0, st, ya, yd, Wfc, aff2, partial, xout, g, \
                       B, b0, NC, fin, c0, x_rs, wmaxp);                                                               \
    TDS_LAUNCH_CHECK();                                                                                                \
    break;
    switch (nb) {
      TDS_HPF(1) TDS_HPF(2) TDS_HPF(3) TDS_HPF(4) TDS_HPF(5) TDS_HPF(6) TDS_HPF(7) TDS_HPF(8)
      default: return -1;
    }
#undef TDS_HPF
  }
  if (fin.sync != nullptr) return labels != nullptr ? 1 : 0;
  hipLaunchKernelGGL(head_logits_kernel, dim3(BN), dim3(256), 0, st, partial, nwg, sums, bias, logits, BN, NC);
  TDS_LAUNCH_CHECK();
  return 0;
}

// partial: double [32][npass * nblk][2], npass = ceil(B / 8)
int tds_head_bwd_pb_npass(int B) { return (B + HP_MAXB - 1) / HP_MAXB; }

int tds_head_bwd_pb(const unsigned short* ya, TdsYaDec yd, const float* Wfc, const float* aff2, const float* dlogits, unsigned short* g2m,
                    double* partial, float* dW, float* Wupd, int B, int Q, int NC, float scale, float lr, int c0,
                    int c1, uint32_t* gpart, float* g2inv, hipStream_t st, const TdsHeadBwdFin* hf) {
  if (B < 1 || NC < 1 || NC > 10 || Q < 1 || c0 < 0 || c1 > 32 || c0 >= c1) return -1;
  const uint32_t* wmaxp = hp_wmax_buf(Q, st);
  if (wmaxp == nullptr) return -5;
  const int wrows = hp_grid(pb_geom(Q)).per_channel();
  const int npass = tds_head_bwd_pb_npass(B);
  if (Wupd && npass != 1) return -2;  // the fused SGD step needs the whole dW in one pass
  const PBGeom g = pb_geom(Q);
  HBFin fin{};
  if (hf != nullptr) {
    if (npass != 1 || c0 != 0 || c1 != 32 || hp_grid_b(g).per_channel() > HP_THREADS) return -3;
    fin.sync = tds_sync_words(kSyncHeadBwd, st);
    if (fin.sync == nullptr) return -4;
    fin.cmax = hf->cmax;
    fin.stats = hf->stats;
    fin.gamma = hf->gamma;
    fin.dgamma = hf->dgamma;
    fin.dbeta = hf->dbeta;
    fin.kbuf = hf->kbuf;
    fin.n = (int64_t)B * (2 * Q) * (2 * Q);
    fin.B = B;
    fin.dbfc = hf->dbfc;
    fin.scale = scale;
    fin.mag = hf->mag;
  }
  const int nwg = (c1 - c0) * hp_grid_b(g).per_channel();
  for (int pass = 0; pass < npass; ++pass) {
    const int b0 = pass * HP_MAXB;
    const int nb = B - b0 < HP_MAXB ? B - b0 : HP_MAXB;
    const bool acc = pass > 0;
#define TDS_HPB_E(NBV, WD, AC, UP, KP)                                                                             \
  hipLaunchKernelGGL((head_bwd_pb_kernel<NBV, WD, AC, UP, KP>), dim3(nwg), dim3(HP_THREADS), 0, st, ya, yd, Wfc, aff2, \
                     dlogits, g2m, partial, dW, Wupd, g, b0, pass, npass, NC, scale, lr, c0, gpart, fin, wmaxp, wrows, \
                     B, g2inv);
#define TDS_HPB(NBV)                                   \
  case NBV:                                            \
    if (!dW && Wupd) {                                 \
      TDS_HPB_E(NBV, true, false, true, false)         \
    } else if (!dW) {                                  \
      TDS_HPB_E(NBV, false, false, false, true)        \
    } else if (acc) {                                  \
      TDS_HPB_E(NBV, true, true, false, true)          \
    } else if (Wupd) {                                 \
      TDS_HPB_E(NBV, true, false, true, true)          \
    } else {                                           \
      TDS_HPB_E(NBV, true, false, false, true)         \
    }                                                  \
    TDS_LAUNCH_CHECK();                                \
    break;
    switch (nb) {
      TDS_HPB(1) TDS_HPB(2) TDS_HPB(3) TDS_HPB(4) TDS_HPB(5) TDS_HPB(6) TDS_HPB(7) TDS_HPB(8)
      default: return -1;
    }
#undef TDS_HPB
#undef TDS_HPB_E
  }
  return 0;
}
