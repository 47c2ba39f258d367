// Zero-suppressed encoding of the fc input rows X for the fc-gradient exchanges
// (parallel/zs.py has the format and the torch reference; parallel/factored.py the protocol).
// X is a ReLU output; the exchange sends its non-zero values plus a bitmask and rebuilds X bit
// for bit, so the exchanged gradient is bitwise the dense exchange's.
//
// Pages of 2048 flat elements, one 256-thread workgroup per page, thread t owns elements
// 8t .. 8t+7 of its page (one byte of the mask).  meta[p*65] = the page's value offset,
// meta[p*65 + 1 + j] = mask word j (bit i <-> element 32j + i, "non-zero" = any bit set).
//   encode: zs_encode -- ONE pass over X, 8 pages per workgroup: mask words, the counts, the
//           tile's value offset by a decoupled look-back over the preceding tiles' published
//           counts, and the values compacted through LDS into coalesced stores (dropped past
//           the capacity).  (Three
//           passes -- count, a one-workgroup scan, compaction -- took 71 + 80 + 143 us at the
//           3000^2 bench shape, on the compute stream.)
//   decode: zs_expand (values back to their places, zeros elsewhere)
// The segmented form (zs_seg_*, the sharded exchange) keeps the three-pass scheme: its offsets
// restart per segment.
#include <map>
#include <mutex>
#include <tuple>
#include <type_traits>

#include "common.h"
#include "launchers.h"
#include "pooled_layout.h"

namespace tds {

constexpr int ZS_PAGE = 2048;
constexpr int ZS_META = 1 + ZS_PAGE / 32;

// this thread's 8 elements as raw bits (zeros past n)
__device__ __forceinline__ void zs_load8(const uint32_t* __restrict__ x, int64_t e0, int64_t n, uint32_t (&v)[8]) {
  if (e0 + 8 <= n && (e0 & 3) == 0 && (reinterpret_cast<uintptr_t>(x) & 15) == 0) {
    const uint4 a = *reinterpret_cast<const uint4*>(x + e0), b = *reinterpret_cast<const uint4*>(x + e0 + 4);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  } else {
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = e0 + i < n ? x[e0 + i] : 0u;
  }
}

__device__ __forceinline__ uint32_t zs_byte(const uint32_t (&v)[8]) {
  uint32_t m = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) m |= (v[i] != 0u ? 1u : 0u) << i;
  return m;
}

// exclusive prefix of one value per thread over the 256-thread workgroup (+ the total)
__device__ __forceinline__ int zs_block_scan(int v, int* sh, int& total) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  int incl = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int o = __shfl_up(incl, d, 64);
    if (lane >= d) incl += o;
  }
  if (lane == 63) sh[wv] = incl;
  __syncthreads();
  int base = 0;
  total = 0;
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    const int s = sh[w];
    if (w < wv) base += s;
    total += s;
  }
  __syncthreads();
  return base + incl - v;
}

// Single-pass encode over TILES of ZS_TILE pages (one workgroup each, the tile's X in
// registers: 8 elements x 8 pages per thread).  Tile order is the order workgroups START (a
// ticket from a counter; the workgroup drawing the last ticket resets it for the next call), so
// every tile a workgroup looks back at belongs to a workgroup already running or done -- nothing
// depends on the dispatcher's order or placement (cdna_hip_programming.md, Guideline 16).  Each
// tile publishes a 64-bit status word (the value travels inside the atomic word: no payload to
// make visible): [63:40] the call's epoch (24 bits; words of earlier calls never match), [39:38]
// 1 = the tile's own count, 2 = its inclusive prefix, [37:0] the value.  Wave 0 walks back from
// tile t-1, 64 tiles per round (one status word per lane), adding counts up to the nearest
// inclusive prefix.  Measured at the bench shape (44 K pages): one page per workgroup spent
// 550-590 us in the single ticket counter's same-address atomics and the walk; 8 pages per
// workgroup cut both by 8x.  Status words and the counter belong to one (device, stream).
constexpr int ZS_ST_VAL = 38, ZS_ST_EPOCH = 40;
constexpr int ZS_TILE = 8;

__device__ __forceinline__ void zs_status_store(unsigned long long* p, unsigned long long v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned long long zs_status_load(unsigned long long* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <class SRC>
__global__ __launch_bounds__(256) void zs_encode_kernel(SRC x, int64_t n, int64_t npages,
                                                        int* __restrict__ meta, uint32_t* __restrict__ vals,
                                                        int64_t cap, int64_t* __restrict__ nnz,
                                                        unsigned long long* __restrict__ status,
                                                        unsigned long long* __restrict__ ticket,
                                                        unsigned long long epoch) {
  __shared__ uint32_t bytes[ZS_TILE][256];
  __shared__ uint32_t lv[ZS_PAGE];
  __shared__ int sh[4];
  __shared__ int ptot[ZS_TILE];
  __shared__ long long s_tile, s_prefix;
  const int tid = threadIdx.x;
  if (tid == 0) {
    const unsigned long long t = atomicAdd(ticket, 1ull);
    if (t == (unsigned long long)gridDim.x - 1) zs_status_store(ticket, 0ull);  // every ticket is out
    s_tile = (long long)t;
  }
  __syncthreads();
  const int64_t tile = s_tile, p0 = tile * ZS_TILE;
  uint32_t v[ZS_TILE][8];
  int ex[ZS_TILE];
#pragma unroll
  for (int k = 0; k < ZS_TILE; ++k) zs_load8(x, (p0 + k) * ZS_PAGE + 8 * (int64_t)tid, n, v[k]);
  int tile_total = 0;
#pragma unroll
  for (int k = 0; k < ZS_TILE; ++k) {
    const uint32_t m = zs_byte(v[k]);
    bytes[k][tid] = m;
    int total;
    ex[k] = zs_block_scan(__builtin_popcount(m), sh, total);  // (its barriers order bytes)
    if (tid == 0) ptot[k] = total;
    tile_total += total;
  }
  if (tid < 64) {  // wave 0: the look-back, 64 predecessor tiles per round (lane i <-> tile q - i)
    const unsigned long long tag = epoch << ZS_ST_EPOCH, agg = 1ull << ZS_ST_VAL, inc = 2ull << ZS_ST_VAL;
    const unsigned long long vmask = (1ull << ZS_ST_VAL) - 1;
    long long prefix = 0;
    if (tile > 0) {
      if (tid == 0) zs_status_store(status + tile, tag | agg | (unsigned long long)tile_total);
      for (int64_t q = tile - 1;; q -= 64) {
        const int64_t qi = q - tid;
        // tiles before the first count as an inclusive prefix of 0
        unsigned long long w = qi >= 0 ? 0ull : (tag | inc);
        bool ready = qi < 0;
        while (__builtin_amdgcn_ballot_w64(!ready) != 0ull) {
          if (!ready) {
            w = zs_status_load(status + qi);
            ready = (w >> ZS_ST_EPOCH) == epoch && ((w >> ZS_ST_VAL) & 3ull) != 0ull;
          }
        }
        const unsigned long long incl = __builtin_amdgcn_ballot_w64(((w >> ZS_ST_VAL) & 3ull) == 2ull);
        const int first = incl ? __builtin_ctzll(incl) : 64;  // the nearest inclusive prefix
        prefix += wave_sum(tid <= first ? (long long)(w & vmask) : 0ll);
        if (incl) break;
      }
    }
    if (tid == 0) {
      zs_status_store(status + tile, tag | inc | (unsigned long long)(prefix + tile_total));
      s_prefix = prefix;
      if (tile == (int64_t)gridDim.x - 1) *nnz = prefix + tile_total;
    }
  }
  __syncthreads();
  long long o = s_prefix;
#pragma unroll
  for (int k = 0; k < ZS_TILE; ++k) {
    const int64_t p = p0 + k;
    if (p >= npages) break;  // (workgroup-uniform)
    if (tid == 0) meta[p * ZS_META] = (int)o;
    if (tid < 64)
      meta[p * ZS_META + 1 + tid] = (int)(bytes[k][4 * tid] | (bytes[k][4 * tid + 1] << 8) |
                                          (bytes[k][4 * tid + 2] << 16) | (bytes[k][4 * tid + 3] << 24));
    int pos = ex[k];
#pragma unroll
    for (int i = 0; i < 8; ++i)
      if (v[k][i] != 0u) lv[pos++] = v[k][i];
    __syncthreads();
    const int total = ptot[k];
    for (int i = tid; i < total; i += 256)
      if (o + i < cap) vals[o + i] = lv[i];
    o += total;
    __syncthreads();  // lv is rewritten by the next page
  }
}

__global__ __launch_bounds__(256) void zs_expand_kernel(const int* __restrict__ meta, const uint32_t* __restrict__ vals,
                                                        int64_t cap, uint32_t* __restrict__ out, int64_t n) {
  __shared__ int sh[4];
  const int64_t p = blockIdx.x;
  const uint32_t w = (uint32_t)meta[p * ZS_META + 1 + (threadIdx.x >> 2)];
  const uint32_t m = (w >> (8 * (threadIdx.x & 3))) & 0xffu;
  int total;
  const int ex = zs_block_scan(__builtin_popcount(m), sh, total);
  int64_t pos = (int64_t)meta[p * ZS_META] + ex;
  uint32_t v[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    v[i] = 0u;
    if ((m >> i) & 1u) {
      v[i] = pos < cap ? vals[pos] : 0u;
      ++pos;
    }
  }
  const int64_t e0 = p * ZS_PAGE + 8 * (int64_t)threadIdx.x;
  if (e0 + 8 <= n && (reinterpret_cast<uintptr_t>(out) & 15) == 0) {
    *reinterpret_cast<uint4*>(out + e0) = make_uint4(v[0], v[1], v[2], v[3]);
    *reinterpret_cast<uint4*>(out + e0 + 4) = make_uint4(v[4], v[5], v[6], v[7]);
  } else {
#pragma unroll
    for (int i = 0; i < 8; ++i)
      if (e0 + i < n) out[e0 + i] = v[i];
  }
}

// ---------------------------------------------------------------------------- segmented
// The sharded exchange encodes each (row, destination shard) slice of X as a SEGMENT of its own
// (offsets restart per segment, values go to a fixed-capacity slot per segment), so every
// destination's part is one contiguous meta range and one run of value slots.  A page table
// (built once per layout on the host, parallel/zs.py) gives each page its element start in the
// source (encode) or destination (decode) tensor, its element count (<= 2048) and its segment;
// each segment's pages are consecutive.
struct ZSPages {
  const int64_t* start;  // element start of page g
  const int* cnt;        // elements in page g
  const int* seg;        // segment of page g
};

__device__ __forceinline__ void zs_load_n(const uint32_t* __restrict__ x, int64_t e0, int n, uint32_t (&v)[8]) {
  const int t0 = 8 * (int)threadIdx.x;
  if (t0 + 8 <= n && ((reinterpret_cast<uintptr_t>(x + e0 + t0)) & 15) == 0) {
    const uint4 a = *reinterpret_cast<const uint4*>(x + e0 + t0), b = *reinterpret_cast<const uint4*>(x + e0 + t0 + 4);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  } else {
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = t0 + i < n ? x[e0 + t0 + i] : 0u;
  }
}

__global__ __launch_bounds__(256) void zs_seg_count_kernel(const uint32_t* __restrict__ x, ZSPages pg,
                                                           int* __restrict__ meta, int* __restrict__ counts) {
  __shared__ uint32_t bytes[256];
  __shared__ int sh[4];
  const int64_t g = blockIdx.x;
  uint32_t v[8];
  zs_load_n(x, pg.start[g], pg.cnt[g], v);
  const uint32_t m = zs_byte(v);
  bytes[threadIdx.x] = m;
  int total;
  (void)zs_block_scan(__builtin_popcount(m), sh, total);
  if (threadIdx.x < 64) {
    const int j = threadIdx.x;
    meta[g * ZS_META + 1 + j] =
        (int)(bytes[4 * j] | (bytes[4 * j + 1] << 8) | (bytes[4 * j + 2] << 16) | (bytes[4 * j + 3] << 24));
  }
  if (threadIdx.x == 0) counts[g] = total;
}

// one workgroup per segment: page offsets within the segment, the segment's count
__global__ __launch_bounds__(1024) void zs_seg_scan_kernel(const int* __restrict__ counts, const int* __restrict__ first,
                                                           const int* __restrict__ npg, int* __restrict__ meta,
                                                           int64_t* __restrict__ nnz) {
  __shared__ int64_t part[1024];
  const int t = threadIdx.x, sg = blockIdx.x;
  const int64_t f = first[sg], np = npg[sg];
  const int64_t per = (np + 1023) / 1024, q0 = t * per, q1 = min(np, q0 + per);
  int64_t s = 0;
  for (int64_t q = q0; q < q1; ++q) s += counts[f + q];
  part[t] = s;
  __syncthreads();
  for (int d = 1; d < 1024; d <<= 1) {
    const int64_t o = t >= d ? part[t - d] : 0;
    __syncthreads();
    part[t] += o;
    __syncthreads();
  }
  int64_t run = part[t] - s;
  for (int64_t q = q0; q < q1; ++q) {
    meta[(f + q) * ZS_META] = (int)run;
    run += counts[f + q];
  }
  if (t == 1023) nnz[sg] = part[1023];
}

__global__ __launch_bounds__(256) void zs_seg_compact_kernel(const uint32_t* __restrict__ x, ZSPages pg,
                                                             const int* __restrict__ meta, uint32_t* __restrict__ vals,
                                                             int64_t cap) {
  __shared__ int sh[4];
  const int64_t g = blockIdx.x;
  uint32_t v[8];
  zs_load_n(x, pg.start[g], pg.cnt[g], v);
  const uint32_t m = zs_byte(v);
  int total;
  const int ex = zs_block_scan(__builtin_popcount(m), sh, total);
  int64_t pos = (int64_t)meta[g * ZS_META] + ex;
  uint32_t* slot = vals + (int64_t)pg.seg[g] * cap;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    if (v[i] != 0u) {
      if (pos < cap) slot[pos] = v[i];
      ++pos;
    }
  }
}

// decode: page g's mask/offset at meta[g], its values in slot pg.seg[g] (capacity cap), its
// elements to out[pg.start[g] ..]
__global__ __launch_bounds__(256) void zs_seg_expand_kernel(const int* __restrict__ meta, ZSPages pg,
                                                            const uint32_t* __restrict__ vals, int64_t cap,
                                                            uint32_t* __restrict__ out) {
  __shared__ int sh[4];
  const int64_t g = blockIdx.x;
  const uint32_t w = (uint32_t)meta[g * ZS_META + 1 + (threadIdx.x >> 2)];
  const uint32_t m = (w >> (8 * (threadIdx.x & 3))) & 0xffu;
  int total;
  const int ex = zs_block_scan(__builtin_popcount(m), sh, total);
  int64_t pos = (int64_t)meta[g * ZS_META] + ex;
  const uint32_t* slot = vals + (int64_t)pg.seg[g] * cap;
  const int n = pg.cnt[g], t0 = 8 * (int)threadIdx.x;
  uint32_t* o = out + pg.start[g];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    uint32_t v = 0u;
    if ((m >> i) & 1u) {
      v = pos < cap ? slot[pos] : 0u;
      ++pos;
    }
    if (t0 + i < n) o[t0 + i] = v;
  }
}

// ---------------------------------------------------------------------------- fused update
// dW (=/+=) scale * dYᵀX, or the update-only W -= lr * scale * dYᵀX (linear_dw's contract), with
// X given zero-suppressed: the all-gathered encodings of the W source ranks (rank r: meta at
// meta + r*mstride, values at vals + r*cap; its `rows` rows of K columns encoded flat).  Row
// m = r*rows + b of dY pairs with local row b of rank r.  The rows are decoded in registers:
// no dense X is written and read back (zs_expand + linear_dw moved 2 x 360 MB per source rank
// more at the bench shape).
//
// A workgroup takes 1024 columns (4 per thread, one 16-B piece of each output row).  For each X
// row the span lies in at most 2 pages: their 2 x 64 mask words are loaded into LDS and turned
// into exclusive popcount prefixes (one wave per page), so a thread finds its 4 values' offset
// with one LDS read and a popcount.  Needs K % 4 == 0 (a thread's 4 columns share a mask word).
constexpr int ZD_COLS = 1024;

template <int NN>
__global__ __launch_bounds__(256) void linear_dw_zs_kernel(const float* __restrict__ g, const int* __restrict__ meta,
                                                           int64_t mstride, const uint32_t* __restrict__ vals,
                                                           int64_t cap, int rows, int M, int64_t K,
                                                           float* __restrict__ dW, int64_t ldw,
                                                           float* __restrict__ db, float scale, int acc,
                                                           float upd_lr) {
  __shared__ int pre[2][2][64];   // [buffer][page of the span][word]: value offset of the word
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  if (db && blockIdx.x == 0 && tid < NN) {
    float t = 0.f;
    for (int m = 0; m < M; ++m) t += g[m * NN + tid];
    db[tid] = acc ? db[tid] + scale * t : scale * t;
  }
  const int64_t nblk = (K + ZD_COLS - 1) / ZD_COLS;
  for (int64_t blk = blockIdx.x; blk < nblk; blk += gridDim.x) {
    const int64_t c0 = blk * ZD_COLS, col = c0 + 4 * tid;
    const bool cv = col < K;
    float4 s[NN];
#pragma unroll
    for (int n = 0; n < NN; ++n) s[n] = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int m = 0; m < M; ++m) {
      const int r = m / rows, b = m - r * rows;
      const int* mr = meta + r * mstride;
      const int64_t e0 = (int64_t)b * K + c0, pg0 = e0 / ZS_PAGE;
      const int buf = m & 1;
      if (wv < 2) {  // wave w: page pg0 + w of the span (beyond the rank's pages: never read)
        const int64_t pg = pg0 + wv;
        const int64_t npg = ((int64_t)rows * K + ZS_PAGE - 1) / ZS_PAGE;
        int cnt = 0, off = 0;
        if (pg < npg) {
          cnt = __builtin_popcount((uint32_t)mr[pg * ZS_META + 1 + lane]);
          off = mr[pg * ZS_META];
        }
        int incl = cnt;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
          const int o = __shfl_up(incl, d, 64);
          if (lane >= d) incl += o;
        }
        pre[buf][wv][lane] = off + incl - cnt;
      }
      __syncthreads();  // (double-buffered: the next row's prefixes go to the other buffer)
      float4 xv = make_float4(0.f, 0.f, 0.f, 0.f);
      if (cv) {
        const int64_t e = (int64_t)b * K + col;
        const int64_t pg = e / ZS_PAGE;
        const int pos = (int)(e - pg * ZS_PAGE), wj = pos >> 5, bit = pos & 31;
        const uint32_t w = (uint32_t)mr[pg * ZS_META + 1 + wj];
        const uint32_t m4 = (w >> bit) & 0xFu;
        if (m4) {
          int64_t o = (int64_t)pre[buf][(int)(pg - pg0)][wj] + __builtin_popcount(w & ((1u << bit) - 1u));
          const uint32_t* vr = vals + r * cap;
          float x4[4];
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            x4[k] = 0.f;
            if ((m4 >> k) & 1u) x4[k] = __uint_as_float(vr[o++]);
          }
          xv = make_float4(x4[0], x4[1], x4[2], x4[3]);
        }
      }
#pragma unroll
      for (int n = 0; n < NN; ++n) {
        const float gv = g[m * NN + n];
        s[n].x = fmaf(gv, xv.x, s[n].x);
        s[n].y = fmaf(gv, xv.y, s[n].y);
        s[n].z = fmaf(gv, xv.z, s[n].z);
        s[n].w = fmaf(gv, xv.w, s[n].w);
      }
    }
    if (cv) {
#pragma unroll
      for (int n = 0; n < NN; ++n) {
        float4* ptr = reinterpret_cast<float4*>(dW + (int64_t)n * ldw + col);
        const float4 v = make_float4(scale * s[n].x, scale * s[n].y, scale * s[n].z, scale * s[n].w);
        if (upd_lr != 0.f) {
          const float4 w0 = *ptr;
          *ptr = make_float4(w0.x - upd_lr * v.x, w0.y - upd_lr * v.y, w0.z - upd_lr * v.z, w0.w - upd_lr * v.w);
        } else if (acc) {
          const float4 w0 = *ptr;
          *ptr = make_float4(w0.x + v.x, w0.y + v.y, w0.z + v.z, w0.w + v.w);
        } else {
          *ptr = v;
        }
      }
    }
    __syncthreads();  // the prefix buffers are rewritten by the next block's first rows
  }
}

}  // namespace tds

using namespace tds;

int tds_linear_dw_zs(const float* dy, const int* meta, int64_t mstride, const float* vals, int64_t cap, int rows,
                     int M, int N, int64_t K, float* dW, int64_t ldw, float* db, float scale, int acc, float upd_lr,
                     hipStream_t st) {
  if (M < 1 || rows < 1 || M % rows || K % 4 || ldw % 4 || ((uintptr_t)dW & 15) || (N != 10 && N != 16)) return -1;
  int64_t grid = (K + ZD_COLS - 1) / ZD_COLS;
  if (grid > 8192) grid = 8192;
  const uint32_t* v = reinterpret_cast<const uint32_t*>(vals);
  if (N == 10)
    hipLaunchKernelGGL(linear_dw_zs_kernel<10>, dim3((unsigned)grid), dim3(256), 0, st, dy, meta, mstride, v, cap, rows,
                       M, K, dW, ldw, db, scale, acc, upd_lr);
  else
    hipLaunchKernelGGL(linear_dw_zs_kernel<16>, dim3((unsigned)grid), dim3(256), 0, st, dy, meta, mstride, v, cap, rows,
                       M, K, dW, ldw, db, scale, acc, upd_lr);
  TDS_LAUNCH_CHECK();
  return 0;
}

void tds_zs_seg_encode(const float* x, const int64_t* pg_start, const int* pg_cnt, const int* pg_seg, int64_t npages,
                       const int* seg_first, const int* seg_npg, int nseg, int* meta, int* counts, float* vals,
                       int64_t cap, int64_t* seg_nnz, hipStream_t st) {
  const ZSPages pg{pg_start, pg_cnt, pg_seg};
  const uint32_t* xb = reinterpret_cast<const uint32_t*>(x);
  hipLaunchKernelGGL(zs_seg_count_kernel, dim3((unsigned)npages), dim3(256), 0, st, xb, pg, meta, counts);
  TDS_LAUNCH_CHECK();
  hipLaunchKernelGGL(zs_seg_scan_kernel, dim3((unsigned)nseg), dim3(1024), 0, st, counts, seg_first, seg_npg, meta,
                     seg_nnz);
  TDS_LAUNCH_CHECK();
  hipLaunchKernelGGL(zs_seg_compact_kernel, dim3((unsigned)npages), dim3(256), 0, st, xb, pg, meta,
                     reinterpret_cast<uint32_t*>(vals), cap);
  TDS_LAUNCH_CHECK();
}

void tds_zs_seg_decode(const int* meta, const int64_t* pg_start, const int* pg_cnt, const int* pg_seg, int64_t npages,
                       const float* vals, int64_t cap, float* out, hipStream_t st) {
  const ZSPages pg{pg_start, pg_cnt, pg_seg};
  hipLaunchKernelGGL(zs_seg_expand_kernel, dim3((unsigned)npages), dim3(256), 0, st, meta, pg,
                     reinterpret_cast<const uint32_t*>(vals), cap, reinterpret_cast<uint32_t*>(out));
  TDS_LAUNCH_CHECK();
}

int64_t tds_zs_npages(int64_t n) { return (n + ZS_PAGE - 1) / ZS_PAGE; }

namespace {
// Look-back state of one (device, stream): status words (zeroed once when allocated; grown by a
// fresh allocation, the old one is kept -- a kernel may still be using it), the ticket counter
// and the call epoch.
struct ZSLookback {
  unsigned long long* status = nullptr;
  int64_t capacity = 0;
  unsigned long long* ticket = nullptr;
  unsigned long long epoch = 0;
};

bool zs_lookback(int64_t P, hipStream_t st, unsigned long long*& status, unsigned long long*& ticket,
                 unsigned long long& epoch) {
  static std::mutex mu;
  static std::map<std::pair<int, hipStream_t>, ZSLookback> cache;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return false;
  std::lock_guard<std::mutex> lock(mu);
  ZSLookback& e = cache[{dev, st}];
  if (e.ticket == nullptr) {
    if (hipMalloc(&e.ticket, sizeof(unsigned long long)) != hipSuccess) return false;
    if (hipMemsetAsync(e.ticket, 0, sizeof(unsigned long long), st) != hipSuccess) return false;
  }
  if (e.capacity < P || ++e.epoch >= (1ull << 24)) {
    const int64_t c = P > e.capacity ? std::max<int64_t>(P, 2 * e.capacity) : e.capacity;
    unsigned long long* fresh = nullptr;
    if (hipMalloc(&fresh, c * sizeof(unsigned long long)) != hipSuccess) return false;
    if (hipMemsetAsync(fresh, 0, c * sizeof(unsigned long long), st) != hipSuccess) return false;
    e.status = fresh;
    e.capacity = c;
    e.epoch = 1;  // zeroed words carry epoch 0
  }
  status = e.status;
  ticket = e.ticket;
  epoch = e.epoch;
  return true;
}
}  // namespace

void tds_zs_encode(const float* x, int64_t n, int* meta, float* vals, int64_t cap, int64_t* nnz, hipStream_t st) {
  const int64_t P = tds_zs_npages(n);
  unsigned long long *status = nullptr, *ticket = nullptr, epoch = 0;
  if (!zs_lookback((P + ZS_TILE - 1) / ZS_TILE, st, status, ticket, epoch)) {
    tds_launch_fail("zs_encode: look-back state allocation failed");
    return;
  }
  const int64_t tiles = (P + ZS_TILE - 1) / ZS_TILE;
  hipLaunchKernelGGL(zs_encode_kernel<const uint32_t*>, dim3((unsigned)tiles), dim3(256), 0, st,
                     reinterpret_cast<const uint32_t*>(x), n, P, meta, reinterpret_cast<uint32_t*>(vals), cap, nnz,
                     status, ticket, epoch);
  TDS_LAUNCH_CHECK();
}

void tds_zs_decode(const int* meta, const float* vals, int64_t cap, float* out, int64_t n, hipStream_t st) {
  const int64_t P = tds_zs_npages(n);
  hipLaunchKernelGGL(zs_expand_kernel, dim3((unsigned)P), dim3(256), 0, st, meta,
                     reinterpret_cast<const uint32_t*>(vals), cap, reinterpret_cast<uint32_t*>(out), n);
  TDS_LAUNCH_CHECK();
}
