// Shared device helpers for the gfx950 (MI355X, CDNA4) kernels.
//
// Everything here assumes wave64: lane = threadIdx.x & 63, 64-bit ballots,
// shuffles over 64 lanes.  No CUDA spellings, no dual paths.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#define TDS_WAVE 64

// Launch-status plumbing (launch_status.hip): every host launcher calls TDS_LAUNCH_CHECK()
// right after its hipLaunchKernelGGL, which records the first failed launch of the calling
// thread (bad grid / block / LDS size, missing code object ...); launchers that refuse a shape
// record it with tds_launch_fail().  The binding layer (csrc/*.cpp) takes the record after every
// op and raises, so a bad launch is a Python exception, never silently skipped work.
void tds_note_launch(hipError_t e, const char* where, int line);
void tds_launch_fail(const char* what);
#define TDS_LAUNCH_CHECK() tds_note_launch(hipGetLastError(), __func__, __LINE__)

namespace tds {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef short bf16x4 __attribute__((ext_vector_type(4)));

// Streaming stores of the step's large tensors (y2, ya, p1, idx1, g2m, the fc weight update):
// non-temporal.  A/B on MI355X against plain stores, bench 3 x alternating: 3.64 vs 3.80 ms per
// step (layer-1 forward -68 us, conv2 forward -12 us, head backward -18 us;
// tools/gpu_sessions/r2_split2.sh).  dp1 keeps plain stores: the layer-1 backward reads it
// right after the conv2 backward (nt there measured +15 us).
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void st_stream(float* p, float v) {
  __builtin_nontemporal_store(v, p);
}
__device__ __forceinline__ void st_stream(uint32_t* p, uint32_t v) {
  __builtin_nontemporal_store(v, p);
}
__device__ __forceinline__ void st_stream(float4* p, float4 v) {
  __builtin_nontemporal_store(__builtin_bit_cast(f32x4, v), reinterpret_cast<f32x4*>(p));
}
__device__ __forceinline__ void st_stream(float2* p, float2 v) {
  __builtin_nontemporal_store(__builtin_bit_cast(f32x2, v), reinterpret_cast<f32x2*>(p));
}
__device__ __forceinline__ void st_stream(uint2* p, uint2 v) {
  __builtin_nontemporal_store(__builtin_bit_cast(u32x2, v), reinterpret_cast<u32x2*>(p));
}

__device__ __forceinline__ int lane_id() { return threadIdx.x & (TDS_WAVE - 1); }
__device__ __forceinline__ int wave_id() { return threadIdx.x / TDS_WAVE; }

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, TDS_WAVE);
  return v;
}

template <typename T>
__device__ __forceinline__ T wave_max(T v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    T o = __shfl_xor(v, off, TDS_WAVE);
    v = v > o ? v : o;
  }
  return v;
}

// Block-wide sum of one value per thread; result valid in every thread.
// `scratch` must hold blockDim.x / 64 elements.
template <typename T>
__device__ __forceinline__ T block_sum(T v, T* scratch) {
  v = wave_sum(v);
  const int nw = blockDim.x / TDS_WAVE;
  __syncthreads();
  if (lane_id() == 0) scratch[wave_id()] = v;
  __syncthreads();
  T r = 0;
  for (int i = 0; i < nw; ++i) r += scratch[i];
  return r;
}

// Block-wide max (same contract as block_sum).
template <typename T>
__device__ __forceinline__ T block_max(T v, T* scratch) {
  v = wave_max(v);
  const int nw = blockDim.x / TDS_WAVE;
  __syncthreads();
  if (lane_id() == 0) scratch[wave_id()] = v;
  __syncthreads();
  T r = scratch[0];
  for (int i = 1; i < nw; ++i) r = r > scratch[i] ? r : scratch[i];
  return r;
}

// Round-to-nearest-even f32 -> bf16 bits (finite inputs; NaN stays NaN via cast path).
__device__ __forceinline__ unsigned short f32_to_bf16_bits(float f) {
  unsigned int u = __float_as_uint(f);
  u += 0x7FFFu + ((u >> 16) & 1u);
  return (unsigned short)(u >> 16);
}
__device__ __forceinline__ float bf16_bits_to_f32(unsigned short h) {
  return __uint_as_float(((unsigned int)h) << 16);
}

// XCD-aware bijective block remap (cdna_hip_programming.md §5 "XCD swizzle must be
// bijective"): consecutive logical tiles land on the same XCD so neighbours
// share that XCD's L2.  Speed only; correctness never depends on placement.
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  const int nx = 8;
  if (nwg < nx) return orig;
  const int q = nwg / nx, r = nwg % nx;
  const int x = orig % nx;
  const int base = (x < r) ? x * (q + 1) : r * (q + 1) + (x - r) * q;
  return base + orig / nx;
}

// Wave-uniform raw buffer descriptor over [base, base + bytes): lanes whose voffset is past
// `bytes` read zeros / drop stores (hardware range check).  The two readfirstlane halves are
// widened as UNSIGNED: readfirstlane returns int, and OR-ing a sign-extended low word into the
// address corrupts the high word whenever bit 31 of the base is set (an allocation-dependent
// memory fault).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t tds_buffer_rsrc(const void* base, uint32_t bytes) {
  const uint64_t v = reinterpret_cast<uint64_t>(base);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)v);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  // every field wave-uniform (readfirstlane): a descriptor the compiler cannot prove uniform
  // gets a waterfall loop around each buffer instruction
  return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(((uint64_t)hi << 32) | (uint64_t)lo), (short)0,
                                           (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}

// ---------------------------------------------------------------------------- in-launch finalizers
// A producer kernel whose per-workgroup partials used to go to a separate reduce / finalize launch
// (6-8 us each at the bench shape, almost all of it the kernel boundary) reduces them itself: the
// LAST workgroup of a group to arrive reduces the group's rows, the last group-reducer finalizes.
// Hand-off per cdna_hip_programming.md Guideline 16, counter form with WRITE-THROUGH payload:
//   producer: every handed-off value stored sc1 (st_agent: an agent-scope relaxed atomic store,
//             global_store ... sc1) -> every wave s_waitcnt vmcnt(0) -> barrier -> lane 0 relaxed
//             agent fetch_add on the counter.  No release fence: an agent release is a
//             buffer_wbl2 of the XCD's whole L2, and in the streaming kernels (the conv2 forward's
//             y2h / ya, the head backward's g2m / weight update, all non-temporal stores that sit
//             dirty in L2) one per workgroup cost +0.34 ms per step (r5_s2);
//   the workgroup that draws n - 1 is the reducer: agent acquire fence (this CU's L1) -> vmcnt(0)
//   -> barrier, then every wave reads the rows with lane-indexed vector loads (never through the
//   scalar cache: Pitfall 6).
// Counters live in a per-(device, stream) word buffer zeroed when it is allocated
// (tds_sync_words); the reducer resets its counter to 0 for the next launch on that stream.
// `flag` is one int of the kernel's own LDS (the broadcast of "I am last").
__device__ __forceinline__ bool tds_arrive(uint32_t* counter, uint32_t n, int* flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t t = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const bool last = t == n - 1;
    if (last) {
      __hip_atomic_store(counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    *flag = last ? 1 : 0;
  }
  __syncthreads();
  return *flag != 0;
}
// stores of handed-off data: write-through (sc1)
__device__ __forceinline__ void st_agent(double* p, double v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_agent(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Sum of nrows rows of ncols doubles (row r at base + r * rstride), in a fixed order, by one
// 256-thread workgroup in ONE round of loads: thread t takes column t % ncols of row group t / ncols
// (G = 256 / ncols groups, rows g, g + G, ...; at most WRS_MAXL loads each, all issued before the
// first add), the G group sums meet in LDS (part: G * ncols doubles) and threads t < ncols add them
// in group order.  A reducer that walked its rows as a dependent chain paid one global round trip
// (~1-2 us) per step, which made the in-launch finalizers slower than the launches they replaced
// (r5_s3).  Returns the column sum in threads t < ncols (0 elsewhere).  Needs ncols <= 256 and
// 1 <= nrows <= WRS_MAXL * (256 / ncols).  Every thread of the workgroup must call it.
// Rows past nrows are loaded CLAMPED to the last row and dropped at the add: with the load under
// `r < nrows ? load : 0` the compiler put each load in its own branch and waited for it there, so
// the "one round" was 16 dependent round trips (r5_s47, found in the ISA).
constexpr int WRS_MAXL = 16;
// (column c of row r at base + r * rstride + (c >> 1) * cstride2 + (c & 1): cstride2 = 2 for
// contiguous rows; the conv2 forward's [channel][workgroup][2] partials use cstride2 = 2 * nwg)
__device__ __forceinline__ double wide_row_sum(const double* base, int nrows, int ncols, int64_t rstride,
                                               double* part, int64_t cstride2 = 2) {
  const int t = (int)threadIdx.x, G = 256 / ncols;
  const int col = t % ncols, grp = t / ncols;
  const int64_t coff = (int64_t)(col >> 1) * cstride2 + (col & 1);
  double s = 0.0;
  if (grp < G) {
    double v[WRS_MAXL];
#pragma unroll
    for (int k = 0; k < WRS_MAXL; ++k) {
      v[k] = base[(int64_t)min(grp + k * G, nrows - 1) * rstride + coff];  // (clamped, see above)
    }
#pragma unroll
    for (int k = 0; k < WRS_MAXL; ++k) s += grp + k * G < nrows ? v[k] : 0.0;
    part[grp * ncols + col] = s;
  }
  __syncthreads();
  double tot = 0.0;
  if (t < ncols)
    for (int q = 0; q < G; ++q) tot += part[q * ncols + t];
  __syncthreads();  // part may be reused
  return tot;
}

// max of nrows rows of ncols (<= 256) uint32 (row r at base + r * rstride), one round of loads,
// threads t < ncols get the column max (same contract as wide_row_sum; part: 256 words)
__device__ __forceinline__ uint32_t wide_row_max(const uint32_t* base, int nrows, int ncols, int64_t rstride,
                                                 uint32_t* part) {
  const int t = (int)threadIdx.x, G = 256 / ncols;
  const int col = t % ncols, grp = t / ncols;
  uint32_t m = 0u;
  if (grp < G) {
    uint32_t v[WRS_MAXL];
#pragma unroll
    for (int k = 0; k < WRS_MAXL; ++k) {
      v[k] = base[(int64_t)min(grp + k * G, nrows - 1) * rstride + col];  // (clamped: a repeat leaves the max)
    }
#pragma unroll
    for (int k = 0; k < WRS_MAXL; ++k) m = max(m, v[k]);
    part[grp * ncols + col] = m;
  }
  __syncthreads();
  uint32_t tot = 0u;
  if (t < ncols)
    for (int q = 0; q < G; ++q) tot = max(tot, part[q * ncols + t]);
  __syncthreads();
  return tot;
}

// call sites of the in-launch finalizers (tds_sync_words: kSyncWordsPerSite counters each)
enum TdsSyncSite {
  kSyncHeadFwd = 0, kSyncConv2Fwd = 1, kSyncHeadBwd = 2, kSyncL1Bwd = 3, kSyncXMoments = 4, kSyncL1Gram = 5,
  kSyncL1Fin = 6
};
constexpr int kSyncSites = 8, kSyncWordsPerSite = 256;

// The head backward's pooled gradient g2m is PLANAR, [B][32][Q][Q] (the fc flatten order):
// its producer streams the fc weight planes and writes g2m in the same long per-channel runs
// (head_bwd_stream_kernel).  Channels 4*c4 .. 4*c4+3 of pooled position (py, px) of image b:
__device__ __forceinline__ float4 g2m_planar4(const float* __restrict__ g2m, int b, int c4, int py, int px, int Q) {
  const int64_t QQ = (int64_t)Q * Q;
  const float* g = g2m + ((int64_t)b * 32 + 4 * c4) * QQ + (int64_t)py * Q + px;
  return make_float4(g[0], g[QQ], g[2 * QQ], g[3 * QQ]);
}

}  // namespace tds
