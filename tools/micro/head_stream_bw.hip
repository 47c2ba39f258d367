// Memory-system probe for the fc head forward stream (csrc/kernels/head_pb.hip): per block row
// of 4 pooled rows, 5 image planes of ya (pooled-blocked, one contiguous run per plane) and 10
// class planes of the fc weight (4 row runs of Q floats) of one channel.  Variants:
//   PF  : register double-buffering of the next chunk's loads (1) or not (0)
//   NT  : nontemporal loads
//   TPB : threads per workgroup
//   HB  : block rows per workgroup
// plus a plain contiguous float4 read of the same byte count as the ceiling.
// Build: hipcc --offload-arch=gfx950 -O3 tools/micro/head_stream_bw.hip -o /tmp/head_stream_bw
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

constexpr int NB = 5, NC = 10;

typedef float f4v __attribute__((ext_vector_type(4)));
template <bool NT>
__device__ __forceinline__ float4 ld4(const float* p) {
  if constexpr (NT) {
    const f4v v = __builtin_nontemporal_load(reinterpret_cast<const f4v*>(p));
    return float4{v.x, v.y, v.z, v.w};
  }
  return *reinterpret_cast<const float4*>(p);
}

template <int TPB, int HB, bool PF, bool NT>
__global__ __launch_bounds__(TPB) void head_like(const float* __restrict__ ya, const float* __restrict__ W,
                                                 float* __restrict__ out, int Q, int Q4, int Q8) {
  const int nband = (Q4 + HB - 1) / HB;
  const int c = blockIdx.x / nband, band = blockIdx.x % nband;
  const long QQ = (long)Q * Q, plane = (long)Q4 * Q8 * 32;
  const int nch = (Q8 * 8 + TPB - 1) / TPB;
  const int R0 = band * HB, nit = (min(Q4, R0 + HB) - R0) * nch;
  float acc[NB][NC] = {};
  struct L {
    float4 y[NB], w[NC];
  };
  auto issue = [&](int i, L& l) {
    const int R = R0 + i / nch, f = (i % nch) * TPB + threadIdx.x;
    const int blk = f >> 3, part = f & 7, prow = part >> 1, half = part & 1;
    const bool ok = blk < Q8 && 4 * R + prow < Q && blk * 8 + half * 4 + 3 < Q;
    const long yi = (((long)c * Q4 + R) * Q8 + blk) * 32 + part * 4;
    const float* wr = W + (long)c * QQ + (long)(4 * R + prow) * Q + blk * 8 + half * 4;
#pragma unroll
    for (int b = 0; b < NB; ++b) l.y[b] = ok ? ld4<NT>(ya + b * 32 * plane + yi) : float4{0, 0, 0, 0};
#pragma unroll
    for (int j = 0; j < NC; ++j) l.w[j] = ok ? ld4<NT>(wr + (long)j * 32 * QQ) : float4{0, 0, 0, 0};
  };
  L cur, nxt;
  if (nit > 0) issue(0, cur);
  for (int i = 0; i < nit; ++i) {
    if constexpr (PF) {
      if (i + 1 < nit) issue(i + 1, nxt);
    }
#pragma unroll
    for (int j = 0; j < NC; ++j)
#pragma unroll
      for (int b = 0; b < NB; ++b)
        acc[b][j] += cur.y[b].x * cur.w[j].x + cur.y[b].y * cur.w[j].y + cur.y[b].z * cur.w[j].z + cur.y[b].w * cur.w[j].w;
    if constexpr (PF) {
      cur = nxt;
    } else {
      if (i + 1 < nit) issue(i + 1, cur);
    }
  }
  float s = 0.f;
#pragma unroll
  for (int b = 0; b < NB; ++b)
#pragma unroll
    for (int j = 0; j < NC; ++j) s += acc[b][j];
  if (s == 12345.f) out[threadIdx.x] = s;
}

__global__ void plain_read(const float4* __restrict__ in, float* __restrict__ out, long n4) {
  float4 a{0, 0, 0, 0};
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) {
    const float4 v = in[i];
    a.x += v.x;
    a.y += v.y;
  }
  if (a.x == 12345.f) out[0] = a.y;
}

template <int TPB, int HB, bool PF, bool NT>
void run(const char* name, const float* ya, const float* W, float* out, int Q) {
  const int Q4 = (Q + 3) / 4, Q8 = (Q + 7) / 8;
  const int grid = 32 * ((Q4 + HB - 1) / HB);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int w = 0; w < 3; ++w) hipLaunchKernelGGL((head_like<TPB, HB, PF, NT>), dim3(grid), dim3(TPB), 0, 0, ya, W, out, Q, Q4, Q8);
  hipEventRecord(a);
  const int iters = 20;
  for (int w = 0; w < iters; ++w) hipLaunchKernelGGL((head_like<TPB, HB, PF, NT>), dim3(grid), dim3(TPB), 0, 0, ya, W, out, Q, Q4, Q8);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0.f;
  hipEventElapsedTime(&ms, a, b);
  ms /= iters;
  const double bytes = (double)NB * 32 * Q4 * Q8 * 32 * 4 + (double)NC * 32 * Q * Q * 4;
  std::printf("%-28s TPB %4d HB %2d PF %d NT %d grid %6d  %.3f ms  %.2f TB/s\n", name, TPB, HB, (int)PF, (int)NT, grid, ms,
              bytes / ms / 1e9);
}

int main(int argc, char** argv) {
  const int Q = argc > 1 ? std::atoi(argv[1]) : 750;
  const int Q4 = (Q + 3) / 4, Q8 = (Q + 7) / 8;
  const size_t ny = (size_t)NB * 32 * Q4 * Q8 * 32, nw = (size_t)NC * 32 * Q * Q;
  float *ya, *W, *out;
  hipMalloc(&ya, ny * 4);
  hipMalloc(&W, nw * 4 + 64);
  hipMalloc(&out, 4096);
  hipMemset(ya, 0, ny * 4);
  hipMemset(W, 0, nw * 4);
  {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const long n4 = (long)(nw / 4);
    for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(plain_read, dim3(4096), dim3(256), 0, 0, (const float4*)W, out, n4);
    hipEventRecord(a);
    for (int w = 0; w < 20; ++w) hipLaunchKernelGGL(plain_read, dim3(4096), dim3(256), 0, 0, (const float4*)W, out, n4);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0.f;
    hipEventElapsedTime(&ms, a, b);
    std::printf("plain contiguous read       %.3f ms  %.2f TB/s\n", ms / 20, nw * 4.0 / (ms / 20) / 1e9);
  }
  run<256, 4, true, false>("regs-prefetch", ya, W, out, Q);
  run<256, 4, false, false>("no-prefetch", ya, W, out, Q);
  run<256, 4, true, true>("regs-prefetch nt", ya, W, out, Q);
  run<256, 4, false, true>("no-prefetch nt", ya, W, out, Q);
  run<512, 4, false, false>("no-prefetch", ya, W, out, Q);
  run<256, 1, false, false>("no-prefetch", ya, W, out, Q);
  run<256, 2, true, false>("regs-prefetch", ya, W, out, Q);
  run<256, 8, true, false>("regs-prefetch", ya, W, out, Q);
  run<128, 4, true, false>("regs-prefetch", ya, W, out, Q);
  run<1024, 1, false, false>("no-prefetch", ya, W, out, Q);
  hipFree(ya);
  hipFree(W);
  hipFree(out);
  return 0;
}
