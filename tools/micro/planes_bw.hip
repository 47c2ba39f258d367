// Memory-system probe for the head kernels' access pattern (tools/micro/README in
// docs/KERNELS.md): NR read planes + NW write planes of N floats each, every element
// of the output needing the same position of every plane.  A workgroup handles a run
// of RUN consecutive positions of all planes; lanes take VX consecutive floats.
// Build: hipcc --offload-arch=gfx950 -O3 tools/micro/planes_bw.hip -o planes_bw
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

template <int VX> struct V { typedef float __attribute__((ext_vector_type(VX))) T; };
template <> struct V<1> { typedef float T; };

template <int VX, int NR, int NWR>
__global__ __launch_bounds__(256) void planes(const float* __restrict__ in, float* __restrict__ out, long n, int run) {
  typedef typename V<VX>::T T;
  const long nrun = n / run;
  for (long r = blockIdx.x; r < nrun; r += gridDim.x) {
    for (int i = threadIdx.x * VX; i < run; i += 256 * VX) {
      const long pos = r * run + i;
      T acc;
      T v[NR];
#pragma unroll
      for (int k = 0; k < NR; ++k) v[k] = *reinterpret_cast<const T*>(in + (long)k * n + pos);
      acc = v[0];
#pragma unroll
      for (int k = 1; k < NR; ++k) acc = acc * 0.5f + v[k];
#pragma unroll
      for (int k = 0; k < NWR; ++k) *reinterpret_cast<T*>(out + (long)k * n + pos) = acc + (float)k;
    }
  }
}

template <int VX>
__global__ __launch_bounds__(256) void copy(const float* __restrict__ in, float* __restrict__ out, long n) {
  typedef typename V<VX>::T T;
  for (long i = ((long)blockIdx.x * 256 + threadIdx.x) * VX; i < n; i += (long)gridDim.x * 256 * VX)
    *reinterpret_cast<T*>(out + i) = *reinterpret_cast<const T*>(in + i) * 2.f;
}

int main() {
  const long n = 18000000;  // one fc plane-set column count (32*750*750)
  const int NR = 15, NWR = 11;
  float *in, *out;
  hipMalloc(&in, sizeof(float) * n * NR);
  hipMalloc(&out, sizeof(float) * n * NWR);
  hipMemset(in, 0, sizeof(float) * n * NR);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  auto timeit = [&](const char* name, double gb, auto launch) {
    for (int w = 0; w < 2; ++w) launch();
    hipEventRecord(a);
    for (int w = 0; w < 5; ++w) launch();
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    ms /= 5;
    printf("%-40s %8.3f ms  %6.2f TB/s\n", name, ms, gb / ms);
  };
  const double gb = (double)n * 4 * (NR + NWR) / 1e9;
  for (int grid : {1024, 4096, 16384}) {
    char s[64];
    snprintf(s, 64, "copy float4 grid %d", grid);
    timeit(s, (double)n * NR * 4 * 2 / 1e9, [&] { hipLaunchKernelGGL(copy<4>, dim3(grid), dim3(256), 0, 0, in, out, n * NR < n * NWR ? n * NR : n * NWR); });
  }
  for (int run : {256, 1024, 4096, 16384}) {
    for (int grid : {1024, 4096}) {
      char s[64];
      snprintf(s, 64, "planes vx1 run %d grid %d", run, grid);
      timeit(s, gb, [&] { hipLaunchKernelGGL((planes<1, NR, NWR>), dim3(grid), dim3(256), 0, 0, in, out, n, run); });
      snprintf(s, 64, "planes vx4 run %d grid %d", run, grid);
      timeit(s, gb, [&] { hipLaunchKernelGGL((planes<4, NR, NWR>), dim3(grid), dim3(256), 0, 0, in, out, n, run); });
    }
  }
  return 0;
}
