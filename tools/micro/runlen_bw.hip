// Memory-system probe: bandwidth of the head backward's plane mix as a function of the
// contiguous run a workgroup covers per plane.  Data: NR read and NWR write "tensors", each
// C=32 channel planes of N positions (like W[j][c][pos]).  A 256-thread workgroup iteration
// covers CB channels x L positions (CB*L = 1024 floats: every thread one float4), so each
// plane is touched in runs of L*4 bytes.  NT=1 makes the stores nontemporal.
// Build: hipcc --offload-arch=gfx950 -O3 tools/micro/runlen_bw.hip -o tools/micro/runlen_bw
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f4 __attribute__((ext_vector_type(4)));

template <int L, int NR, int NWR, bool NT>
__global__ __launch_bounds__(256) void runlen(const float* __restrict__ in, float* __restrict__ out, long n) {
  constexpr int CB = 1024 / L, TPC = L / 4;  // channels per iteration, threads per channel
  const int c_in = threadIdx.x / TPC, p4 = threadIdx.x % TPC;
  const long nchunk = n / L;
  const long plane = 32 * n;  // floats between consecutive tensors k
  for (long it = blockIdx.x; it < nchunk * (32 / CB); it += gridDim.x) {
    const long cg = it % (32 / CB), ch = it / (32 / CB);
    const long off = (cg * CB + c_in) * n + ch * L + p4 * 4;
    f4 v[NR];
#pragma unroll
    for (int k = 0; k < NR; ++k) v[k] = *reinterpret_cast<const f4*>(in + k * plane + off);
    f4 acc = v[0];
#pragma unroll
    for (int k = 1; k < NR; ++k) acc = acc * 0.5f + v[k];
#pragma unroll
    for (int k = 0; k < NWR; ++k) {
      f4 o = acc + (float)k;
      if constexpr (NT) __builtin_nontemporal_store(o, reinterpret_cast<f4*>(out + k * plane + off));
      else *reinterpret_cast<f4*>(out + k * plane + off) = o;
    }
  }
}

int main() {
  const long n = 562500;  // 750 x 750 pooled positions per channel plane
  const int NR = 15, NWR = 15;
  float *in, *out;
  hipMalloc(&in, sizeof(float) * n * 32 * NR);
  hipMalloc(&out, sizeof(float) * n * 32 * NWR);
  hipMemset(in, 0, sizeof(float) * n * 32 * NR);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const double gb = (double)n * 32 * 4 * (NR + NWR) / 1e9;
  auto timeit = [&](const char* name, auto launch) {
    for (int w = 0; w < 2; ++w) launch();
    hipEventRecord(a);
    for (int w = 0; w < 5; ++w) launch();
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    ms /= 5;
    printf("%-36s %8.3f ms  %6.2f TB/s\n", name, ms, gb / ms);
  };
#define RUN(LL, NTT)                                                                                     \
  for (int grid : {1024, 4096, 16384}) {                                                               \
    char s[64];                                                                                        \
    snprintf(s, 64, "L %4d nt %d grid %5d", LL, (int)NTT, grid);                                       \
    timeit(s, [&] { hipLaunchKernelGGL((runlen<LL, NR, NWR, NTT>), dim3(grid), dim3(256), 0, 0, in, out, n); }); \
  }
  RUN(32, false) RUN(32, true) RUN(64, true) RUN(128, true) RUN(256, true) RUN(1024, false) RUN(1024, true)
  return 0;
}
