// HBM ceiling for the head backward's traffic mix (csrc/kernels/head_pb.hip head_bwd_pb_kernel:
// per step it reads the fc weight and ya, 1.07 GB, and writes the updated weight and g2m, 1.07 GB).
// Grid-stride float4 streams over buffers of the bench's sizes:
//   read  : read 2.14 GB (sum kept live)
//   copy  : read 1.07 GB, write 1.07 GB (plain stores)
//   copynt: the same with non-temporal stores (as the head backward)
//   rmw   : read A, write A' = A + 1 in place (the weight's own read + write) + read B, write B'
// Build: hipcc --offload-arch=gfx950 -O3 tools/micro/rw_bw.hip -o /tmp/rw_bw
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float f4v __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void k_read(const f4v* __restrict__ a, long n, float* __restrict__ out) {
  f4v s = {0.f, 0.f, 0.f, 0.f};
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) s += a[i];
  if (s.x + s.y + s.z + s.w == 12345.f) out[0] = s.x;
}

template <bool NT>
__global__ __launch_bounds__(256) void k_copy(const f4v* __restrict__ a, f4v* __restrict__ b, long n) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const f4v v = a[i] + 1.f;
    if constexpr (NT) __builtin_nontemporal_store(v, b + i);
    else b[i] = v;
  }
}

template <bool NT>
__global__ __launch_bounds__(256) void k_rmw2(f4v* __restrict__ a, long na, f4v* __restrict__ b, long nb) {
  // the head backward's shape: per element of a (the weight, read and written) one of b (ya read,
  // g2m written) every 2 elements
  for (long i = blockIdx.x * 256L + threadIdx.x; i < na; i += (long)gridDim.x * 256) {
    const f4v v = a[i] + 1.f;
    if constexpr (NT) __builtin_nontemporal_store(v, a + i);
    else a[i] = v;
    if ((i & 1) == 0 && (i >> 1) < nb) {
      const f4v w = b[i >> 1] * 2.f;
      if constexpr (NT) __builtin_nontemporal_store(w, b + (i >> 1));
      else b[i >> 1] = w;
    }
  }
}

int main() {
  const long nw = 714L * 1000 * 1000 / 16, ny = 357L * 1000 * 1000 / 16;  // float4 counts
  f4v *a, *b;
  float* out;
  hipMalloc(&a, (nw + ny) * 16);
  hipMalloc(&b, (nw + ny) * 16);
  hipMalloc(&out, 16);
  hipMemset(a, 0, (nw + ny) * 16);
  hipMemset(b, 0, (nw + ny) * 16);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  auto timeit = [&](const char* name, double gb, auto launch) {
    for (int w = 0; w < 3; ++w) launch();
    hipEventRecord(e0);
    const int it = 20;
    for (int k = 0; k < it; ++k) launch();
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0.f;
    hipEventElapsedTime(&ms, e0, e1);
    ms /= it;
    printf("%-8s %.3f ms  %.2f TB/s (%.2f GB moved)\n", name, ms, gb / ms, gb);
  };
  for (int grid : {1024, 2048, 4096, 8192}) {
    printf("grid %d\n", grid);
    timeit("read", (nw + ny) * 16 * 2 / 1e9,
           [&] { hipLaunchKernelGGL(k_read, dim3(grid), dim3(256), 0, 0, a, nw + ny, out);
                 hipLaunchKernelGGL(k_read, dim3(grid), dim3(256), 0, 0, b, nw + ny, out); });
    timeit("copy", (nw + ny) * 16 * 2 / 1e9,
           [&] { hipLaunchKernelGGL(k_copy<false>, dim3(grid), dim3(256), 0, 0, a, b, nw + ny); });
    timeit("copynt", (nw + ny) * 16 * 2 / 1e9,
           [&] { hipLaunchKernelGGL(k_copy<true>, dim3(grid), dim3(256), 0, 0, a, b, nw + ny); });
    timeit("rmw2nt", (nw + ny) * 16 * 2 / 1e9,
           [&] { hipLaunchKernelGGL(k_rmw2<true>, dim3(grid), dim3(256), 0, 0, a, nw, b, ny); });
  }
  hipFree(a);
  hipFree(b);
  hipFree(out);
  return 0;
}
