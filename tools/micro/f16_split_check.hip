// Bitwise check of the fp16 hi/lo split used by the conv2 backward's staging (bf16x3.h):
//   reference: hi = f16(x), lo = f16(float(x) - float(hi))          (cvt, cvt back, sub, cvt)
//   mix      : hi = f16(x), lo = v_fma_mix{lo,hi}_f16(hi, -1, x)    (one rounding of x - hi)
// over 2^26 values spanning fp16's normal and subnormal range, zeros, and non-finite inputs.
// Build: hipcc -O3 --offload-arch=gfx950 -I../../torch_distributed_sandbox_amd/csrc/kernels f16_split_check.hip -o f16_split_check
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#include "bf16x3.h"

using namespace tds;

__device__ float gen(uint32_t i) {
  uint32_t h = i * 2654435761u;
  h ^= h >> 15;
  h *= 2246822519u;
  h ^= h >> 13;
  // exponent in [-40, 20] (fp16 subnormals start at 2^-14), random mantissa and sign
  const int e = (int)(h % 61u) - 40;
  const float m = 1.0f + (float)((h >> 8) & 0x7FFFFF) * (1.0f / 8388608.0f);
  float v = ldexpf(m, e);
  if (h & 0x80000000u) v = -v;
  if ((i & 0xFFFFF) == 7) v = 0.f;
  if ((i & 0xFFFFF) == 9) v = -0.f;
  if ((i & 0xFFFFF) == 11) v = __builtin_inff();
  if ((i & 0xFFFFF) == 13) v = __builtin_nanf("");
  if ((i & 0xFFFFF) == 15) v = 65504.f + 16.f;  // rounds to inf in fp16
  return v;
}

__global__ void check(uint32_t n, unsigned long long* bad, uint32_t* first) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (2 * i + 1 >= n) return;
  const float a = gen(2 * i), b = gen(2 * i + 1);
  uint32_t h0, l0, h1, l1;
  split2_f16(a, b, h0, l0);
  split2_f16_mix(a, b, h1, l1);
  if (h0 != h1 || l0 != l1) {
    // NaN payloads may differ; count only when either side is not a NaN pattern
    const bool nan = (a != a) || (b != b);
    if (!nan) {
      atomicAdd(bad, 1ull);
      atomicMin(first, 2 * i);
    }
  }
}

int main() {
  const uint32_t n = 1u << 26;
  unsigned long long* bad;
  uint32_t* first;
  (void)hipMalloc(&bad, 8);
  (void)hipMalloc(&first, 4);
  (void)hipMemset(bad, 0, 8);
  (void)hipMemset(first, 0xFF, 4);
  hipLaunchKernelGGL(check, dim3(n / 2 / 256), dim3(256), 0, 0, n, bad, first);
  unsigned long long hb = 0;
  uint32_t hf = 0;
  (void)hipMemcpy(&hb, bad, 8, hipMemcpyDeviceToHost);
  (void)hipMemcpy(&hf, first, 4, hipMemcpyDeviceToHost);
  if (hipGetLastError() != hipSuccess) { printf("hip error\n"); return 2; }
  printf("f16 split check: %u values, %llu mismatches (first at %u)\n", n, hb, hf);
  return hb == 0 ? 0 : 1;
}
