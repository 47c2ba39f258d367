// Texture-path cost of one wave's global load instruction by address pattern (the conv2 backward's
// staging is bound by its load instructions, docs/KERNELS.md "conv2 backward roles"): every wave of
// a full grid issues ITERS loads of one pattern over a 1 MiB, L2-resident buffer (each lane's sum
// kept live), 8 loads in flight per lane.  Reported: ns per wave-instruction per CU.
//   v4_contig  : 16 B per lane, the wave's 1 KiB contiguous (8 full 128-B lines)
//   v4_half    : 16 B per lane, lane quads on 64-B halves of 16 lines 128 B apart (the staging's
//                y2h item loads)
//   v4_lines   : 16 B per lane, every lane its own 128-B line
//   v4_oob     : 16 B per lane, every lane out of the buffer range (buffer-descriptor zeros)
//   b32_contig : 4 B per lane, 256 B contiguous
//   b32_lines  : 4 B per lane, every lane its own 128-B line (the a2 / halo loads)
// Build: hipcc --offload-arch=gfx950 -O3 tools/micro/ta_pattern.hip -o tools/micro/ta_pattern
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int ITERS = 512;
constexpr uint32_t kBuf = 1u << 20;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}

template <int PAT>
__global__ __launch_bounds__(256) void k(const char* __restrict__ buf, float* __restrict__ out, uint32_t salt) {
  const int lane = threadIdx.x & 63;
  const uint32_t wv = (blockIdx.x * 4 + (threadIdx.x >> 6)) * 2654435761u + salt;
  const __amdgpu_buffer_rsrc_t r = rsrc(buf, kBuf);
  uint32_t lo;
  if (PAT == 0) lo = lane * 16;
  else if (PAT == 1) lo = (lane >> 2) * 128 + (lane & 3) * 16;
  else if (PAT == 2) lo = lane * 128;
  else if (PAT == 3) lo = kBuf + 4096 + lane * 16;
  else if (PAT == 4) lo = lane * 4;
  else lo = lane * 128;
  float s = 0.f;
  for (int it = 0; it < ITERS; it += 8) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const uint32_t base = ((wv + (uint32_t)(it + u) * 40503u) & ((kBuf >> 13) - 1)) << 13;  // 8 KiB-aligned
      const uint32_t off = PAT == 3 ? lo : base + lo;
      if (PAT >= 4) {
        v[u] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0));
      } else {
        const uint4 q = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
        v[u] = __uint_as_float(q.x ^ q.y ^ q.z ^ q.w);
      }
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) s += v[u];
  }
  if (s == 1234.5f) out[0] = s;
}

int main() {
  char* buf;
  float* out;
  hipMalloc(&buf, kBuf + 8192);
  hipMalloc(&out, 16);
  hipMemset(buf, 1, kBuf + 8192);
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const char* names[6] = {"v4_contig", "v4_half", "v4_lines", "v4_oob", "b32_contig", "b32_lines"};
  for (int wpc : {4, 8, 16}) {  // waves per CU (workgroups of 4 waves)
    const int grid = cus * wpc / 4;
    for (int pat = 0; pat < 6; ++pat) {
      auto launch = [&](uint32_t salt) {
        switch (pat) {
          case 0: hipLaunchKernelGGL(k<0>, dim3(grid), dim3(256), 0, 0, buf, out, salt); break;
          case 1: hipLaunchKernelGGL(k<1>, dim3(grid), dim3(256), 0, 0, buf, out, salt); break;
          case 2: hipLaunchKernelGGL(k<2>, dim3(grid), dim3(256), 0, 0, buf, out, salt); break;
          case 3: hipLaunchKernelGGL(k<3>, dim3(grid), dim3(256), 0, 0, buf, out, salt); break;
          case 4: hipLaunchKernelGGL(k<4>, dim3(grid), dim3(256), 0, 0, buf, out, salt); break;
          default: hipLaunchKernelGGL(k<5>, dim3(grid), dim3(256), 0, 0, buf, out, salt); break;
        }
      };
      for (int w = 0; w < 3; ++w) launch(w);
      hipEventRecord(e0);
      const int reps = 10;
      for (int k2 = 0; k2 < reps; ++k2) launch(100 + k2);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms = 0.f;
      hipEventElapsedTime(&ms, e0, e1);
      const double per_cu_instr = (double)wpc * ITERS;  // wave-instructions per CU per launch
      printf("waves/CU %2d  %-10s  %.3f ms/launch  %.2f ns per wave-instruction per CU\n", wpc, names[pat],
             ms / reps, ms / reps * 1e6 / per_cu_instr);
    }
  }
  hipFree(buf);
  hipFree(out);
  return 0;
}
