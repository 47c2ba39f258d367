// CU budget of the persistent kernels and CU-masked compute streams (SURVEY.md §7.2 step 6,
// the xGMI comm design: leave CUs to RCCL's kernels while the backward overlaps a collective).
//
// The persistent conv / layer-1 kernels launch one (or k) workgroups per CU and stride over
// their tiles, so a kernel on a CU-masked stream must size its grid to the CUs it may use, or
// the surplus workgroups queue behind the first wave.  tds_device_cus() is that count:
// multiProcessorCount (cached per device) minus the reserve set by tds_set_cu_reserve().
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <atomic>
#include <mutex>
#include <utility>
#include <cstdint>
#include <vector>

#include "launchers.h"

namespace {
constexpr int kMaxDev = 64;
std::atomic<int> g_cus[kMaxDev];
std::atomic<int> g_reserve{0};
std::atomic<bool> g_striped{true};  // mask-bit numbering of the last compute mask (tds_cu_masked_stream)

// Index of CU bit `cu` inside its XCD under either numbering (see tds_cu_masked_stream).
inline int cu_local(int cu, int nxcd, int per, bool striped) { return striped ? cu / nxcd : cu % per; }
}  // namespace

int tds_device_cus() {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDev) dev = 0;
  int n = g_cus[dev].load(std::memory_order_relaxed);
  if (n <= 0) {
    hipDeviceProp_t prop;
    n = (hipGetDeviceProperties(&prop, dev) == hipSuccess && prop.multiProcessorCount > 0) ? prop.multiProcessorCount
                                                                                            : 256;
    g_cus[dev].store(n, std::memory_order_relaxed);
  }
  const int r = g_reserve.load(std::memory_order_relaxed);
  return n - r >= 8 ? n - r : 8;
}

void tds_set_cu_reserve(int n) { g_reserve.store(n > 0 ? n : 0, std::memory_order_relaxed); }

int tds_cu_reserve() { return g_reserve.load(std::memory_order_relaxed); }

// Every CU-masked stream this file creates, for tds_cu_release_streams.
static std::mutex g_masked_mu;
static std::vector<hipStream_t> g_masked;
static std::mutex g_comm_mu, g_side_mu;
static std::vector<std::pair<std::pair<int, int>, hipStream_t>> g_comm_cache, g_side_cache;
static void note_masked(hipStream_t s) {
  std::lock_guard<std::mutex> g(g_masked_mu);
  g_masked.push_back(s);
}

// A stream of `device` whose kernels may use every CU but `reserve` of them, reserve/8 per XCD
// (hipExtStreamCreateWithCUMask).  Two numberings of the mask bits are possible: `striped`
// (bit c -> XCD c % 8, the order the dispatcher deals workgroups round-robin to the XCDs) and
// `blocked` (XCD by XCD, 32 bits each).  A mask built for the wrong one leaves some XCDs with
// fewer CUs than the persistent grid gives them workgroups, which then run in two rounds (the
// whole step +60-70 %).  Returns nullptr on failure (or a reserve that is not a multiple of 8).
// The stream lives for the process.
hipStream_t tds_cu_masked_stream(int device, int reserve, bool striped) {
  if (reserve < 0 || reserve % 8 != 0) return nullptr;
  int prev = 0;
  if (hipGetDevice(&prev) != hipSuccess) return nullptr;
  if (hipSetDevice(device) != hipSuccess) return nullptr;
  hipDeviceProp_t prop;
  hipStream_t s = nullptr;
  if (hipGetDeviceProperties(&prop, device) == hipSuccess) {
    const int n = prop.multiProcessorCount, nxcd = 8, per = n / nxcd, rx = reserve / nxcd;
    if (n % nxcd == 0 && per - rx >= 1) {
      std::vector<uint32_t> mask((n + 31) / 32, 0u);
      for (int cu = 0; cu < n; ++cu) {
        if (cu_local(cu, nxcd, per, striped) < per - rx) mask[cu / 32] |= 1u << (cu % 32);
      }
      if (hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data()) != hipSuccess) s = nullptr;
    }
  }
  (void)hipSetDevice(prev);
  if (s) {
    g_striped.store(striped, std::memory_order_relaxed);
    note_masked(s);
  }
  return s;
}

// The communication side of the split: a stream of `device` confined to the CUs the compute
// stream leaves out (the exact complement of tds_cu_masked_stream's mask for the current reserve,
// in the same bit numbering), so RCCL's kernels -- launched on the communicator's stream -- land
// on CUs no persistent compute workgroup waits for.  nullptr when no CUs are reserved.  Cached
// per (device, reserve, numbering); the streams live for the process.
hipStream_t tds_cu_comm_stream(int device) {
  const int reserve = g_reserve.load(std::memory_order_relaxed);
  const bool striped = g_striped.load(std::memory_order_relaxed);
  if (reserve <= 0 || reserve % 8 != 0 || device < 0 || device >= kMaxDev) return nullptr;
  const int key = reserve * 2 + (striped ? 1 : 0);
  auto& cache = g_comm_cache;
  std::lock_guard<std::mutex> g(g_comm_mu);
  for (auto& e : cache)
    if (e.first.first == device && e.first.second == key) return e.second;
  int prev = 0;
  if (hipGetDevice(&prev) != hipSuccess) return nullptr;
  if (hipSetDevice(device) != hipSuccess) return nullptr;
  hipDeviceProp_t prop;
  hipStream_t s = nullptr;
  if (hipGetDeviceProperties(&prop, device) == hipSuccess) {
    const int n = prop.multiProcessorCount, nxcd = 8, per = n / nxcd, rx = reserve / nxcd;
    if (n % nxcd == 0 && per - rx >= 1) {
      std::vector<uint32_t> mask((n + 31) / 32, 0u);
      for (int cu = 0; cu < n; ++cu)
        if (cu_local(cu, nxcd, per, striped) >= per - rx) mask[cu / 32] |= 1u << (cu % 32);
      if (hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data()) != hipSuccess) s = nullptr;
    }
  }
  (void)hipSetDevice(prev);
  if (s) {
    cache.push_back({{device, key}, s});
    note_masked(s);
  }
  return s;
}

// A further stream of `device` on one side of the current split (comm: the reserved CUs; else
// the compute CUs), distinct from the communicator's and the compute stream: DDP's side work
// (the exchange's dW formation, the deferred SGD step) runs there so it neither lands on CUs a
// persistent compute workgroup waits for nor queues behind RCCL's kernels.  nullptr when no
// CUs are reserved.  Cached per (device, reserve, numbering, side).
hipStream_t tds_cu_side_stream(int device, bool comm) {
  const int reserve = g_reserve.load(std::memory_order_relaxed);
  const bool striped = g_striped.load(std::memory_order_relaxed);
  if (reserve <= 0 || reserve % 8 != 0 || device < 0 || device >= kMaxDev) return nullptr;
  const int key = (reserve * 2 + (striped ? 1 : 0)) * 2 + (comm ? 1 : 0);
  auto& cache = g_side_cache;
  std::lock_guard<std::mutex> g(g_side_mu);
  for (auto& e : cache)
    if (e.first.first == device && e.first.second == key) return e.second;
  int prev = 0;
  if (hipGetDevice(&prev) != hipSuccess) return nullptr;
  if (hipSetDevice(device) != hipSuccess) return nullptr;
  hipDeviceProp_t prop;
  hipStream_t s = nullptr;
  if (hipGetDeviceProperties(&prop, device) == hipSuccess) {
    const int n = prop.multiProcessorCount, nxcd = 8, per = n / nxcd, rx = reserve / nxcd;
    if (n % nxcd == 0 && per - rx >= 1) {
      std::vector<uint32_t> mask((n + 31) / 32, 0u);
      for (int cu = 0; cu < n; ++cu)
        if ((cu_local(cu, nxcd, per, striped) >= per - rx) == comm) mask[cu / 32] |= 1u << (cu % 32);
      if (hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data()) != hipSuccess) s = nullptr;
    }
  }
  (void)hipSetDevice(prev);
  if (s) {
    cache.push_back({{device, key}, s});
    note_masked(s);
  }
  return s;
}

// Synchronize and destroy every CU-masked stream created here; the caches forget them.  For the
// end of a single-process run that used the split (bench.py --reserve-cus): left to process
// exit, the HIP runtime's teardown of their HSA queues and rocprofiler-sdk's own finalization
// race -- under rocprofv3 the tool's __cxa_finalize handler faults inside libhsa-runtime64 on a
// queue page already unmapped (frames resolved with tools/micro/exit_maps.py,
// tools/gpu_sessions/r3_s16.sh).  The caller must no longer use the streams (nor the torch
// ExternalStream objects around them).  Returns how many were destroyed.
int tds_cu_release_streams() {
  std::vector<hipStream_t> all;
  {
    std::lock_guard<std::mutex> g(g_masked_mu);
    all.swap(g_masked);
  }
  {
    std::lock_guard<std::mutex> g(g_comm_mu);
    g_comm_cache.clear();
  }
  {
    std::lock_guard<std::mutex> g(g_side_mu);
    g_side_cache.clear();
  }
  int n = 0;
  for (hipStream_t s : all) {
    (void)hipStreamSynchronize(s);
    if (hipStreamDestroy(s) == hipSuccess) ++n;
  }
  g_reserve.store(0, std::memory_order_relaxed);
  return n;
}

// ---- one-GPU rehearsal of a collective's CU footprint -----------------------------------
// RCCL's generic kernel on gfx950 takes 256 threads, 19.7 KB of LDS and 261-280 VGPRs per
// workgroup (librccl code-object metadata), one workgroup per channel, resident for the whole
// collective.  comm_spin_kernel holds the same LDS for `us` microseconds on each of its
// workgroups (constant 100 MHz clock), so a single-GPU step can be timed with a "collective"
// in flight: a persistent compute kernel cannot place a workgroup on a CU the spin occupies.
__global__ __launch_bounds__(256) void comm_spin_kernel(int64_t ticks, int* sink) {
  extern __shared__ int lds[];
  const int64_t t0 = (int64_t)__builtin_amdgcn_s_memrealtime();
  lds[threadIdx.x] = (int)threadIdx.x;
  int acc = 0;
  while ((int64_t)__builtin_amdgcn_s_memrealtime() - t0 < ticks) {
    __builtin_amdgcn_s_sleep(8);
    acc += lds[(threadIdx.x + acc) & 255];
  }
  if (acc == 0x7fffffff) sink[blockIdx.x] = acc;  // never true: keeps the loop
}

void tds_comm_spin(int64_t us, int nblocks, int lds_bytes, int* sink, hipStream_t st) {
  hipLaunchKernelGGL(comm_spin_kernel, dim3(nblocks), dim3(256), (size_t)lds_bytes, st, us * 100, sink);
}

// Where workgroups land: each workgroup holds 64 KiB of LDS for ~`us` microseconds (so the
// dispatcher spreads them over the CUs it may use) and records its XCC and HW_ID (CU, SE).
__global__ __launch_bounds__(64) void cu_probe_kernel(int64_t ticks, int* out) {
  extern __shared__ int lds[];
  const int64_t t0 = (int64_t)__builtin_amdgcn_s_memrealtime();
  int hwid, xcc;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hwid));
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  lds[threadIdx.x] = hwid;
  while ((int64_t)__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
  if (threadIdx.x == 0) {
    out[2 * blockIdx.x] = xcc;
    out[2 * blockIdx.x + 1] = lds[0];
  }
}

void tds_cu_probe(int64_t us, int nblocks, int* out, hipStream_t st) {
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(cu_probe_kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                            64 * 1024);
  hipLaunchKernelGGL(cu_probe_kernel, dim3(nblocks), dim3(64), 64 * 1024, st, us * 100, out);
}
