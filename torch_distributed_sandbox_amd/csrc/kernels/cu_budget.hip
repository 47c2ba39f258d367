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
#include <cstdint>
#include <vector>

#include "launchers.h"

namespace {
constexpr int kMaxDev = 64;
std::atomic<int> g_cus[kMaxDev];
std::atomic<int> g_reserve{0};
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

// A stream of `device` whose kernels may use every CU but `reserve` of them, reserve/8 per XCD
// (hipExtStreamCreateWithCUMask).  The mask is in the driver's logical CU numbering, which on
// MI355X runs XCD by XCD (32 CUs each): masking the top CUs of the chip instead left one XCD
// with half its CUs, and the workgroups dispatched round-robin to it (one persistent workgroup
// per CU) ran in two rounds -- the whole step took +70 %.  Returns nullptr on failure (or a
// reserve that is not a multiple of 8).  The stream lives for the process.
hipStream_t tds_cu_masked_stream(int device, int reserve) {
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
      for (int cu = 0; cu < n; ++cu)
        if (cu % per < per - rx) mask[cu / 32] |= 1u << (cu % 32);
      if (hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data()) != hipSuccess) s = nullptr;
    }
  }
  (void)hipSetDevice(prev);
  return s;
}
