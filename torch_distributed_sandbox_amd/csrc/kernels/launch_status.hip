// First failed kernel launch of the calling host thread (see TDS_LAUNCH_CHECK in common.h).
#include <cstdio>
#include <cstring>

#include "common.h"
#include "launchers.h"

namespace {
thread_local char g_msg[256] = {0};
thread_local int g_failed = 0;
}  // namespace

void tds_note_launch(hipError_t e, const char* where, int line) {
  if (e == hipSuccess || g_failed) return;
  g_failed = 1;
  std::snprintf(g_msg, sizeof(g_msg), "kernel launch failed in %s (line %d): %s", where, line, hipGetErrorString(e));
}

void tds_launch_fail(const char* what) {
  if (g_failed) return;
  g_failed = 1;
  std::snprintf(g_msg, sizeof(g_msg), "launcher refused: %s", what);
}

int tds_take_launch_error(char* buf, int n) {
  if (!g_failed) return 0;
  if (buf && n > 0) {
    std::strncpy(buf, g_msg, (size_t)n - 1);
    buf[n - 1] = 0;
  }
  g_failed = 0;
  g_msg[0] = 0;
  return 1;
}

// Deliberately bad launch for tests: an LDS request above the 160 KiB a workgroup can have.
__global__ void tds_probe_kernel(int* out) {
  extern __shared__ int s[];
  s[threadIdx.x] = (int)threadIdx.x;
  __syncthreads();
  if (out) out[threadIdx.x] = s[threadIdx.x];
}

void tds_launch_probe(int* out, int lds_bytes, int threads, hipStream_t st) {
  hipLaunchKernelGGL(tds_probe_kernel, dim3(1), dim3(threads), lds_bytes, st, out);
  TDS_LAUNCH_CHECK();
}
