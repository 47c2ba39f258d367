// First failed kernel launch of the calling host thread (see TDS_LAUNCH_CHECK in common.h).
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <tuple>
#include <utility>

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

// Counter words of the in-launch finalizers (common.h tds_arrive): one zeroed block per (device,
// stream), kSyncWordsPerSite words per call site.  Zeroed once, on the stream, when allocated;
// every reducer resets the counter it used, so each launch on that stream finds it at 0.
uint32_t* tds_sync_words(int site, hipStream_t st) {
  if (site < 0 || site >= tds::kSyncSites) return nullptr;
  static std::mutex mu;
  static std::map<std::pair<int, hipStream_t>, uint32_t*> cache;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  std::lock_guard<std::mutex> lock(mu);
  uint32_t*& w = cache[{dev, st}];
  if (w == nullptr) {
    const size_t bytes = (size_t)tds::kSyncSites * tds::kSyncWordsPerSite * sizeof(uint32_t);
    if (hipMalloc(&w, bytes) != hipSuccess) {
      w = nullptr;
      return nullptr;
    }
    if (hipMemsetAsync(w, 0, bytes, st) != hipSuccess) return nullptr;
  }
  return w + (size_t)site * tds::kSyncWordsPerSite;
}

// A zeroed 64-bit accumulator block per (device, stream, key) of at least n words (grown by
// reallocation when a larger n is asked for; zeroed on the stream when allocated).  Its users
// atomically add exact integer sums into it and the consumer zeroes what it read, so each launch on
// that stream finds it at 0 (like tds_sync_words' counters).
unsigned long long* tds_zeroed_u64(int key, size_t n, hipStream_t st) {
  static std::mutex mu;
  static std::map<std::tuple<int, hipStream_t, int>, std::pair<unsigned long long*, size_t>> cache;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  std::lock_guard<std::mutex> lock(mu);
  auto& e = cache[{dev, st, key}];
  if (e.first == nullptr || e.second < n) {
    if (e.first != nullptr) {  // (the stream's earlier launches may still use the old block)
      if (hipStreamSynchronize(st) != hipSuccess) return nullptr;
      (void)hipFree(e.first);
      e.first = nullptr;
    }
    if (hipMalloc(&e.first, n * sizeof(unsigned long long)) != hipSuccess) {
      e.first = nullptr;
      return nullptr;
    }
    e.second = n;
    if (hipMemsetAsync(e.first, 0, n * sizeof(unsigned long long), st) != hipSuccess) return nullptr;
  }
  return e.first;
}

// TDS_FUSED_FIN=0 restores the separate finalize launches (A/B timing and a fallback)
bool tds_fused_fin_enabled() {
  static const bool on = [] {
    const char* e = std::getenv("TDS_FUSED_FIN");
    return !(e && e[0] == '0');
  }();
  return on;
}
