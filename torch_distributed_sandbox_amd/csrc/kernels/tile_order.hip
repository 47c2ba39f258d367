// Host-built, device-resident tile order tables for the persistent conv2 kernels
// (conv2_common.h: blocked_tile / tds_tile_order).
#include <mutex>
#include <map>
#include <tuple>
#include <vector>

#include "conv2_common.h"

namespace tds {

// host mirror of blocked_tile<BC, GR, GC>
static void host_blocked_tile(int t, int per_img, int tiles_r, int tiles_c, int& b, int& tr, int& tc) {
  constexpr int BC = 32, GR = 16, GC = 4;
  b = t / per_img;
  int off = t - b * per_img;
  const int band = off / (BC * tiles_r);
  off -= band * BC * tiles_r;
  const int wj = std::min(BC, tiles_c - band * BC);
  const int gr = off / (GR * wj);
  off -= gr * GR * wj;
  const int hg = std::min(GR, tiles_r - gr * GR);
  const int cg = off / (GC * hg);
  off -= cg * GC * hg;
  const int wc = std::min(GC, wj - cg * GC);
  const int r = off / wc;
  tr = gr * GR + r;
  tc = band * BC + cg * GC + (off - r * wc);
}

const int* tds_tile_order(int B, int tiles_r, int tiles_c) {
  static std::mutex mu;
  static std::map<std::tuple<int, int, int, int>, int*> cache;
  int dev = 0;
  (void)hipGetDevice(&dev);
  const auto key = std::make_tuple(dev, B, tiles_r, tiles_c);
  std::lock_guard<std::mutex> lock(mu);
  auto it = cache.find(key);
  if (it != cache.end()) return it->second;
  if (B > 255 || tiles_r > 4095 || tiles_c > 4095) return nullptr;
  const int per_img = tiles_r * tiles_c, total = per_img * B;
  std::vector<int> h(total);
  for (int t = 0; t < total; ++t) {
    int b, tr, tc;
    host_blocked_tile(t, per_img, tiles_r, tiles_c, b, tr, tc);
    h[t] = (b << 24) | (tr << 12) | tc;
  }
  int* d = nullptr;
  if (hipMalloc(&d, sizeof(int) * (size_t)total) != hipSuccess) return nullptr;
  if (hipMemcpy(d, h.data(), sizeof(int) * (size_t)total, hipMemcpyHostToDevice) != hipSuccess) return nullptr;
  cache[key] = d;
  return d;
}

}  // namespace tds
