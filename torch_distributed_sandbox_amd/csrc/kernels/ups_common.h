// Bilinear u8 upsample arithmetic (PIL-like: half-pixel centres, edge clamp, round to the nearest
// level) shared by every kernel that produces an upsampled image: elementwise.hip's upsample
// kernels and ups_moments.hip's upsample + x moments.  The multiply-adds are explicit fmaf so the
// compiler's contraction choices cannot make two kernels disagree on a level.
#pragma once

namespace tds {

constexpr int kUpsMaxW = 256;  // widest source the row kernel stages
constexpr int kUpsImg = 4096;  // sources up to this many pixels are staged whole (28x28 = 784)
constexpr int kUpsRows = 8;    // output rows per workgroup when the source is staged whole

// source taps of output coordinate X (scale s = n_src / n_dst): i0, i1 = min(i0 + 1, n - 1), weight a of i1
__device__ __forceinline__ void ups_taps(int X, float s, int n, int& i0, int& i1, float& a) {
  float f = fmaf((float)X + 0.5f, s, -0.5f);
  f = fminf(fmaxf(f, 0.f), (float)(n - 1));
  i0 = (int)f;
  i1 = min(i0 + 1, n - 1);
  a = f - (float)i0;
}

__device__ __forceinline__ float ups_lerp(float a, float b, float t) { return fmaf(t, b, (1.f - t) * a); }

// the level of an interpolated value (a convex combination of levels: the clamp never binds)
__device__ __forceinline__ float ups_level(float v) { return fminf(fmaxf(rintf(v), 0.f), 255.f); }

}  // namespace tds
