// Cross entropy of up to 1024 rows by ONE 256-thread workgroup (mean over the rows whose label is not
// ignore_index, torch's CrossEntropyLoss defaults otherwise): the body of elementwise.hip's
// ce_small_kernel, shared with the head forward's in-launch finalizer (head_pb.hip HPFin), which
// forms the loss and dlogits right after the logits when the batch's labels came with it.  logits
// may point to LDS.  Every thread of the workgroup must call it.  Labels outside [0, N) other than
// ignore_index give a NaN loss (and NaN dlogits rows) instead of reading past the row.
#pragma once
#include "common.h"

namespace tds {

__device__ __forceinline__ void ce_small_block(const float* logits, const int64_t* __restrict__ labels,
                                               float* __restrict__ dlogits, float* __restrict__ loss_out,
                                               float* __restrict__ inv_count_out, int M, int N,
                                               int64_t ignore_index, float label_smoothing) {
  __shared__ float rl[1024];
  __shared__ float sh[16];
  const int lane = lane_id(), nw = blockDim.x / TDS_WAVE;
  const float eps = label_smoothing;
  for (int row = wave_id(); row < M; row += nw) {
    const float* z = logits + (int64_t)row * N;
    float mx = -INFINITY;
    for (int j = lane; j < N; j += TDS_WAVE) mx = fmaxf(mx, z[j]);
    mx = wave_max(mx);
    float sm = 0.f, zsum = 0.f;
    for (int j = lane; j < N; j += TDS_WAVE) { sm += __expf(z[j] - mx); zsum += z[j]; }
    sm = wave_sum(sm);
    zsum = wave_sum(zsum);
    const float lse = mx + __logf(sm);
    const int64_t lab = labels[row];
    const bool valid = lab != ignore_index;
    // a label outside [0, N) that is not ignore_index (torch raises 'Target out of bounds'): z is
    // read at a clamped index, and the row's loss and dlogits are NaN, so the step's loss is NaN
    const bool bad = valid && (lab < 0 || lab >= N);
    const int64_t lz = bad ? 0 : lab;
    if (lane == 0) rl[row] = bad ? NAN : valid ? (1.f - eps) * (lse - z[lz]) + eps * (lse - zsum / (float)N) : 0.f;
    for (int j = lane; j < N; j += TDS_WAVE) {
      float d = 0.f;
      if (valid) d = bad ? NAN : __expf(z[j] - lse) - ((j == lz ? (1.f - eps) : 0.f) + eps / (float)N);
      dlogits[(int64_t)row * N + j] = d;
    }
  }
  __syncthreads();  // rl complete; this block's dlogits writes visible to the block
  float l = 0.f, c = 0.f;
  for (int r = threadIdx.x; r < M; r += blockDim.x) {
    l += rl[r];
    c += labels[r] != ignore_index ? 1.f : 0.f;
  }
  l = block_sum(l, sh);
  c = block_sum(c, sh);
  const float inv = c > 0.f ? 1.f / c : 0.f;
  for (int64_t i = threadIdx.x; i < (int64_t)M * N; i += blockDim.x) dlogits[i] *= inv;
  if (threadIdx.x == 0) {
    loss_out[0] = c > 0.f ? l * inv : NAN;
    inv_count_out[0] = inv;
  }
}

}  // namespace tds
