// Memory-bound elementwise / small kernels for the ConvNet hot path.
//
//  * relu fwd/bwd              (reference: nn.ReLU in mnist_onegpu.py:17,22 -> aten clamp_min / threshold_backward)
//  * maxpool 2x2/2 fwd/bwd     (nn.MaxPool2d(2,2), mnist_onegpu.py:18,23) with a 1-byte argmax instead of int64
//  * bilinear u8 upsample      (transforms.Resize(IMAGE_SHAPE)+ToTensor, mnist_onegpu.py:53) done on device
//  * SGD step                  (torch.optim.SGD(params, 1e-4), mnist_onegpu.py:49)
//  * cross-entropy fwd+bwd     (nn.CrossEntropyLoss, mnist_onegpu.py:48) fused in one launch
//
// All kernels are wave64, 16-byte vectorised where the layout allows, grid-capped
// at ~2048 blocks with grid-stride loops (Guideline 11).
#include <cstdlib>

#include "common.h"
#include "launchers.h"
#include "ce_small.h"
#include "ups_common.h"

namespace tds {

static inline int grid_for(int64_t n, int block, int64_t per_thread = 1) {
  int64_t g = (n + (int64_t)block * per_thread - 1) / ((int64_t)block * per_thread);
  if (g < 1) g = 1;
  if (g > 4096) g = 4096;
  return (int)g;
}

// ---------------------------------------------------------------- ReLU
__global__ void relu_fwd_kernel(const float* __restrict__ x, float* __restrict__ y, int64_t n) {
  const int64_t n4 = ((((uintptr_t)x) | ((uintptr_t)y)) & 15) ? 0 : n / 4;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const float4* x4 = reinterpret_cast<const float4*>(x);
  float4* y4 = reinterpret_cast<float4*>(y);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 v = x4[i];
    v.x = fmaxf(v.x, 0.f); v.y = fmaxf(v.y, 0.f); v.z = fmaxf(v.z, 0.f); v.w = fmaxf(v.w, 0.f);
    y4[i] = v;
  }
  for (int64_t i = n4 * 4 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    y[i] = fmaxf(x[i], 0.f);
}

// threshold_backward(grad, out, 0): grad where out > 0 else 0
__global__ void relu_bwd_kernel(const float* __restrict__ g, const float* __restrict__ out,
                                float* __restrict__ dx, int64_t n) {
  const int64_t n4 = ((((uintptr_t)g) | ((uintptr_t)out) | ((uintptr_t)dx)) & 15) ? 0 : n / 4;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const float4* g4 = reinterpret_cast<const float4*>(g);
  const float4* o4 = reinterpret_cast<const float4*>(out);
  float4* d4 = reinterpret_cast<float4*>(dx);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 a = g4[i], o = o4[i];
    a.x = o.x > 0.f ? a.x : 0.f; a.y = o.y > 0.f ? a.y : 0.f;
    a.z = o.z > 0.f ? a.z : 0.f; a.w = o.w > 0.f ? a.w : 0.f;
    d4[i] = a;
  }
  for (int64_t i = n4 * 4 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    dx[i] = out[i] > 0.f ? g[i] : 0.f;
}

// ---------------------------------------------------------------- MaxPool 2x2 stride 2 (floor)
// One thread per output element; the two input rows are read as float2 pairs.
// Tie-break = first maximum in scan order (matches aten max_pool2d); NaN wins.
__global__ void maxpool2_fwd_kernel(const float* __restrict__ x, float* __restrict__ y,
                                    uint8_t* __restrict__ idx, int64_t planes, int H, int W) {
  const int OH = H / 2, OW = W / 2;
  const int64_t total = planes * OH * OW;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t o = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; o < total; o += stride) {
    const int ox = (int)(o % OW);
    const int64_t t = o / OW;
    const int oy = (int)(t % OH);
    const int64_t p = t / OH;
    const float* base = x + (p * H + 2 * oy) * (int64_t)W + 2 * ox;
    float v0 = base[0], v1 = base[1], v2 = base[W], v3 = base[W + 1];
    float m = v0; int a = 0;
    if (v1 > m || isnan(v1)) { m = v1; a = 1; }
    if (v2 > m || isnan(v2)) { m = v2; a = 2; }
    if (v3 > m || isnan(v3)) { m = v3; a = 3; }
    y[o] = m;
    if (idx) idx[o] = (uint8_t)a;
  }
}

// Gather form of the backward: every input element reads the gradient of its
// window iff it was the argmax (no scatter, no zero-fill pass, fully coalesced).
__global__ void maxpool2_bwd_kernel(const float* __restrict__ gy, const uint8_t* __restrict__ idx,
                                    float* __restrict__ gx, int64_t planes, int H, int W) {
  const int OH = H / 2, OW = W / 2;
  const int64_t total = planes * H * (int64_t)W;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
    const int x = (int)(i % W);
    const int64_t t = i / W;
    const int y = (int)(t % H);
    const int64_t p = t / H;
    const int oy = y >> 1, ox = x >> 1;
    float g = 0.f;
    if (oy < OH && ox < OW) {
      const int64_t o = (p * OH + oy) * OW + ox;
      const int a = ((y & 1) << 1) | (x & 1);
      if (idx[o] == a) g = gy[o];
    }
    gx[i] = g;
  }
}

// ---------------------------------------------------------------- bilinear u8 upsample (PIL-like)
// dst[b,0,Y,X] = round(bilinear(src[b], half-pixel centres, edge clamp)) / 255.
// PIL's antialiased BILINEAR for magnification reduces to this triangle filter
// with renormalised edge taps == clamp.
// One workgroup per output row (grid = H x B): the row's vertical taps and the two
// source rows are fixed, so there is no 64-bit index arithmetic in the loop.  The two
// source rows (w <= 256 bytes each) are staged in LDS as floats; each thread writes 4
// consecutive pixels with one 16-byte store (plain, not non-temporal: the 180 MB
// image is read again right away by the layer-1 kernels and can stay in the MALL).  The arithmetic order is exactly the
// per-pixel formula above, so the result is bit-identical to the scalar form.
// (kUpsMaxW / kUpsImg / kUpsRows and the per-pixel arithmetic: ups_common.h)

// one output row Y from the two source rows r0 (y0), r1 (y1) in LDS
template <bool U8OUT>
__device__ __forceinline__ void ups_row(const float* r0, const float* r1, float ay, void* __restrict__ dstv, int b,
                                        int Y, int w, int H, int W, float sx) {
  auto lvl = [&](int X) {
    int x0, x1;
    float ax;
    ups_taps(X, sx, w, x0, x1, ax);
    return ups_level(ups_lerp(ups_lerp(r0[x0], r0[x1], ax), ups_lerp(r1[x0], r1[x1], ax), ay));
  };
  if constexpr (U8OUT) {
    uint8_t* d8 = reinterpret_cast<uint8_t*>(dstv) + ((int64_t)b * H + Y) * W;
    const int W4 = ((((uintptr_t)d8) & 3) == 0) ? (W >> 2) : 0;
    for (int q = threadIdx.x; q < W4; q += blockDim.x) {
      const int X = q << 2;
      const uint32_t v = (uint32_t)lvl(X) | ((uint32_t)lvl(X + 1) << 8) | ((uint32_t)lvl(X + 2) << 16) |
                         ((uint32_t)lvl(X + 3) << 24);
      reinterpret_cast<uint32_t*>(d8)[q] = v;
    }
    for (int X = (W4 << 2) + threadIdx.x; X < W; X += blockDim.x) d8[X] = (uint8_t)lvl(X);
  } else {
    float* d = reinterpret_cast<float*>(dstv) + ((int64_t)b * H + Y) * W;
    auto pix = [&](int X) { return lvl(X) * (1.f / 255.f); };
    const bool vec = ((((uintptr_t)d) & 15) == 0);
    const int W4 = vec ? (W >> 2) : 0;
    for (int q = threadIdx.x; q < W4; q += blockDim.x) {
      const int X = q << 2;
      f32x4 v;
      v[0] = pix(X); v[1] = pix(X + 1); v[2] = pix(X + 2); v[3] = pix(X + 3);
      reinterpret_cast<f32x4*>(d)[q] = v;
    }
    for (int X = (W4 << 2) + threadIdx.x; X < W; X += blockDim.x) d[X] = pix(X);
  }
}

__device__ __forceinline__ void ups_vtaps(int Y, int h, float sy, int& y0, int& y1, float& ay) {
  ups_taps(Y, sy, h, y0, y1, ay);
}

// One workgroup per output row (grid = H x B): the row's two source rows staged in LDS.
// U8OUT: the rounded level itself (uint8), i.e. ToTensor's input before its 1/255 -- the fused
// ConvNet plan folds that scale into conv1 (convnet_fused.hip, x_autocorr.hip).
template <bool U8OUT>
__global__ void __launch_bounds__(256) upsample_bilinear_u8_kernel(const uint8_t* __restrict__ src,
                                                                   void* __restrict__ dstv, int B, int h, int w,
                                                                   int H, int W) {
  __shared__ float rows[2][kUpsMaxW];
  const int Y = blockIdx.x, b = blockIdx.y;
  const float sy = (float)h / (float)H, sx = (float)w / (float)W;
  int y0, y1;
  float ay;
  ups_vtaps(Y, h, sy, y0, y1, ay);
  const uint8_t* s = src + (int64_t)b * h * w;
  for (int x = threadIdx.x; x < w; x += blockDim.x) {
    rows[0][x] = (float)s[y0 * w + x];
    rows[1][x] = (float)s[y1 * w + x];
  }
  __syncthreads();
  ups_row<U8OUT>(rows[0], rows[1], ay, dstv, b, Y, w, H, W, sx);
}

// Small sources (h*w <= kUpsImg, the 28x28 MNIST digits): the whole source image staged once per
// workgroup and kUpsRows output rows per workgroup (grid = ceil(H / kUpsRows) x B); a thread keeps
// the horizontal taps of its 4 columns in registers for all the rows (the kernel is VALU-bound: one
// row per workgroup recomputed them per pixel and ran at 38 us for 5 x 3000^2).  Same arithmetic
// per pixel as ups_row, so the output is bit-identical to the row kernel.
template <bool U8OUT>
__global__ void __launch_bounds__(256) upsample_bilinear_u8_img_kernel(const uint8_t* __restrict__ src,
                                                                       void* __restrict__ dstv, int B, int h, int w,
                                                                       int H, int W) {
  __shared__ float img[kUpsImg];
  const int b = blockIdx.y, Yb = blockIdx.x * kUpsRows;
  const float sy = (float)h / (float)H, sx = (float)w / (float)W;
  const uint8_t* s = src + (int64_t)b * h * w;
  for (int i = threadIdx.x; i < h * w; i += blockDim.x) img[i] = (float)s[i];
  __syncthreads();
  const int nr = min(kUpsRows, H - Yb);
  // rows of this workgroup start 4-byte (u8) / 16-byte (fp32) aligned only when W allows it
  const bool vec = (W & 3) == 0;
  const int W4 = vec ? (W >> 2) : 0;
  for (int q = threadIdx.x; q < W4; q += blockDim.x) {
    int x0[4], x1[4];
    float ax[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) ups_taps(4 * q + k, sx, w, x0[k], x1[k], ax[k]);
    for (int r = 0; r < nr; ++r) {
      int y0, y1;
      float ay;
      ups_vtaps(Yb + r, h, sy, y0, y1, ay);
      const float* r0 = img + y0 * w;
      const float* r1 = img + y1 * w;
      float lv[4];
#pragma unroll
      for (int k = 0; k < 4; ++k)
        lv[k] = ups_level(ups_lerp(ups_lerp(r0[x0[k]], r0[x1[k]], ax[k]), ups_lerp(r1[x0[k]], r1[x1[k]], ax[k]), ay));
      const int64_t row = (int64_t)b * H + Yb + r;
      if constexpr (U8OUT) {
        reinterpret_cast<uint32_t*>(reinterpret_cast<uint8_t*>(dstv) + row * W)[q] =
            (uint32_t)lv[0] | ((uint32_t)lv[1] << 8) | ((uint32_t)lv[2] << 16) | ((uint32_t)lv[3] << 24);
      } else {
        f32x4 v;
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] = lv[k] * (1.f / 255.f);
        reinterpret_cast<f32x4*>(reinterpret_cast<float*>(dstv) + row * W)[q] = v;
      }
    }
  }
  if (W4 * 4 < W) {  // the unvectorised remainder (every column when W % 4 != 0)
    for (int r = 0; r < nr; ++r) {
      int y0, y1;
      float ay;
      ups_vtaps(Yb + r, h, sy, y0, y1, ay);
      const float* r0 = img + y0 * w;
      const float* r1 = img + y1 * w;
      for (int X = W4 * 4 + threadIdx.x; X < W; X += blockDim.x) {
        int a0, a1;
        float a;
        ups_taps(X, sx, w, a0, a1, a);
        const float v = ups_level(ups_lerp(ups_lerp(r0[a0], r0[a1], a), ups_lerp(r1[a0], r1[a1], a), ay));
        const int64_t o = ((int64_t)b * H + Yb + r) * W + X;
        if constexpr (U8OUT) reinterpret_cast<uint8_t*>(dstv)[o] = (uint8_t)v;
        else reinterpret_cast<float*>(dstv)[o] = v * (1.f / 255.f);
      }
    }
  }
}

// ---------------------------------------------------------------- SGD over a tensor list
// Plain SGD (torch.optim.SGD defaults: momentum 0, dampening 0, no nesterov):
//   g' = g + wd * p ; if momentum: buf = mom*buf + (1-damp)*g' (first step buf = g'); p -= lr * g'
__global__ void sgd_multi_kernel(SgdChunkTable tab, float lr, float wd, float momentum, float dampening,
                                 int nesterov, int first_step) {
  const int ti = blockIdx.y;
  if (ti >= tab.n) return;
  float* __restrict__ p = tab.param[ti];
  const float* __restrict__ g = tab.grad[ti];
  float* __restrict__ buf = tab.mom[ti];
  const int64_t n = tab.numel[ti];
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const bool vec = ((((uintptr_t)p) | ((uintptr_t)g) | ((uintptr_t)buf)) & 15) == 0 && momentum == 0.f && wd == 0.f;
  if (vec) {
    const int64_t n4 = n / 4;
    float4* p4 = reinterpret_cast<float4*>(p);
    const float4* g4 = reinterpret_cast<const float4*>(g);
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
      float4 a = p4[i]; const float4 b = g4[i];
      a.x -= lr * b.x; a.y -= lr * b.y; a.z -= lr * b.z; a.w -= lr * b.w;
      p4[i] = a;
    }
    for (int64_t i = n4 * 4 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
      p[i] -= lr * g[i];
    return;
  }
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    float d = g[i];
    if (wd != 0.f) d += wd * p[i];
    if (momentum != 0.f) {
      float b = first_step ? d : momentum * buf[i] + (1.f - dampening) * d;
      buf[i] = b;
      d = nesterov ? d + momentum * b : b;
    }
    p[i] -= lr * d;
  }
}

// ---------------------------------------------------------------- cross entropy (mean, ignore_index)
// One wave per row, classes strided over lanes.  Writes per-row loss, the
// "dlogits for grad_out == 1" and the valid-row count; a second tiny kernel
// finalises the mean.  M is small (global batch rows), N is #classes.
__global__ void ce_rows_kernel(const float* __restrict__ logits, const int64_t* __restrict__ labels,
                               float* __restrict__ row_loss, float* __restrict__ dlogits,
                               int M, int N, int64_t ignore_index, float label_smoothing) {
  const int row = blockIdx.x * (blockDim.x / TDS_WAVE) + wave_id();
  if (row >= M) return;
  const int lane = lane_id();
  const float* z = logits + (int64_t)row * N;
  float mx = -INFINITY;
  for (int j = lane; j < N; j += TDS_WAVE) mx = fmaxf(mx, z[j]);
  mx = wave_max(mx);
  float s = 0.f, zsum = 0.f;
  for (int j = lane; j < N; j += TDS_WAVE) { s += __expf(z[j] - mx); zsum += z[j]; }
  s = wave_sum(s);
  zsum = wave_sum(zsum);
  const float lse = mx + __logf(s);
  const int64_t lab = labels[row];
  const bool valid = lab != ignore_index;
  const float eps = label_smoothing;
  if (lane == 0) {
    float l = 0.f;
    if (valid) {
      const float nll = lse - z[lab];
      const float smooth = lse - zsum / (float)N;
      l = (1.f - eps) * nll + eps * smooth;
    }
    row_loss[row] = valid ? l : 0.f;
  }
  for (int j = lane; j < N; j += TDS_WAVE) {
    float d = 0.f;
    if (valid) {
      const float p = __expf(z[j] - lse);
      const float tgt = (j == lab ? (1.f - eps) : 0.f) + eps / (float)N;
      d = p - tgt;
    }
    dlogits[(int64_t)row * N + j] = d;  // un-normalised; scaled by 1/valid in finalize
  }
}

__global__ void ce_finalize_kernel(const float* __restrict__ row_loss, const int64_t* __restrict__ labels,
                                   float* __restrict__ dlogits, float* __restrict__ loss_out,
                                   float* __restrict__ inv_count_out, int M, int N, int64_t ignore_index) {
  __shared__ float sh[16];
  float l = 0.f, c = 0.f;
  for (int r = threadIdx.x; r < M; r += blockDim.x) {
    l += row_loss[r];
    c += labels[r] != ignore_index ? 1.f : 0.f;
  }
  l = block_sum(l, sh);
  c = block_sum(c, sh);
  const float inv = c > 0.f ? 1.f / c : 0.f;  // PyTorch: mean over zero valid rows is NaN; we give 0/0
  for (int64_t i = threadIdx.x; i < (int64_t)M * N; i += blockDim.x) dlogits[i] *= inv;
  if (threadIdx.x == 0) {
    loss_out[0] = c > 0.f ? l * inv : NAN;
    inv_count_out[0] = inv;
  }
}

// Cross entropy of up to 1024 rows in ONE workgroup (the training batch: the two-kernel form
// below is two launches for 5 x 10 logits): waves take rows round-robin (the per-row math of
// ce_rows_kernel), then the block reduces loss and valid count and scales dlogits by 1/count.
__global__ __launch_bounds__(256) void ce_small_kernel(const float* __restrict__ logits,
                                                       const int64_t* __restrict__ labels,
                                                       float* __restrict__ dlogits, float* __restrict__ loss_out,
                                                       float* __restrict__ inv_count_out, int M, int N,
                                                       int64_t ignore_index, float label_smoothing) {
  ce_small_block(logits, labels, dlogits, loss_out, inv_count_out, M, N, ignore_index, label_smoothing);  // (ce_small.h)
}

// dlogits *= grad_out (scalar tensor on device) — keeps the backward sync-free.
__global__ void scale_by_device_scalar_kernel(const float* __restrict__ in, const float* __restrict__ s,
                                              float* __restrict__ out, int64_t n) {
  const float k = s[0];
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = in[i] * k;
}

}  // namespace tds

using namespace tds;

void tds_relu_fwd(const float* x, float* y, int64_t n, hipStream_t st) {
  hipLaunchKernelGGL(relu_fwd_kernel, dim3(grid_for(n, 256, 16)), dim3(256), 0, st, x, y, n);
  TDS_LAUNCH_CHECK();
}
void tds_relu_bwd(const float* g, const float* out, float* dx, int64_t n, hipStream_t st) {
  hipLaunchKernelGGL(relu_bwd_kernel, dim3(grid_for(n, 256, 16)), dim3(256), 0, st, g, out, dx, n);
  TDS_LAUNCH_CHECK();
}
void tds_maxpool2_fwd(const float* x, float* y, uint8_t* idx, int64_t planes, int H, int W, hipStream_t st) {
  const int64_t total = planes * (H / 2) * (int64_t)(W / 2);
  if (total == 0) return;
  hipLaunchKernelGGL(maxpool2_fwd_kernel, dim3(grid_for(total, 256, 4)), dim3(256), 0, st, x, y, idx, planes, H, W);
  TDS_LAUNCH_CHECK();
}
void tds_maxpool2_bwd(const float* gy, const uint8_t* idx, float* gx, int64_t planes, int H, int W, hipStream_t st) {
  const int64_t total = planes * H * (int64_t)W;
  if (total == 0) return;
  hipLaunchKernelGGL(maxpool2_bwd_kernel, dim3(grid_for(total, 256, 4)), dim3(256), 0, st, gy, idx, gx, planes, H, W);
  TDS_LAUNCH_CHECK();
}
void tds_upsample_bilinear_u8(const uint8_t* src, void* dst, bool u8_out, int B, int h, int w, int H, int W,
                              hipStream_t st) {
  if ((int64_t)B * H * W == 0) return;
  if (w > kUpsMaxW || h < 1 || B > 65535) {  // the op wrapper rejects these shapes first (ops.cpp)
    tds_launch_fail("upsample_bilinear_u8: unsupported shape");
    return;
  }
  // whole-source kernel for small sources: 31.0 us vs 37.6 us for the row kernel at 5 x 3000^2, bench
  // 2.891 / 2.899 vs 2.915 / 2.929 ms per step same box (tools/gpu_sessions/r3_s23.sh; its first form,
  // without the hoisted taps, measured 44 us).  TDS_UPS_IMG=0 selects the row kernel (A/B only).
  static const bool img = [] {
    const char* e = std::getenv("TDS_UPS_IMG");
    return !(e && e[0] == '0');
  }();
  if (img && h * w <= kUpsImg) {
    const dim3 grid((H + kUpsRows - 1) / kUpsRows, B);
    if (u8_out)
      hipLaunchKernelGGL(upsample_bilinear_u8_img_kernel<true>, grid, dim3(256), 0, st, src, dst, B, h, w, H, W);
    else
      hipLaunchKernelGGL(upsample_bilinear_u8_img_kernel<false>, grid, dim3(256), 0, st, src, dst, B, h, w, H, W);
  } else if (u8_out) {
    hipLaunchKernelGGL(upsample_bilinear_u8_kernel<true>, dim3(H, B), dim3(256), 0, st, src, dst, B, h, w, H, W);
  } else {
    hipLaunchKernelGGL(upsample_bilinear_u8_kernel<false>, dim3(H, B), dim3(256), 0, st, src, dst, B, h, w, H, W);
  }
  TDS_LAUNCH_CHECK();
}
void tds_sgd_multi(const SgdChunkTable& tab, float lr, float wd, float momentum, float dampening, int nesterov,
                   int first_step, int64_t max_numel, hipStream_t st) {
  if (tab.n == 0) return;
  int gx = grid_for(max_numel, 256, 16);
  if (gx > 1024) gx = 1024;
  hipLaunchKernelGGL(sgd_multi_kernel, dim3(gx, tab.n), dim3(256), 0, st, tab, lr, wd, momentum, dampening,
                     nesterov, first_step);
  TDS_LAUNCH_CHECK();
}
void tds_cross_entropy(const float* logits, const int64_t* labels, float* row_loss, float* dlogits, float* loss,
                       float* inv_count, int M, int N, int64_t ignore_index, float label_smoothing, hipStream_t st) {
  if (M <= 1024) {
    hipLaunchKernelGGL(ce_small_kernel, dim3(1), dim3(256), 0, st, logits, labels, dlogits, loss, inv_count, M, N,
                       ignore_index, label_smoothing);
    TDS_LAUNCH_CHECK();
    return;
  }
  const int rows_per_block = 4;
  hipLaunchKernelGGL(ce_rows_kernel, dim3((M + rows_per_block - 1) / rows_per_block), dim3(64 * rows_per_block), 0, st,
                     logits, labels, row_loss, dlogits, M, N, ignore_index, label_smoothing);
  TDS_LAUNCH_CHECK();
  hipLaunchKernelGGL(ce_finalize_kernel, dim3(1), dim3(256), 0, st, row_loss, labels, dlogits, loss, inv_count, M, N,
                     ignore_index);
  TDS_LAUNCH_CHECK();
}
void tds_scale_by_device_scalar(const float* in, const float* s, float* out, int64_t n, hipStream_t st) {
  hipLaunchKernelGGL(scale_by_device_scalar_kernel, dim3(grid_for(n, 256, 4)), dim3(256), 0, st, in, s, out, n);
  TDS_LAUNCH_CHECK();
}
