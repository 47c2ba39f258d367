// Training-mode BatchNorm2d for NCHW fp32 (reference: nn.BatchNorm2d(16/32),
// mnist_onegpu.py:16,21 -> cudnn_batch_norm / native_batch_norm_backward,
// SURVEY.md §2.4 K2, K6, K18, K24).
//
// Semantics reproduced: batch statistics over (N,H,W), biased variance for
// normalisation, unbiased variance into running_var, momentum (default 0.1),
// eps 1e-5, num_batches_tracked += 1.
//
// Reductions: each workgroup reduces a contiguous chunk of one channel with
// per-thread fp64 accumulators (45M elements per channel at 3000^2), writes
// one fp64 partial per chunk; a finalize kernel folds the partials in a fixed
// order (deterministic, no atomics).  Apply passes are written as per-channel
// affine maps y = a[c]*x + b[c] (+ReLU), which is also how the backward is
// expressed: dx = k1[c]*dy + k2[c]*x + k3[c].
#include "common.h"
#include "launchers.h"

namespace tds {

// partial[(c*nchunk + k)*2 + {0,1}] = {sum x, sum x^2} (MODE 0)
//                                    or {sum dy, sum dy*(x-mean)} (MODE 1)
template <int MODE>
__global__ __launch_bounds__(256) void bn_reduce_kernel(const float* __restrict__ x, const float* __restrict__ dy,
                                                        const float* __restrict__ mean, double* __restrict__ partial,
                                                        int B, int C, int64_t HW, int nchunk) {
  __shared__ double sh[8];
  const int c = blockIdx.y;
  const int k = blockIdx.x;
  // chunk k = (plane b, slice s) so a workgroup streams one contiguous range
  const int cpp = nchunk / B;  // chunks per plane
  const int b = k / cpp;
  const int s = k - b * cpp;
  const int64_t per = ((HW + cpp - 1) / cpp + 3) & ~(int64_t)3;
  const int64_t e0 = (int64_t)s * per;
  const int64_t e1 = e0 + per < HW ? e0 + per : HW;
  const int64_t base = ((int64_t)b * C + c) * HW;
  const float* xp = x + base;
  const float* dp = MODE == 1 ? dy + base : nullptr;
  double s0 = 0.0, s1 = 0.0;
  const float mu = MODE == 1 ? mean[c] : 0.f;
  const bool vec = ((((uintptr_t)xp) | (MODE == 1 ? (uintptr_t)dp : 0)) & 15) == 0 && e1 > e0;
  int64_t e = e0;
  if (vec) {
    const int64_t nv = (e1 - e0) / 4;
    for (int64_t q = threadIdx.x; q < nv; q += blockDim.x) {
      const float4 v = *reinterpret_cast<const float4*>(xp + e0 + 4 * q);
      if (MODE == 0) {
        s0 += (double)((v.x + v.y) + (v.z + v.w));
        s1 += (double)v.x * v.x + (double)v.y * v.y + (double)v.z * v.z + (double)v.w * v.w;
      } else {
        const float4 d = *reinterpret_cast<const float4*>(dp + e0 + 4 * q);
        s0 += (double)((d.x + d.y) + (d.z + d.w));
        s1 += (double)d.x * (v.x - mu) + (double)d.y * (v.y - mu) + (double)d.z * (v.z - mu) + (double)d.w * (v.w - mu);
      }
    }
    e = e0 + nv * 4;
  }
  for (int64_t i = e + threadIdx.x; i < e1; i += blockDim.x) {
    const float v = xp[i];
    if (MODE == 0) {
      s0 += (double)v;
      s1 += (double)v * (double)v;
    } else {
      const float d = dp[i];
      s0 += (double)d;
      s1 += (double)d * (double)(v - mu);
    }
  }
  s0 = block_sum(s0, sh);
  s1 = block_sum(s1, sh);
  if (threadIdx.x == 0) {
    partial[((int64_t)c * nchunk + k) * 2 + 0] = s0;
    partial[((int64_t)c * nchunk + k) * 2 + 1] = s1;
  }
}

// One thread per channel: fold partials, produce mean/invstd (+ running stats)
// and the apply affine a = gamma*invstd, b = beta - mean*a.
__global__ void bn_fwd_finalize_kernel(const double* __restrict__ partial, int C, int nchunk, int64_t n, float eps,
                                       float momentum, const float* __restrict__ gamma, const float* __restrict__ beta,
                                       float* __restrict__ save_mean, float* __restrict__ save_invstd,
                                       float* __restrict__ running_mean, float* __restrict__ running_var,
                                       int64_t* __restrict__ num_batches, float* __restrict__ aff_a,
                                       float* __restrict__ aff_b) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c == 0 && num_batches) num_batches[0] += 1;
  if (c >= C) return;
  double s = 0.0, ss = 0.0;
  for (int k = 0; k < nchunk; ++k) {
    s += partial[((int64_t)c * nchunk + k) * 2];
    ss += partial[((int64_t)c * nchunk + k) * 2 + 1];
  }
  const double mean = s / (double)n;
  double var = ss / (double)n - mean * mean;
  if (var < 0.0) var = 0.0;
  const float invstd = (float)(1.0 / sqrt(var + (double)eps));
  save_mean[c] = (float)mean;
  save_invstd[c] = invstd;
  if (running_mean) {
    const double unbiased = n > 1 ? var * (double)n / (double)(n - 1) : var;
    running_mean[c] = (float)((1.0 - momentum) * running_mean[c] + momentum * mean);
    running_var[c] = (float)((1.0 - momentum) * running_var[c] + momentum * unbiased);
  }
  const float g = gamma ? gamma[c] : 1.f;
  const float bt = beta ? beta[c] : 0.f;
  aff_a[c] = g * invstd;
  aff_b[c] = bt - (float)mean * g * invstd;
}

// eval-mode affine from running stats
__global__ void bn_eval_affine_kernel(const float* __restrict__ rm, const float* __restrict__ rv, int C, float eps,
                                      const float* __restrict__ gamma, const float* __restrict__ beta,
                                      float* __restrict__ aff_a, float* __restrict__ aff_b) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const float invstd = rsqrtf(rv[c] + eps);
  const float g = gamma ? gamma[c] : 1.f;
  aff_a[c] = g * invstd;
  aff_b[c] = (beta ? beta[c] : 0.f) - rm[c] * g * invstd;
}

// y = a[c]*x + b[c] (+ relu).  grid.y = B*C planes, grid.x strides the plane.
__global__ __launch_bounds__(256) void bn_apply_kernel(const float* __restrict__ x, const float* __restrict__ aff_a,
                                                       const float* __restrict__ aff_b, float* __restrict__ y, int C,
                                                       int64_t HW, int relu) {
  const int64_t plane = blockIdx.y;
  const int c = (int)(plane % C);
  const float a = aff_a[c], bb = aff_b[c];
  const float* xp = x + plane * HW;
  float* yp = y + plane * HW;
  const bool vec = (((uintptr_t)xp | (uintptr_t)yp) & 15) == 0;
  const int64_t n4 = vec ? HW / 4 : 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
    float4 v = reinterpret_cast<const float4*>(xp)[i];
    v.x = fmaf(a, v.x, bb); v.y = fmaf(a, v.y, bb); v.z = fmaf(a, v.z, bb); v.w = fmaf(a, v.w, bb);
    if (relu) { v.x = fmaxf(v.x, 0.f); v.y = fmaxf(v.y, 0.f); v.z = fmaxf(v.z, 0.f); v.w = fmaxf(v.w, 0.f); }
    reinterpret_cast<float4*>(yp)[i] = v;
  }
  for (int64_t i = n4 * 4 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < HW; i += (int64_t)gridDim.x * blockDim.x) {
    float v = fmaf(a, xp[i], bb);
    yp[i] = relu ? fmaxf(v, 0.f) : v;
  }
}

// backward finalize: dgamma, dbeta and the dx affine (k1, k2, k3)
__global__ void bn_bwd_finalize_kernel(const double* __restrict__ partial, int C, int nchunk, int64_t n,
                                       const float* __restrict__ gamma, const float* __restrict__ mean,
                                       const float* __restrict__ invstd, float* __restrict__ dgamma,
                                       float* __restrict__ dbeta, float* __restrict__ k1, float* __restrict__ k2,
                                       float* __restrict__ k3) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  double sdy = 0.0, sdyx = 0.0;
  for (int k = 0; k < nchunk; ++k) {
    sdy += partial[((int64_t)c * nchunk + k) * 2];
    sdyx += partial[((int64_t)c * nchunk + k) * 2 + 1];
  }
  const double is = invstd[c];
  const double g = gamma ? gamma[c] : 1.0;
  if (dgamma) dgamma[c] = (float)(sdyx * is);
  if (dbeta) dbeta[c] = (float)sdy;
  // dx = g*is*(dy - sdy/n - (x-mu)*is^2*sdyx/n)
  const double a1 = g * is;
  const double a2 = -g * is * is * is * sdyx / (double)n;
  const double a3 = -g * is * sdy / (double)n - a2 * (double)mean[c];
  k1[c] = (float)a1;
  k2[c] = (float)a2;
  k3[c] = (float)a3;
}

__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(const float* __restrict__ dy, const float* __restrict__ x,
                                                           const float* __restrict__ k1, const float* __restrict__ k2,
                                                           const float* __restrict__ k3, float* __restrict__ dx, int C,
                                                           int64_t HW) {
  const int64_t plane = blockIdx.y;
  const int c = (int)(plane % C);
  const float a1 = k1[c], a2 = k2[c], a3 = k3[c];
  const float* dp = dy + plane * HW;
  const float* xp = x + plane * HW;
  float* op = dx + plane * HW;
  const bool vec = (((uintptr_t)dp | (uintptr_t)xp | (uintptr_t)op) & 15) == 0;
  const int64_t n4 = vec ? HW / 4 : 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
    const float4 d = reinterpret_cast<const float4*>(dp)[i];
    const float4 v = reinterpret_cast<const float4*>(xp)[i];
    float4 o;
    o.x = fmaf(a1, d.x, fmaf(a2, v.x, a3)); o.y = fmaf(a1, d.y, fmaf(a2, v.y, a3));
    o.z = fmaf(a1, d.z, fmaf(a2, v.z, a3)); o.w = fmaf(a1, d.w, fmaf(a2, v.w, a3));
    reinterpret_cast<float4*>(op)[i] = o;
  }
  for (int64_t i = n4 * 4 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < HW; i += (int64_t)gridDim.x * blockDim.x)
    op[i] = fmaf(a1, dp[i], fmaf(a2, xp[i], a3));
}

// chunks per channel = B * chunks-per-plane; aim for ~2048 workgroups in
// total with >= 16K elements each.
static int chunks_for(int B, int64_t HW, int C) {
  int64_t k = 2048 / ((int64_t)(C > 0 ? C : 1) * B);
  if (k < 1) k = 1;
  const int64_t max_k = (HW + 16383) / 16384;
  if (k > max_k) k = max_k;
  if (k < 1) k = 1;
  return (int)(k * B);
}

static dim3 plane_grid(int64_t HW, int64_t planes) {
  int64_t gx = (HW / 4 + 255) / 256;
  if (gx < 1) gx = 1;
  if (gx > 64) gx = 64;
  return dim3((unsigned)gx, (unsigned)planes);
}

}  // namespace tds

using namespace tds;

int tds_bn_num_chunks(int B, int C, int64_t HW) { return chunks_for(B, HW, C); }

void tds_bn_fwd_train(const float* x, int B, int C, int64_t HW, float eps, float momentum, const float* gamma,
                      const float* beta, float* save_mean, float* save_invstd, float* running_mean, float* running_var,
                      int64_t* num_batches, float* aff_a, float* aff_b, double* partial, int nchunk, hipStream_t st) {
  hipLaunchKernelGGL(bn_reduce_kernel<0>, dim3(nchunk, C), dim3(256), 0, st, x, nullptr, nullptr, partial, B, C, HW,
                     nchunk);
  TDS_LAUNCH_CHECK();
  hipLaunchKernelGGL(bn_fwd_finalize_kernel, dim3((C + 63) / 64), dim3(64), 0, st, partial, C, nchunk,
                     (int64_t)B * HW, eps, momentum, gamma, beta, save_mean, save_invstd, running_mean, running_var,
                     num_batches, aff_a, aff_b);
  TDS_LAUNCH_CHECK();
}

void tds_bn_eval_affine(const float* rm, const float* rv, int C, float eps, const float* gamma, const float* beta,
                        float* aff_a, float* aff_b, hipStream_t st) {
  hipLaunchKernelGGL(bn_eval_affine_kernel, dim3((C + 63) / 64), dim3(64), 0, st, rm, rv, C, eps, gamma, beta, aff_a,
                     aff_b);
  TDS_LAUNCH_CHECK();
}

void tds_bn_apply(const float* x, const float* aff_a, const float* aff_b, float* y, int B, int C, int64_t HW, int relu,
                  hipStream_t st) {
  hipLaunchKernelGGL(bn_apply_kernel, plane_grid(HW, (int64_t)B * C), dim3(256), 0, st, x, aff_a, aff_b, y, C, HW, relu);
  TDS_LAUNCH_CHECK();
}

void tds_bn_bwd(const float* dy, const float* x, int B, int C, int64_t HW, const float* gamma, const float* mean,
                const float* invstd, float* dx, float* dgamma, float* dbeta, float* kbuf /*3*C*/, double* partial,
                int nchunk, hipStream_t st) {
  hipLaunchKernelGGL(bn_reduce_kernel<1>, dim3(nchunk, C), dim3(256), 0, st, x, dy, mean, partial, B, C, HW, nchunk);
  TDS_LAUNCH_CHECK();
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3((C + 63) / 64), dim3(64), 0, st, partial, C, nchunk, (int64_t)B * HW,
                     gamma, mean, invstd, dgamma, dbeta, kbuf, kbuf + C, kbuf + 2 * C);
  TDS_LAUNCH_CHECK();
  if (dx) {
    hipLaunchKernelGGL(bn_bwd_apply_kernel, plane_grid(HW, (int64_t)B * C), dim3(256), 0, st, dy, x, kbuf, kbuf + C,
                       kbuf + 2 * C, dx, C, HW);
    TDS_LAUNCH_CHECK();
  }
}
