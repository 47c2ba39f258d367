// Skinny fully-connected layer: M (batch rows) and N (classes) tiny, K huge.
// Reference: nn.LazyLinear(10) on a flattened [B, 32*(H/4)^2] activation
// (mnist_onegpu.py:24,29-30 -> addmm / mm / sum).
// At 3000^2 the weight is [10, 18e6] (720 MB): all three products are pure
// HBM streams, so they are written as split-K streams over every CU, not as
// MFMA tiles (M=5 would waste >90% of any MFMA shape).
//
//  fwd : partial[blk][m*N+n] = sum_{k in blk} x[m,k] W[n,k]  -> reduce (+bias), fixed order
//  bwd : one pass over k: dx[m,k] = sum_n dy[m,n] W[n,k];
//                         dW[n,k] = scale * sum_m dy[m,n] x[m,k]  (optionally accumulated)
//        db[n] = scale * sum_m dy[m,n]
#include "common.h"
#include "launchers.h"

namespace tds {

template <int MAXM, int MAXN>
__global__ __launch_bounds__(256) void linear_fwd_splitk_kernel(const float* __restrict__ x, const float* __restrict__ W,
                                                                float* __restrict__ partial, int M, int N, int64_t K,
                                                                int64_t kchunk) {
  __shared__ float red[4][MAXM * MAXN];
  float acc[MAXM][MAXN];
#pragma unroll
  for (int m = 0; m < MAXM; ++m)
#pragma unroll
    for (int n = 0; n < MAXN; ++n) acc[m][n] = 0.f;
  const int64_t k0 = (int64_t)blockIdx.x * kchunk;
  int64_t k1 = k0 + kchunk;
  if (k1 > K) k1 = K;
  bool vec = (K % 4 == 0) && ((((uintptr_t)x) | ((uintptr_t)W)) & 15) == 0;
  int64_t kv_end = k0;
  if (vec) {
    kv_end = k0 + ((k1 - k0) / 4) * 4;
    for (int64_t k = k0 + 4 * threadIdx.x; k < kv_end; k += 4 * blockDim.x) {
      float4 xv[MAXM];
#pragma unroll
      for (int m = 0; m < MAXM; ++m)
        if (m < M) xv[m] = *reinterpret_cast<const float4*>(x + (int64_t)m * K + k);
#pragma unroll
      for (int n = 0; n < MAXN; ++n) {
        if (n < N) {
          const f32x4 wt = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(W + (int64_t)n * K + k));
          const float4 wv = float4{wt[0], wt[1], wt[2], wt[3]};
#pragma unroll
          for (int m = 0; m < MAXM; ++m)
            if (m < M) acc[m][n] += xv[m].x * wv.x + xv[m].y * wv.y + xv[m].z * wv.z + xv[m].w * wv.w;
        }
      }
    }
  }
  for (int64_t k = kv_end + threadIdx.x; k < k1; k += blockDim.x) {
#pragma unroll
    for (int n = 0; n < MAXN; ++n)
      if (n < N) {
        const float wv = W[(int64_t)n * K + k];
#pragma unroll
        for (int m = 0; m < MAXM; ++m)
          if (m < M) acc[m][n] += x[(int64_t)m * K + k] * wv;
      }
  }
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int m = 0; m < MAXM; ++m)
#pragma unroll
    for (int n = 0; n < MAXN; ++n) {
      const float s = wave_sum(acc[m][n]);
      if (lane == 0) red[wv][m * MAXN + n] = s;
    }
  __syncthreads();
  for (int i = threadIdx.x; i < M * N; i += blockDim.x) {
    const int m = i / N, n = i - (i / N) * N;
    const float s = red[0][m * MAXN + n] + red[1][m * MAXN + n] + red[2][m * MAXN + n] + red[3][m * MAXN + n];
    partial[(int64_t)blockIdx.x * M * N + i] = s;
  }
}

__global__ void linear_fwd_reduce_kernel(const float* __restrict__ partial, const float* __restrict__ bias,
                                         float* __restrict__ out, int M, int N, int nblk) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= M * N) return;
  double s = 0.0;
  for (int b = 0; b < nblk; ++b) s += partial[(int64_t)b * M * N + i];
  out[i] = (float)s + (bias ? bias[i % N] : 0.f);
}

template <int MAXM, int MAXN>
__global__ __launch_bounds__(256) void linear_bwd_skinny_kernel(const float* __restrict__ dy, const float* __restrict__ x,
                                                                const float* __restrict__ W, float* __restrict__ dx,
                                                                float* __restrict__ dW, float* __restrict__ db, int M,
                                                                int N, int64_t K, float scale, int acc_w) {
  float g[MAXM][MAXN];
#pragma unroll
  for (int m = 0; m < MAXM; ++m)
#pragma unroll
    for (int n = 0; n < MAXN; ++n) g[m][n] = (m < M && n < N) ? dy[m * N + n] : 0.f;
  if (db && blockIdx.x == 0 && threadIdx.x < N) {
    float s = 0.f;
    for (int m = 0; m < M; ++m) s += dy[m * N + threadIdx.x];
    db[threadIdx.x] = acc_w ? db[threadIdx.x] + scale * s : scale * s;
  }
  const bool vec = (K % 4 == 0) && ((((uintptr_t)x) | ((uintptr_t)W) | ((uintptr_t)dx) | ((uintptr_t)dW)) & 15) == 0;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  if (vec) {
    const int64_t K4 = K / 4;
    for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < K4; q += stride) {
      const int64_t k = 4 * q;
      if (dx) {
        float4 o[MAXM];
#pragma unroll
        for (int m = 0; m < MAXM; ++m) o[m] = float4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int n = 0; n < MAXN; ++n)
          if (n < N) {
            const float4 wv = *reinterpret_cast<const float4*>(W + (int64_t)n * K + k);
#pragma unroll
            for (int m = 0; m < MAXM; ++m) {
              o[m].x += g[m][n] * wv.x; o[m].y += g[m][n] * wv.y; o[m].z += g[m][n] * wv.z; o[m].w += g[m][n] * wv.w;
            }
          }
#pragma unroll
        for (int m = 0; m < MAXM; ++m)
          if (m < M) *reinterpret_cast<float4*>(dx + (int64_t)m * K + k) = o[m];
      }
      if (dW) {
        float4 xv[MAXM];
#pragma unroll
        for (int m = 0; m < MAXM; ++m)
          xv[m] = m < M ? *reinterpret_cast<const float4*>(x + (int64_t)m * K + k) : float4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int n = 0; n < MAXN; ++n)
          if (n < N) {
            float4 s = float4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int m = 0; m < MAXM; ++m) {
              s.x += g[m][n] * xv[m].x; s.y += g[m][n] * xv[m].y; s.z += g[m][n] * xv[m].z; s.w += g[m][n] * xv[m].w;
            }
            float4* dst = reinterpret_cast<float4*>(dW + (int64_t)n * K + k);
            if (acc_w) {
              const float4 old = *dst;
              s.x = old.x + scale * s.x; s.y = old.y + scale * s.y; s.z = old.z + scale * s.z; s.w = old.w + scale * s.w;
            } else {
              s.x *= scale; s.y *= scale; s.z *= scale; s.w *= scale;
            }
            *dst = s;
          }
      }
    }
    return;
  }
  for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < K; k += stride) {
    if (dx) {
#pragma unroll
      for (int m = 0; m < MAXM; ++m)
        if (m < M) {
          float s = 0.f;
#pragma unroll
          for (int n = 0; n < MAXN; ++n)
            if (n < N) s += g[m][n] * W[(int64_t)n * K + k];
          dx[(int64_t)m * K + k] = s;
        }
    }
    if (dW) {
#pragma unroll
      for (int n = 0; n < MAXN; ++n)
        if (n < N) {
          float s = 0.f;
#pragma unroll
          for (int m = 0; m < MAXM; ++m)
            if (m < M) s += g[m][n] * x[(int64_t)m * K + k];
          float* d = dW + (int64_t)n * K + k;
          *d = acc_w ? *d + scale * s : scale * s;
        }
    }
  }
}

// Weight gradient of a linear layer from (grad_output, input) rows:
//   dW[n][k] (= or +=) scale * sum_m g[m][n] x[m][k],  db[n] (= or +=) scale * sum_m g[m][n]
// M <= 64 rows (e.g. the all-gathered rows of every rank), N <= 16 outputs, any K; dW rows
// are ldw apart (ldw = K for a dense matrix, > K for a column shard written in place into
// the full [N, ldw] gradient, parallel/factored.py sharded path).
// Exact fp32 on v_mfma_f32_16x16x4_f32: A[n][m] = g[m][n] stays in registers, B = 4 rows x
// 16 columns of x per step; memory-bound on reading x and writing dW.
__global__ __launch_bounds__(256) void linear_dw_mfma_kernel(const float* __restrict__ g, const float* __restrict__ x,
                                                             float* __restrict__ dW, float* __restrict__ db, int M,
                                                             int N, int64_t K, int64_t ldw, float scale, int acc,
                                                             float upd_lr) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int li = lane & 15, gq = lane >> 4;
  const int steps = (M + 3) / 4;
  float a[16];
#pragma unroll
  for (int s = 0; s < 16; ++s) {
    const int m = 4 * s + gq;
    a[s] = (m < M && li < N) ? g[m * N + li] : 0.f;
  }
  if (db && blockIdx.x == 0 && threadIdx.x < N) {
    float t = 0.f;
    for (int m = 0; m < M; ++m) t += g[m * N + threadIdx.x];
    db[threadIdx.x] = acc ? db[threadIdx.x] + scale * t : scale * t;
  }
  const int64_t ncb = (K + 15) / 16;
  for (int64_t cb = (int64_t)blockIdx.x * 4 + wv; cb < ncb; cb += (int64_t)gridDim.x * 4) {
    const int64_t col = cb * 16 + li;
    const bool cv = col < K;
    f32x4 d = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      if (s < steps) {
        const int m = 4 * s + gq;
        const float bv = (m < M && cv) ? x[(int64_t)m * K + col] : 0.f;
        d = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s], bv, d, 0, 0, 0);
      }
    }
    if (cv) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = 4 * gq + r;
        if (n < N) {
          float* ptr = dW + (int64_t)n * ldw + col;
          const float v = scale * d[r];
          if (upd_lr != 0.f) {
            *ptr = *ptr - upd_lr * v;  // update-only: dW is the weight, torch SGD p -= lr * g
          } else {
            *ptr = acc ? *ptr + v : v;
          }
        }
      }
    }
  }
}

// Same contract as linear_dw_mfma_kernel, for the aligned case (K, ldw multiples of 4, 16-B
// aligned rows): a streaming VALU kernel, 4 columns per thread.  The fc exchange's update is
// one pass over the 720 MB weight (read + write) and every rank's rows of x: it is bound by
// HBM, and the MFMA kernel above moves it in 64-B pieces (16 columns x one float per lane, one
// column block in flight per wave): 754 us for 1.8 GB at the bench shape.  Here every access is
// a 16-B-per-lane vector (1 KiB per wave instruction) and a thread has its NN weight rows and 8
// x rows in flight at once.  g (dY, tiny and wave-uniform) comes through scalar loads.
template <int NN>
__global__ __launch_bounds__(256) void linear_dw_vec_kernel(const float* __restrict__ g, const float* __restrict__ x,
                                                            float* __restrict__ dW, float* __restrict__ db, int M,
                                                            int64_t K, int64_t ldw, float scale, int acc,
                                                            float upd_lr) {
  if (db && blockIdx.x == 0 && threadIdx.x < NN) {
    float t = 0.f;
    for (int m = 0; m < M; ++m) t += g[m * NN + threadIdx.x];
    db[threadIdx.x] = acc ? db[threadIdx.x] + scale * t : scale * t;
  }
  const bool rmw = upd_lr != 0.f || acc;
  const int64_t nq = K / 4;
  for (int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x; q < nq; q += (int64_t)gridDim.x * 256) {
    const int64_t col = 4 * q;
    float4 w[NN];
    if (rmw) {
#pragma unroll
      for (int n = 0; n < NN; ++n) w[n] = *reinterpret_cast<const float4*>(dW + (int64_t)n * ldw + col);
    }
    float4 s[NN];
#pragma unroll
    for (int n = 0; n < NN; ++n) s[n] = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int m0 = 0; m0 < M; m0 += 8) {
      float4 xv[8];
#pragma unroll
      for (int i = 0; i < 8; ++i)
        xv[i] = m0 + i < M ? __builtin_bit_cast(float4, __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(
                                                              x + (int64_t)(m0 + i) * K + col)))
                           : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        if (m0 + i < M) {
#pragma unroll
          for (int n = 0; n < NN; ++n) {
            const float gv = g[(m0 + i) * NN + n];
            s[n].x = fmaf(gv, xv[i].x, s[n].x);
            s[n].y = fmaf(gv, xv[i].y, s[n].y);
            s[n].z = fmaf(gv, xv[i].z, s[n].z);
            s[n].w = fmaf(gv, xv[i].w, s[n].w);
          }
        }
      }
    }
#pragma unroll
    for (int n = 0; n < NN; ++n) {
      const float4 v = make_float4(scale * s[n].x, scale * s[n].y, scale * s[n].z, scale * s[n].w);
      float4 o;
      if (upd_lr != 0.f) {  // update-only: dW is the weight, torch SGD p -= lr * g
        o = make_float4(w[n].x - upd_lr * v.x, w[n].y - upd_lr * v.y, w[n].z - upd_lr * v.z, w[n].w - upd_lr * v.w);
      } else if (acc) {
        o = make_float4(w[n].x + v.x, w[n].y + v.y, w[n].z + v.z, w[n].w + v.w);
      } else {
        o = v;
      }
      *reinterpret_cast<float4*>(dW + (int64_t)n * ldw + col) = o;
    }
  }
}

}  // namespace tds

using namespace tds;

int tds_linear_fwd_nblk(int64_t K) {
  int64_t nb = (K + 8191) / 8192;  // >= 8K columns per workgroup
  if (nb > 1024) nb = 1024;
  if (nb < 1) nb = 1;
  return (int)nb;
}

int tds_linear_fwd_skinny(const float* x, const float* W, const float* bias, float* out, float* partial, int M, int N,
                          int64_t K, int nblk, hipStream_t st) {
  if (N > 16 || M > 8) return -1;
  int64_t kchunk = (K + nblk - 1) / nblk;
  kchunk = (kchunk + 3) & ~(int64_t)3;
#define TDS_LF(MM)                                                                                              \
  hipLaunchKernelGGL((linear_fwd_splitk_kernel<MM, 16>), dim3(nblk), dim3(256), 0, st, x, W, partial, M, N, K, \
                     kchunk)
  if (M <= 1) TDS_LF(1);
  else if (M <= 2) TDS_LF(2);
  else if (M <= 4) TDS_LF(4);
  else TDS_LF(8);
  TDS_LAUNCH_CHECK();
#undef TDS_LF
  hipLaunchKernelGGL(linear_fwd_reduce_kernel, dim3((M * N + 255) / 256), dim3(256), 0, st, partial, bias, out, M, N,
                     nblk);
  TDS_LAUNCH_CHECK();
  return 0;
}

int tds_linear_bwd_skinny(const float* dy, const float* x, const float* W, float* dx, float* dW, float* db, int M,
                          int N, int64_t K, float scale, int acc_w, hipStream_t st) {
  if (N > 16 || M > 8) return -1;
  int64_t g = (K / 4 + 255) / 256;
  if (g > 2048) g = 2048;
  if (g < 1) g = 1;
#define TDS_LB(MM)                                                                                               \
  hipLaunchKernelGGL((linear_bwd_skinny_kernel<MM, 16>), dim3((unsigned)g), dim3(256), 0, st, dy, x, W, dx, dW, db, \
                     M, N, K, scale, acc_w)
  if (M <= 1) TDS_LB(1);
  else if (M <= 2) TDS_LB(2);
  else if (M <= 4) TDS_LB(4);
  else TDS_LB(8);
  TDS_LAUNCH_CHECK();
#undef TDS_LB
  return 0;
}

int tds_linear_dw(const float* dy, const float* x, float* dW, float* db, int M, int N, int64_t K, int64_t ldw,
                  float scale, int acc, float upd_lr, hipStream_t st) {
  if (M > 64 || N > 16 || M < 1 || ldw < K) return -1;
  const bool aligned = K % 4 == 0 && ldw % 4 == 0 && ((uintptr_t)x & 15) == 0 && ((uintptr_t)dW & 15) == 0;
  if (aligned && (N == 10 || N == 16)) {
    int64_t grid = (K / 4 + 255) / 256;
    if (grid > 4096) grid = 4096;
    if (grid < 1) grid = 1;
    if (N == 10)
      hipLaunchKernelGGL(linear_dw_vec_kernel<10>, dim3((unsigned)grid), dim3(256), 0, st, dy, x, dW, db, M, K, ldw,
                         scale, acc, upd_lr);
    else
      hipLaunchKernelGGL(linear_dw_vec_kernel<16>, dim3((unsigned)grid), dim3(256), 0, st, dy, x, dW, db, M, K, ldw,
                         scale, acc, upd_lr);
    TDS_LAUNCH_CHECK();
    return 0;
  }
  int64_t ncb = (K + 15) / 16;
  int64_t grid = (ncb + 3) / 4;
  if (grid > 8192) grid = 8192;
  hipLaunchKernelGGL(linear_dw_mfma_kernel, dim3((unsigned)grid), dim3(256), 0, st, dy, x, dW, db, M, N, K, ldw,
                     scale, acc, upd_lr);
  TDS_LAUNCH_CHECK();
  return 0;
}
