// x autocorrelation for the closed-form BN1 statistics (the conv1
// batch-norm moments come from the Gram of the 5x5 input patches instead of a pass over the
// 16-channel conv1 output).  Built with -fno-slp-vectorize (_build.HIP_FILE_FLAGS).
#include "common.h"
#include "launchers.h"

namespace tds {

// ============================================================================ x autocorrelation (Gram of conv1 patches)
// full[b][dy+4][dx+4] = sum_u x(u) x(u+d) over the image (0 outside), d in [-4,4]^2 with
// (dy > 0) or (dy == 0 and dx >= 0) computed, the rest by symmetry in the finalize.
// A thread owns a 4-column x AC_RB-row block of pixels and keeps the rows it multiplies
// (AC_RB + 4 rows x 12 columns: cols c-4 .. c+7) in registers: no LDS, no barriers (the
// LDS-tiled form with two barriers per 16 x 64 tile ran at 0.19 ms, latency bound).  A wave
// covers 256 consecutive columns, so every row load is a 1 KB run; neighbours' halo reloads hit
// L2.  Loads go through one buffer descriptor per wave, based at the wave's first image: a
// wave's lanes span at most two images of any size that matters, so lane offsets stay under
// 4 GiB for images up to 2^29 pixels (23170^2) whatever the batch; lanes outside the image read
// zeros by the descriptor's range check.  Each fp32
// accumulator sums 4 * AC_RB = 64 products; waves reduce in fp32, the workgroup in fp64
// (partial[wg][42], slot 41 = plain sum).  Requires W % 4 == 0.
// rows per thread: sweep on MI355X (isolated layer-1 forward, which includes this kernel):
// 4 -> 0.488 ms, 8 -> 0.435, 16 -> 0.407 (tools/gpu_sessions/r2_acrb.sh)
constexpr int AC_RB = 16;
// the uint8 path's moments are exact u32 sums: a thread adds 4 * AC_RB products of <= 255^2 and
// a wave 64 threads' sums (x_autocorr_u8_kernel), which must stay below 2^32
static_assert((unsigned long long)AC_RB * 4ull * 64ull * 65025ull < (1ull << 32),
              "AC_RB too large: the u8 moments' u32 wave sums would overflow");

static int x_autocorr_num_wg(int B, int H, int W) {
  if (W % 4 != 0 || B < 1 || H < 1) return 0;
  const int64_t threads = (int64_t)B * ((H + AC_RB - 1) / AC_RB) * (W / 4);
  return (int)((threads + 255) / 256);
}

// Border strips (the Gram's edge corrections, l1_build_gram): for image b, line L in {row 0, 1,
// H-2, H-1, col 0, 1, W-2, W-1} and d in [-4,4]^2, strips[b][L][d] = sum over the line of
// x(u) x(u+d); d index 81 = the plain line sum.  One workgroup per (d, L, b); l1_build_gram
// sums the images in a fixed order.  (One workgroup per (d, L) looping over the batch ran 35 us,
// latency-bound on its serial loop.)  Measured alternatives, all slower: the border workgroups
// as the first 656 of the autocorrelation's own launch (they held its slots: 167 us for both
// vs 99 + 35 us), the two kernels on separate streams (176 + 94 us overlapped), and workgroups
// per (line, dy, line chunk) with the 9 dx products per pixel and chunk partials folded in
// l1_gram (45 us here + 11 us more in l1_gram).
template <typename T>
__device__ void x_border_block(const T* __restrict__ x, double* __restrict__ strips, int H, int W, int di, int L,
                               int b, double* sh) {
  const int dy = di / 9 - 4, dx = di % 9 - 4;
  const bool plain = di == 81;
  const bool is_row = L < 4;
  const int fixed = is_row ? (L < 2 ? L : H - 4 + L) : (L < 6 ? L - 4 : W - 8 + L);
  const int len = is_row ? W : H;
  double s = 0.0;
  const T* xb = x + (int64_t)b * H * W;
  for (int i = threadIdx.x; i < len; i += blockDim.x) {
    const int r = is_row ? fixed : i, c = is_row ? i : fixed;
    if (r < 0 || r >= H || c < 0 || c >= W) continue;
    const float u = (float)xb[(int64_t)r * W + c];
    if (plain) {
      s += u;
    } else {
      const int r2 = r + dy, c2 = c + dx;
      if (r2 >= 0 && r2 < H && c2 >= 0 && c2 < W) s += (double)u * (double)xb[(int64_t)r2 * W + c2];
    }
  }
  s = block_sum(s, sh);
  if (threadIdx.x == 0) strips[((int64_t)b * 8 + L) * 82 + di] = s;
}

template <typename T>
__global__ __launch_bounds__(256) void x_border_kernel(const T* __restrict__ x, double* __restrict__ strips, int B,
                                                       int H, int W) {
  __shared__ double sh[8];
  x_border_block(x, strips, H, W, blockIdx.x, blockIdx.y, blockIdx.z, sh);
}

// Workgroups nac .. nac + 656 B - 1 of the launch (after every autocorrelation workgroup) are
// border-strip workgroups (d, L, b): they fill the CUs the autocorrelation's tail frees.
__global__ __launch_bounds__(256, 3) void x_autocorr_kernel(const float* __restrict__ x, double* __restrict__ partial,
                                                         int B, int H, int W, double* __restrict__ strips, int nac) {
  __shared__ double red[4][42];
  if ((int)blockIdx.x >= nac) {
    __shared__ double sh[8];
    const int j = (int)blockIdx.x - nac;
    x_border_block(x, strips, H, W, j % 82, (j / 82) % 8, j / 656, sh);
    return;
  }
  const int blk = blockIdx.x;
  const int tid = threadIdx.x;
  const int ncg = W / 4, nband = (H + AC_RB - 1) / AC_RB;
  const int64_t gt = (int64_t)blk * 256 + tid;
  float acc[42];
#pragma unroll
  for (int i = 0; i < 42; ++i) acc[i] = 0.f;
  if (gt < (int64_t)B * nband * ncg) {
    const int cg = (int)(gt % ncg);
    const int64_t rest = gt / ncg;
    const int band = (int)(rest % nband), b = (int)(rest / nband);
    const int c = 4 * cg, r0 = band * AC_RB;
    const int b0 = __builtin_amdgcn_readfirstlane(b);  // first active lane: the wave's lowest image
    const int64_t img = (int64_t)H * W;
    const int64_t span = (int64_t)(B - b0) * img * 4;
    const __amdgpu_buffer_rsrc_t rx =
        tds_buffer_rsrc(x + (int64_t)b0 * img, (uint32_t)(span < 0xFFFFFFF0LL ? span : 0xFFFFFFF0LL));
    constexpr uint32_t kOob = 0xFFFFFFF0u;
    const uint32_t base = (uint32_t)(((int64_t)(b - b0) * img + c) * 4);
    const bool has_l = c >= 4, has_r = c + 4 < W;
    auto ld_row = [&](int r, float (&row)[12]) {
      const uint32_t o = base + (uint32_t)r * (uint32_t)W * 4u;
      const bool in = r < H;
      const float4 v0 = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rx, in && has_l ? o - 16 : kOob, 0, 0));
      const float4 v1 = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rx, in ? o : kOob, 0, 0));
      const float4 v2 = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rx, in && has_r ? o + 16 : kOob, 0, 0));
      row[0] = v0.x; row[1] = v0.y; row[2] = v0.z; row[3] = v0.w;
      row[4] = v1.x; row[5] = v1.y; row[6] = v1.z; row[7] = v1.w;
      row[8] = v2.x; row[9] = v2.y; row[10] = v2.z; row[11] = v2.w;
    };
    // 5-row ring (own row + 4 below) plus the next row in flight
    float w[5][12], nx[12];
#pragma unroll
    for (int i = 0; i < 5; ++i) ld_row(r0 + i, w[i]);
#pragma unroll 1
    for (int i = 0; i < AC_RB; ++i) {
      if (i + 1 < AC_RB) ld_row(r0 + i + 5, nx);
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        const float u = w[0][4 + p];  // rows >= H loaded as zeros
        int k = 0;
#pragma unroll
        for (int dx = 0; dx <= 4; ++dx) acc[k++] += u * w[0][4 + p + dx];
#pragma unroll
        for (int dy = 1; dy <= 4; ++dy)
#pragma unroll
          for (int dx = -4; dx <= 4; ++dx) acc[k++] += u * w[dy][4 + p + dx];
        acc[41] += u;
      }
#pragma unroll
      for (int k = 0; k < 4; ++k)
#pragma unroll
        for (int q = 0; q < 12; ++q) w[k][q] = w[k + 1][q];
#pragma unroll
      for (int q = 0; q < 12; ++q) w[4][q] = nx[q];
    }
  }
  const int lane = tid & 63, wv = tid >> 6;
#pragma unroll
  for (int i = 0; i < 42; ++i) {
    const float s = wave_sum(acc[i]);
    if (lane == 0) red[wv][i] = s;
  }
  __syncthreads();
  if (tid < 42) partial[(int64_t)blk * 42 + tid] = (red[0][tid] + red[1][tid]) + (red[2][tid] + red[3][tid]);
}


// The same sums over uint8 levels (the fused plan's input when the batch is handed over as
// ToTensor's levels, ops/functional.py upsample_bilinear_u8(levels=True)): every product is an
// integer <= 255^2, so the sums are EXACT in u32 (a thread's accumulator <= 64 * 255^2, a wave's
// <= 2^28) and one v_dot4_u32_u8 takes a pixel quad's 4 products of one offset: the partner
// quad of offset dx is a byte window of the row's three dwords (v_alignbyte).  41 dot4 + <= 41
// alignbyte per quad and row instead of 168 FMAs.  Rows are 12-byte runs (cols c-4 .. c+7), 3
// dword loads per row; the level image is a quarter of the fp32 bytes.
__global__ __launch_bounds__(256, 3) void x_autocorr_u8_kernel(const uint8_t* __restrict__ x,
                                                            double* __restrict__ partial, int B, int H, int W,
                                                            double* __restrict__ strips, int nac) {
  __shared__ double red[4][42];
  if ((int)blockIdx.x >= nac) {
    __shared__ double sh[8];
    const int j = (int)blockIdx.x - nac;
    x_border_block(x, strips, H, W, j % 82, (j / 82) % 8, j / 656, sh);
    return;
  }
  const int blk = blockIdx.x;
  const int tid = threadIdx.x;
  const int ncg = W / 4, nband = (H + AC_RB - 1) / AC_RB;
  const int64_t gt = (int64_t)blk * 256 + tid;
  uint32_t acc[42];
#pragma unroll
  for (int i = 0; i < 42; ++i) acc[i] = 0u;
  if (gt < (int64_t)B * nband * ncg) {
    const int cg = (int)(gt % ncg);
    const int64_t rest = gt / ncg;
    const int band = (int)(rest % nband), b = (int)(rest / nband);
    const int c = 4 * cg, r0 = band * AC_RB;
    const int b0 = __builtin_amdgcn_readfirstlane(b);
    const int64_t img = (int64_t)H * W;
    const int64_t span = (int64_t)(B - b0) * img;
    const __amdgpu_buffer_rsrc_t rx =
        tds_buffer_rsrc(x + (int64_t)b0 * img, (uint32_t)(span < 0xFFFFFFF0LL ? span : 0xFFFFFFF0LL));
    constexpr uint32_t kOob = 0xFFFFFFF0u;
    const uint32_t base = (uint32_t)((int64_t)(b - b0) * img + c);
    const bool has_l = c >= 4, has_r = c + 4 < W;
    // (offsets made out of range by OR-ing the high bits: no short-circuit branch, whose merges
    // made the compiler wait for each row's loads at once)
    auto ld_row = [&](int r, uint32_t (&row)[3]) {
      const uint32_t o = base + (uint32_t)r * (uint32_t)W;
      const uint32_t oob = r < H ? 0u : kOob;
      row[0] = __builtin_amdgcn_raw_buffer_load_b32(rx, (o - 4) | oob | (has_l ? 0u : kOob), 0, 0);
      row[1] = __builtin_amdgcn_raw_buffer_load_b32(rx, o | oob, 0, 0);
      row[2] = __builtin_amdgcn_raw_buffer_load_b32(rx, (o + 4) | oob | (has_r ? 0u : kOob), 0, 0);
    };
    // bytes s .. s+3 of a row's 12 (s = 4 + dx in 0..8)
    auto win = [](const uint32_t (&row)[3], int s) -> uint32_t {
      return (s & 3) == 0 ? row[s >> 2] : __builtin_amdgcn_alignbyte(row[(s >> 2) + 1], row[s >> 2], s & 3);
    };
    // (fully unrolled, every row's loads can issue early: measured no faster, 73 vs 70 us in the
    // step, tools/gpu_sessions/r4_s23.sh -- kept rolled)
    uint32_t w[5][3], nx[3];
#pragma unroll
    for (int i = 0; i < 5; ++i) ld_row(r0 + i, w[i]);
#pragma unroll 1
    for (int i = 0; i < AC_RB; ++i) {
      if (i + 1 < AC_RB) ld_row(r0 + i + 5, nx);
      const uint32_t u = w[0][1];  // this thread's 4 pixels (rows >= H loaded as zeros)
      int k = 0;
#pragma unroll
      for (int dx = 0; dx <= 4; ++dx) acc[k] = __builtin_amdgcn_udot4(u, win(w[0], 4 + dx), acc[k], false), ++k;
#pragma unroll
      for (int dy = 1; dy <= 4; ++dy)
#pragma unroll
        for (int dx = -4; dx <= 4; ++dx) acc[k] = __builtin_amdgcn_udot4(u, win(w[dy], 4 + dx), acc[k], false), ++k;
      acc[41] = __builtin_amdgcn_udot4(u, 0x01010101u, acc[41], false);
#pragma unroll
      for (int k2 = 0; k2 < 4; ++k2)
#pragma unroll
        for (int q = 0; q < 3; ++q) w[k2][q] = w[k2 + 1][q];
#pragma unroll
      for (int q = 0; q < 3; ++q) w[4][q] = nx[q];
    }
  }
  const int lane = tid & 63, wv = tid >> 6;
#pragma unroll
  for (int i = 0; i < 42; ++i) {
    const uint32_t s = wave_sum(acc[i]);
    if (lane == 0) red[wv][i] = (double)s;
  }
  __syncthreads();
  if (tid < 42) partial[(int64_t)blk * 42 + tid] = (red[0][tid] + red[1][tid]) + (red[2][tid] + red[3][tid]);
}

}  // namespace tds

using namespace tds;

int tds_x_autocorr_num_wg(int B, int H, int W) { return x_autocorr_num_wg(B, H, W); }

void tds_x_border(const float* x, double* strips, int B, int H, int W, hipStream_t st) {
  hipLaunchKernelGGL(x_border_kernel<float>, dim3(82, 8, B), dim3(256), 0, st, x, strips, B, H, W);
  TDS_LAUNCH_CHECK();
}

// x moments for BN1: autocorrelation partials [nwg][42] and per-image border strips [B][8][82] in
// one launch, the border workgroups behind the autocorrelation's (measured: layer-1 forward 0.407 ->
// 0.402 ms against two launches, tools/gpu_sessions/r2_acmerge.sh)
void tds_x_moments(const float* x, double* ac_partial, int nwg, double* strips, int B, int H, int W, hipStream_t st) {
  if (nwg < 1 || nwg != x_autocorr_num_wg(B, H, W)) {  // the partial buffer is sized by tds_x_autocorr_num_wg
    tds_launch_fail("x_autocorr: workgroup count does not match the shape (needs W % 4 == 0)");
    return;
  }
  hipLaunchKernelGGL(x_autocorr_kernel, dim3(nwg + 656 * B), dim3(256), 0, st, x, ac_partial, B, H, W, strips, nwg);
  TDS_LAUNCH_CHECK();
}

// the same moments of uint8 levels (x = levels / 255 is scaled in l1_gram), one launch
void tds_x_moments_u8(const uint8_t* x, double* ac_partial, int nwg, double* strips, int B, int H, int W,
                      hipStream_t st, bool border_wgs) {
  if (nwg < 1 || nwg != x_autocorr_num_wg(B, H, W)) {
    tds_launch_fail("x_autocorr_u8: workgroup count does not match the shape (needs W % 4 == 0)");
    return;
  }
  // (without the border workgroups: 60 vs 76 us for the moments op at the bench shape, r5_s22)
  hipLaunchKernelGGL(x_autocorr_u8_kernel, dim3(nwg + (border_wgs ? 656 * B : 0)), dim3(256), 0, st, x, ac_partial, B,
                     H, W, strips, nwg);
  TDS_LAUNCH_CHECK();
}

void tds_x_border_u8(const uint8_t* x, double* strips, int B, int H, int W, hipStream_t st) {
  hipLaunchKernelGGL(x_border_kernel<uint8_t>, dim3(82, 8, B), dim3(256), 0, st, x, strips, B, H, W);
  TDS_LAUNCH_CHECK();
}
