// Plan-level ops of the fused ConvNet execution (torch.ops.tdsa.fused_*).
// Each op = a few kernel launches on the current stream, all shapes checked on
// the host first.  Activation formats:
//   p1          [B,P,P,16] fp16 (conv2's single-rounded operand)
//   y2h         [B,P,P,32] fp16 (the conv2 output the backward re-reads, bias-free, scaled)
//   ya          [B,32,PB] fp16: pooled-blocked planes (kernels/pooled_layout.h), the y2h value at
//               each window's argmax: y2 = h d + b2 (kernels/launchers.h TdsYaDec)
//   g2m         [B,32,Q,Q] fp16: planar pooled gradient at a per-channel power-of-two scale 2^e_c
//               bounded by the head forward's max |W| per channel and class (kernels/head_pb.hip);
//               kbuf[96 + c] = 2^-e_c (kbuf = [k1 | k2 | k3 | g2m scales], 128 floats)
//   mag         int32 workspace [mag_numel(B, P)]: the step's magnitude bounds (float bits) behind
//               the conv2 backward's fp16 gradient scale -- [0,32) max |y2 - b2| per channel, [32]
//               max |g2m|, then per-workgroup maxima from the conv2 forward (ypart [32][nwg])
//               and the head backward (gpart [32][npass][nblk]), written with plain stores and
//               reduced into [0,33) by the BN2-backward finalize
#include <ATen/ATen.h>
#include <c10/core/DeviceGuard.h>
#include <c10/hip/HIPStream.h>
#include <torch/library.h>

#include <algorithm>
#include <cstdlib>
#include <map>
#include <mutex>
#include <tuple>

#include "kernels/launchers.h"
#include "launch_check.h"

namespace {

using at::Tensor;
using tds_bind::check_launches;

hipStream_t stream_of(const Tensor& t) { return c10::hip::getCurrentHIPStream(t.device().index()).stream(); }

void need(const Tensor& t, at::ScalarType dt, std::vector<int64_t> shape, const char* name) {
  TORCH_CHECK(t.defined() && t.is_cuda(), "tdsa fused: ", name, " must be a GPU tensor");
  TORCH_CHECK(t.scalar_type() == dt, "tdsa fused: ", name, " has dtype ", t.scalar_type(), ", expected ", dt);
  TORCH_CHECK(t.is_contiguous(), "tdsa fused: ", name, " must be contiguous");
  TORCH_CHECK(t.sizes() == at::IntArrayRef(shape), "tdsa fused: ", name, " has shape ", t.sizes(), ", expected ",
              at::IntArrayRef(shape));
}

const float* optf(const c10::optional<Tensor>& t, int64_t n, const char* name) {
  if (!t.has_value() || !t->defined()) return nullptr;
  need(*t, at::kFloat, {n}, name);
  return t->data_ptr<float>();
}

// Gradient sink: a caller-provided destination (the parameter's slot in the DDP bucket,
// ops/grad_sink.py) or a fresh tensor -- the small parameter gradients land in the bucket
// straight from their finalize kernels instead of one copy kernel each.
Tensor sink_or_empty(const c10::optional<Tensor>& out, std::vector<int64_t> shape, const Tensor& like,
                     const char* name) {
  if (out.has_value() && out->defined()) {
    need(*out, at::kFloat, shape, name);
    TORCH_CHECK(out->device() == like.device(), "tdsa fused: ", name, " on the wrong device");
    return *out;
  }
  return at::empty(shape, like.options().dtype(at::kFloat));
}

// layer-1 conv workgroups per CU (grid-stride tile loop).  Sweep on MI355X (isolated layer-1
// forward, ms): 2 -> 0.524, 4 -> 0.443, 6 -> 0.433, 8 -> 0.429; bench 3.62-3.63 vs 3.64-3.68 ms
// per step at 4 (tools/gpu_sessions/r2_l1wg.sh)
int l1_wg() { return tds_fused_num_wg(8); }

// layer-1 backward workgroups per CU: 4 waves each.  Round 3 (124-126 VGPRs, 4 fit a CU): 4 -> 0.318
// ms, 3 -> 0.351 ms (tools/gpu_sessions/r3_s21.sh).  Round 4's fp16 weight gradient runs at 87
// VGPRs, so 5 fit (<= 102): 4 / 5 / 6 -> 0.143 / 0.138 / 0.145 ms (r4_s47.sh).  Capped by what the
// launched variant's registers allow (hipOccupancyMaxActiveBlocksPerMultiprocessor): the fp32-image
// variant needs more VGPRs than the level-input one, and a 5th workgroup that cannot be resident
// only adds a second, partial wave of workgroups.
int l1b_wg(bool levels) { return tds_fused_num_wg(std::min(5, tds_l1_bwd_max_per_cu(levels))); }

// Device copy of the blocked tile order (tds_tile_order_fill) per (device, shape), from the
// torch caching allocator, built once.  The map is never destroyed (no frees at process exit).
// On the device as per-workgroup lists: *sw / *sk are the strides of (workgroup, k-th tile of that
// workgroup) in the device table.

const int* tile_order(const Tensor& like, int B, int tiles_r, int tiles_c, int nwg, int* sw, int* sk) {
  static std::mutex mu;
  static auto* cache = new std::map<std::tuple<int, int, int, int, int>, Tensor>();
  // 16-row groups for both conv2 kernels: for the backward's 256 workgroups (32 per XCD
  // round) 4 / 8 / 16 / 32 rows measured 1.585 / 1.603 / 1.572 / 1.564 ms -- within noise
  const int gr = 16;
  const int64_t total = (int64_t)B * tiles_r * tiles_c;
  const int64_t rows = (total + nwg - 1) / nwg;
  *sw = (int)rows;
  *sk = 1;
  const auto key = std::make_tuple((int)like.get_device(), B, tiles_r, tiles_c, nwg);
  std::lock_guard<std::mutex> lock(mu);
  auto it = cache->find(key);
  if (it != cache->end()) return it->second.data_ptr<int>();
  auto host = at::empty({total}, at::TensorOptions().dtype(at::kInt));
  const int rc = tds_tile_order_fill(host.data_ptr<int>(), B, tiles_r, tiles_c, gr);
  TORCH_CHECK(rc == 0, "tdsa fused: tile order table needs B <= 255 and <= 4095 tiles per side (B=", B,
              ", tiles ", tiles_r, " x ", tiles_c, ")");
  // (the conv2 forward walking p1 last-to-first, the reverse of the layer-1 conv's writes, measured
  // 385.2 -> 389.0 us, r5_s50: the forward keeps its order)
  // on the device as per-workgroup lists: work index t = w + kk * nwg at [w][kk] (rows =
  // ceil(total / nwg), the tail padded with the list's last entry), so one workgroup's
  // consecutive tiles share a scalar-cache line (16 entries) instead of one line each
  auto l = at::empty({(int64_t)nwg, rows}, at::TensorOptions().dtype(at::kInt));
  const int* src = host.data_ptr<int>();
  int* dst = l.data_ptr<int>();
  for (int64_t w = 0; w < nwg; ++w)
    for (int64_t k = 0; k < rows; ++k) dst[w * rows + k] = src[std::min(w + k * nwg, total - 1)];
  Tensor dev = l.to(like.device());
  (*cache)[key] = dev;
  return dev.data_ptr<int>();
}

// Device copy of the rolling conv2 backward's walk table (tds_conv2_bwd_walk) per (device,
// shape, workgroups), from the torch caching allocator, built once.
// On the device the table is stored per workgroup ([nwg][rows], rows returned): one
// workgroup's consecutive tiles then share a scalar-cache line (16 entries) -- the host layout
// [rows][nwg] put each tile's entry on a line of its own, a scalar miss per tile in every wave.
const int* bwd_walk(const Tensor& like, int B, int tiles_r, int tiles_c, int nwg, int* sw, int* sk) {
  static std::mutex mu;
  static auto* cache = new std::map<std::tuple<int, int, int, int, int>, Tensor>();
  // tiles per vertical segment (a segment start re-stages 4 rows); r2_seg.sh: 24 / 48 / 96 / 200
  // tiles = 1.551 / 1.534 / 1.546 / 1.584 ms
  constexpr int kSeg = 48;
  const auto key = std::make_tuple((int)like.get_device(), B, tiles_r, tiles_c, nwg);
  std::lock_guard<std::mutex> lock(mu);
  auto it = cache->find(key);
  if (it != cache->end()) {
    *sw = (int)(it->second.numel() / nwg);
    *sk = 1;
    return it->second.data_ptr<int>();
  }
  const int64_t n = tds_conv2_bwd_walk(nullptr, B, tiles_r, tiles_c, nwg, kSeg);
  TORCH_CHECK(n > 0, "tdsa fused: conv2 backward walk needs B <= 63 and <= 4095 tiles per side (B=", B, ", tiles ",
              tiles_r, " x ", tiles_c, ")");
  auto host = at::empty({n / nwg, (int64_t)nwg}, at::TensorOptions().dtype(at::kInt));
  tds_conv2_bwd_walk(host.data_ptr<int>(), B, tiles_r, tiles_c, nwg, kSeg);
  *sw = (int)(n / nwg);
  *sk = 1;
  Tensor dev = host.t().contiguous().to(like.device());
  (*cache)[key] = dev;
  return dev.data_ptr<int>();
}

int64_t pb_plane(int64_t P) { return tds_pb_plane((int)(P / 2)); }

// ---------------------------------------------------------------- the step's magnitude-bound workspace
constexpr int64_t kG2mSlack = 32;   // fp16 elements (64 B) past g2m's end its allocations carry (conv2_bwd.hip GB runs)
constexpr int64_t kMagParts = 64;   // ypart offset in the mag workspace
constexpr int64_t kMagScales = 40;  // conv2 epilogue scales (csrc/kernels/conv2_common.h)
int64_t mag_ypart_count() { return (int64_t)tds_conv2_fwd2_num_wg(); }
int64_t mag_gpart_count(int64_t B, int64_t P) {
  return (int64_t)32 * tds_head_bwd_pb_npass((int)B) * tds_head_bwd_pb_nblk((int)(P / 2));
}
int64_t mag_numel(int64_t B, int64_t P) { return kMagParts + 32 * mag_ypart_count() + mag_gpart_count(B, P); }

uint32_t* opt_mag(const c10::optional<Tensor>& mag, int64_t numel = 33) {
  if (!mag.has_value() || !mag->defined()) return nullptr;
  TORCH_CHECK(mag->is_cuda() && mag->scalar_type() == at::kInt && mag->is_contiguous() && mag->numel() >= numel,
              "mag (magnitude-bound workspace) must be a contiguous int32 GPU tensor of >= ", numel,
              " elements (ops.mag_numel)");
  return reinterpret_cast<uint32_t*>(mag->data_ptr<int>());
}

// ---------------------------------------------------------------- layer 1 forward
// returns (p1 carrier, idx1, stats1[mean16|invstd16], ac_partial, strips)
// x: fp32 images, or uint8 levels (ToTensor's input: x = level / 255, folded into the kernels)
void check_l1_input(const Tensor& x, const char* what) {
  TORCH_CHECK(x.is_cuda() && (x.scalar_type() == at::kFloat || x.scalar_type() == at::kByte) && x.is_contiguous(),
              what, ": x must be a contiguous fp32 or uint8 GPU tensor");
  TORCH_CHECK(x.dim() == 4 && x.size(1) == 1, what, ": x must be [B,1,H,W]");
  TORCH_CHECK(x.size(2) == x.size(3) && x.size(2) >= 8, what, ": square images with H >= 8");
  TORCH_CHECK(x.size(0) >= 1 && x.size(0) <= 32, what, ": 1 <= B <= 32 per rank");
}

// The weight-independent half of the BN1 statistics: the x autocorrelation sums (42 doubles)
// and the per-image border strips (B x 8 x 82 doubles).  conv1 is linear in x, so BN1's batch mean and
// variance are these moments contracted with w1 (tds_l1_gram); they depend on the batch only,
// which lets an input pipeline produce them with the batch (on its own stream, beside the
// previous step's backward) and hand them to fused_l1_forward.
// the x moments' per-workgroup partials [nac][42] and the border strips (no reduction yet); uint8
// levels without border_wgs: the partials only (tds_l1_reduce_gram's border workgroups form the strips)
static std::tuple<Tensor, Tensor, int> x_moment_parts(const Tensor& x, bool border_wgs) {
  const int64_t B = x.size(0), H = x.size(2), W = x.size(3);
  hipStream_t st = stream_of(x);
  auto fo = x.options().dtype(at::kDouble);
  // one thread per 4 x 16 pixel block: each fp32 partial covers 64 products (fp64 beyond)
  const int nac = tds_x_autocorr_num_wg((int)B, (int)H, (int)W);
  TORCH_CHECK(nac > 0, "l1_input_stats: W % 4 == 0 required (autocorrelation kernel)");
  auto ac = at::empty({(int64_t)nac * 42}, fo);
  auto strips = at::empty({B * 8 * 82}, fo);
  if (x.scalar_type() == at::kByte)
    tds_x_moments_u8(x.data_ptr<uint8_t>(), ac.data_ptr<double>(), nac, strips.data_ptr<double>(), (int)B, (int)H,
                     (int)W, st, border_wgs);
  else
    tds_x_moments(x.data_ptr<float>(), ac.data_ptr<double>(), nac, strips.data_ptr<double>(), (int)B, (int)H, (int)W,
                  st);
  return {ac, strips, nac};
}

std::tuple<Tensor, Tensor> l1_input_stats(const Tensor& x) {
  check_l1_input(x, "l1_input_stats");
  c10::DeviceGuard guard(x.device());
  hipStream_t st = stream_of(x);
  Tensor ac, strips;
  int nac = 0;
  std::tie(ac, strips, nac) = x_moment_parts(x, true);
  auto asum = at::empty({42}, x.options().dtype(at::kDouble));
  tds_reduce_partials(ac.data_ptr<double>(), asum.data_ptr<double>(), 42, nac, 42, 0, 42, st);
  check_launches("l1_input_stats");
  return {asum, strips};
}

// returns (p1 [B,P,P,16] fp16, idx1, stats1 [mean16|invstd16], gram, p1_scale [1]: the power of two
// p1 is stored at -- 1 unless BN1's affine could push p1 past fp16's range, convnet_fused.hip)
std::tuple<Tensor, Tensor, Tensor, Tensor, Tensor> fused_l1_forward(
    const Tensor& x, const Tensor& w1, const Tensor& b1, const c10::optional<Tensor>& gamma1,
    const c10::optional<Tensor>& beta1, const c10::optional<Tensor>& rm1, const c10::optional<Tensor>& rv1,
    const c10::optional<Tensor>& nbt1, double momentum, double eps, const c10::optional<Tensor>& asum_in,
    const c10::optional<Tensor>& strips_in, const c10::optional<Tensor>& mag, const c10::optional<Tensor>& w2,
    const c10::optional<Tensor>& wp_out, const c10::optional<Tensor>& wd_out) {
  check_l1_input(x, "fused_l1_forward");
  // mag (optional): the Gram launch stores 1 / p1_scale at mag[kMagScales + 1] for the conv2
  // kernels (the weight packing, conv2_pack(write_p1=False), then runs ahead on a side stream)
  uint32_t* p1inv = opt_mag(mag, kMagScales + 2) ? opt_mag(mag) + kMagScales + 1 : nullptr;
  // w2 + wp_out + wd_out (with mag): conv2's weights packed by workgroups of the Gram launch (or,
  // on the paths without that launch, by the packing kernel right after the Gram) -- conv2_pack's
  // outputs without its launch between layer 1 and conv2
  const bool pack = w2.has_value() && w2->defined();
  const float* pw2 = nullptr;
  short *pwp = nullptr, *pwd = nullptr;
  if (pack) {
    TORCH_CHECK(p1inv != nullptr && wp_out.has_value() && wd_out.has_value(),
                "fused_l1_forward: packing conv2's weights needs mag, wp_out and wd_out");
    need(*w2, at::kFloat, {32, 16, 5, 5}, "conv2.weight");
    TORCH_CHECK(reinterpret_cast<uintptr_t>(w2->data_ptr()) % 16 == 0, "fused_l1_forward: conv2.weight must be 16-B aligned");
    need(*wp_out, at::kShort, {13 * 2 * 4 * 16 * 8}, "conv2 fwd pack");
    need(*wd_out, at::kShort, {25 * 4 * 16 * 8}, "conv2 dgrad pack");
    pw2 = w2->data_ptr<float>();
    pwp = wp_out->data_ptr<int16_t>();
    pwd = wd_out->data_ptr<int16_t>();
  }
  bool packed = false;
  const int64_t B = x.size(0), H = x.size(2), W = x.size(3);
  need(w1, at::kFloat, {16, 1, 5, 5}, "conv1.weight");
  need(b1, at::kFloat, {16}, "conv1.bias");
  const float* g = optf(gamma1, 16, "bn1.weight");
  const float* be = optf(beta1, 16, "bn1.bias");
  float* rm = const_cast<float*>(optf(rm1, 16, "bn1.running_mean"));
  float* rv = const_cast<float*>(optf(rv1, 16, "bn1.running_var"));
  int64_t* nb = nullptr;
  if (nbt1.has_value() && nbt1->defined()) {
    TORCH_CHECK(nbt1->is_cuda() && nbt1->scalar_type() == at::kLong && nbt1->numel() == 1, "bn1.num_batches_tracked");
    nb = nbt1->data_ptr<int64_t>();
  }
  c10::DeviceGuard guard(x.device());
  hipStream_t st = stream_of(x);
  const int64_t P = H / 2;
  auto fo = x.options().dtype(at::kFloat);
  const bool levels = x.scalar_type() == at::kByte;
  // x autocorrelation + border strips (precomputed by the input pipeline, or here) -> Gram G /
  // patch sums S -> BN1 statistics in closed form
  auto gram = at::empty({650}, fo.dtype(at::kDouble));
  auto sums = at::empty({32}, fo.dtype(at::kDouble));
  auto stats = at::empty({32}, fo);
  auto aff = at::empty({33}, fo);  // a16 | b16 | p1 scale
  // the moments' partials (from the fused upsample, ops.upsample_levels_moments, or here) -> their
  // reduction and the Gram in one launch (tds_l1_reduce_gram), uint8 levels' border strips formed
  // by workgroups of that launch
  auto reduce_gram = [&](const Tensor& ac, int nac, Tensor& strips, bool border) {
    auto asum = at::empty({42}, fo.dtype(at::kDouble));
    if (tds_l1_reduce_gram(ac.data_ptr<double>(), nac, asum.data_ptr<double>(), strips.data_ptr<double>(),
                           x.data_ptr(), levels, (int)B, (int)H, (int)W, w1.data_ptr<float>(), gram.data_ptr<double>(),
                           sums.data_ptr<double>(), b1.data_ptr<float>(), (float)eps, (float)momentum, g, be,
                           stats.data_ptr<float>(), rm, rv, nb, aff.data_ptr<float>(), st, border, p1inv, pw2, pwp, pwd,
                           pack ? opt_mag(mag) : nullptr)) {
      packed = pack;
      return;
    }
    if (border) tds_x_border_u8(x.data_ptr<uint8_t>(), strips.data_ptr<double>(), (int)B, (int)H, (int)W, st);
    tds_reduce_partials(ac.data_ptr<double>(), asum.data_ptr<double>(), 42, nac, 42, 0, 42, st);
    tds_l1_gram(asum.data_ptr<double>(), strips.data_ptr<double>(), x.data_ptr(), levels, (int)B, (int)H, (int)W,
                w1.data_ptr<float>(), gram.data_ptr<double>(), sums.data_ptr<double>(), b1.data_ptr<float>(),
                (float)eps, (float)momentum, g, be, stats.data_ptr<float>(), rm, rv, nb, aff.data_ptr<float>(), st,
                p1inv);
  };
  const bool pre = asum_in.has_value() && asum_in->defined();
  if (pre && asum_in->numel() != 42) {
    // autocorrelation partials [rows][42] of this batch (ops.upsample_levels_moments), strips not yet formed
    TORCH_CHECK(levels, "fused_l1_forward: precomputed moment partials need a uint8 level batch");
    TORCH_CHECK(!(strips_in.has_value() && strips_in->defined()), "fused_l1_forward: partials come without strips");
    TORCH_CHECK(asum_in->numel() % 42 == 0 && asum_in->numel() / 42 <= INT32_MAX, "fused_l1_forward: partials [rows][42]");
    need(*asum_in, at::kDouble, {asum_in->numel()}, "precomputed autocorrelation partials");
    // (the in-launch border: the strips accumulate elsewhere and this buffer carries the Gram body's
    // corner table, 16 * 81 + 16 doubles; [B][8][82] strips on the fallback path)
    auto strips = at::empty({std::max<int64_t>(B * 8 * 82, 16 * 81 + 16)}, fo.dtype(at::kDouble));
    reduce_gram(*asum_in, (int)(asum_in->numel() / 42), strips, true);
  } else if (pre) {
    TORCH_CHECK(strips_in.has_value() && strips_in->defined(), "fused_l1_forward: asum without strips");
    need(*asum_in, at::kDouble, {42}, "precomputed autocorrelation sums");
    need(*strips_in, at::kDouble, {B * 8 * 82}, "precomputed border strips");
    tds_l1_gram(asum_in->data_ptr<double>(), strips_in->data_ptr<double>(), x.data_ptr(), levels, (int)B, (int)H,
                (int)W, w1.data_ptr<float>(), gram.data_ptr<double>(), sums.data_ptr<double>(), b1.data_ptr<float>(),
                (float)eps, (float)momentum, g, be, stats.data_ptr<float>(), rm, rv, nb, aff.data_ptr<float>(), st,
                p1inv);
  } else {
    Tensor ac, strips;
    int nac = 0;
    std::tie(ac, strips, nac) = x_moment_parts(x, !levels);
    if (levels) strips = at::empty({std::max<int64_t>(B * 8 * 82, 16 * 81 + 16)}, fo.dtype(at::kDouble));
    reduce_gram(ac, nac, strips, levels);
  }
  if (pack && !packed)
    tds_conv2_pack_weights(pw2, pwp, pwd, opt_mag(mag), nullptr, st, /*write_p1=*/false);
  // the single conv1 pass: conv + BN1 affine + ReLU + pool -> p1 (fp16), argmax
  auto p1 = at::empty({B, P, P, 16}, fo.dtype(at::kHalf));
  auto idx1 = at::empty({B, P, P, 16}, fo.dtype(at::kByte));
  tds_l1_apply(x.data_ptr(), levels, w1.data_ptr<float>(), b1.data_ptr<float>(), aff.data_ptr<float>(),
               p1.data_ptr(), idx1.data_ptr<uint8_t>(), l1_wg(), (int)B, (int)H, (int)W, st);
  check_launches("fused_l1_forward");
  return {p1, idx1, stats, gram, aff.narrow(0, 32, 1)};
}

// ---------------------------------------------------------------- conv2 forward
// fp16 hi/lo weight packs of the conv2 forward and data gradient; resets mag when given
// With mag: weights packed at a power-of-two scale that keeps them in fp16's normal range, the
// scale and p1_scale's inverse recorded in mag for the conv2 epilogues (conv2_pack.hip).
std::tuple<Tensor, Tensor> conv2_pack(const Tensor& w2, const c10::optional<Tensor>& mag,
                                      const c10::optional<Tensor>& p1_scale, bool write_p1) {
  need(w2, at::kFloat, {32, 16, 5, 5}, "conv2.weight");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(w2.data_ptr()) % 16 == 0, "conv2_pack: conv2.weight must be 16-B aligned");
  const float* ps = optf(p1_scale, 1, "p1_scale");
  c10::DeviceGuard guard(w2.device());
  auto wp = at::empty({13 * 2 * 4 * 16 * 8}, w2.options().dtype(at::kShort));
  auto wd = at::empty({25 * 4 * 16 * 8}, w2.options().dtype(at::kShort));
  tds_conv2_pack_weights(w2.data_ptr<float>(), wp.data_ptr<int16_t>(), wd.data_ptr<int16_t>(), opt_mag(mag), ps,
                         stream_of(w2), write_p1);
  check_launches("conv2_pack");
  return {wp, wd};
}

unsigned short* ya_out(const Tensor& ya) { return reinterpret_cast<unsigned short*>(ya.data_ptr<at::Half>()); }

// ya's decode (kernels/launchers.h TdsYaDec): conv2.bias and the conv2 pack's scales in mag (none:
// d = 1, as fused_conv2_forward stores ya without mag)
TdsYaDec ya_dec(const Tensor& b2, const c10::optional<Tensor>& mag) {
  need(b2, at::kFloat, {32}, "conv2.bias (ya's decode)");
  uint32_t* m = opt_mag(mag, kMagScales + 3);
  return TdsYaDec{b2.data_ptr<float>(), m ? m + kMagScales : nullptr};
}

// returns (y2h [B,P,P,32] fp16: the conv2 output bias-free at the y2h scale mag[kMagScales + 2]
// (1 without mag; kernels/conv2_common.h), BN2 partials, ya [B,32,PB] fp16: y2h at each 2x2 window's
// argmax of the BN2 output, resolved by the sign of gamma2, a2 [B,P/2,P/2,2] int32: those argmaxes
// as 2-bit codes (kernels/conv2_common.h), for the backward)
std::tuple<Tensor, Tensor, Tensor, Tensor> fused_conv2_forward(const Tensor& p1, const Tensor& wp, const Tensor& b2,
                                                       const c10::optional<Tensor>& gamma2,
                                                       const c10::optional<Tensor>& mag) {
  TORCH_CHECK(p1.dim() == 4 && p1.size(1) == p1.size(2) && p1.size(3) == 16, "fused_conv2_forward: p1 [B,P,P,16]");
  const int64_t B = p1.size(0), P = p1.size(1);
  need(p1, at::kHalf, {B, P, P, 16}, "p1");
  need(wp, at::kShort, {13 * 2 * 4 * 16 * 8}, "conv2 fwd pack");
  need(b2, at::kFloat, {32}, "conv2.bias");
  const float* g = optf(gamma2, 32, "bn2.weight");
  TORCH_CHECK(B <= 255 && P >= 2, "fused_conv2_forward: 1 <= batch <= 255 and P >= 2");
  c10::DeviceGuard guard(p1.device());
  const int nwg = tds_conv2_fwd2_num_wg();
  int tr = 0, tc = 0;
  tds_conv2_fwd2_tiles((int)P, &tr, &tc);
  int sw = 0, sk = 0;
  const int* order = tile_order(p1, (int)B, tr, tc, nwg, &sw, &sk);
  auto y2 = at::empty({B, P, P, 32}, p1.options().dtype(at::kHalf));  // y2h (kernels/conv2_common.h)
  auto ya = at::empty({B, 32, pb_plane(P)}, p1.options().dtype(at::kHalf));
  auto partial = at::empty({32 * nwg * 2}, p1.options().dtype(at::kDouble));
  auto a2 = at::empty({B, P / 2, P / 2, 2}, p1.options().dtype(at::kInt));
  tds_conv2_fwd2(p1.data_ptr(), wp.data_ptr<int16_t>(), b2.data_ptr<float>(), g, y2.data_ptr(),
                 ya_out(ya), reinterpret_cast<uint32_t*>(a2.data_ptr<int>()), partial.data_ptr<double>(),
                 opt_mag(mag, kMagParts + 32 * mag_ypart_count()) ? opt_mag(mag) + kMagParts : nullptr,
                 opt_mag(mag) ? opt_mag(mag) + kMagScales : nullptr, order, nwg, sw, sk, (int)B, (int)P, stream_of(p1));
  check_launches("fused_conv2_forward");
  return {y2, partial, ya, a2};
}

// The conv2 forward with BN2 finalized inside its launch (conv2_fwd2.hip f2_finalize): returns (y2h,
// ya, a2 as fused_conv2_forward, stats2 [mean32|invstd32], aff2 [a32|b32]); the running statistics
// and num_batches_tracked are updated, and mag[0..32) gets max |y2 - b2| per channel (the conv2
// backward's magnitude bound; fused_head_backward(ypart_done=True) then leaves it).
std::tuple<Tensor, Tensor, Tensor, Tensor, Tensor> fused_conv2_forward_bn(
    const Tensor& p1, const Tensor& wp, const Tensor& b2, const c10::optional<Tensor>& gamma2,
    const c10::optional<Tensor>& beta2, const c10::optional<Tensor>& rm2, const c10::optional<Tensor>& rv2,
    const c10::optional<Tensor>& nbt2, double momentum, double eps, const c10::optional<Tensor>& mag) {
  TORCH_CHECK(p1.dim() == 4 && p1.size(1) == p1.size(2) && p1.size(3) == 16, "fused_conv2_forward_bn: p1 [B,P,P,16]");
  const int64_t B = p1.size(0), P = p1.size(1);
  need(p1, at::kHalf, {B, P, P, 16}, "p1");
  need(wp, at::kShort, {13 * 2 * 4 * 16 * 8}, "conv2 fwd pack");
  need(b2, at::kFloat, {32}, "conv2.bias");
  const float* g = optf(gamma2, 32, "bn2.weight");
  TORCH_CHECK(B <= 255 && P >= 2, "fused_conv2_forward_bn: 1 <= batch <= 255 and P >= 2");
  int64_t* nb = nullptr;
  if (nbt2.has_value() && nbt2->defined()) {
    TORCH_CHECK(nbt2->is_cuda() && nbt2->scalar_type() == at::kLong && nbt2->numel() == 1, "bn2.num_batches_tracked");
    nb = nbt2->data_ptr<int64_t>();
  }
  c10::DeviceGuard guard(p1.device());
  const int nwg = tds_conv2_fwd2_num_wg();
  int tr = 0, tc = 0;
  tds_conv2_fwd2_tiles((int)P, &tr, &tc);
  int sw = 0, sk = 0;
  const int* order = tile_order(p1, (int)B, tr, tc, nwg, &sw, &sk);
  auto y2 = at::empty({B, P, P, 32}, p1.options().dtype(at::kHalf));
  auto ya = at::empty({B, 32, pb_plane(P)}, p1.options().dtype(at::kHalf));
  auto a2 = at::empty({B, P / 2, P / 2, 2}, p1.options().dtype(at::kInt));
  const int ndw = tds_conv2_fwd2_fin_doubles(nwg), nuw = tds_conv2_fwd2_fin_words(nwg);
  auto partial = at::empty({32 * nwg * 2 + ndw}, p1.options().dtype(at::kDouble));
  auto uwork = at::empty({nuw}, p1.options().dtype(at::kInt));
  auto stats = at::empty({64}, p1.options().dtype(at::kFloat));
  auto aff = at::empty({64}, p1.options().dtype(at::kFloat));
  uint32_t* m = opt_mag(mag, kMagParts + 32 * mag_ypart_count());
  TdsBnFin fin{};
  fin.beta = optf(beta2, 32, "bn2.bias");
  fin.eps = (float)eps;
  fin.momentum = (float)momentum;
  fin.stats = stats.data_ptr<float>();
  fin.running_mean = const_cast<float*>(optf(rm2, 32, "bn2.running_mean"));
  fin.running_var = const_cast<float*>(optf(rv2, 32, "bn2.running_var"));
  fin.num_batches = nb;
  fin.aff = aff.data_ptr<float>();
  fin.mag = m;
  fin.dwork = partial.data_ptr<double>() + 32 * nwg * 2;
  fin.uwork = reinterpret_cast<uint32_t*>(uwork.data_ptr<int>());
  tds_conv2_fwd2(p1.data_ptr(), wp.data_ptr<int16_t>(), b2.data_ptr<float>(), g, y2.data_ptr(), ya_out(ya),
                 reinterpret_cast<uint32_t*>(a2.data_ptr<int>()), partial.data_ptr<double>(), m ? m + kMagParts : nullptr,
                 m ? m + kMagScales : nullptr, order, nwg, sw, sk, (int)B, (int)P, stream_of(p1), &fin);
  check_launches("fused_conv2_forward_bn");
  return {y2, ya, a2, stats, aff};
}

// The head forward on a finished BN2 affine (fused_conv2_forward_bn's aff2): logits only, finished
// inside the head's launch (head_pb.hip HPFin) for B <= 8
Tensor fused_head_forward_aff(const Tensor& ya, const Tensor& aff2, const Tensor& b2, const c10::optional<Tensor>& mag,
                              const Tensor& wfc, const c10::optional<Tensor>& bfc, int64_t P,
                              const c10::optional<Tensor>& x_out) {
  TORCH_CHECK(ya.dim() == 3 && ya.size(1) == 32, "fused_head_forward_aff: ya must be [B,32,PB]");
  const int64_t B = ya.size(0), Q = P / 2;
  TORCH_CHECK(Q >= 4 && B >= 1, "fused_head_forward_aff: needs P/2 >= 4 pooled columns and B >= 1");
  need(ya, at::kHalf, {B, 32, pb_plane(P)}, "ya (fp16)");
  need(aff2, at::kFloat, {64}, "aff2");
  TORCH_CHECK(wfc.dim() == 2 && wfc.size(1) == 32 * Q * Q && wfc.size(0) >= 1 && wfc.size(0) <= 10,
              "fc.weight must be [<=10, 32*Q*Q]");
  const int64_t NC = wfc.size(0);
  need(wfc, at::kFloat, {NC, 32 * Q * Q}, "fc.weight");
  const float* bf = optf(bfc, NC, "fc.bias");
  float* xo = nullptr;
  if (x_out.has_value() && x_out->defined()) {
    need(*x_out, at::kFloat, {B, 32 * Q * Q}, "x_out (fc input rows)");
    xo = x_out->data_ptr<float>();
  }
  c10::DeviceGuard guard(ya.device());
  const int nblk = 32 * tds_head_pb_nblk((int)Q);
  auto part = at::empty({(int64_t)(nblk + 32) * B * NC}, ya.options().dtype(at::kDouble));
  auto lsum = at::empty({B * NC}, ya.options().dtype(at::kDouble));
  auto logits = at::empty({B, NC}, ya.options().dtype(at::kFloat));
  const int rc = tds_head_fwd_pb(ya_out(ya), ya_dec(b2, mag), wfc.data_ptr<float>(), bf, aff2.data_ptr<float>(),
                                 part.data_ptr<double>(), lsum.data_ptr<double>(), logits.data_ptr<float>(), xo, (int)B,
                                 (int)Q, (int)NC, stream_of(ya));
  TORCH_CHECK(rc == 0, "fused_head_forward_aff: unsupported shape");
  check_launches("fused_head_forward_aff");
  return logits;
}

// fused_head_forward_aff with the batch's labels: the mean cross-entropy loss (torch's
// CrossEntropyLoss defaults: ignore_index -100, no label smoothing) and dlogits formed by the
// head forward's finalizing workgroup right after the logits (ce_small.h) -- one launch fewer than
// logits then ops.cross_entropy, with the same arithmetic.  Returns (logits, loss, dlogits).
std::tuple<Tensor, Tensor, Tensor> fused_head_forward_aff_ce(const Tensor& ya, const Tensor& aff2, const Tensor& b2,
                                                             const c10::optional<Tensor>& mag, const Tensor& wfc,
                                                             const c10::optional<Tensor>& bfc, int64_t P,
                                                             const Tensor& labels, const c10::optional<Tensor>& x_out) {
  TORCH_CHECK(ya.dim() == 3 && ya.size(1) == 32, "fused_head_forward_aff_ce: ya must be [B,32,PB]");
  const int64_t B = ya.size(0), Q = P / 2;
  TORCH_CHECK(Q >= 4 && B >= 1, "fused_head_forward_aff_ce: needs P/2 >= 4 pooled columns and B >= 1");
  need(ya, at::kHalf, {B, 32, pb_plane(P)}, "ya (fp16)");
  need(aff2, at::kFloat, {64}, "aff2");
  TORCH_CHECK(wfc.dim() == 2 && wfc.size(1) == 32 * Q * Q && wfc.size(0) >= 1 && wfc.size(0) <= 10,
              "fc.weight must be [<=10, 32*Q*Q]");
  const int64_t NC = wfc.size(0);
  need(wfc, at::kFloat, {NC, 32 * Q * Q}, "fc.weight");
  need(labels, at::kLong, {B}, "labels");
  TORCH_CHECK(labels.device() == ya.device(), "fused_head_forward_aff_ce: labels must be on ya's device");
  const float* bf = optf(bfc, NC, "fc.bias");
  float* xo = nullptr;
  if (x_out.has_value() && x_out->defined()) {  // (the activation exchange's fc input rows)
    need(*x_out, at::kFloat, {B, 32 * Q * Q}, "x_out (fc input rows)");
    xo = x_out->data_ptr<float>();
  }
  c10::DeviceGuard guard(ya.device());
  hipStream_t st = stream_of(ya);
  const int nblk = 32 * tds_head_pb_nblk((int)Q);
  auto part = at::empty({(int64_t)(nblk + 32) * B * NC}, ya.options().dtype(at::kDouble));
  auto lsum = at::empty({B * NC}, ya.options().dtype(at::kDouble));
  auto logits = at::empty({B, NC}, ya.options().dtype(at::kFloat));
  auto dlogits = at::empty({B, NC}, ya.options().dtype(at::kFloat));
  auto loss = at::empty({}, ya.options().dtype(at::kFloat));
  auto inv = at::empty({1}, ya.options().dtype(at::kFloat));
  const int rc = tds_head_fwd_pb(ya_out(ya), ya_dec(b2, mag), wfc.data_ptr<float>(), bf, aff2.data_ptr<float>(),
                                 part.data_ptr<double>(), lsum.data_ptr<double>(), logits.data_ptr<float>(), xo,
                                 (int)B, (int)Q, (int)NC, st, true, labels.data_ptr<int64_t>(),
                                 dlogits.data_ptr<float>(), loss.data_ptr<float>(), inv.data_ptr<float>());
  TORCH_CHECK(rc >= 0, "fused_head_forward_aff_ce: unsupported shape");
  if (rc == 0) {  // (the finalizer was not in the launch: the separate CE)
    auto row_loss = at::empty({B}, ya.options().dtype(at::kFloat));
    tds_cross_entropy(logits.data_ptr<float>(), labels.data_ptr<int64_t>(), row_loss.data_ptr<float>(),
                      dlogits.data_ptr<float>(), loss.data_ptr<float>(), inv.data_ptr<float>(), (int)B, (int)NC, -100,
                      0.f, st);
  }
  check_launches("fused_head_forward_aff_ce");
  return {logits, loss, dlogits};
}

// The head forward in channel-range launches (the activation exchange's column groups, parallel/
// factored.py: each group's fc input rows can be encoded and start travelling while the next range
// runs).  head_forward_range_ws allocates the step's shared workspace -- (partials, sums, logits,
// dlogits, loss, 1/count) -- and fused_head_forward_range runs channels [c0, c1) over it, writing
// that range's X rows into x_out [B, (c1-c0)*Q*Q]; the launch that completes the 32nd channel
// finishes the logits (and, with labels, the cross-entropy) inside itself (head_pb.hip HPFin).
std::tuple<Tensor, Tensor, Tensor, Tensor, Tensor, Tensor> head_forward_range_ws(const Tensor& ya, const Tensor& wfc,
                                                                                 int64_t P) {
  const int64_t B = ya.size(0), Q = P / 2, NC = wfc.size(0);
  const int nblk = 32 * tds_head_pb_nblk((int)Q);
  auto o = ya.options().dtype(at::kFloat);
  return {at::empty({(int64_t)(nblk + 32) * B * NC}, o.dtype(at::kDouble)), at::empty({B * NC}, o.dtype(at::kDouble)),
          at::empty({B, NC}, o), at::empty({B, NC}, o), at::empty({}, o), at::empty({1}, o)};
}

void fused_head_forward_range(const Tensor& ya, const Tensor& aff2, const Tensor& b2, const c10::optional<Tensor>& mag,
                              const Tensor& wfc, const c10::optional<Tensor>& bfc,
                              int64_t P, int64_t c0, int64_t c1, const Tensor& part, const Tensor& lsum,
                              const Tensor& logits, const Tensor& dlogits, const Tensor& loss, const Tensor& inv,
                              const c10::optional<Tensor>& labels, const c10::optional<Tensor>& x_out) {
  TORCH_CHECK(ya.dim() == 3 && ya.size(1) == 32, "fused_head_forward_range: ya must be [B,32,PB]");
  const int64_t B = ya.size(0), Q = P / 2;
  TORCH_CHECK(Q >= 4 && B >= 1 && B <= 8, "fused_head_forward_range: needs P/2 >= 4 and 1 <= B <= 8 (one pass)");
  TORCH_CHECK(0 <= c0 && c0 < c1 && c1 <= 32, "fused_head_forward_range: channels 0 <= c0 < c1 <= 32");
  need(ya, at::kHalf, {B, 32, pb_plane(P)}, "ya (fp16)");
  need(aff2, at::kFloat, {64}, "aff2");
  TORCH_CHECK(wfc.dim() == 2 && wfc.size(1) == 32 * Q * Q && wfc.size(0) >= 1 && wfc.size(0) <= 10,
              "fc.weight must be [<=10, 32*Q*Q]");
  const int64_t NC = wfc.size(0);
  need(wfc, at::kFloat, {NC, 32 * Q * Q}, "fc.weight");
  const float* bf = optf(bfc, NC, "fc.bias");
  const int nblk = 32 * tds_head_pb_nblk((int)Q);
  need(part, at::kDouble, {(int64_t)(nblk + 32) * B * NC}, "head partials");
  need(lsum, at::kDouble, {B * NC}, "logit sums");
  need(logits, at::kFloat, {B, NC}, "logits");
  need(dlogits, at::kFloat, {B, NC}, "dlogits");
  need(loss, at::kFloat, {}, "loss");
  need(inv, at::kFloat, {1}, "1/count");
  const int64_t* lab = nullptr;
  if (labels.has_value() && labels->defined()) {
    need(*labels, at::kLong, {B}, "labels");
    lab = labels->data_ptr<int64_t>();
  }
  float* xo = nullptr;
  if (x_out.has_value() && x_out->defined()) {
    need(*x_out, at::kFloat, {B, (c1 - c0) * Q * Q}, "x_out (the range's fc input rows)");
    xo = x_out->data_ptr<float>();
  }
  c10::DeviceGuard guard(ya.device());
  const int rc = tds_head_fwd_pb(ya_out(ya), ya_dec(b2, mag), wfc.data_ptr<float>(), bf, aff2.data_ptr<float>(),
                                 part.data_ptr<double>(), lsum.data_ptr<double>(), logits.data_ptr<float>(), xo, (int)B,
                                 (int)Q, (int)NC, stream_of(ya), true, lab, dlogits.data_ptr<float>(),
                                 loss.data_ptr<float>(), inv.data_ptr<float>(), (int)c0, (int)c1);
  TORCH_CHECK(rc >= 0, "fused_head_forward_range: unsupported shape or no in-launch finalize (TDS_FUSED_FIN=0)");
  check_launches("fused_head_forward_range");
}

// The activation exchange's "pooled" source (parallel/factored.py): the ranks all-gather ya and a
// 128-float record of the head constants their forward used (head_pooled_record: aff2 | the ya
// scale words | b2), and every rank forms the fc step from them (head_update_pooled; kernels/
// head_pb.hip head_upd_pb_kernel).  mode 0: wfc -= lr * scale * dl_all^T X (update only), 1: out =
// scale * dl_all^T X, 2: out += scale * dl_all^T X; X recomputed from each rank's ya with that rank's
// record, bitwise the rows its head forward used.
Tensor head_pooled_record(const Tensor& aff2, const Tensor& b2, const c10::optional<Tensor>& mag) {
  need(aff2, at::kFloat, {64}, "aff2");
  need(b2, at::kFloat, {32}, "conv2.bias");
  uint32_t* m = opt_mag(mag, kMagScales + 3);
  c10::DeviceGuard guard(aff2.device());
  auto rec = at::empty({128}, aff2.options());
  tds_head_pooled_record(aff2.data_ptr<float>(), b2.data_ptr<float>(), m ? m + kMagScales : nullptr,
                         rec.data_ptr<float>(), stream_of(aff2));
  check_launches("head_pooled_record");
  return rec;
}

void head_update_pooled(const Tensor& dl_all, const Tensor& ya_all, const Tensor& rec_all, const Tensor& wfc,
                        const c10::optional<Tensor>& out, int64_t P, double scale, double lr, int64_t mode) {
  TORCH_CHECK(ya_all.dim() == 4 && ya_all.size(2) == 32, "head_update_pooled: ya_all must be [W,B,32,PB]");
  const int64_t Wr = ya_all.size(0), B = ya_all.size(1), Q = P / 2;
  TORCH_CHECK(Q >= 4 && B >= 1 && B <= 8, "head_update_pooled: needs P/2 >= 4 and 1 <= B <= 8 images per rank");
  TORCH_CHECK(mode >= 0 && mode <= 2, "head_update_pooled: mode 0 (update), 1 (=) or 2 (+=)");
  need(ya_all, at::kHalf, {Wr, B, 32, pb_plane(P)}, "ya_all");
  need(rec_all, at::kFloat, {Wr, 128}, "rec_all");
  TORCH_CHECK(wfc.dim() == 2 && wfc.size(1) == 32 * Q * Q && wfc.size(0) >= 1 && wfc.size(0) <= 10,
              "fc.weight must be [<=10, 32*Q*Q]");
  const int64_t NC = wfc.size(0);
  need(wfc, at::kFloat, {NC, 32 * Q * Q}, "fc.weight");
  need(dl_all, at::kFloat, {Wr * B, NC}, "dl_all");
  float* o = wfc.data_ptr<float>();
  if (mode != 0) {
    TORCH_CHECK(out.has_value() && out->defined(), "head_update_pooled: modes 1 and 2 write into out");
    need(*out, at::kFloat, {NC, 32 * Q * Q}, "out (dW)");
    o = out->data_ptr<float>();
  } else {
    TORCH_CHECK(lr > 0.0, "head_update_pooled: mode 0 needs lr > 0");
  }
  // (the weight-layout stores pick their width from the row's alignment class: 16-B aligned bases)
  TORCH_CHECK(reinterpret_cast<uintptr_t>(o) % 16 == 0 && reinterpret_cast<uintptr_t>(wfc.data_ptr()) % 16 == 0,
              "head_update_pooled: fc.weight and out must be 16-B aligned");
  c10::DeviceGuard guard(wfc.device());
  const int rc = tds_head_upd_pb(ya_out(ya_all), B * 32 * pb_plane(P), rec_all.data_ptr<float>(), (int)Wr,
                                 dl_all.data_ptr<float>(), wfc.data_ptr<float>(), o, (int)B, (int)Q, (int)NC,
                                 (float)scale, (float)lr, (int)mode, stream_of(wfc));
  TORCH_CHECK(rc == 0, "head_update_pooled: unsupported shape");
  check_launches("head_update_pooled");
}

// ---------------------------------------------------------------- head forward (BN2 finalize + fc)
// returns (logits, stats2 [mean32|invstd32], aff2 [a32|b32])
std::tuple<Tensor, Tensor, Tensor> fused_head_forward(
    const Tensor& ya, const Tensor& partial2, const Tensor& b2, const c10::optional<Tensor>& gamma2,
    const c10::optional<Tensor>& beta2, const c10::optional<Tensor>& rm2, const c10::optional<Tensor>& rv2,
    const c10::optional<Tensor>& nbt2, double momentum, double eps, const Tensor& wfc, const c10::optional<Tensor>& bfc,
    int64_t P, const c10::optional<Tensor>& x_out, const c10::optional<Tensor>& mag) {
  TORCH_CHECK(ya.dim() == 3 && ya.size(1) == 32, "fused_head_forward: ya must be [B,32,PB]");
  const int64_t B = ya.size(0), Q = P / 2;
  TORCH_CHECK(Q >= 4 && B >= 1, "fused_head_forward: needs P/2 >= 4 pooled columns and B >= 1");
  need(ya, at::kHalf, {B, 32, pb_plane(P)}, "ya (fp16)");
  TORCH_CHECK(partial2.is_cuda() && partial2.scalar_type() == at::kDouble && partial2.numel() % 64 == 0, "partial2");
  const int nch = (int)(partial2.numel() / 64);
  need(b2, at::kFloat, {32}, "conv2.bias");
  const float* g = optf(gamma2, 32, "bn2.weight");
  const float* be = optf(beta2, 32, "bn2.bias");
  float* rm = const_cast<float*>(optf(rm2, 32, "bn2.running_mean"));
  float* rv = const_cast<float*>(optf(rv2, 32, "bn2.running_var"));
  int64_t* nb = nullptr;
  if (nbt2.has_value() && nbt2->defined()) {
    TORCH_CHECK(nbt2->is_cuda() && nbt2->scalar_type() == at::kLong && nbt2->numel() == 1, "bn2.num_batches_tracked");
    nb = nbt2->data_ptr<int64_t>();
  }
  TORCH_CHECK(wfc.dim() == 2 && wfc.size(1) == 32 * Q * Q && wfc.size(0) >= 1 && wfc.size(0) <= 10,
              "fc.weight must be [<=10, 32*Q*Q]");
  const int64_t NC = wfc.size(0);
  need(wfc, at::kFloat, {NC, 32 * Q * Q}, "fc.weight");
  const float* bf = optf(bfc, NC, "fc.bias");
  float* xo = nullptr;
  if (x_out.has_value() && x_out->defined()) {
    need(*x_out, at::kFloat, {B, 32 * Q * Q}, "x_out (fc input rows)");
    xo = x_out->data_ptr<float>();
  }
  c10::DeviceGuard guard(ya.device());
  hipStream_t st = stream_of(ya);
  auto stats = at::empty({64}, ya.options().dtype(at::kFloat));
  auto aff = at::empty({64}, ya.options().dtype(at::kFloat));
  tds_bn_reduce_finalize(partial2.data_ptr<double>(), 32, nch, B * P * P, b2.data_ptr<float>(), (float)eps,
                         (float)momentum, g, be, stats.data_ptr<float>(), rm, rv, nb, aff.data_ptr<float>(), st);
  const int nblk = 32 * tds_head_pb_nblk((int)Q);
  auto part = at::empty({(int64_t)(nblk + 32) * B * NC}, ya.options().dtype(at::kDouble));
  auto lsum = at::empty({B * NC}, ya.options().dtype(at::kDouble));
  auto logits = at::empty({B, NC}, ya.options().dtype(at::kFloat));
  const int rc = tds_head_fwd_pb(ya_out(ya), ya_dec(b2, mag), wfc.data_ptr<float>(), bf, aff.data_ptr<float>(),
                                 part.data_ptr<double>(), lsum.data_ptr<double>(), logits.data_ptr<float>(), xo, (int)B,
                                 (int)Q, (int)NC, st);
  TORCH_CHECK(rc == 0, "fused_head_forward: unsupported shape");
  check_launches("fused_head_forward");
  return {logits, stats, aff};
}

// ---------------------------------------------------------------- head backward
// fc / pool / ReLU / BN2 backward up to the pooled gradient g2m and the BN2 backward constants
// kbuf = [k1|k2|k3] (dy2 = k1*dz + k2*y2 + k3, rebuilt tile by tile inside the conv2 backward).
// update_lr > 0: the plain-SGD step of fc.weight runs in the same pass (W -= lr * dW).
// returns (dW [into dw_out if given; empty when !compute_dw], db_fc, dgamma2, dbeta2, g2m, kbuf)
// BN2 partial-sum workspace (doubles) of the head backward for B images at pooled size P/2
// Host copy of the conv2 backward walk table (CPU int tensor [rows, nwg]) for tests/inspection.
Tensor conv2_bwd_walk_table(int64_t B, int64_t tiles_r, int64_t tiles_c, int64_t nwg, int64_t seg) {
  const int64_t n = tds_conv2_bwd_walk(nullptr, (int)B, (int)tiles_r, (int)tiles_c, (int)nwg, (int)seg);
  TORCH_CHECK(n > 0, "conv2_bwd_walk_table: unsupported sizes");
  auto t = at::empty({n / nwg, nwg}, at::TensorOptions().dtype(at::kInt));
  tds_conv2_bwd_walk(t.data_ptr<int>(), (int)B, (int)tiles_r, (int)tiles_c, (int)nwg, (int)seg);
  return t;
}

// Per-wave barrier-wait clocks of the last conv2 backward launch of a TDS_CONV2_DIAG=13 diag
// build ([nwg][8][wait, total] shader-clock cycles; zeros in production builds).
Tensor conv2_bwd_clock_dump(int64_t nwg) {
  auto t = at::zeros({nwg, 8, 2}, at::TensorOptions().dtype(at::kInt));
  const int n = tds_conv2_bwd_clock_read(reinterpret_cast<uint32_t*>(t.data_ptr<int>()), (int)(nwg * 16));
  TORCH_CHECK(n >= 0, "conv2_bwd_clock_dump: hipMemcpyFromSymbol failed");
  return t;
}

// the BN2 partials [32][npass * nblk][4] (fp32 dz / stored dz sums), then 16 doubles = g2m's 32 per-channel scales 2^-e_c (fp32)
// for the K-chunked launches (the finalizing call copies them into kbuf[96..128))
int64_t head_bwd_workspace(int64_t B, int64_t P) {
  const int Q = (int)(P / 2);
  return (int64_t)32 * tds_head_bwd_pb_npass((int)B) * tds_head_bwd_pb_nblk(Q) * 4 + 16;
}

// Channels [c_begin, c_end) of the head backward (K-chunked fc gradient): the caller passes the
// same g2m_out / partial_out to every chunk and finalize=True on the last one, which then runs
// the BN2 backward finalize and the bias gradient (outputs 1-3 and 5 are empty before that).
std::tuple<Tensor, Tensor, Tensor, Tensor, Tensor, Tensor> fused_head_backward(
    const Tensor& dlogits, const Tensor& ya, const Tensor& stats2, const Tensor& aff2, const Tensor& b2,
    const c10::optional<Tensor>& gamma2, const Tensor& wfc, int64_t P, const c10::optional<Tensor>& dw_out,
    double scale, bool compute_dw, double update_lr, const c10::optional<Tensor>& dbfc_out,
    const c10::optional<Tensor>& dg_out, const c10::optional<Tensor>& dbe_out, bool keep_dw, int64_t c_begin,
    int64_t c_end, bool finalize, const c10::optional<Tensor>& g2m_out, const c10::optional<Tensor>& partial_out,
    const c10::optional<Tensor>& mag, bool ypart_done) {
  TORCH_CHECK(ya.dim() == 3 && ya.size(1) == 32, "fused_head_backward: ya must be [B,32,PB]");
  const int64_t B = ya.size(0), Q = P / 2;
  TORCH_CHECK(Q >= 4 && B >= 1, "fused_head_backward: needs P/2 >= 4 pooled columns and B >= 1");
  TORCH_CHECK(0 <= c_begin && c_begin < c_end && c_end <= 32, "fused_head_backward: bad channel range");
  need(ya, at::kHalf, {B, 32, pb_plane(P)}, "ya (fp16)");
  const int64_t NC = wfc.size(0);
  need(wfc, at::kFloat, {NC, 32 * Q * Q}, "fc.weight");
  need(dlogits, at::kFloat, {B, NC}, "dlogits");
  need(stats2, at::kFloat, {64}, "stats2");
  need(aff2, at::kFloat, {64}, "aff2");
  const float* g = optf(gamma2, 32, "bn2.weight");
  const TdsYaDec yd = ya_dec(b2, mag);
  c10::DeviceGuard guard(ya.device());
  hipStream_t st = stream_of(ya);
  const bool upd = update_lr > 0.0;
  TORCH_CHECK(keep_dw || upd, "fused_head_backward: keep_dw=False needs update_lr > 0 (update-only step)");
  const bool whole = c_begin == 0 && c_end == 32;
  TORCH_CHECK(whole || !upd, "fused_head_backward: the fused SGD step runs on the whole weight only");
  Tensor dW;  // undefined (None) for an update-only step
  if (!compute_dw) {
    dW = at::empty({0}, wfc.options());
  } else if (!keep_dw) {
  } else if (dw_out.has_value() && dw_out->defined()) {
    need(*dw_out, at::kFloat, {NC, 32 * Q * Q}, "dW_out");
    dW = *dw_out;
  } else {
    TORCH_CHECK(whole, "fused_head_backward: a channel chunk writes into dw_out");
    dW = at::empty_like(wfc);
  }
  TORCH_CHECK(!upd || (compute_dw && tds_head_bwd_pb_npass((int)B) == 1),
              "fused_head_backward: update_lr needs compute_dw and a batch of <= 8 images");
  Tensor g2m;
  if (g2m_out.has_value() && g2m_out->defined()) {
    need(*g2m_out, at::kHalf, {B, 32, Q, Q}, "g2m_out");
    g2m = *g2m_out;
  } else {
    TORCH_CHECK(whole, "fused_head_backward: a channel chunk writes into g2m_out");
    // planar (the fc flatten order), with the 64 B of slack the conv2 backward's row loads may
    // touch past the last row (conv2_bwd.hip BRStager GB)
    g2m = at::empty({B * 32 * Q * Q + kG2mSlack}, ya.options().dtype(at::kHalf))
              .narrow(0, 0, B * 32 * Q * Q)
              .view({B, 32, Q, Q});
  }
  const int nblk = tds_head_bwd_pb_nblk((int)Q), npass = tds_head_bwd_pb_npass((int)B);
  Tensor partial;
  if (partial_out.has_value() && partial_out->defined()) {
    need(*partial_out, at::kDouble, {head_bwd_workspace(B, P)}, "partial_out");
    partial = *partial_out;
  } else {
    TORCH_CHECK(whole, "fused_head_backward: a channel chunk writes into partial_out");
    partial = at::empty({head_bwd_workspace(B, P)}, ya.options().dtype(at::kDouble));
  }
  // g2m's per-channel scales 2^-e_c: straight into kbuf[96..128) for a whole-weight call, into the
  // workspace tail for the channel chunks (copied at the finalizing call)
  auto kbuf = at::empty({128}, ya.options().dtype(at::kFloat));
  float* g2inv_tail = reinterpret_cast<float*>(partial.data_ptr<double>() + (int64_t)32 * npass * nblk * 4);
  float* g2inv = whole ? kbuf.data_ptr<float>() + 96 : g2inv_tail;
  auto* g2p = reinterpret_cast<unsigned short*>(g2m.data_ptr<at::Half>());
  uint32_t* gp = opt_mag(mag, mag_numel(B, P)) ? opt_mag(mag) + kMagParts + 32 * mag_ypart_count() : nullptr;
  // the BN2 backward finalize inside the head backward's launch (head_pb.hip HBFin): one pass over
  // all channels, with the conv2 forward having reduced its magnitude parts (ypart_done)
  // (its one-round reducer takes at most 256 workgroups per channel: past that -- images beyond
  // ~2048^2 pooled -- the separate finalize below)
  const bool fin_in = finalize && whole && npass == 1 && ypart_done && nblk <= 256 && tds_fused_fin_enabled();
  if (fin_in) {
    auto dgamma = sink_or_empty(dg_out, {32}, ya, "dgamma2_out");
    auto dbeta = sink_or_empty(dbe_out, {32}, ya, "dbeta2_out");
    auto dbfc = sink_or_empty(dbfc_out, {NC}, ya, "dbfc_out");
    auto cmax = at::empty({32}, ya.options().dtype(at::kInt));
    TdsHeadBwdFin hf{reinterpret_cast<uint32_t*>(cmax.data_ptr<int>()), stats2.data_ptr<float>(), g,
                     dgamma.data_ptr<float>(), dbeta.data_ptr<float>(), kbuf.data_ptr<float>(), dbfc.data_ptr<float>(),
                     opt_mag(mag, mag_numel(B, P))};
    const int rc = tds_head_bwd_pb(ya_out(ya), yd, wfc.data_ptr<float>(), aff2.data_ptr<float>(),
                                   dlogits.data_ptr<float>(), g2p, partial.data_ptr<double>(),
                                   compute_dw && dW.defined() ? dW.data_ptr<float>() : nullptr,
                                   upd ? const_cast<float*>(wfc.data_ptr<float>()) : nullptr, (int)B, (int)Q, (int)NC,
                                   (float)scale, (float)update_lr, 0, 32, gp, g2inv, st, &hf);
    TORCH_CHECK(rc == 0, "fused_head_backward: unsupported shape (rc ", rc, ")");
    check_launches("fused_head_backward");
    return {dW, dbfc, dgamma, dbeta, g2m, kbuf};
  }
  const int rc = tds_head_bwd_pb(ya_out(ya), yd, wfc.data_ptr<float>(), aff2.data_ptr<float>(),
                                 dlogits.data_ptr<float>(), g2p, partial.data_ptr<double>(),
                                 compute_dw && dW.defined() ? dW.data_ptr<float>() : nullptr,
                                 upd ? const_cast<float*>(wfc.data_ptr<float>()) : nullptr, (int)B, (int)Q, (int)NC,
                                 (float)scale, (float)update_lr, (int)c_begin, (int)c_end, gp, g2inv, st);
  TORCH_CHECK(rc == 0, "fused_head_backward: unsupported shape (rc ", rc, ")");
  if (!finalize) {
    check_launches("fused_head_backward");
    const Tensor none = at::empty({0}, ya.options().dtype(at::kFloat));
    return {dW, none, none, none, g2m, none};
  }
  auto dgamma = sink_or_empty(dg_out, {32}, ya, "dgamma2_out");
  auto dbeta = sink_or_empty(dbe_out, {32}, ya, "dbeta2_out");
  if (!whole) kbuf.narrow(0, 96, 32).copy_(partial.narrow(0, (int64_t)32 * npass * nblk * 4, 16).view(at::kFloat));
  auto dbfc = sink_or_empty(dbfc_out, {NC}, ya, "dbfc_out");
  uint32_t* m = opt_mag(mag, mag_numel(B, P));
  tds_bn_bwd_finalize2(partial.data_ptr<double>(), 32, npass * nblk, B * P * P, g, stats2.data_ptr<float>(),
                       dgamma.data_ptr<float>(), dbeta.data_ptr<float>(), kbuf.data_ptr<float>(), dlogits.data_ptr<float>(),
                       (int)B, (int)NC, dbfc.data_ptr<float>(), (float)scale, m && !ypart_done ? m + kMagParts : nullptr,
                       (int)mag_ypart_count(), m ? m + kMagParts + 32 * mag_ypart_count() : nullptr,
                       (int)mag_gpart_count(B, P), m, st);
  check_launches("fused_head_backward");
  return {dW, dbfc, dgamma, dbeta, g2m, kbuf};
}

// ---------------------------------------------------------------- conv2 backward
// BN2/ReLU/pool backward fused into conv2 dgrad + wgrad: (y2h, a2, g2m, aff2, kbuf, b2, p1) -> (dp1h, dw2,
// db2); dp1h's decode factor lands in mag[kMagScales + 4] (fused_l1_backward's dp1_dec)
std::tuple<Tensor, Tensor, Tensor> fused_conv2_backward_y2(const Tensor& y2, const Tensor& a2, const Tensor& g2m,
                                                           const Tensor& aff2,
                                                           const Tensor& kbuf, const Tensor& b2, const Tensor& mag,
                                                           const Tensor& p1,
                                                           const Tensor& wd, double scale,
                                                           const c10::optional<Tensor>& dw_out,
                                                           const c10::optional<Tensor>& db_out) {
  const int64_t B = p1.size(0), P = p1.size(1);
  need(p1, at::kHalf, {B, P, P, 16}, "p1");
  opt_mag(mag, kMagScales + 5);  // the magnitude bounds of the forward / head backward, the y2h decode, the
                                 // dp1h factors (kernels/conv2_common.h; mag[kMagScales + 4] is written)
  need(y2, at::kHalf, {B, P, P, 32}, "y2h (fused_conv2_forward's)");
  need(a2, at::kInt, {B, P / 2, P / 2, 2}, "a2 (fused_conv2_forward's pooling argmax codes)");
  need(b2, at::kFloat, {32}, "conv2.bias");
  need(g2m, at::kHalf, {B, 32, P / 2, P / 2}, "g2m (fused_head_backward's, fp16 at the scales in kbuf[96..128))");
  TORCH_CHECK((int64_t)g2m.storage().nbytes() >= (g2m.storage_offset() + g2m.numel() + kG2mSlack) * 2,
              "fused_conv2_backward_y2: g2m needs ", kG2mSlack, " fp16 elements of slack after it (as "
              "fused_head_backward allocates it): the staging's row loads may read past the last row");
  need(aff2, at::kFloat, {64}, "aff2");
  need(kbuf, at::kFloat, {128}, "kbuf");
  need(wd, at::kShort, {25 * 4 * 16 * 8}, "conv2 dgrad pack");
  TORCH_CHECK(B <= 63 && P >= 2, "fused_conv2_backward_y2: 1 <= batch <= 63 and P >= 2");
  c10::DeviceGuard guard(p1.device());
  hipStream_t st = stream_of(p1);
  const int nwg = tds_conv2_bwd3_num_wg();
  int tr = 0, tc = 0;
  tds_conv2_bwd3_tiles((int)P, &tr, &tc);
  int sw = 0, sk = 0;
  const int* order = bwd_walk(p1, (int)B, tr, tc, nwg, &sw, &sk);
  auto dp1 = at::empty({B, P, (P + 3) / 4, 16, 4}, p1.options().dtype(at::kHalf));  // dp1h (kernels/conv2_common.h)
  auto slab = at::empty({(int64_t)nwg * 26 * 512}, p1.options().dtype(at::kFloat));
  auto dw2 = sink_or_empty(dw_out, {32, 16, 5, 5}, p1, "dw2_out");
  auto db2 = sink_or_empty(db_out, {32}, p1, "db2_out");
  tds_conv2_bwd3(y2.data_ptr(), reinterpret_cast<const uint32_t*>(a2.data_ptr<int>()),
                 reinterpret_cast<const unsigned short*>(g2m.data_ptr<at::Half>()), aff2.data_ptr<float>(), kbuf.data_ptr<float>(),
                 b2.data_ptr<float>(), reinterpret_cast<uint32_t*>(mag.data_ptr<int>()), p1.data_ptr(),
                 wd.data_ptr<int16_t>(),
                 dp1.data_ptr(), slab.data_ptr<float>(), order, nwg, sw, sk, (int)B, (int)P, st);
  tds_conv2_wgrad_reduce(slab.data_ptr<float>(), nwg, dw2.data_ptr<float>(), db2.data_ptr<float>(), (float)scale, st);
  check_launches("fused_conv2_backward_y2");
  return {dp1, dw2, db2};
}

// CU budget (cu_budget.hip): reserve CUs for RCCL's kernels; persistent kernels size their
// grids to the rest; a CU-masked stream for the compute (returned as a raw handle, wrapped in
// torch.cuda.ExternalStream by utils/streams.py)
void set_cu_reserve(int64_t n) { tds_set_cu_reserve((int)n); }
int64_t cu_reserve() { return tds_cu_reserve(); }
int64_t device_cus() { return tds_device_cus(); }
int64_t cu_masked_stream(int64_t device, int64_t reserve, bool striped) {
  hipStream_t s = tds_cu_masked_stream((int)device, (int)reserve, striped);
  TORCH_CHECK(s != nullptr, "cu_masked_stream: hipExtStreamCreateWithCUMask failed (device ", device, ", reserve ",
              reserve, ")");
  return (int64_t)reinterpret_cast<intptr_t>(s);
}

// the communication stream of the CU split (0 when no CUs are reserved)
int64_t cu_comm_stream(int64_t device) { return (int64_t)reinterpret_cast<intptr_t>(tds_cu_comm_stream((int)device)); }

int64_t cu_release_streams() { return tds_cu_release_streams(); }

// a further stream on one side of the CU split (0 when no CUs are reserved)
int64_t cu_side_stream(int64_t device, bool comm) {
  return (int64_t)reinterpret_cast<intptr_t>(tds_cu_side_stream((int)device, comm));
}

// one-GPU rehearsal of a collective's CU footprint (cu_budget.hip): `nblocks` workgroups of 256
// threads holding `lds_bytes` of LDS each for `us` microseconds, on the current stream
// Device-to-device copy on the current stream of dst's device by the copy engines (SDMA, no compute
// units: hipMemcpyDeviceToDeviceNoCU) or, nocu = false, the runtime's blit kernel -- the bulk
// payload of the fc exchange rehearsed on one GPU (bench.py --sim-sdma-mb)
void copy_engine(const Tensor& dst, const Tensor& src, bool nocu) {
  TORCH_CHECK(dst.is_cuda() && src.is_cuda() && dst.is_contiguous() && src.is_contiguous() &&
                  dst.nbytes() == src.nbytes(), "copy_engine: contiguous GPU tensors of equal size");
  c10::DeviceGuard guard(dst.device());
  const hipError_t e = hipMemcpyAsync(dst.data_ptr(), src.data_ptr(), dst.nbytes(),
                                      nocu ? hipMemcpyDeviceToDeviceNoCU : hipMemcpyDeviceToDevice, stream_of(dst));
  TORCH_CHECK(e == hipSuccess, "copy_engine: hipMemcpyAsync failed: ", hipGetErrorString(e));
}

void comm_spin(const Tensor& like, int64_t us, int64_t nblocks, int64_t lds_bytes) {
  TORCH_CHECK(like.is_cuda(), "comm_spin: needs a GPU tensor");
  TORCH_CHECK(us >= 0 && us <= 1000000 && nblocks >= 1 && nblocks <= 1024 && lds_bytes >= 1024 &&
                  lds_bytes <= 64 * 1024,
              "comm_spin: 0 <= us <= 1e6, 1 <= nblocks <= 1024, 1 KiB <= lds <= 64 KiB");
  c10::DeviceGuard guard(like.device());
  auto sink = at::empty({nblocks}, like.options().dtype(at::kInt));
  tds_comm_spin(us, (int)nblocks, (int)lds_bytes, sink.data_ptr<int>(), stream_of(like));
  check_launches("comm_spin");
}

// where the current stream's workgroups land: [nblocks, 2] int32 (XCC id, HW_ID register)
Tensor cu_probe(const Tensor& like, int64_t us, int64_t nblocks) {
  TORCH_CHECK(like.is_cuda() && us >= 0 && us <= 100000 && nblocks >= 1 && nblocks <= 65536, "cu_probe: arguments");
  c10::DeviceGuard guard(like.device());
  auto out = at::empty({nblocks, 2}, like.options().dtype(at::kInt));
  tds_cu_probe(us, (int)nblocks, out.data_ptr<int>(), stream_of(like));
  check_launches("cu_probe");
  return out;
}

// test hook: one launch of a trivial kernel with the given dynamic LDS / block size (a request
// beyond the hardware limits must surface as an exception through check_launches)
void launch_probe(const Tensor& like, int64_t lds_bytes, int64_t threads) {
  TORCH_CHECK(like.is_cuda(), "launch_probe: needs a GPU tensor");
  c10::DeviceGuard guard(like.device());
  tds_launch_probe(nullptr, (int)lds_bytes, (int)threads, stream_of(like));
  check_launches("launch_probe");
}

// ---------------------------------------------------------------- layer 1 backward
std::tuple<Tensor, Tensor, Tensor, Tensor> fused_l1_backward(const Tensor& dp1, const Tensor& dp1_dec,
                                                             const Tensor& x, const Tensor& p1,
                                                             const Tensor& idx1, const Tensor& w1, const Tensor& b1,
                                                             const c10::optional<Tensor>& gamma1, const Tensor& stats1,
                                                             const Tensor& gram, double scale,
                                                             const c10::optional<Tensor>& dw_out,
                                                             const c10::optional<Tensor>& db_out,
                                                             const c10::optional<Tensor>& dg_out,
                                                             const c10::optional<Tensor>& dbe_out) {
  TORCH_CHECK(x.dim() == 4 && x.size(1) == 1, "fused_l1_backward: x");
  const int64_t B = x.size(0), H = x.size(2), W = x.size(3), P = H / 2;
  const bool levels = x.scalar_type() == at::kByte;
  need(x, levels ? at::kByte : at::kFloat, {B, 1, H, W}, "x");
  need(dp1, at::kHalf, {B, P, (W / 2 + 3) / 4, 16, 4}, "dp1h (fused_conv2_backward_y2's)");
  TORCH_CHECK(dp1_dec.is_cuda() && dp1_dec.scalar_type() == at::kInt && dp1_dec.numel() >= 1,
              "dp1_dec: the dp1h decode factor (int32 GPU view of mag[kMagScales + 4])");
  need(p1, at::kHalf, {B, P, P, 16}, "p1");
  need(idx1, at::kByte, {B, P, P, 16}, "idx1");
  need(w1, at::kFloat, {16, 1, 5, 5}, "conv1.weight");
  need(b1, at::kFloat, {16}, "conv1.bias");
  need(stats1, at::kFloat, {32}, "stats1");
  need(gram, at::kDouble, {650}, "gram");
  const float* g = optf(gamma1, 16, "bn1.weight");
  c10::DeviceGuard guard(x.device());
  hipStream_t st = stream_of(x);
  const int nwg = l1b_wg(levels), rows = tds_l1_bwd_rows(nwg);
  auto partial = at::empty({(int64_t)rows * 16 * 27}, x.options().dtype(at::kDouble));
  auto dw1 = sink_or_empty(dw_out, {16, 1, 5, 5}, x, "dw1_out");
  auto db1 = sink_or_empty(db_out, {16}, x, "db1_out");
  auto dg = sink_or_empty(dg_out, {16}, x, "dgamma1_out");
  auto dbe = sink_or_empty(dbe_out, {16}, x, "dbeta1_out");
  // (the reduction and the closed-form gradients inside this launch measured slower than the one
  // small launch below: its 1280 partial rows of 432 doubles need several dependent rounds of loads
  // in one workgroup, l1 backward 0.172 ms vs 0.131 + 2 x 0.007, r5_s3)
  tds_l1_bwd(x.data_ptr(), levels, dp1.data_ptr(), reinterpret_cast<const uint32_t*>(dp1_dec.data_ptr<int>()),
             p1.data_ptr(), idx1.data_ptr<uint8_t>(), partial.data_ptr<double>(), nwg, (int)B, (int)H, (int)W, st);
  auto bsum = at::empty({16 * 27}, x.options().dtype(at::kDouble));
  // the partials' reduction and the closed-form gradients in one launch (tds_l1_reduce_finalize)
  if (!tds_l1_reduce_finalize(partial.data_ptr<double>(), rows, bsum.data_ptr<double>(), gram.data_ptr<double>(),
                              B * H * W, w1.data_ptr<float>(), b1.data_ptr<float>(), g, stats1.data_ptr<float>(),
                              dw1.data_ptr<float>(), db1.data_ptr<float>(), dg.data_ptr<float>(), dbe.data_ptr<float>(),
                              (float)scale, st)) {
    tds_reduce_partials(partial.data_ptr<double>(), bsum.data_ptr<double>(), 16 * 27, rows, 16 * 27, 0, 16 * 27, st);
    tds_l1_finalize(bsum.data_ptr<double>(), gram.data_ptr<double>(), B * H * W, w1.data_ptr<float>(),
                    b1.data_ptr<float>(), g, stats1.data_ptr<float>(), dw1.data_ptr<float>(), db1.data_ptr<float>(),
                    dg.data_ptr<float>(), dbe.data_ptr<float>(), (float)scale, st);
  }
  check_launches("fused_l1_backward");
  return {dw1, db1, dg, dbe};
}

// ---------------------------------------------------------------- zero-suppressed X exchange
// (parallel/zs.py: format; kernels/zs_exchange.hip)
Tensor zs_encode(const Tensor& x, const Tensor& meta_out, const Tensor& values_out) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kFloat && x.is_contiguous(), "zs_encode: x fp32 contiguous GPU");
  const int64_t n = x.numel(), P = tds_zs_npages(n);
  TORCH_CHECK(n > 0, "zs_encode: empty x");
  need(meta_out, at::kInt, {P * 65}, "zs meta_out");
  TORCH_CHECK(values_out.is_cuda() && values_out.scalar_type() == at::kFloat && values_out.is_contiguous() &&
                  values_out.dim() == 1,
              "zs_encode: values_out fp32 1-d contiguous GPU");
  TORCH_CHECK(x.device() == meta_out.device() && x.device() == values_out.device(), "zs_encode: one device");
  TORCH_CHECK(n < ((int64_t)1 << 31), "zs_encode: the format's int32 offsets need < 2^31 elements");
  c10::DeviceGuard guard(x.device());
  auto nnz = at::empty({}, x.options().dtype(at::kLong));
  tds_zs_encode(x.data_ptr<float>(), n, meta_out.data_ptr<int>(), values_out.data_ptr<float>(), values_out.numel(),
                nnz.data_ptr<int64_t>(), stream_of(x));
  check_launches("zs_encode");
  return nnz;
}

void zs_decode(const Tensor& meta, const Tensor& values, const Tensor& out) {
  TORCH_CHECK(out.is_cuda() && out.scalar_type() == at::kFloat && out.is_contiguous(), "zs_decode: out fp32 GPU");
  const int64_t n = out.numel(), P = tds_zs_npages(n);
  TORCH_CHECK(n > 0, "zs_decode: empty out");
  need(meta, at::kInt, {P * 65}, "zs meta");
  TORCH_CHECK(values.is_cuda() && values.scalar_type() == at::kFloat && values.is_contiguous(),
              "zs_decode: values fp32 contiguous GPU");
  c10::DeviceGuard guard(out.device());
  tds_zs_decode(meta.data_ptr<int>(), values.data_ptr<float>(), values.numel(), out.data_ptr<float>(), n,
                stream_of(out));
  check_launches("zs_decode");
}

// dW (=/+=) scale dyᵀX or W -= update_lr * scale dyᵀX with X as the all-gathered zero-suppressed
// rows: meta [W, P*65 + 2] int32 (the records + each rank's count), values [W, cap] fp32, `rows`
// rows of K columns per rank; dy [W*rows, N].  The counts must not exceed cap (the caller checks).
void linear_dw_zs(const Tensor& dy, const Tensor& meta, const Tensor& values, int64_t rows, const Tensor& dw,
                  const c10::optional<Tensor>& db, double scale, bool accumulate, double update_lr) {
  TORCH_CHECK(dy.is_cuda() && dy.scalar_type() == at::kFloat && dy.is_contiguous() && dy.dim() == 2,
              "linear_dw_zs: dy fp32 [M, N] contiguous GPU");
  const int64_t M = dy.size(0), N = dy.size(1);
  TORCH_CHECK(dw.is_cuda() && dw.scalar_type() == at::kFloat && dw.dim() == 2 && dw.size(0) == N && dw.stride(1) == 1,
              "linear_dw_zs: dW [N, K] unit-stride rows");
  const int64_t K = dw.size(1);
  TORCH_CHECK(rows >= 1 && M % rows == 0, "linear_dw_zs: dy rows must be W x rows");
  const int64_t W = M / rows, P = tds_zs_npages(rows * K);
  TORCH_CHECK(meta.is_cuda() && meta.scalar_type() == at::kInt && meta.is_contiguous() && meta.dim() == 2 &&
                  meta.size(0) == W && meta.size(1) >= P * 65,
              "linear_dw_zs: meta int32 [W, >= npages*65]");
  TORCH_CHECK(values.is_cuda() && values.scalar_type() == at::kFloat && values.is_contiguous() && values.dim() == 2 &&
                  values.size(0) == W,
              "linear_dw_zs: values fp32 [W, cap]");
  TORCH_CHECK(rows * K < ((int64_t)1 << 31), "linear_dw_zs: int32 offsets");
  float* dbp = nullptr;
  if (db.has_value() && db->defined()) {
    need(*db, at::kFloat, {N}, "db");
    dbp = db->data_ptr<float>();
  }
  c10::DeviceGuard guard(dy.device());
  const int rc = tds_linear_dw_zs(dy.data_ptr<float>(), meta.data_ptr<int>(), meta.size(1), values.data_ptr<float>(),
                                  values.size(1), (int)rows, (int)M, (int)N, K, dw.data_ptr<float>(), dw.stride(0), dbp,
                                  (float)scale, accumulate ? 1 : 0, (float)update_lr, stream_of(dy));
  TORCH_CHECK(rc == 0, "linear_dw_zs: unsupported shape (K % 4, 16-B aligned rows, N in {10, 16})");
  check_launches("linear_dw_zs");
}

void check_pages(const Tensor& start, const Tensor& cnt, const Tensor& seg, const Tensor& like) {
  TORCH_CHECK(start.is_cuda() && start.scalar_type() == at::kLong && start.dim() == 1 && start.is_contiguous(),
              "zs pages: start int64 [npages]");
  need(cnt, at::kInt, {start.numel()}, "zs pages: cnt");
  need(seg, at::kInt, {start.numel()}, "zs pages: seg");
  TORCH_CHECK(start.device() == like.device(), "zs pages: one device");
}

// segmented encode (parallel/zs.py SegLayout): returns seg_nnz [nseg] int64
Tensor zs_seg_encode(const Tensor& x, const Tensor& pg_start, const Tensor& pg_cnt, const Tensor& pg_seg,
                     const Tensor& seg_first, const Tensor& seg_npg, const Tensor& meta_out, const Tensor& values_out,
                     int64_t cap) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kFloat && x.is_contiguous(), "zs_seg_encode: x fp32 GPU");
  check_pages(pg_start, pg_cnt, pg_seg, x);
  const int64_t P = pg_start.numel(), S = seg_first.numel();
  need(seg_first, at::kInt, {S}, "zs seg_first");
  need(seg_npg, at::kInt, {S}, "zs seg_npg");
  need(meta_out, at::kInt, {P * 65}, "zs meta_out");
  TORCH_CHECK(values_out.is_cuda() && values_out.scalar_type() == at::kFloat && values_out.numel() == S * cap &&
                  values_out.is_contiguous(),
              "zs_seg_encode: values_out fp32 [nseg * cap]");
  c10::DeviceGuard guard(x.device());
  auto counts = at::empty({P}, x.options().dtype(at::kInt));
  auto nnz = at::empty({S}, x.options().dtype(at::kLong));
  if (P > 0)
    tds_zs_seg_encode(x.data_ptr<float>(), pg_start.data_ptr<int64_t>(), pg_cnt.data_ptr<int>(), pg_seg.data_ptr<int>(),
                      P, seg_first.data_ptr<int>(), seg_npg.data_ptr<int>(), (int)S, meta_out.data_ptr<int>(),
                      counts.data_ptr<int>(), values_out.data_ptr<float>(), cap, nnz.data_ptr<int64_t>(), stream_of(x));
  else
    nnz.zero_();
  check_launches("zs_seg_encode");
  return nnz;
}

void zs_seg_decode(const Tensor& meta, const Tensor& pg_start, const Tensor& pg_cnt, const Tensor& pg_seg,
                   const Tensor& values, int64_t cap, const Tensor& out) {
  TORCH_CHECK(out.is_cuda() && out.scalar_type() == at::kFloat && out.is_contiguous(), "zs_seg_decode: out fp32 GPU");
  check_pages(pg_start, pg_cnt, pg_seg, out);
  const int64_t P = pg_start.numel();
  need(meta, at::kInt, {P * 65}, "zs meta");
  TORCH_CHECK(values.is_cuda() && values.scalar_type() == at::kFloat && values.is_contiguous(), "zs_seg_decode: values");
  c10::DeviceGuard guard(out.device());
  if (P > 0)
    tds_zs_seg_decode(meta.data_ptr<int>(), pg_start.data_ptr<int64_t>(), pg_cnt.data_ptr<int>(), pg_seg.data_ptr<int>(),
                      P, values.data_ptr<float>(), cap, out.data_ptr<float>(), stream_of(out));
  check_launches("zs_seg_decode");
}

}  // namespace

TORCH_LIBRARY_FRAGMENT(tdsa, m) {
  m.def("zs_encode(Tensor x, Tensor(a!) meta_out, Tensor(b!) values_out) -> Tensor", &zs_encode);
  m.def(
      "linear_dw_zs(Tensor dy, Tensor meta, Tensor values, int rows, Tensor(a!) dw, Tensor(b!)? db, float scale, "
      "bool accumulate, float update_lr=0.0) -> ()",
      &linear_dw_zs);
  m.def(
      "zs_seg_encode(Tensor x, Tensor pg_start, Tensor pg_cnt, Tensor pg_seg, Tensor seg_first, Tensor seg_npg, "
      "Tensor(a!) meta_out, Tensor(b!) values_out, int cap) -> Tensor",
      &zs_seg_encode);
  m.def(
      "zs_seg_decode(Tensor meta, Tensor pg_start, Tensor pg_cnt, Tensor pg_seg, Tensor values, int cap, "
      "Tensor(a!) out) -> ()",
      &zs_seg_decode);
  m.def("zs_decode(Tensor meta, Tensor values, Tensor(a!) out) -> ()", &zs_decode);
  m.def(
      "fused_l1_forward(Tensor x, Tensor w1, Tensor b1, Tensor? gamma1, Tensor? beta1, Tensor(a!)? rm1, "
      "Tensor(b!)? rv1, Tensor(c!)? nbt1, float momentum, float eps, Tensor? asum=None, Tensor? strips=None, "
      "Tensor(d!)? mag=None, Tensor? w2=None, Tensor(e!)? wp_out=None, Tensor(f!)? wd_out=None) -> "
      "(Tensor, Tensor, Tensor, Tensor, Tensor)",
      &fused_l1_forward);
  m.def("l1_input_stats(Tensor x) -> (Tensor, Tensor)", &l1_input_stats);
  m.def("conv2_pack(Tensor w2, Tensor(a!)? mag=None, Tensor? p1_scale=None, bool write_p1=True) -> (Tensor, Tensor)",
        &conv2_pack);
  m.def(
      "fused_conv2_forward(Tensor p1, Tensor wp, Tensor b2, Tensor? gamma2, Tensor(a!)? mag=None) -> "
      "(Tensor, Tensor, Tensor, Tensor)",
      &fused_conv2_forward);
  m.def(
      "fused_head_forward(Tensor ya, Tensor partial2, Tensor b2, Tensor? gamma2, Tensor? beta2, Tensor(a!)? rm2, "
      "Tensor(b!)? rv2, Tensor(c!)? nbt2, float momentum, float eps, Tensor wfc, Tensor? bfc, int P, "
      "Tensor(d!)? x_out=None, Tensor? mag=None) -> (Tensor, Tensor, Tensor)",
      &fused_head_forward);
  m.def(
      "fused_head_backward(Tensor dlogits, Tensor ya, Tensor stats2, Tensor aff2, Tensor b2, Tensor? gamma2, "
      "Tensor(e!) wfc, "
      "int P, Tensor(a!)? dw_out, float scale, bool compute_dw=True, float update_lr=0.0, "
      "Tensor(b!)? dbfc_out=None, Tensor(c!)? dg_out=None, Tensor(d!)? dbe_out=None, bool keep_dw=True, "
      "int c_begin=0, int c_end=32, bool finalize=True, Tensor(f!)? g2m_out=None, Tensor(g!)? partial_out=None, "
      "Tensor(h!)? mag=None, bool ypart_done=False) -> (Tensor, Tensor, Tensor, Tensor, Tensor, Tensor)",
      &fused_head_backward);
  m.def(
      "fused_conv2_forward_bn(Tensor p1, Tensor wp, Tensor b2, Tensor? gamma2, Tensor? beta2, Tensor(a!)? rm2, "
      "Tensor(b!)? rv2, Tensor(c!)? nbt2, float momentum, float eps, Tensor(d!)? mag=None) -> "
      "(Tensor, Tensor, Tensor, Tensor, Tensor)",
      &fused_conv2_forward_bn);
  m.def("fused_head_forward_aff(Tensor ya, Tensor aff2, Tensor b2, Tensor? mag, Tensor wfc, Tensor? bfc, int P, "
        "Tensor(a!)? x_out=None) -> Tensor",
        &fused_head_forward_aff);
  m.def("fused_head_forward_aff_ce(Tensor ya, Tensor aff2, Tensor b2, Tensor? mag, Tensor wfc, Tensor? bfc, int P, "
        "Tensor labels, "
        "Tensor(a!)? x_out=None) -> (Tensor, Tensor, Tensor)",
        &fused_head_forward_aff_ce);
  m.def("head_bwd_workspace(int B, int P) -> int", &head_bwd_workspace);
  m.def("head_forward_range_ws(Tensor ya, Tensor wfc, int P) -> (Tensor, Tensor, Tensor, Tensor, Tensor, Tensor)",
        &head_forward_range_ws);
  m.def(
      "fused_head_forward_range(Tensor ya, Tensor aff2, Tensor b2, Tensor? mag, Tensor wfc, Tensor? bfc, int P, int c0, "
      "int c1, Tensor(a!) part, "
      "Tensor(b!) lsum, Tensor(c!) logits, Tensor(d!) dlogits, Tensor(e!) loss, Tensor(f!) inv, Tensor? labels=None, "
      "Tensor(g!)? x_out=None) -> ()",
      &fused_head_forward_range);
  m.def("head_pooled_record(Tensor aff2, Tensor b2, Tensor? mag=None) -> Tensor", &head_pooled_record);
  m.def(
      "head_update_pooled(Tensor dl_all, Tensor ya_all, Tensor rec_all, Tensor(a!) wfc, Tensor(b!)? out, int P, "
      "float scale, float lr, int mode) -> ()",
      &head_update_pooled);
  m.def("mag_numel(int B, int P) -> int", &mag_numel);
  m.def("mag_ypart_count() -> int", &mag_ypart_count);
  m.def("conv2_bwd_clock_dump(int nwg) -> Tensor", &conv2_bwd_clock_dump);
  m.def("conv2_bwd_walk_table(int B, int tiles_r, int tiles_c, int nwg, int seg) -> Tensor", &conv2_bwd_walk_table);
  m.def(
      "fused_conv2_backward_y2(Tensor y2, Tensor a2, Tensor g2m, Tensor aff2, Tensor kbuf, Tensor b2, Tensor(c!) mag, Tensor p1, "
      "Tensor wd, "
      "float scale, Tensor(a!)? dw_out=None, Tensor(b!)? db_out=None) -> (Tensor, Tensor, Tensor)",
      &fused_conv2_backward_y2);
  m.def(
      "fused_l1_backward(Tensor dp1, Tensor dp1_dec, Tensor x, Tensor p1, Tensor idx1, Tensor w1, Tensor b1, Tensor? gamma1, "
      "Tensor stats1, Tensor gram, float scale, Tensor(a!)? dw_out=None, Tensor(b!)? db_out=None, "
      "Tensor(c!)? dg_out=None, Tensor(d!)? dbe_out=None) -> (Tensor, Tensor, Tensor, Tensor)",
      &fused_l1_backward);
  m.def("launch_probe(Tensor like, int lds_bytes, int threads) -> ()", &launch_probe);
  m.def("set_cu_reserve(int n) -> ()", &set_cu_reserve);
  m.def("cu_reserve() -> int", &cu_reserve);
  m.def("device_cus() -> int", &device_cus);
  m.def("cu_masked_stream(int device, int reserve, bool striped=True) -> int", &cu_masked_stream);
  m.def("comm_spin(Tensor like, int us, int nblocks, int lds_bytes) -> ()", &comm_spin);
  m.def("copy_engine(Tensor(a!) dst, Tensor src, bool nocu=True) -> ()", &copy_engine);
  m.def("cu_probe(Tensor like, int us, int nblocks) -> Tensor", &cu_probe);
  m.def("cu_comm_stream(int device) -> int", &cu_comm_stream);
  m.def("cu_release_streams() -> int", &cu_release_streams);
  m.def("cu_side_stream(int device, bool comm) -> int", &cu_side_stream);
}
