// Plan-level ops of the fused ConvNet execution (torch.ops.tdsa.fused_*).
// Each op = a few kernel launches on the current stream, all shapes checked on
// the host first.  Tensor "carriers": packed bf16 hi|lo activations are handed
// to autograd as float32 tensors of the same byte size, so that gradients line
// up shape-for-shape:
//   p1 carrier  [B,P,P,16] f32  == bytes of bf16 [B,P,P,32] (hi16|lo16)   <-> dp1  [B,P,P,16] f32
//   y2          [B,P,P,32] f32                                           <-> dy2 carrier [B,P,P,32] f32
//                                                                            == bytes of bf16 [B,P,P,64]
#include <ATen/ATen.h>
#include <c10/core/DeviceGuard.h>
#include <c10/hip/HIPStream.h>
#include <torch/library.h>

#include "kernels/launchers.h"

namespace {

using at::Tensor;

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

int l1_wg() { return tds_fused_num_wg(4); }

// ---------------------------------------------------------------- layer 1 forward
// returns (p1 carrier, idx1, stats1[mean16|invstd16], ac_partial, strips)
std::tuple<Tensor, Tensor, Tensor, Tensor> fused_l1_forward(
    const Tensor& x, const Tensor& w1, const Tensor& b1, const c10::optional<Tensor>& gamma1,
    const c10::optional<Tensor>& beta1, const c10::optional<Tensor>& rm1, const c10::optional<Tensor>& rv1,
    const c10::optional<Tensor>& nbt1, double momentum, double eps) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kFloat && x.is_contiguous(), "fused_l1_forward: x");
  TORCH_CHECK(x.dim() == 4 && x.size(1) == 1, "fused_l1_forward: x must be [B,1,H,W]");
  const int64_t B = x.size(0), H = x.size(2), W = x.size(3);
  TORCH_CHECK(H == W && H >= 8, "fused_l1_forward: square images with H >= 8");
  TORCH_CHECK(B >= 1 && B <= 32, "fused_l1_forward: 1 <= B <= 32 per rank");
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
  auto fo = x.options();
  // x autocorrelation + border strips -> Gram G / patch sums S -> BN1 statistics in closed form
  // one thread per 4 x 8 pixel block: each fp32 partial covers 32 products (fp64 beyond)
  const int nac = tds_x_autocorr_num_wg((int)B, (int)H, (int)W);
  TORCH_CHECK(nac > 0, "fused_l1_forward: x must be < 2 GiB with W % 4 == 0 (autocorrelation kernel)");
  auto ac = at::empty({(int64_t)nac * 42}, fo.dtype(at::kDouble));
  auto strips = at::empty({9 * 82}, fo.dtype(at::kDouble));
  tds_x_autocorr(x.data_ptr<float>(), ac.data_ptr<double>(), nac, strips.data_ptr<double>(), (int)B, (int)H, (int)W,
                 st);
  auto asum = at::empty({42}, fo.dtype(at::kDouble));
  tds_reduce_partials(ac.data_ptr<double>(), asum.data_ptr<double>(), 42, nac, 42, 0, 42, st);
  auto gram = at::empty({650}, fo.dtype(at::kDouble));
  auto sums = at::empty({32}, fo.dtype(at::kDouble));
  tds_l1_gram(asum.data_ptr<double>(), strips.data_ptr<double>(), x.data_ptr<float>(), (int)B, (int)H, (int)W,
              w1.data_ptr<float>(), gram.data_ptr<double>(), sums.data_ptr<double>(), st);
  auto stats = at::empty({32}, fo);
  auto aff = at::empty({32}, fo);
  tds_bn_finalize_shifted(sums.data_ptr<double>(), 16, 1, B * H * W, b1.data_ptr<float>(), (float)eps,
                          (float)momentum, g, be, stats.data_ptr<float>(), rm, rv, nb, aff.data_ptr<float>(), st);
  // the single conv1 pass: conv + BN1 affine + ReLU + pool -> p1, argmax
  auto p1 = at::empty({B, P, P, 16}, fo);  // carrier of bf16 [B,P,P,32]
  auto idx1 = at::empty({B, P, P, 16}, fo.dtype(at::kByte));
  tds_l1_apply(x.data_ptr<float>(), w1.data_ptr<float>(), b1.data_ptr<float>(), aff.data_ptr<float>(), p1.data_ptr(),
               idx1.data_ptr<uint8_t>(), l1_wg(), (int)B, (int)H, (int)W, st);
  return {p1, idx1, stats, gram};
}

// ---------------------------------------------------------------- conv2 forward
std::tuple<Tensor, Tensor> conv2_pack(const Tensor& w2) {
  need(w2, at::kFloat, {32, 16, 5, 5}, "conv2.weight");
  c10::DeviceGuard guard(w2.device());
  auto wp = at::empty({2 * 13 * 2 * 4 * 16 * 8}, w2.options().dtype(at::kShort));
  auto wd = at::empty({2 * 25 * 4 * 16 * 8}, w2.options().dtype(at::kShort));
  tds_conv2_pack_weights(w2.data_ptr<float>(), wp.data_ptr<int16_t>(), wd.data_ptr<int16_t>(), stream_of(w2));
  return {wp, wd};
}

std::tuple<Tensor, Tensor> fused_conv2_forward(const Tensor& p1, const Tensor& wp, const Tensor& b2) {
  TORCH_CHECK(p1.dim() == 4 && p1.size(1) == p1.size(2) && p1.size(3) == 16, "fused_conv2_forward: p1 carrier");
  const int64_t B = p1.size(0), P = p1.size(1);
  need(p1, at::kFloat, {B, P, P, 16}, "p1");
  need(wp, at::kShort, {2 * 13 * 2 * 4 * 16 * 8}, "conv2 fwd pack");
  need(b2, at::kFloat, {32}, "conv2.bias");
  TORCH_CHECK(B <= 255 && P <= 32760, "fused_conv2_forward: batch <= 255 and P <= 32760 (tile-order table packing)");
  c10::DeviceGuard guard(p1.device());
  const int nwg = tds_conv2_fwd_num_wg();
  auto y2 = at::empty({B, P, P, 32}, p1.options());
  auto partial = at::empty({32 * nwg * 2}, p1.options().dtype(at::kDouble));
  tds_conv2_fwd_bf16x3(p1.data_ptr(), wp.data_ptr<int16_t>(), b2.data_ptr<float>(), y2.data_ptr<float>(),
                       partial.data_ptr<double>(), nwg, (int)B, (int)P, stream_of(p1));
  return {y2, partial};
}

// ---------------------------------------------------------------- head forward (BN2 finalize + fc)
// returns (logits, stats2 [mean32|invstd32], aff2 [a32|b32])
std::tuple<Tensor, Tensor, Tensor> fused_head_forward(
    const Tensor& y2, const Tensor& partial2, const Tensor& b2, const c10::optional<Tensor>& gamma2,
    const c10::optional<Tensor>& beta2, const c10::optional<Tensor>& rm2, const c10::optional<Tensor>& rv2,
    const c10::optional<Tensor>& nbt2, double momentum, double eps, const Tensor& wfc, const c10::optional<Tensor>& bfc,
    const c10::optional<Tensor>& x_out, const c10::optional<Tensor>& ya_out) {
  TORCH_CHECK(y2.dim() == 4 && y2.size(3) == 32 && y2.size(1) == y2.size(2), "fused_head_forward: y2");
  const int64_t B = y2.size(0), P = y2.size(1), Q = P / 2;
  need(y2, at::kFloat, {B, P, P, 32}, "y2");
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
  TORCH_CHECK(wfc.dim() == 2 && wfc.size(1) == 32 * Q * Q && wfc.size(0) <= 10, "fc.weight must be [<=10, 32*Q*Q]");
  const int64_t NC = wfc.size(0);
  need(wfc, at::kFloat, {NC, 32 * Q * Q}, "fc.weight");
  const float* bf = optf(bfc, NC, "fc.bias");
  float* xo = nullptr;
  if (x_out.has_value() && x_out->defined()) {
    need(*x_out, at::kFloat, {B, 32 * Q * Q}, "x_out (fc input rows)");
    xo = x_out->data_ptr<float>();
  }
  float* yo = nullptr;
  if (ya_out.has_value() && ya_out->defined()) {
    need(*ya_out, at::kFloat, {B, 32 * Q * Q}, "ya_out (y2 at the pooling argmax)");
    yo = ya_out->data_ptr<float>();
  }
  c10::DeviceGuard guard(y2.device());
  hipStream_t st = stream_of(y2);
  auto sums2 = at::empty({64}, y2.options().dtype(at::kDouble));
  tds_reduce_partials(partial2.data_ptr<double>(), sums2.data_ptr<double>(), 64, nch, 2, (int64_t)nch * 2, 2, st);
  auto stats = at::empty({64}, y2.options());
  auto aff = at::empty({64}, y2.options());
  tds_bn_finalize_shifted(sums2.data_ptr<double>(), 32, 1, B * P * P, b2.data_ptr<float>(), (float)eps,
                          (float)momentum, g, be, stats.data_ptr<float>(), rm, rv, nb, aff.data_ptr<float>(), st);
  const int nblk = tds_head_fwd_nblk((int)Q);
  auto part = at::empty({(int64_t)nblk * B * NC}, y2.options().dtype(at::kDouble));
  auto lsum = at::empty({B * NC}, y2.options().dtype(at::kDouble));
  auto logits = at::empty({B, NC}, y2.options());
  const int rc = tds_head_fwd(y2.data_ptr<float>(), wfc.data_ptr<float>(), bf, aff.data_ptr<float>(),
                              part.data_ptr<double>(), lsum.data_ptr<double>(), logits.data_ptr<float>(), xo, yo, (int)B,
                              (int)P, (int)NC, st);
  TORCH_CHECK(rc == 0, "fused_head_forward: unsupported B/NC");
  return {logits, stats, aff};
}

// ---------------------------------------------------------------- head backward
struct HeadBwd {
  Tensor dW, dbfc, dgamma, dbeta, g2m, kbuf;
};

// fc / pool2 / ReLU / BN2 backward up to the pooled gradient g2m and the BN2 backward
// constants kbuf = [k1|k2|k3] (dy2 = k1*dz + k2*y2 + k3)
static HeadBwd head_backward_core(const Tensor& dlogits, const Tensor& y2, const Tensor& stats2, const Tensor& aff2,
                                  const c10::optional<Tensor>& gamma2, const Tensor& wfc,
                                  const c10::optional<Tensor>& dw_out, double scale, bool compute_dw,
                                  const c10::optional<Tensor>& ya = c10::nullopt, double update_lr = 0.0,
                                  const c10::optional<Tensor>& dbfc_out = c10::nullopt,
                                  const c10::optional<Tensor>& dg_out = c10::nullopt,
                                  const c10::optional<Tensor>& dbe_out = c10::nullopt) {
  const int64_t B = y2.size(0), P = y2.size(1), Q = P / 2;
  need(y2, at::kFloat, {B, P, P, 32}, "y2");
  const int64_t NC = wfc.size(0);
  need(wfc, at::kFloat, {NC, 32 * Q * Q}, "fc.weight");
  need(dlogits, at::kFloat, {B, NC}, "dlogits");
  need(stats2, at::kFloat, {64}, "stats2");
  need(aff2, at::kFloat, {64}, "aff2");
  const float* g = optf(gamma2, 32, "bn2.weight");
  hipStream_t st = stream_of(y2);
  HeadBwd r;
  if (!compute_dw) {
    r.dW = at::empty({0}, wfc.options());
  } else if (dw_out.has_value() && dw_out->defined()) {
    need(*dw_out, at::kFloat, {NC, 32 * Q * Q}, "dW_out");
    r.dW = *dw_out;
  } else {
    r.dW = at::empty_like(wfc);
  }
  r.g2m = at::empty({B, 32, Q, Q}, y2.options());  // planar (fc flatten order)
  const bool use_ya = ya.has_value() && ya->defined() && tds_head_bwd_ya_supported((int)B, (int)P, (int)NC);
  int nblk = use_ya ? tds_head_bwd_ya_nblk((int)B, (int)P, (int)NC) : tds_head_bwd_nblk((int)Q);
  auto partial = at::empty({(int64_t)32 * nblk * 2}, y2.options().dtype(at::kDouble));
  int rc;
  rc = -1;
  if (use_ya) {
    // saved argmax values: stream ya (B*32*Q*Q floats) instead of y2
    need(*ya, at::kFloat, {B, 32 * Q * Q}, "ya");
    // update_lr > 0: also apply SGD to wfc in place (optimizer step fused into the backward)
    rc = tds_head_bwd_ya(ya->data_ptr<float>(), wfc.data_ptr<float>(), aff2.data_ptr<float>(),
                         dlogits.data_ptr<float>(), compute_dw ? r.dW.data_ptr<float>() : nullptr,
                         r.g2m.data_ptr<float>(), partial.data_ptr<double>(), (int)B, (int)P, (int)NC, (float)scale,
                         (update_lr > 0.0 && compute_dw) ? const_cast<float*>(wfc.data_ptr<float>()) : nullptr,
                         (float)update_lr, st);
  }
  TORCH_CHECK(update_lr <= 0.0 || (use_ya && rc == 0 && compute_dw),
              "fused_head_backward_g2m: update_lr needs the saved-argmax (ya) path with compute_dw");
  if (rc != 0) {
    if (nblk != tds_head_bwd_nblk((int)Q)) {
      nblk = tds_head_bwd_nblk((int)Q);
      partial = at::empty({(int64_t)32 * nblk * 2}, y2.options().dtype(at::kDouble));
    }
    rc = tds_head_bwd(y2.data_ptr<float>(), wfc.data_ptr<float>(), aff2.data_ptr<float>(), dlogits.data_ptr<float>(),
                      compute_dw ? r.dW.data_ptr<float>() : nullptr, r.g2m.data_ptr<float>(),
                      partial.data_ptr<double>(), (int)B, (int)P, (int)NC, (float)scale, st);
  }
  TORCH_CHECK(rc == 0, "fused_head_backward: unsupported B/NC");
  auto sums = at::empty({64}, y2.options().dtype(at::kDouble));
  tds_reduce_partials(partial.data_ptr<double>(), sums.data_ptr<double>(), 64, nblk, 2, (int64_t)nblk * 2, 2, st);
  r.dgamma = sink_or_empty(dg_out, {32}, y2, "dgamma2_out");
  r.dbeta = sink_or_empty(dbe_out, {32}, y2, "dbeta2_out");
  r.kbuf = at::empty({96}, y2.options());
  tds_bn_bwd_finalize2(sums.data_ptr<double>(), 32, 1, B * P * P, g, stats2.data_ptr<float>(),
                       r.dgamma.data_ptr<float>(), r.dbeta.data_ptr<float>(), r.kbuf.data_ptr<float>(), st);
  r.dbfc = sink_or_empty(dbfc_out, {NC}, y2, "dbfc_out");
  at::sum_out(r.dbfc, dlogits, {0});
  if (scale != 1.0) r.dbfc.mul_(scale);
  return r;
}

// returns (dW [written into dw_out if given; empty when !compute_dw], db_fc, dgamma2, dbeta2, dy2 carrier)
std::tuple<Tensor, Tensor, Tensor, Tensor, Tensor> fused_head_backward(
    const Tensor& dlogits, const Tensor& y2, const Tensor& stats2, const Tensor& aff2,
    const c10::optional<Tensor>& gamma2, const Tensor& wfc, const c10::optional<Tensor>& dw_out, double scale,
    bool compute_dw) {
  c10::DeviceGuard guard(y2.device());
  HeadBwd r = head_backward_core(dlogits, y2, stats2, aff2, gamma2, wfc, dw_out, scale, compute_dw);
  const int64_t B = y2.size(0), P = y2.size(1);
  auto dy2 = at::empty({B, P, P, 32}, y2.options());  // carrier of bf16 [B,P,P,64]
  tds_dy2_build(y2.data_ptr<float>(), r.g2m.data_ptr<float>(), aff2.data_ptr<float>(), r.kbuf.data_ptr<float>(),
                dy2.data_ptr(), (int)B, (int)P, stream_of(y2));
  return {r.dW, r.dbfc, r.dgamma, r.dbeta, dy2};
}

// Head backward up to the pooled gradient: returns (dW, db_fc, dgamma2, dbeta2, g2m, kbuf).
// The conv2 backward then runs fused with the BN2/pool backward (fused_conv2_backward_y2),
// so dy2 is never materialised.
std::tuple<Tensor, Tensor, Tensor, Tensor, Tensor, Tensor> fused_head_backward_g2m(
    const Tensor& dlogits, const Tensor& y2, const Tensor& stats2, const Tensor& aff2,
    const c10::optional<Tensor>& gamma2, const Tensor& wfc, const c10::optional<Tensor>& dw_out, double scale,
    bool compute_dw, const c10::optional<Tensor>& ya, double update_lr, const c10::optional<Tensor>& dbfc_out,
    const c10::optional<Tensor>& dg_out, const c10::optional<Tensor>& dbe_out) {
  c10::DeviceGuard guard(y2.device());
  HeadBwd r = head_backward_core(dlogits, y2, stats2, aff2, gamma2, wfc, dw_out, scale, compute_dw, ya, update_lr,
                                 dbfc_out, dg_out, dbe_out);
  return {r.dW, r.dbfc, r.dgamma, r.dbeta, r.g2m, r.kbuf};
}

// ---------------------------------------------------------------- conv2 backward
std::tuple<Tensor, Tensor, Tensor> fused_conv2_backward(const Tensor& dy2, const Tensor& p1, const Tensor& wd,
                                                        bool need_dp1, double scale) {
  const int64_t B = p1.size(0), P = p1.size(1);
  need(p1, at::kFloat, {B, P, P, 16}, "p1");
  need(dy2, at::kFloat, {B, P, P, 32}, "dy2 carrier");
  need(wd, at::kShort, {2 * 25 * 4 * 16 * 8}, "conv2 dgrad pack");
  c10::DeviceGuard guard(p1.device());
  hipStream_t st = stream_of(p1);
  const int nwg = tds_conv2_num_wg();
  Tensor dp1 = need_dp1 ? at::empty({B, P, P, 16}, p1.options()) : at::empty({0}, p1.options());
  if (need_dp1) tds_conv2_dgrad_bf16x3(dy2.data_ptr(), wd.data_ptr<int16_t>(), dp1.data_ptr<float>(), nwg, (int)B,
                                       (int)P, st);
  auto slab = at::empty({(int64_t)nwg * 26 * 512}, p1.options());
  auto dw2 = at::empty({32, 16, 5, 5}, p1.options());
  auto db2 = at::empty({32}, p1.options());
  tds_conv2_wgrad_bf16x3(dy2.data_ptr(), p1.data_ptr(), slab.data_ptr<float>(), dw2.data_ptr<float>(),
                         db2.data_ptr<float>(), (float)scale, nwg, (int)B, (int)P, st);
  return {dp1, dw2, db2};
}

// BN2/ReLU/pool backward fused into conv2 dgrad + wgrad: (y2, g2m, aff2, kbuf, p1) -> (dp1, dw2, db2)
std::tuple<Tensor, Tensor, Tensor> fused_conv2_backward_y2(const Tensor& y2, const Tensor& g2m, const Tensor& aff2,
                                                           const Tensor& kbuf, const Tensor& p1, const Tensor& wd,
                                                           double scale, const c10::optional<Tensor>& dw_out,
                                                           const c10::optional<Tensor>& db_out) {
  const int64_t B = p1.size(0), P = p1.size(1), Q = P / 2;
  need(p1, at::kFloat, {B, P, P, 16}, "p1");
  need(y2, at::kFloat, {B, P, P, 32}, "y2");
  need(g2m, at::kFloat, {B, 32, Q, Q}, "g2m");
  need(aff2, at::kFloat, {64}, "aff2");
  need(kbuf, at::kFloat, {96}, "kbuf");
  need(wd, at::kShort, {2 * 25 * 4 * 16 * 8}, "conv2 dgrad pack");
  TORCH_CHECK(B <= 255 && P <= 32760, "fused_conv2_backward_y2: batch <= 255 and P <= 32760 (tile-order table packing)");
  c10::DeviceGuard guard(p1.device());
  hipStream_t st = stream_of(p1);
  const int nwg = tds_conv2_bwd_fused_num_wg();
  auto dp1 = at::empty({B, P, P, 16}, p1.options());
  auto slab = at::empty({(int64_t)nwg * 26 * 512}, p1.options());
  auto dw2 = sink_or_empty(dw_out, {32, 16, 5, 5}, p1, "dw2_out");
  auto db2 = sink_or_empty(db_out, {32}, p1, "db2_out");
  tds_conv2_bwd_fused(y2.data_ptr<float>(), g2m.data_ptr<float>(), aff2.data_ptr<float>(), kbuf.data_ptr<float>(),
                      p1.data_ptr(), wd.data_ptr<int16_t>(), dp1.data_ptr<float>(), slab.data_ptr<float>(),
                      dw2.data_ptr<float>(), db2.data_ptr<float>(), (float)scale, nwg, (int)B, (int)P, st);
  return {dp1, dw2, db2};
}

// ---------------------------------------------------------------- layer 1 backward
std::tuple<Tensor, Tensor, Tensor, Tensor> fused_l1_backward(const Tensor& dp1, const Tensor& x, const Tensor& p1,
                                                             const Tensor& idx1, const Tensor& w1, const Tensor& b1,
                                                             const c10::optional<Tensor>& gamma1, const Tensor& stats1,
                                                             const Tensor& gram, double scale,
                                                             const c10::optional<Tensor>& dw_out,
                                                             const c10::optional<Tensor>& db_out,
                                                             const c10::optional<Tensor>& dg_out,
                                                             const c10::optional<Tensor>& dbe_out) {
  TORCH_CHECK(x.dim() == 4 && x.size(1) == 1, "fused_l1_backward: x");
  const int64_t B = x.size(0), H = x.size(2), W = x.size(3), P = H / 2;
  need(x, at::kFloat, {B, 1, H, W}, "x");
  need(dp1, at::kFloat, {B, P, P, 16}, "dp1");
  need(p1, at::kFloat, {B, P, P, 16}, "p1");
  need(idx1, at::kByte, {B, P, P, 16}, "idx1");
  need(w1, at::kFloat, {16, 1, 5, 5}, "conv1.weight");
  need(b1, at::kFloat, {16}, "conv1.bias");
  need(stats1, at::kFloat, {32}, "stats1");
  need(gram, at::kDouble, {650}, "gram");
  const float* g = optf(gamma1, 16, "bn1.weight");
  c10::DeviceGuard guard(x.device());
  hipStream_t st = stream_of(x);
  const int nwg = tds_fused_num_wg(3), rows = tds_l1_bwd_rows(nwg);  // 3 workgroups fit a CU (156 VGPRs)
  auto partial = at::empty({(int64_t)rows * 16 * 27}, x.options().dtype(at::kDouble));
  tds_l1_bwd(x.data_ptr<float>(), dp1.data_ptr<float>(), p1.data_ptr(), idx1.data_ptr<uint8_t>(), w1.data_ptr<float>(),
             b1.data_ptr<float>(), partial.data_ptr<double>(), nwg, (int)B, (int)H, (int)W, st);
  auto bsum = at::empty({16 * 27}, x.options().dtype(at::kDouble));
  tds_reduce_partials(partial.data_ptr<double>(), bsum.data_ptr<double>(), 16 * 27, rows, 16 * 27, 0, 16 * 27, st);
  auto dw1 = sink_or_empty(dw_out, {16, 1, 5, 5}, x, "dw1_out");
  auto db1 = sink_or_empty(db_out, {16}, x, "db1_out");
  auto dg = sink_or_empty(dg_out, {16}, x, "dgamma1_out");
  auto dbe = sink_or_empty(dbe_out, {16}, x, "dbeta1_out");
  tds_l1_finalize(bsum.data_ptr<double>(), gram.data_ptr<double>(), B * H * W, w1.data_ptr<float>(),
                  b1.data_ptr<float>(), g, stats1.data_ptr<float>(), dw1.data_ptr<float>(), db1.data_ptr<float>(),
                  dg.data_ptr<float>(), dbe.data_ptr<float>(), (float)scale, st);
  return {dw1, db1, dg, dbe};
}

}  // namespace

TORCH_LIBRARY_FRAGMENT(tdsa, m) {
  m.def(
      "fused_l1_forward(Tensor x, Tensor w1, Tensor b1, Tensor? gamma1, Tensor? beta1, Tensor(a!)? rm1, "
      "Tensor(b!)? rv1, Tensor(c!)? nbt1, float momentum, float eps) -> (Tensor, Tensor, Tensor, Tensor)",
      &fused_l1_forward);
  m.def("conv2_pack(Tensor w2) -> (Tensor, Tensor)", &conv2_pack);
  m.def("fused_conv2_forward(Tensor p1, Tensor wp, Tensor b2) -> (Tensor, Tensor)", &fused_conv2_forward);
  m.def(
      "fused_head_forward(Tensor y2, Tensor partial2, Tensor b2, Tensor? gamma2, Tensor? beta2, Tensor(a!)? rm2, "
      "Tensor(b!)? rv2, Tensor(c!)? nbt2, float momentum, float eps, Tensor wfc, Tensor? bfc, Tensor(d!)? x_out=None, "
      "Tensor(e!)? ya_out=None) "
      "-> (Tensor, Tensor, Tensor)",
      &fused_head_forward);
  m.def(
      "fused_head_backward(Tensor dlogits, Tensor y2, Tensor stats2, Tensor aff2, Tensor? gamma2, Tensor wfc, "
      "Tensor(a!)? dw_out, float scale, bool compute_dw=True) -> (Tensor, Tensor, Tensor, Tensor, Tensor)",
      &fused_head_backward);
  m.def("fused_conv2_backward(Tensor dy2, Tensor p1, Tensor wd, bool need_dp1, float scale) -> (Tensor, Tensor, Tensor)",
        &fused_conv2_backward);
  m.def(
      "fused_head_backward_g2m(Tensor dlogits, Tensor y2, Tensor stats2, Tensor aff2, Tensor? gamma2, Tensor wfc, "
      "Tensor(a!)? dw_out, float scale, bool compute_dw=True, Tensor? ya=None, float update_lr=0.0, "
      "Tensor(b!)? dbfc_out=None, Tensor(c!)? dg_out=None, Tensor(d!)? dbe_out=None) -> "
      "(Tensor, Tensor, Tensor, Tensor, Tensor, Tensor)",
      &fused_head_backward_g2m);
  m.def(
      "fused_conv2_backward_y2(Tensor y2, Tensor g2m, Tensor aff2, Tensor kbuf, Tensor p1, Tensor wd, float scale, "
      "Tensor(a!)? dw_out=None, Tensor(b!)? db_out=None) -> (Tensor, Tensor, Tensor)",
      &fused_conv2_backward_y2);
  m.def(
      "fused_l1_backward(Tensor dp1, Tensor x, Tensor p1, Tensor idx1, Tensor w1, Tensor b1, Tensor? gamma1, "
      "Tensor stats1, Tensor gram, float scale, Tensor(a!)? dw_out=None, Tensor(b!)? db_out=None, "
      "Tensor(c!)? dg_out=None, Tensor(d!)? dbe_out=None) -> (Tensor, Tensor, Tensor, Tensor)",
      &fused_l1_backward);
}
