// Torch op registration for the gfx950 kernels (namespace torch.ops.tdsa).
//
// Every op checks device/dtype/contiguity/shape on the host before launching
// (a mis-shaped launch of a hand-written kernel can fault the whole GPU box),
// launches on the current HIP stream, and never synchronises, so the ops are
// safe to capture into hipGraphs.  Only "cuda" (= HIP on ROCm) tensors are
// accepted: CPU tensors are routed to reference implementations by the Python
// layer, never silently here.
#include <ATen/ATen.h>
#include <c10/core/DeviceGuard.h>
#include <c10/hip/HIPStream.h>
#include <torch/library.h>

#include <vector>

#include "kernels/launchers.h"
#include "launch_check.h"

namespace {

using at::Tensor;
using tds_bind::check_launches;

hipStream_t cur_stream(const Tensor& t) { return c10::hip::getCurrentHIPStream(t.device().index()).stream(); }

void check_f32_dev(const Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), "tdsa: ", name, " must be a GPU tensor (got ", t.device(), ")");
  TORCH_CHECK(t.scalar_type() == at::kFloat, "tdsa: ", name, " must be float32 (got ", t.scalar_type(), ")");
  TORCH_CHECK(t.is_contiguous(), "tdsa: ", name, " must be contiguous");
}

void check_opt(const c10::optional<Tensor>& t, const char* name, int64_t numel) {
  if (t.has_value() && t->defined()) {
    check_f32_dev(*t, name);
    TORCH_CHECK(t->numel() == numel, "tdsa: ", name, " has ", t->numel(), " elements, expected ", numel);
  }
}

const float* opt_ptr(const c10::optional<Tensor>& t) {
  return (t.has_value() && t->defined()) ? t->data_ptr<float>() : nullptr;
}
float* opt_mut_ptr(const c10::optional<Tensor>& t) {
  return (t.has_value() && t->defined()) ? t->data_ptr<float>() : nullptr;
}

// ------------------------------------------------------------------ elementwise
Tensor relu_fwd(const Tensor& x) {
  check_f32_dev(x, "x");
  c10::DeviceGuard g(x.device());
  auto y = at::empty_like(x);
  tds_relu_fwd(x.data_ptr<float>(), y.data_ptr<float>(), x.numel(), cur_stream(x));
  check_launches("relu_fwd");
  return y;
}

Tensor relu_bwd(const Tensor& grad, const Tensor& out) {
  check_f32_dev(grad, "grad");
  check_f32_dev(out, "out");
  TORCH_CHECK(grad.sizes() == out.sizes(), "tdsa.relu_bwd: shape mismatch");
  c10::DeviceGuard g(grad.device());
  auto dx = at::empty_like(grad);
  tds_relu_bwd(grad.data_ptr<float>(), out.data_ptr<float>(), dx.data_ptr<float>(), grad.numel(), cur_stream(grad));
  check_launches("relu_bwd");
  return dx;
}

std::tuple<Tensor, Tensor> maxpool2_fwd(const Tensor& x) {
  check_f32_dev(x, "x");
  TORCH_CHECK(x.dim() == 4, "tdsa.maxpool2_fwd: expected NCHW");
  c10::DeviceGuard g(x.device());
  const int64_t B = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  auto y = at::empty({B, C, H / 2, W / 2}, x.options());
  auto idx = at::empty({B, C, H / 2, W / 2}, x.options().dtype(at::kByte));
  tds_maxpool2_fwd(x.data_ptr<float>(), y.data_ptr<float>(), idx.data_ptr<uint8_t>(), B * C, (int)H, (int)W,
                   cur_stream(x));
  check_launches("maxpool2_fwd");
  return {y, idx};
}

Tensor maxpool2_bwd(const Tensor& gy, const Tensor& idx, int64_t H, int64_t W) {
  check_f32_dev(gy, "grad");
  TORCH_CHECK(idx.is_cuda() && idx.scalar_type() == at::kByte && idx.is_contiguous(), "tdsa.maxpool2_bwd: bad idx");
  TORCH_CHECK(gy.dim() == 4 && gy.sizes() == idx.sizes() && gy.size(2) == H / 2 && gy.size(3) == W / 2,
              "tdsa.maxpool2_bwd: shape mismatch");
  c10::DeviceGuard g(gy.device());
  auto gx = at::empty({gy.size(0), gy.size(1), H, W}, gy.options());
  tds_maxpool2_bwd(gy.data_ptr<float>(), idx.data_ptr<uint8_t>(), gx.data_ptr<float>(), gy.size(0) * gy.size(1),
                   (int)H, (int)W, cur_stream(gy));
  check_launches("maxpool2_bwd");
  return gx;
}

// levels=True: the rounded uint8 levels (ToTensor's input) instead of level / 255 in fp32
Tensor upsample_bilinear_u8(const Tensor& src, int64_t H, int64_t W, bool levels) {
  TORCH_CHECK(src.is_cuda() && src.scalar_type() == at::kByte && src.is_contiguous() && src.dim() == 3,
              "tdsa.upsample_bilinear_u8: expected contiguous uint8 [B,h,w] on GPU");
  TORCH_CHECK(src.size(1) >= 1 && src.size(2) >= 1 && src.size(2) <= 256 && src.size(0) <= 65535 && H >= 1 &&
                  W >= 1 && H <= INT32_MAX && W <= INT32_MAX,
              "tdsa.upsample_bilinear_u8: source width must be 1..256 and batch <= 65535");
  c10::DeviceGuard g(src.device());
  auto dst = at::empty({src.size(0), 1, H, W}, src.options().dtype(levels ? at::kByte : at::kFloat));
  tds_upsample_bilinear_u8(src.data_ptr<uint8_t>(), dst.data_ptr(), levels, (int)src.size(0), (int)src.size(1),
                           (int)src.size(2), (int)H, (int)W, cur_stream(src));
  check_launches("upsample_bilinear_u8");
  return dst;
}

// The uint8 level upsample fused with the x autocorrelation partials behind BN1's statistics
// (ups_moments.hip): returns (levels [B,1,H,W] uint8, partials [rows * 42] fp64) for
// fused_l1_forward's precomputed-moments argument.  Shapes the fused kernel does not take (W % 4,
// sources past 4096 pixels) get the plain upsample and an empty partials tensor.
std::tuple<Tensor, Tensor> upsample_levels_moments(const Tensor& src, int64_t H, int64_t W) {
  TORCH_CHECK(src.is_cuda() && src.scalar_type() == at::kByte && src.is_contiguous() && src.dim() == 3,
              "tdsa.upsample_levels_moments: expected contiguous uint8 [B,h,w] on GPU");
  TORCH_CHECK(H >= 1 && W >= 1 && H <= INT32_MAX && W <= INT32_MAX && src.size(0) <= 65535,
              "tdsa.upsample_levels_moments: bad output shape");
  c10::DeviceGuard g(src.device());
  const int B = (int)src.size(0), h = (int)src.size(1), w = (int)src.size(2);
  const int rows = tds_ups_moments_rows(B, h, w, (int)H, (int)W);
  if (rows == 0 || (int64_t)H * W > 0xFFFFFFF0LL)
    return {upsample_bilinear_u8(src, H, W, true), at::empty({0}, src.options().dtype(at::kDouble))};
  auto dst = at::empty({B, 1, H, W}, src.options());
  auto part = at::empty({(int64_t)rows * 42}, src.options().dtype(at::kDouble));
  tds_ups_moments_u8(src.data_ptr<uint8_t>(), dst.data_ptr<uint8_t>(), part.data_ptr<double>(), rows, B, h, w, (int)H,
                     (int)W, cur_stream(src));
  check_launches("upsample_levels_moments");
  return {dst, part};
}

void sgd_step_(at::TensorList params, at::TensorList grads, at::TensorList moms, double lr, double wd,
               double momentum, double dampening, bool nesterov, bool first_step) {
  TORCH_CHECK(params.size() == grads.size(), "tdsa.sgd_step_: params/grads length mismatch");
  TORCH_CHECK(momentum == 0.0 || moms.size() == params.size(), "tdsa.sgd_step_: momentum buffers missing");
  if (params.empty()) return;
  c10::DeviceGuard g(params[0].device());
  hipStream_t st = cur_stream(params[0]);
  size_t i = 0;
  while (i < params.size()) {
    SgdChunkTable tab;
    tab.n = 0;
    int64_t maxn = 0;
    for (; i < params.size() && tab.n < TDS_SGD_MAX_TENSORS; ++i) {
      check_f32_dev(params[i], "param");
      check_f32_dev(grads[i], "grad");
      TORCH_CHECK(params[i].numel() == grads[i].numel(), "tdsa.sgd_step_: param/grad numel mismatch");
      tab.param[tab.n] = params[i].data_ptr<float>();
      tab.grad[tab.n] = grads[i].data_ptr<float>();
      tab.mom[tab.n] = momentum != 0.0 ? moms[i].data_ptr<float>() : nullptr;
      tab.numel[tab.n] = params[i].numel();
      maxn = std::max(maxn, params[i].numel());
      tab.n++;
    }
    tds_sgd_multi(tab, (float)lr, (float)wd, (float)momentum, (float)dampening, nesterov ? 1 : 0, first_step ? 1 : 0,
                  maxn, st);
  }
  check_launches("sgd_step_");
}

std::tuple<Tensor, Tensor> cross_entropy(const Tensor& logits, const Tensor& labels, int64_t ignore_index,
                                         double label_smoothing) {
  check_f32_dev(logits, "logits");
  TORCH_CHECK(logits.dim() == 2, "tdsa.cross_entropy: logits must be [M,N]");
  TORCH_CHECK(labels.is_cuda() && labels.scalar_type() == at::kLong && labels.is_contiguous() &&
                  labels.numel() == logits.size(0),
              "tdsa.cross_entropy: labels must be int64 [M] on GPU");
  c10::DeviceGuard g(logits.device());
  const int M = (int)logits.size(0), N = (int)logits.size(1);
  auto row_loss = at::empty({M}, logits.options());
  auto dlogits = at::empty_like(logits);
  auto loss = at::empty({}, logits.options());
  auto inv = at::empty({1}, logits.options());
  tds_cross_entropy(logits.data_ptr<float>(), labels.data_ptr<int64_t>(), row_loss.data_ptr<float>(),
                    dlogits.data_ptr<float>(), loss.data_ptr<float>(), inv.data_ptr<float>(), M, N, ignore_index,
                    (float)label_smoothing, cur_stream(logits));
  check_launches("cross_entropy");
  return {loss, dlogits};
}

Tensor scale_by_scalar(const Tensor& x, const Tensor& s) {
  check_f32_dev(x, "x");
  check_f32_dev(s, "scalar");
  TORCH_CHECK(s.numel() == 1, "tdsa.scale_by_scalar: scalar must have one element");
  c10::DeviceGuard g(x.device());
  auto y = at::empty_like(x);
  tds_scale_by_device_scalar(x.data_ptr<float>(), s.data_ptr<float>(), y.data_ptr<float>(), x.numel(), cur_stream(x));
  check_launches("scale_by_scalar");
  return y;
}

// ------------------------------------------------------------------ conv (generic NCHW)
void check_conv(const Tensor& x, const Tensor& w, int64_t pad) {
  check_f32_dev(x, "input");
  check_f32_dev(w, "weight");
  TORCH_CHECK(x.dim() == 4 && w.dim() == 4, "tdsa.conv2d: expected 4-D input and weight");
  TORCH_CHECK(w.size(1) == x.size(1), "tdsa.conv2d: channel mismatch");
  TORCH_CHECK(w.size(2) == w.size(3), "tdsa.conv2d: square kernels only");
  const int64_t ks = w.size(2);
  TORCH_CHECK(ks == 1 || ks == 3 || ks == 5, "tdsa.conv2d: kernel size must be 1, 3 or 5");
  TORCH_CHECK(2 * pad == ks - 1, "tdsa.conv2d: only 'same' padding (pad = (k-1)/2) is supported");
  TORCH_CHECK(x.size(1) <= 64, "tdsa.conv2d: Cin <= 64");
}

Tensor conv2d_fwd(const Tensor& x, const Tensor& w, const c10::optional<Tensor>& bias, int64_t pad) {
  check_conv(x, w, pad);
  check_opt(bias, "bias", w.size(0));
  c10::DeviceGuard g(x.device());
  const int B = (int)x.size(0), Cin = (int)x.size(1), H = (int)x.size(2), W = (int)x.size(3);
  const int Cout = (int)w.size(0), KS = (int)w.size(2);
  auto out = at::empty({B, Cout, H, W}, x.options());
  const int rc = tds_conv2d_fwd_f32(x.data_ptr<float>(), w.data_ptr<float>(), opt_ptr(bias), out.data_ptr<float>(), B,
                                    Cin, Cout, H, W, KS, (int)pad, cur_stream(x));
  TORCH_CHECK(rc == 0, "tdsa.conv2d_fwd: unsupported configuration (rc=", rc, ")");
  check_launches("conv2d_fwd");
  return out;
}

Tensor conv2d_dgrad(const Tensor& gy, const Tensor& w, int64_t pad) {
  check_f32_dev(gy, "grad_output");
  check_f32_dev(w, "weight");
  TORCH_CHECK(gy.dim() == 4 && w.dim() == 4 && gy.size(1) == w.size(0), "tdsa.conv2d_dgrad: shape mismatch");
  const int64_t ks = w.size(2);
  TORCH_CHECK(w.size(2) == w.size(3) && (ks == 1 || ks == 3 || ks == 5) && 2 * pad == ks - 1,
              "tdsa.conv2d_dgrad: unsupported kernel/padding");
  TORCH_CHECK(gy.size(1) <= 64, "tdsa.conv2d_dgrad: Cout <= 64");
  c10::DeviceGuard g(gy.device());
  const int Cout = (int)w.size(0), Cin = (int)w.size(1), KS = (int)ks;
  auto wt = at::empty({Cin, Cout, KS, KS}, w.options());
  hipStream_t st = cur_stream(gy);
  tds_conv2d_flip_weights(w.data_ptr<float>(), wt.data_ptr<float>(), Cout, Cin, KS, st);
  const int B = (int)gy.size(0), H = (int)gy.size(2), W = (int)gy.size(3);
  auto dx = at::empty({B, Cin, H, W}, gy.options());
  const int rc = tds_conv2d_fwd_f32(gy.data_ptr<float>(), wt.data_ptr<float>(), nullptr, dx.data_ptr<float>(), B, Cout,
                                    Cin, H, W, KS, (int)(KS - 1 - pad), st);
  TORCH_CHECK(rc == 0, "tdsa.conv2d_dgrad: unsupported configuration (rc=", rc, ")");
  check_launches("conv2d_dgrad");
  return dx;
}

std::tuple<Tensor, Tensor> conv2d_wgrad(const Tensor& x, const Tensor& gy, int64_t ks, int64_t pad, bool need_bias) {
  check_f32_dev(x, "input");
  check_f32_dev(gy, "grad_output");
  TORCH_CHECK(x.dim() == 4 && gy.dim() == 4 && x.size(0) == gy.size(0) && x.size(2) == gy.size(2) &&
                  x.size(3) == gy.size(3),
              "tdsa.conv2d_wgrad: shape mismatch");
  TORCH_CHECK((ks == 1 || ks == 3 || ks == 5) && 2 * pad == ks - 1, "tdsa.conv2d_wgrad: unsupported kernel/padding");
  TORCH_CHECK(x.size(1) <= 32, "tdsa.conv2d_wgrad: Cin <= 32");
  c10::DeviceGuard g(x.device());
  const int B = (int)x.size(0), Cin = (int)x.size(1), H = (int)x.size(2), W = (int)x.size(3);
  const int Cout = (int)gy.size(1);
  auto dw = at::empty({Cout, Cin, ks, ks}, x.options());
  auto db = at::empty({need_bias ? Cout : 0}, x.options());
  const int num_wg = 512;
  const int64_t slab_floats = tds_conv2d_wgrad_f32(nullptr, nullptr, nullptr, nullptr, nullptr, B, Cin, Cout, H, W,
                                                   (int)ks, (int)pad, 1.f, 0, num_wg, nullptr);
  TORCH_CHECK(slab_floats > 0, "tdsa.conv2d_wgrad: unsupported configuration");
  auto slab = at::empty({slab_floats}, x.options());
  const int64_t rc = tds_conv2d_wgrad_f32(x.data_ptr<float>(), gy.data_ptr<float>(), dw.data_ptr<float>(),
                                          need_bias ? db.data_ptr<float>() : nullptr, slab.data_ptr<float>(), B, Cin,
                                          Cout, H, W, (int)ks, (int)pad, 1.f, 0, num_wg, cur_stream(x));
  TORCH_CHECK(rc == 0, "tdsa.conv2d_wgrad: launch failed (rc=", rc, ")");
  check_launches("conv2d_wgrad");
  return {dw, db};
}

// ------------------------------------------------------------------ batchnorm (NCHW)
std::tuple<Tensor, Tensor, Tensor> bn_fwd_train(const Tensor& x, const c10::optional<Tensor>& gamma,
                                                const c10::optional<Tensor>& beta,
                                                const c10::optional<Tensor>& running_mean,
                                                const c10::optional<Tensor>& running_var,
                                                const c10::optional<Tensor>& num_batches, double momentum, double eps,
                                                bool relu) {
  check_f32_dev(x, "input");
  TORCH_CHECK(x.dim() == 4, "tdsa.bn_fwd_train: expected NCHW");
  const int B = (int)x.size(0), C = (int)x.size(1);
  const int64_t HW = x.size(2) * x.size(3);
  TORCH_CHECK((int64_t)B * HW > 0, "tdsa.bn_fwd_train: empty input");
  check_opt(gamma, "weight", C);
  check_opt(beta, "bias", C);
  check_opt(running_mean, "running_mean", C);
  check_opt(running_var, "running_var", C);
  const bool has_nb = num_batches.has_value() && num_batches->defined();
  if (has_nb)
    TORCH_CHECK(num_batches->is_cuda() && num_batches->scalar_type() == at::kLong && num_batches->numel() == 1,
                "tdsa.bn_fwd_train: num_batches_tracked must be an int64 scalar on GPU");
  c10::DeviceGuard g(x.device());
  hipStream_t st = cur_stream(x);
  auto mean = at::empty({C}, x.options());
  auto invstd = at::empty({C}, x.options());
  auto aff = at::empty({2 * C}, x.options());
  const int nchunk = tds_bn_num_chunks(B, C, HW);
  auto partial = at::empty({(int64_t)C * nchunk * 2}, x.options().dtype(at::kDouble));
  tds_bn_fwd_train(x.data_ptr<float>(), B, C, HW, (float)eps, (float)momentum, opt_ptr(gamma), opt_ptr(beta),
                   mean.data_ptr<float>(), invstd.data_ptr<float>(), opt_mut_ptr(running_mean),
                   opt_mut_ptr(running_var), has_nb ? num_batches->data_ptr<int64_t>() : nullptr,
                   aff.data_ptr<float>(), aff.data_ptr<float>() + C, partial.data_ptr<double>(), nchunk, st);
  auto y = at::empty_like(x);
  tds_bn_apply(x.data_ptr<float>(), aff.data_ptr<float>(), aff.data_ptr<float>() + C, y.data_ptr<float>(), B, C, HW,
               relu ? 1 : 0, st);
  check_launches("bn_fwd_train");
  return {y, mean, invstd};
}

Tensor bn_fwd_eval(const Tensor& x, const c10::optional<Tensor>& gamma, const c10::optional<Tensor>& beta,
                   const Tensor& running_mean, const Tensor& running_var, double eps, bool relu) {
  check_f32_dev(x, "input");
  TORCH_CHECK(x.dim() == 4, "tdsa.bn_fwd_eval: expected NCHW");
  const int B = (int)x.size(0), C = (int)x.size(1);
  const int64_t HW = x.size(2) * x.size(3);
  check_opt(gamma, "weight", C);
  check_opt(beta, "bias", C);
  check_f32_dev(running_mean, "running_mean");
  check_f32_dev(running_var, "running_var");
  c10::DeviceGuard g(x.device());
  hipStream_t st = cur_stream(x);
  auto aff = at::empty({2 * C}, x.options());
  tds_bn_eval_affine(running_mean.data_ptr<float>(), running_var.data_ptr<float>(), C, (float)eps, opt_ptr(gamma),
                     opt_ptr(beta), aff.data_ptr<float>(), aff.data_ptr<float>() + C, st);
  auto y = at::empty_like(x);
  tds_bn_apply(x.data_ptr<float>(), aff.data_ptr<float>(), aff.data_ptr<float>() + C, y.data_ptr<float>(), B, C, HW,
               relu ? 1 : 0, st);
  check_launches("bn_fwd_eval");
  return y;
}

std::tuple<Tensor, Tensor, Tensor> bn_bwd(const Tensor& dy, const Tensor& x, const c10::optional<Tensor>& gamma,
                                          const Tensor& mean, const Tensor& invstd, bool need_dx) {
  check_f32_dev(dy, "grad_output");
  check_f32_dev(x, "input");
  TORCH_CHECK(dy.sizes() == x.sizes() && x.dim() == 4, "tdsa.bn_bwd: shape mismatch");
  const int B = (int)x.size(0), C = (int)x.size(1);
  const int64_t HW = x.size(2) * x.size(3);
  check_opt(gamma, "weight", C);
  check_f32_dev(mean, "save_mean");
  check_f32_dev(invstd, "save_invstd");
  c10::DeviceGuard g(x.device());
  hipStream_t st = cur_stream(x);
  const int nchunk = tds_bn_num_chunks(B, C, HW);
  auto partial = at::empty({(int64_t)C * nchunk * 2}, x.options().dtype(at::kDouble));
  auto kbuf = at::empty({3 * C}, x.options());
  auto dgamma = at::empty({C}, x.options());
  auto dbeta = at::empty({C}, x.options());
  Tensor dx = need_dx ? at::empty_like(x) : at::empty({0}, x.options());
  tds_bn_bwd(dy.data_ptr<float>(), x.data_ptr<float>(), B, C, HW, opt_ptr(gamma), mean.data_ptr<float>(),
             invstd.data_ptr<float>(), need_dx ? dx.data_ptr<float>() : nullptr, dgamma.data_ptr<float>(),
             dbeta.data_ptr<float>(), kbuf.data_ptr<float>(), partial.data_ptr<double>(), nchunk, st);
  check_launches("bn_bwd");
  return {dx, dgamma, dbeta};
}

// ------------------------------------------------------------------ linear (skinny)
Tensor linear_fwd(const Tensor& x, const Tensor& w, const c10::optional<Tensor>& b) {
  check_f32_dev(x, "input");
  check_f32_dev(w, "weight");
  TORCH_CHECK(x.dim() == 2 && w.dim() == 2 && x.size(1) == w.size(1), "tdsa.linear_fwd: shape mismatch");
  TORCH_CHECK(x.size(0) <= 8 && w.size(0) <= 16, "tdsa.linear_fwd: skinny kernel needs M<=8, N<=16");
  check_opt(b, "bias", w.size(0));
  c10::DeviceGuard g(x.device());
  const int M = (int)x.size(0), N = (int)w.size(0);
  const int64_t K = x.size(1);
  auto out = at::empty({M, N}, x.options());
  const int nblk = tds_linear_fwd_nblk(K);
  auto partial = at::empty({(int64_t)nblk * M * N}, x.options());
  const int rc = tds_linear_fwd_skinny(x.data_ptr<float>(), w.data_ptr<float>(), opt_ptr(b), out.data_ptr<float>(),
                                       partial.data_ptr<float>(), M, N, K, nblk, cur_stream(x));
  TORCH_CHECK(rc == 0, "tdsa.linear_fwd: unsupported shape");
  check_launches("linear_fwd");
  return out;
}

// Writes dW/db into caller-provided buffers (e.g. views of a DDP bucket) with
// an optional scale (1/world for pre-averaged buckets) and accumulate flag.
Tensor linear_bwd_into(const Tensor& dy, const Tensor& x, const Tensor& w, const c10::optional<Tensor>& dw_out,
                       const c10::optional<Tensor>& db_out, double scale, bool accumulate, bool need_dx) {
  check_f32_dev(dy, "grad_output");
  check_f32_dev(x, "input");
  check_f32_dev(w, "weight");
  TORCH_CHECK(dy.dim() == 2 && x.dim() == 2 && w.dim() == 2 && dy.size(0) == x.size(0) && dy.size(1) == w.size(0) &&
                  x.size(1) == w.size(1),
              "tdsa.linear_bwd_into: shape mismatch");
  TORCH_CHECK(x.size(0) <= 8 && w.size(0) <= 16, "tdsa.linear_bwd_into: skinny kernel needs M<=8, N<=16");
  check_opt(dw_out, "dW", w.numel());
  check_opt(db_out, "db", w.size(0));
  c10::DeviceGuard g(x.device());
  const int M = (int)x.size(0), N = (int)w.size(0);
  const int64_t K = x.size(1);
  Tensor dx = need_dx ? at::empty_like(x) : at::empty({0}, x.options());
  const int rc = tds_linear_bwd_skinny(dy.data_ptr<float>(), x.data_ptr<float>(), w.data_ptr<float>(),
                                       need_dx ? dx.data_ptr<float>() : nullptr, opt_mut_ptr(dw_out),
                                       opt_mut_ptr(db_out), M, N, K, (float)scale, accumulate ? 1 : 0, cur_stream(x));
  TORCH_CHECK(rc == 0, "tdsa.linear_bwd_into: unsupported shape");
  check_launches("linear_bwd_into");
  return dx;
}

// dW (= or +=) scale * dy^T x, db (= or +=) scale * sum_rows dy   (dy [M,N], x [M,K], N <= 16).
// dW may be a column slice of a wider row-major matrix (unit column stride, any row stride):
// the sharded fc exchange writes its shard straight into the full gradient.  More than 64
// rows run as 64-row passes that accumulate.
// update_lr != 0: UPDATE-ONLY -- dw is the weight itself (or a column slice of it) and receives
// the plain SGD step dw -= update_lr * (scale * dy^T x) with no gradient materialised (the fc
// exchange's optimizer-in-backward, parallel/factored.py); db is still written as a gradient.
void linear_dw(const Tensor& dy, const Tensor& x, const Tensor& dw, const c10::optional<Tensor>& db, double scale,
               bool accumulate, double update_lr) {
  check_f32_dev(dy, "grad_output");
  check_f32_dev(x, "input");
  TORCH_CHECK(dw.is_cuda() && dw.scalar_type() == at::kFloat, "tdsa.linear_dw: dW must be a float32 GPU tensor");
  TORCH_CHECK(dy.dim() == 2 && x.dim() == 2 && dw.dim() == 2 && dy.size(0) == x.size(0) && dw.size(0) == dy.size(1) &&
                  dw.size(1) == x.size(1),
              "tdsa.linear_dw: shape mismatch");
  TORCH_CHECK(dw.stride(1) == 1 && dw.stride(0) >= dw.size(1), "tdsa.linear_dw: dW rows must be unit-stride");
  TORCH_CHECK(dy.size(1) <= 16 && dy.size(0) >= 1, "tdsa.linear_dw: needs 1 <= rows and outputs <= 16");
  check_opt(db, "db", dw.size(0));
  c10::DeviceGuard g(x.device());
  const int64_t M = dy.size(0), N = dy.size(1), K = x.size(1);
  for (int64_t m0 = 0; m0 < M; m0 += 64) {
    const int64_t mc = std::min<int64_t>(64, M - m0);
    const int rc = tds_linear_dw(dy.data_ptr<float>() + m0 * N, x.data_ptr<float>() + m0 * K, dw.data_ptr<float>(),
                                 opt_mut_ptr(db), (int)mc, (int)N, K, dw.stride(0), (float)scale,
                                 (accumulate || m0 > 0) ? 1 : 0, (float)update_lr, cur_stream(x));
    TORCH_CHECK(rc == 0, "tdsa.linear_dw: bad launch shape");
  }
  check_launches("linear_dw");
}

}  // namespace

TORCH_LIBRARY(tdsa, m) {
  m.def("relu_fwd(Tensor x) -> Tensor", &relu_fwd);
  m.def("relu_bwd(Tensor grad, Tensor out) -> Tensor", &relu_bwd);
  m.def("maxpool2_fwd(Tensor x) -> (Tensor, Tensor)", &maxpool2_fwd);
  m.def("maxpool2_bwd(Tensor grad, Tensor idx, int H, int W) -> Tensor", &maxpool2_bwd);
  m.def("upsample_bilinear_u8(Tensor src, int H, int W, bool levels=False) -> Tensor", &upsample_bilinear_u8);
  m.def("upsample_levels_moments(Tensor src, int H, int W) -> (Tensor, Tensor)", &upsample_levels_moments);
  m.def(
      "sgd_step_(Tensor(a!)[] params, Tensor[] grads, Tensor(b!)[] moms, float lr, float weight_decay, float momentum, "
      "float dampening, bool nesterov, bool first_step) -> ()",
      &sgd_step_);
  m.def("cross_entropy(Tensor logits, Tensor labels, int ignore_index, float label_smoothing) -> (Tensor, Tensor)",
        &cross_entropy);
  m.def("scale_by_scalar(Tensor x, Tensor s) -> Tensor", &scale_by_scalar);
  m.def("conv2d_fwd(Tensor x, Tensor w, Tensor? b, int pad) -> Tensor", &conv2d_fwd);
  m.def("conv2d_dgrad(Tensor grad, Tensor w, int pad) -> Tensor", &conv2d_dgrad);
  m.def("conv2d_wgrad(Tensor x, Tensor grad, int ks, int pad, bool need_bias) -> (Tensor, Tensor)", &conv2d_wgrad);
  m.def(
      "bn_fwd_train(Tensor x, Tensor? gamma, Tensor? beta, Tensor(a!)? running_mean, Tensor(b!)? running_var, "
      "Tensor(c!)? num_batches, float momentum, float eps, bool relu) -> (Tensor, Tensor, Tensor)",
      &bn_fwd_train);
  m.def("bn_fwd_eval(Tensor x, Tensor? gamma, Tensor? beta, Tensor running_mean, Tensor running_var, float eps, "
        "bool relu) -> Tensor",
        &bn_fwd_eval);
  m.def("bn_bwd(Tensor dy, Tensor x, Tensor? gamma, Tensor mean, Tensor invstd, bool need_dx) -> (Tensor, Tensor, "
        "Tensor)",
        &bn_bwd);
  m.def("linear_fwd(Tensor x, Tensor w, Tensor? b) -> Tensor", &linear_fwd);
  m.def(
      "linear_bwd_into(Tensor dy, Tensor x, Tensor w, Tensor(a!)? dw_out, Tensor(b!)? db_out, float scale, "
      "bool accumulate, bool need_dx) -> Tensor",
      &linear_bwd_into);
  m.def("linear_dw(Tensor dy, Tensor x, Tensor(a!) dw, Tensor(b!)? db, float scale, bool accumulate, "
        "float update_lr=0.0) -> ()",
        &linear_dw);
}
