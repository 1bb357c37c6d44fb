// PyTorch operators over the C ABI (liblievae_torch.so, loaded with torch.ops.load_library):
// the fused metric op z = mu·exp(v) -> ZYZ -> block D(z)·F (reparameterize.py:269-273,
// vae.py:182, decoders.py:47-56) as a C++ autograd function, so the eager training
// direction runs forward, backward and the autograd bookkeeping without Python frames or
// ctypes argument conversion (the Python autograd.Function path, lie_vae/_ops.py, cost
// ~100 us of host time per forward + backward at config 2 against ~34 us of kernels).
// Host code only: the kernels are the library's (include/lievae.h); this file adds no
// device code and no fallback.
#include <torch/all.h>
#include <torch/library.h>

#include <c10/hip/HIPGraphsC10Utils.h>
#include <c10/hip/HIPStream.h>

#include <c10/core/DeviceGuard.h>

#include <map>
#include <mutex>
#include <utility>

#include "../../include/lievae.h"

namespace {

using at::Tensor;
using torch::autograd::AutogradContext;
using torch::autograd::variable_list;

void check(int rc, const char* what) {
  TORCH_CHECK(rc == LV_OK, what, " failed (", rc, "): ", lv_last_error());
}

void* stream_of(const Tensor& t) {
  return c10::hip::getCurrentHIPStream(t.device().index()).stream();
}

// The backward's workspace, reused per (device, stream) for eager calls (stream order
// serialises its users) -- the same policy as lie_vae/_ops.py; under graph capture a fresh
// allocation from the capture's pool.
Tensor workspace(int64_t n, int64_t L, int64_t C, const Tensor& like, void* stream, size_t& bytes) {
  bytes = lv_group_action_bwd_workspace(n, (int)L, (int)C, 1);
  const int64_t nb = std::max<int64_t>((int64_t)bytes, 1);
  auto opts = like.options().dtype(torch::kUInt8);
  if (c10::hip::currentStreamCaptureStatusMayInitCtx() != c10::hip::CaptureStatus::None)
    return torch::empty({nb}, opts);
  // keyed by (device, stream): the default stream's handle is the same on every device
  static std::mutex mu;
  static std::map<std::pair<int, void*>, Tensor> cache;
  std::lock_guard<std::mutex> lock(mu);
  Tensor& buf = cache[{(int)like.device().index(), stream}];
  if (!buf.defined() || buf.numel() < nb)
    buf = torch::empty({std::max<int64_t>(nb, 1 << 20)}, opts);
  return buf;
}

struct FusedExpAction : public torch::autograd::Function<FusedExpAction> {
  static Tensor forward(AutogradContext* ctx, const std::optional<Tensor>& mu, const Tensor& v,
                        const Tensor& spec, int64_t L, bool transpose, bool out_bf16) {
    // every input on ONE HIP device: the kernels take raw device pointers, so a CPU tensor
    // or a tensor of another GPU must be refused here, before any launch
    TORCH_CHECK(v.is_cuda() && spec.is_cuda() && (!mu.has_value() || !mu->defined() || mu->is_cuda()),
                "lievae::fused_exp_action: device tensors only (no CPU fallback)");
    TORCH_CHECK(spec.device() == v.device() && (!mu.has_value() || !mu->defined() || mu->device() == v.device()),
                "lievae::fused_exp_action: mu, v and spectrum must be on one device (got v on ", v.device(),
                ", spectrum on ", spec.device(), mu.has_value() && mu->defined() ? ", mu on " : "",
                mu.has_value() && mu->defined() ? mu->device().str() : std::string(), ")");
    const c10::DeviceGuard guard(v.device());
    TORCH_CHECK(v.dim() == 2 && v.size(1) == 3, "v must be (n,3)");
    TORCH_CHECK(spec.dim() == 2 && spec.size(0) == (L + 1) * (L + 1), "spectrum must be ((L+1)^2, C)");
    const Tensor vc = v.scalar_type() == torch::kFloat32 && v.is_contiguous() ? v : v.to(torch::kFloat32).contiguous();
    const Tensor fc = spec.scalar_type() == torch::kFloat32 && spec.is_contiguous()
                          ? spec
                          : spec.to(torch::kFloat32).contiguous();
    Tensor muc;
    if (mu.has_value() && mu->defined()) {
      TORCH_CHECK(mu->dim() == 3 && mu->size(0) == v.size(0) && mu->size(1) == 3 && mu->size(2) == 3,
                  "mu must be (n,3,3)");
      muc = mu->scalar_type() == torch::kFloat32 && mu->is_contiguous() ? *mu : mu->to(torch::kFloat32).contiguous();
    }
    const int64_t n = vc.size(0), C = fc.size(1), M = fc.size(0);
    auto out = torch::empty({n, M, C}, vc.options().dtype(out_bf16 ? torch::kBFloat16 : torch::kFloat32));
    auto ang = torch::empty({n, 3}, vc.options());
    check(lv_fused_exp_action_fwd(muc.defined() ? muc.data_ptr<float>() : nullptr, vc.data_ptr<float>(),
                                  fc.data_ptr<float>(), 0, out.data_ptr(),
                                  out_bf16 ? LV_DTYPE_BF16 : LV_DTYPE_F32, ang.data_ptr<float>(), n,
                                  (int)L, (int)C, transpose ? 1 : 0, stream_of(vc)),
          "lv_fused_exp_action_fwd");
    ctx->save_for_backward({muc, vc, fc, ang});
    ctx->saved_data["L"] = L;
    ctx->saved_data["transpose"] = transpose;
    ctx->saved_data["mu_dtype"] = mu.has_value() && mu->defined() ? (int64_t)mu->scalar_type() : (int64_t)-1;
    ctx->saved_data["v_dtype"] = (int64_t)v.scalar_type();
    ctx->saved_data["f_dtype"] = (int64_t)spec.scalar_type();
    return out;
  }

  static variable_list backward(AutogradContext* ctx, variable_list grads) {
    const auto saved = ctx->get_saved_variables();
    const Tensor& mu = saved[0];
    const Tensor& v = saved[1];
    const Tensor& spec = saved[2];
    const Tensor& ang = saved[3];
    const int64_t L = ctx->saved_data["L"].toInt();
    const bool transpose = ctx->saved_data["transpose"].toBool();
    const c10::DeviceGuard guard(v.device());
    Tensor g = grads[0];
    TORCH_CHECK(g.device() == v.device(), "lievae::fused_exp_action backward: gradient on ", g.device(),
                ", inputs on ", v.device());
    g = g.scalar_type() == torch::kFloat32 && g.is_contiguous() ? g : g.to(torch::kFloat32).contiguous();
    const int64_t n = v.size(0), C = spec.size(1);
    auto gspec = torch::empty_like(spec);
    auto gv = torch::empty_like(v);
    Tensor gmu = mu.defined() ? torch::empty_like(mu) : Tensor();
    void* st = stream_of(v);
    size_t wsb = 0;
    Tensor ws = workspace(n, L, C, v, st, wsb);
    check(lv_fused_exp_action_bwd(mu.defined() ? mu.data_ptr<float>() : nullptr, v.data_ptr<float>(),
                                  ang.data_ptr<float>(), spec.data_ptr<float>(), g.data_ptr<float>(),
                                  gmu.defined() ? gmu.data_ptr<float>() : nullptr, gv.data_ptr<float>(),
                                  gspec.data_ptr<float>(), n, (int)L, (int)C, transpose ? 1 : 0,
                                  ws.data_ptr(), wsb, st),
          "lv_fused_exp_action_bwd");
    // gradients in the inputs' dtypes (autograd's contract; the kernels are fp32)
    const int64_t mdt = ctx->saved_data["mu_dtype"].toInt();
    if (gmu.defined() && mdt != (int64_t)torch::kFloat32) gmu = gmu.to((c10::ScalarType)mdt);
    const int64_t vdt = ctx->saved_data["v_dtype"].toInt();
    if (vdt != (int64_t)torch::kFloat32) gv = gv.to((c10::ScalarType)vdt);
    const int64_t fdt = ctx->saved_data["f_dtype"].toInt();
    if (fdt != (int64_t)torch::kFloat32) gspec = gspec.to((c10::ScalarType)fdt);
    return {gmu, gv, gspec, Tensor(), Tensor(), Tensor()};
  }
};

Tensor fused_exp_action(const std::optional<Tensor>& mu, const Tensor& v, const Tensor& spec, int64_t L,
                        bool transpose, bool out_bf16) {
  return FusedExpAction::apply(mu, v, spec, L, transpose, out_bf16);
}

}  // namespace

TORCH_LIBRARY(lievae, m) {
  m.def("fused_exp_action(Tensor? mu, Tensor v, Tensor spec, int L, bool transpose, bool out_bf16) -> Tensor");
}
// One kernel for every device key: the autograd function is the implementation (it checks
// that the tensors are on the GPU and raises otherwise).
TORCH_LIBRARY_IMPL(lievae, CompositeImplicitAutograd, m) {
  m.impl("fused_exp_action", &fused_exp_action);
}
