// Python bindings for apex._C (compiled by the host compiler against torch's
// headers; all device code lives in the torch-free .hip translation units).
#include <ATen/hip/HIPContext.h>
#include <torch/extension.h>

#include <vector>

#include "kernels.h"

namespace {

using at::Tensor;

hipStream_t cur_stream() { return at::hip::getCurrentHIPStream().stream(); }

int dt_code(at::ScalarType t) {
  switch (t) {
    case at::kFloat: return apex::kF32Code;
    case at::kHalf: return apex::kF16Code;
    case at::kBFloat16: return apex::kBF16Code;
    default: TORCH_CHECK(false, "apex._C: unsupported dtype ", t);
  }
  return -1;
}

void check(int rc, const char* what) {
  TORCH_CHECK(rc == 0, "apex._C: ", what, " failed (code ", rc, ")");
}

template <typename T>
T* opt_ptr(const c10::optional<Tensor>& t) {
  return t.has_value() && t->defined() ? t->data_ptr<T>() : nullptr;
}

void* opt_vptr(const c10::optional<Tensor>& t) {
  return t.has_value() && t->defined() ? t->data_ptr() : nullptr;
}

// --------------------------------------------------------------------------
// Multi-tensor plan: device-resident chunk table describing N parallel lists.
// --------------------------------------------------------------------------
struct MTPlan {
  Tensor meta;  // int64 on device
  int nlists = 0, ntensors = 0, nchunks = 0, chunk_size = 0, aligned = 1;
  std::vector<int> dtypes;
  std::vector<int64_t> host_ptrs;

  MTPlan(const std::vector<std::vector<Tensor>>& lists, int64_t chunk) {
    TORCH_CHECK(!lists.empty() && lists.size() <= (size_t)apex::kMaxLists, "bad list count");
    TORCH_CHECK(chunk > 0 && chunk % 8 == 0, "chunk size must be a positive multiple of 8");
    nlists = (int)lists.size();
    ntensors = (int)lists[0].size();
    chunk_size = (int)chunk;
    at::Device dev = at::kCPU;
    for (int l = 0; l < nlists; ++l) {
      TORCH_CHECK((int)lists[l].size() == ntensors, "all tensor lists must have the same length");
      dtypes.push_back(ntensors ? dt_code(lists[l][0].scalar_type()) : 0);
      for (int t = 0; t < ntensors; ++t) {
        const Tensor& x = lists[l][t];
        TORCH_CHECK(x.is_cuda(), "multi-tensor op requires device tensors");
        TORCH_CHECK(x.is_contiguous(), "multi-tensor op requires contiguous tensors");
        TORCH_CHECK(dt_code(x.scalar_type()) == dtypes[l], "list ", l, " mixes dtypes");
        TORCH_CHECK(x.numel() == lists[0][t].numel(), "tensor size mismatch across lists");
        dev = x.device();
      }
    }
    std::vector<int64_t> numel(ntensors), chunk_off(ntensors + 1);
    std::vector<int64_t> chunks;
    for (int t = 0; t < ntensors; ++t) {
      numel[t] = lists[0][t].numel();
      chunk_off[t] = (int64_t)chunks.size();
      const int64_t nc = (numel[t] + chunk - 1) / chunk;
      for (int64_t c = 0; c < nc; ++c) chunks.push_back(((int64_t)t << apex::kChunkShift) | c);
    }
    chunk_off[ntensors] = (int64_t)chunks.size();
    nchunks = (int)chunks.size();
    const int64_t words = apex::mt_meta_words(nlists, ntensors, nchunks);
    Tensor host = at::empty({words}, at::TensorOptions().dtype(at::kLong).pinned_memory(true));
    int64_t* h = host.data_ptr<int64_t>();
    host_ptrs.resize((size_t)nlists * ntensors);
    for (int l = 0; l < nlists; ++l)
      for (int t = 0; t < ntensors; ++t) {
        const int64_t p = (int64_t)(uintptr_t)lists[l][t].data_ptr();
        host_ptrs[(size_t)l * ntensors + t] = p;
        h[(size_t)l * ntensors + t] = p;
        if (p & 15) aligned = 0;
      }
    int64_t* q = h + (int64_t)nlists * ntensors;
    for (int t = 0; t < ntensors; ++t) q[t] = numel[t];
    q += ntensors;
    for (int t = 0; t <= ntensors; ++t) q[t] = chunk_off[t];
    q += ntensors + 1;
    for (int c = 0; c < nchunks; ++c) q[c] = chunks[c];
    // pinned + non_blocking: torch's caching host allocator records the copy's stream
    // event and will not recycle the staging block before the copy has completed
    meta = host.to(dev, /*non_blocking=*/true);
  }

  bool matches(const std::vector<std::vector<Tensor>>& lists) const {
    if ((int)lists.size() != nlists) return false;
    for (int l = 0; l < nlists; ++l) {
      if ((int)lists[l].size() != ntensors) return false;
      for (int t = 0; t < ntensors; ++t)
        if ((int64_t)(uintptr_t)lists[l][t].data_ptr() != host_ptrs[(size_t)l * ntensors + t])
          return false;
    }
    return true;
  }

  apex::MTMeta view() const {
    return apex::mt_meta_view(meta.data_ptr<int64_t>(), nlists, ntensors, nchunks, chunk_size,
                              aligned);
  }

  void scale(const c10::optional<Tensor>& scale_t, double scale, const c10::optional<Tensor>& overflow) {
    TORCH_CHECK(nlists >= 2, "scale needs [in, out]");
    check(apex::mt_scale(view(), dtypes[0], dtypes[1], opt_ptr<float>(scale_t), (float)scale,
                         opt_ptr<int>(overflow), cur_stream()),
          "mt_scale");
  }

  void axpby(double a, double b, int64_t check_arg, const c10::optional<Tensor>& overflow) {
    TORCH_CHECK(nlists >= 3, "axpby needs [x, y, out]");
    check(apex::mt_axpby(view(), dtypes[0], dtypes[1], dtypes[2], (float)a, (float)b,
                         (int)check_arg, opt_ptr<int>(overflow), cur_stream()),
          "mt_axpby");
  }

  // returns (global_norm[1], per_tensor[T] or empty)
  std::vector<Tensor> l2norm(int64_t list, bool per_tensor, const c10::optional<Tensor>& scale_t,
                             double scale, const c10::optional<Tensor>& overflow) {
    auto opts = meta.options().dtype(at::kFloat);
    Tensor partial = at::empty({std::max(nchunks, 1)}, opts);
    Tensor glob = at::zeros({1}, opts);
    Tensor per = per_tensor ? at::zeros({ntensors}, opts) : at::empty({0}, opts);
    check(apex::mt_l2norm(view(), (int)list, dtypes[list], partial.data_ptr<float>(),
                          per_tensor ? per.data_ptr<float>() : nullptr, glob.data_ptr<float>(),
                          opt_ptr<float>(scale_t), (float)scale, opt_ptr<int>(overflow),
                          cur_stream()),
          "mt_l2norm");
    return {glob, per};
  }

  void sgd(double lr, double momentum, double dampening, double wd, bool nesterov, bool first_run,
           bool wd_after_momentum, double grad_scale, const c10::optional<Tensor>& grad_scale_t,
           const c10::optional<Tensor>& noop) {
    apex::SgdArgs a{(float)lr, (float)momentum, (float)dampening, (float)wd, nesterov, first_run,
                    wd_after_momentum, (float)grad_scale, opt_ptr<float>(grad_scale_t),
                    opt_ptr<int>(noop)};
    const int c_dt = nlists > 3 ? dtypes[3] : dtypes[1];
    check(apex::mt_sgd(view(), dtypes[0], dtypes[1], c_dt, a, cur_stream()), "mt_sgd");
  }

  void adam(double lr, double b1, double b2, double eps, double wd, double bc1, double bc2,
            bool adamw, double grad_scale, const c10::optional<Tensor>& grad_scale_t,
            const c10::optional<Tensor>& noop) {
    apex::AdamArgs a{(float)lr, (float)b1, (float)b2, (float)eps, (float)wd, (float)bc1, (float)bc2,
                     adamw, (float)grad_scale, opt_ptr<float>(grad_scale_t), opt_ptr<int>(noop)};
    const int c_dt = nlists > 4 ? dtypes[4] : dtypes[1];
    check(apex::mt_adam(view(), dtypes[0], dtypes[1], c_dt, a, cur_stream()), "mt_adam");
  }

  // lists: g, p, m, v, u(fp32 scratch), [copy]; step: int32[1] device counter
  // workspace is returned so python can read the grad norm (ws[0]).
  Tensor lamb(double lr, double b1, double b2, double eps, double wd, double max_grad_norm,
              bool adamw, bool bias_correction, bool grad_averaging, bool use_nvlamb,
              double grad_scale, const c10::optional<Tensor>& grad_scale_t,
              const c10::optional<Tensor>& noop, const c10::optional<Tensor>& overflow_out,
              Tensor step, const c10::optional<Tensor>& gnorm_in) {
    TORCH_CHECK(nlists >= 5, "lamb needs [g, p, m, v, u, (copy)]");
    TORCH_CHECK(step.scalar_type() == at::kInt && step.is_cuda(), "step must be int32 device");
    Tensor ws = at::empty({4 + 3 * (int64_t)std::max(nchunks, 1) + 2 * (int64_t)ntensors},
                          meta.options().dtype(at::kFloat));
    apex::LambArgs a{(float)lr, (float)b1, (float)b2, (float)eps, (float)wd, (float)max_grad_norm,
                     adamw, bias_correction, grad_averaging, use_nvlamb, (float)grad_scale,
                     opt_ptr<float>(grad_scale_t), opt_ptr<int>(noop), opt_ptr<int>(overflow_out),
                     opt_ptr<float>(gnorm_in)};
    const int c_dt = nlists > 5 ? dtypes[5] : dtypes[1];
    check(apex::mt_lamb(view(), dtypes[0], dtypes[1], c_dt, a, ws.data_ptr<float>(),
                        step.data_ptr<int>(), cur_stream()),
          "mt_lamb");
    return ws;
  }

  void larc(double trust, double eps, double lr, double wd, bool clip) {
    Tensor ws = at::empty({(int64_t)std::max(nchunks, 1) + 2 * (int64_t)ntensors},
                          meta.options().dtype(at::kFloat));
    apex::LarcArgs a{(float)trust, (float)eps, (float)lr, (float)wd, clip};
    check(apex::mt_larc(view(), dtypes[0], dtypes[1], a, ws.data_ptr<float>(), cur_stream()),
          "mt_larc");
  }
};

void update_scale(Tensor scale, Tensor tracker, Tensor overflow, double growth, double backoff,
                  int64_t interval, double min_scale, double max_scale) {
  check(apex::amp_update_scale(scale.data_ptr<float>(), tracker.data_ptr<int>(),
                               overflow.data_ptr<int>(), (float)growth, (float)backoff,
                               (int)interval, (float)min_scale, (float)max_scale, cur_stream()),
        "update_scale");
}

// --------------------------------------------------------------------------
// LayerNorm / RMSNorm
// --------------------------------------------------------------------------
std::vector<Tensor> ln_fwd(Tensor x, int64_t cols, const c10::optional<Tensor>& gamma,
                           const c10::optional<Tensor>& beta, double eps, bool rms) {
  TORCH_CHECK(x.is_cuda() && x.is_contiguous(), "layer_norm: x must be contiguous device tensor");
  const int64_t rows = cols ? x.numel() / cols : 0;
  Tensor y = at::empty_like(x);
  auto fopt = x.options().dtype(at::kFloat);
  Tensor mean = rms ? at::empty({0}, fopt) : at::empty({rows}, fopt);
  Tensor rstd = at::empty({rows}, fopt);
  const int wdt = gamma.has_value() && gamma->defined() ? dt_code(gamma->scalar_type())
                                                        : dt_code(x.scalar_type());
  check(apex::layer_norm_fwd(x.data_ptr(), opt_vptr(gamma), opt_vptr(beta), y.data_ptr(),
                             rms ? nullptr : mean.data_ptr<float>(), rstd.data_ptr<float>(), rows,
                             (int)cols, (float)eps, dt_code(x.scalar_type()), wdt, rms,
                             cur_stream()),
        "layer_norm_fwd");
  return {y, mean, rstd};
}

std::vector<Tensor> ln_bwd(Tensor dy, Tensor x, int64_t cols, const c10::optional<Tensor>& gamma,
                           const c10::optional<Tensor>& beta, Tensor mean, Tensor rstd, bool rms) {
  TORCH_CHECK(dy.is_contiguous() && x.is_contiguous(), "layer_norm_bwd: contiguous inputs");
  const int64_t rows = cols ? x.numel() / cols : 0;
  Tensor dx = at::empty_like(x);
  const bool hg = gamma.has_value() && gamma->defined();
  const bool hb = beta.has_value() && beta->defined();
  Tensor dgamma = hg ? at::empty_like(*gamma) : Tensor();
  Tensor dbeta = hb ? at::empty_like(*beta) : Tensor();
  Tensor ws;
  if (hg || hb)
    ws = at::empty({apex::layer_norm_bwd_ws_floats(rows, (int)cols)}, x.options().dtype(at::kFloat));
  const int wdt = hg ? dt_code(gamma->scalar_type()) : dt_code(x.scalar_type());
  check(apex::layer_norm_bwd(dy.data_ptr(), x.data_ptr(), opt_vptr(gamma),
                             rms ? nullptr : mean.data_ptr<float>(), rstd.data_ptr<float>(),
                             dx.data_ptr(), hg ? dgamma.data_ptr() : nullptr,
                             hb ? dbeta.data_ptr() : nullptr, ws.defined() ? ws.data_ptr<float>() : nullptr,
                             rows, (int)cols, dt_code(x.scalar_type()), wdt, rms, cur_stream()),
        "layer_norm_bwd");
  return {dx, dgamma, dbeta};
}

// --------------------------------------------------------------------------
// softmax cross-entropy
// --------------------------------------------------------------------------
std::vector<Tensor> xent_fwd(Tensor logits, Tensor labels, double smoothing, int64_t ignore_index) {
  TORCH_CHECK(logits.dim() == 2 && logits.is_contiguous(), "xentropy: logits must be [N, V] contiguous");
  TORCH_CHECK(labels.scalar_type() == at::kLong, "xentropy: labels must be int64");
  const int64_t N = logits.size(0);
  const int V = (int)logits.size(1);
  auto fopt = logits.options().dtype(at::kFloat);
  Tensor losses = at::empty({N}, fopt), lse = at::empty({N}, fopt);
  Tensor lab = labels.contiguous();
  check(apex::xentropy_fwd(logits.data_ptr(), lab.data_ptr<int64_t>(), losses.data_ptr<float>(),
                           lse.data_ptr<float>(), N, V, (float)smoothing, ignore_index,
                           dt_code(logits.scalar_type()), cur_stream()),
        "xentropy_fwd");
  return {losses, lse};
}

Tensor xent_bwd(Tensor dloss, Tensor logits, Tensor lse, Tensor labels, double smoothing,
                int64_t ignore_index) {
  const int64_t N = logits.size(0);
  const int V = (int)logits.size(1);
  Tensor dx = at::empty_like(logits);
  Tensor lab = labels.contiguous();
  TORCH_CHECK(dloss.dim() == 1 && dloss.size(0) == N, "xentropy_bwd: dloss must be [N]");
  check(apex::xentropy_bwd(dloss.data_ptr(), dloss.stride(0), dt_code(dloss.scalar_type()),
                           logits.data_ptr(), lse.data_ptr<float>(), lab.data_ptr<int64_t>(),
                           dx.data_ptr(), N, V, (float)smoothing, ignore_index,
                           dt_code(logits.scalar_type()), cur_stream()),
        "xentropy_bwd");
  return dx;
}

}  // namespace

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "apex MI355X (gfx950) HIP kernels";
  m.attr("arch") = "gfx950";
  py::class_<MTPlan>(m, "MTPlan")
      .def(py::init<const std::vector<std::vector<Tensor>>&, int64_t>())
      .def("matches", &MTPlan::matches)
      .def_readonly("nchunks", &MTPlan::nchunks)
      .def_readonly("ntensors", &MTPlan::ntensors)
      .def_readonly("nlists", &MTPlan::nlists)
      .def_readonly("aligned", &MTPlan::aligned)
      .def("scale", &MTPlan::scale)
      .def("axpby", &MTPlan::axpby)
      .def("l2norm", &MTPlan::l2norm)
      .def("sgd", &MTPlan::sgd)
      .def("adam", &MTPlan::adam)
      .def("lamb", &MTPlan::lamb)
      .def("larc", &MTPlan::larc);
  m.def("update_scale", &update_scale);
  m.def("ln_fwd", &ln_fwd);
  m.def("ln_bwd", &ln_bwd);
  m.def("xent_fwd", &xent_fwd);
  m.def("xent_bwd", &xent_bwd);
}
