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
        // elementwise ops only need dense storage walked in the same order in every list
        // (e.g. channels_last conv weights, their grads and optimizer state)
        TORCH_CHECK((x.is_contiguous() && lists[0][t].is_contiguous()) ||
                        (x.is_non_overlapping_and_dense() && x.strides() == lists[0][t].strides()),
                    "multi-tensor op requires dense tensors with matching strides across lists");
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

  // first_run_t: optional int32[1] device flag (nonzero until a non-skipped step ran); when given
  // it replaces the host first_run so an overflow-skipped step does not use it up
  void sgd(double lr, double momentum, double dampening, double wd, bool nesterov, bool first_run,
           bool wd_after_momentum, double grad_scale, const c10::optional<Tensor>& grad_scale_t,
           const c10::optional<Tensor>& noop, const c10::optional<Tensor>& first_run_t) {
    if (first_run_t) TORCH_CHECK(first_run_t->scalar_type() == at::kInt && first_run_t->is_cuda(), "first_run flag must be int32 device");
    apex::SgdArgs a{(float)lr, (float)momentum, (float)dampening, (float)wd, nesterov, first_run,
                    wd_after_momentum, (float)grad_scale, opt_ptr<float>(grad_scale_t),
                    opt_ptr<int>(noop), opt_ptr<int>(first_run_t)};
    const int c_dt = nlists > 3 ? dtypes[3] : dtypes[1];
    check(apex::mt_sgd(view(), dtypes[0], dtypes[1], c_dt, a, cur_stream()), "mt_sgd");
  }

  // step_t: optional int32[1] device step counter; when given it is advanced on the device only by
  // non-skipped steps and the bias corrections come from it (bc1/bc2 ignored)
  void adam(double lr, double b1, double b2, double eps, double wd, double bc1, double bc2,
            bool adamw, double grad_scale, const c10::optional<Tensor>& grad_scale_t,
            const c10::optional<Tensor>& noop, const c10::optional<Tensor>& step_t, bool bias_correction) {
    Tensor scal;
    if (step_t) {
      TORCH_CHECK(step_t->scalar_type() == at::kInt && step_t->is_cuda(), "step must be int32 device");
      scal = at::empty({2}, meta.options().dtype(at::kFloat));
    }
    apex::AdamArgs a{(float)lr, (float)b1, (float)b2, (float)eps, (float)wd, (float)bc1, (float)bc2,
                     adamw, (float)grad_scale, opt_ptr<float>(grad_scale_t), opt_ptr<int>(noop),
                     opt_ptr<int>(step_t), bias_correction, step_t ? scal.data_ptr<float>() : nullptr};
    const int c_dt = nlists > 4 ? dtypes[4] : dtypes[1];
    check(apex::mt_adam(view(), dtypes[0], dtypes[1], c_dt, a, cur_stream()), "mt_adam");
  }

  // lists: g, p, m, v, [copy]; step: int32[1] device counter
  // workspace is returned so python can read the grad norm (ws[0]).
  Tensor lamb(double lr, double b1, double b2, double eps, double wd, double max_grad_norm,
              bool adamw, bool bias_correction, bool grad_averaging, bool use_nvlamb,
              double grad_scale, const c10::optional<Tensor>& grad_scale_t,
              const c10::optional<Tensor>& noop, const c10::optional<Tensor>& overflow_out,
              Tensor step, const c10::optional<Tensor>& gnorm_in) {
    TORCH_CHECK(nlists >= 4, "lamb needs [g, p, m, v, (copy)]");
    TORCH_CHECK(step.scalar_type() == at::kInt && step.is_cuda(), "step must be int32 device");
    Tensor ws = at::empty({4 + 3 * (int64_t)std::max(nchunks, 1) + 2 * (int64_t)ntensors},
                          meta.options().dtype(at::kFloat));
    apex::LambArgs a{(float)lr, (float)b1, (float)b2, (float)eps, (float)wd, (float)max_grad_norm,
                     adamw, bias_correction, grad_averaging, use_nvlamb, (float)grad_scale,
                     opt_ptr<float>(grad_scale_t), opt_ptr<int>(noop), opt_ptr<int>(overflow_out),
                     opt_ptr<float>(gnorm_in)};
    const int c_dt = nlists > 4 ? dtypes[4] : dtypes[1];
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

Tensor out_or_empty(const c10::optional<Tensor>& out, at::IntArrayRef sizes, const at::TensorOptions& opt,
                    const char* what);

// dgamma_out / dbeta_out: optional destinations (a DDP gradient-bucket slot, apex.parallel.grad_target)
std::vector<Tensor> ln_bwd(Tensor dy, Tensor x, int64_t cols, const c10::optional<Tensor>& gamma,
                           const c10::optional<Tensor>& beta, Tensor mean, Tensor rstd, bool rms,
                           const c10::optional<Tensor>& dgamma_out, const c10::optional<Tensor>& dbeta_out) {
  TORCH_CHECK(dy.is_contiguous() && x.is_contiguous(), "layer_norm_bwd: contiguous inputs");
  const int64_t rows = cols ? x.numel() / cols : 0;
  Tensor dx = at::empty_like(x);
  const bool hg = gamma.has_value() && gamma->defined();
  const bool hb = beta.has_value() && beta->defined();
  Tensor dgamma = hg ? out_or_empty(dgamma_out, gamma->sizes(), gamma->options(), "layer_norm_bwd dgamma") : Tensor();
  Tensor dbeta = hb ? out_or_empty(dbeta_out, beta->sizes(), beta->options(), "layer_norm_bwd dbeta") : Tensor();
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

// --------------------------------------------------------------------------
// flash attention: q, k, v, o are [B, S, H, D] (any batch/seq/head strides, D contiguous)
// --------------------------------------------------------------------------
void attn_set(apex::AttnArgs& a, const Tensor& t, int64_t& bs, int64_t& ss, int64_t& hs) {
  TORCH_CHECK(t.dim() == 4 && t.stride(3) == 1, "attention tensors must be [B, S, H, D], D contiguous");
  TORCH_CHECK(t.stride(1) % 8 == 0 && t.stride(2) % 8 == 0 && t.stride(0) % 8 == 0 &&
                  ((uintptr_t)t.data_ptr() & 15) == 0,
              "attention tensors must be 16-byte aligned per row");
  bs = t.stride(0);
  ss = t.stride(1);
  hs = t.stride(2);
}

apex::AttnArgs attn_common(const Tensor& q, const Tensor& k, const Tensor& v, bool causal,
                           double scale, double p_drop, int64_t seed, int64_t offset,
                           const c10::optional<Tensor>& k_lens) {
  apex::AttnArgs a{};
  TORCH_CHECK(q.scalar_type() == k.scalar_type() && q.scalar_type() == v.scalar_type(), "dtype mismatch");
  a.q = q.data_ptr();
  a.k = k.data_ptr();
  a.v = v.data_ptr();
  attn_set(a, q, a.q_bs, a.q_ss, a.q_hs);
  attn_set(a, k, a.k_bs, a.k_ss, a.k_hs);
  attn_set(a, v, a.v_bs, a.v_ss, a.v_hs);
  a.B = (int)q.size(0);
  a.Sq = (int)q.size(1);
  a.H = (int)q.size(2);
  a.D = (int)q.size(3);
  a.Sk = (int)k.size(1);
  TORCH_CHECK(k.size(0) == a.B && k.size(2) == a.H && k.size(3) == a.D && v.sizes() == k.sizes(),
              "k/v shape mismatch");
  TORCH_CHECK(a.D == 32 || a.D == 64 || a.D == 128 || a.D == 256,
              "flash attention supports head dims 32, 64, 128, 256 (pad others)");
  TORCH_CHECK(q.scalar_type() != at::kFloat || a.D <= 128, "fp32 flash attention supports head dims up to 128");
  a.causal = causal;
  a.scale = (float)scale;
  a.scale_log2 = (float)(scale * 1.4426950408889634);
  TORCH_CHECK(p_drop >= 0.0 && p_drop < 1.0, "dropout p must be in [0, 1)");
  // attention dropout draws 8-bit uniforms (keep iff u8 >= thresh, p quantised to 1/256 as in
  // FlashAttention-2); the rescale uses the quantised keep probability, so E[output] is exact
  a.drop_thresh = apex::attn_drop_thresh(p_drop);
  a.drop_scale = p_drop > 0.0 ? (float)(256.0 / (256.0 - a.drop_thresh)) : 1.f;
  a.seed = (uint64_t)seed;
  a.offset = (uint64_t)offset;
  if (k_lens.has_value() && k_lens->defined()) {
    TORCH_CHECK(k_lens->scalar_type() == at::kInt && k_lens->numel() == a.B, "k_lens must be int32 [B]");
    a.k_lens = k_lens->data_ptr<int>();
  }
  return a;
}

// optional additive score bias: a [B|1, H|1, Sq|1, Sk] view (broadcast dims stride 0) in q's dtype,
// key stride 1, 8-byte aligned rows
void attn_set_bias(apex::AttnArgs& a, const c10::optional<Tensor>& bias, const Tensor& q) {
  if (!bias.has_value() || !bias->defined()) return;
  const Tensor& t = *bias;
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == q.scalar_type(), "attention bias must be a device tensor in q's dtype");
  TORCH_CHECK(t.dim() == 4 && t.size(3) == a.Sk && t.stride(3) == 1, "attention bias must be [B|1, H|1, Sq|1, Sk], key-contiguous");
  TORCH_CHECK((t.size(0) == a.B || t.stride(0) == 0 || t.size(0) == 1) && (t.size(1) == a.H || t.size(1) == 1 || t.stride(1) == 0) &&
                  (t.size(2) == a.Sq || t.size(2) == 1 || t.stride(2) == 0),
              "attention bias does not broadcast to [B, H, Sq, Sk]");
  TORCH_CHECK(((uintptr_t)t.data_ptr() & 7) == 0 && t.stride(2) % 4 == 0 && t.stride(1) % 4 == 0 && t.stride(0) % 4 == 0,
              "attention bias rows must be 8-byte aligned");
  TORCH_CHECK(t.scalar_type() != at::kFloat || ((uintptr_t)t.data_ptr() & 15) == 0,
              "fp32 attention bias rows must be 16-byte aligned");
  a.bias = t.data_ptr();
  a.bias_bs = t.size(0) == 1 ? 0 : t.stride(0);
  a.bias_hs = t.size(1) == 1 ? 0 : t.stride(1);
  a.bias_qs = t.size(2) == 1 ? 0 : t.stride(2);
}

// fp8 producer-side codes of an attention output (apex.fp8): a uint8 tensor with `like`'s sizes AND
// strides (so a code sits at its value's element offset), plus the slot's scale / amax
static uint8_t* attn_q8(const c10::optional<Tensor>& codes, const Tensor& like, const char* what) {
  if (!codes.has_value() || !codes->defined()) return nullptr;
  TORCH_CHECK(codes->scalar_type() == at::kByte && codes->sizes() == like.sizes() &&
                  codes->strides() == like.strides() && codes->device() == like.device(),
              what, ": fp8 codes must be a uint8 tensor with the output's sizes and strides");
  return codes->data_ptr<uint8_t>();
}
static void attn_q8_scale(apex::AttnArgs& a, const c10::optional<Tensor>& scale, const c10::optional<Tensor>& amax,
                          int64_t fmt, const Tensor& like) {
  TORCH_CHECK(scale.has_value() && amax.has_value() && scale->scalar_type() == at::kFloat &&
                  amax->scalar_type() == at::kFloat && scale->numel() >= 1 && amax->numel() >= 1 &&
                  scale->device() == like.device() && amax->device() == like.device(),
              "flash attention fp8 codes: q8_scale / q8_amax fp32 device tensors");
  TORCH_CHECK(fmt == 0 || fmt == 1, "flash attention fp8 codes: q8_fmt 0 (e4m3) or 1 (e5m2)");
  a.q8_scale = scale->data_ptr<float>();
  a.q8_amax = amax->data_ptr<float>();
  a.q8_fmt = (int)fmt;
}

std::vector<Tensor> flash_attn_fwd(Tensor q, Tensor k, Tensor v, bool causal, double scale,
                                   double p_drop, int64_t seed, int64_t offset,
                                   const c10::optional<Tensor>& k_lens, const c10::optional<Tensor>& bias,
                                   const c10::optional<Tensor>& q8_out, const c10::optional<Tensor>& q8_scale,
                                   const c10::optional<Tensor>& q8_amax, int64_t q8_fmt) {
  apex::AttnArgs a = attn_common(q, k, v, causal, scale, p_drop, seed, offset, k_lens);
  attn_set_bias(a, bias, q);
  Tensor o = at::empty({a.B, a.Sq, a.H, a.D}, q.options());
  Tensor lse = at::empty({a.B, a.H, a.Sq}, q.options().dtype(at::kFloat));
  a.o = o.data_ptr();
  attn_set(a, o, a.o_bs, a.o_ss, a.o_hs);
  a.lse = lse.data_ptr<float>();
  a.q8o = attn_q8(q8_out, o, "flash_attn_fwd");
  TORCH_CHECK(!(a.q8o && q.scalar_type() == at::kFloat), "flash_attn_fwd: fp8 codes are a 16-bit-input feature");
  if (a.q8o) attn_q8_scale(a, q8_scale, q8_amax, q8_fmt, o);
  a.mask_words = 2 * (((int64_t)a.Sk + 31) / 32);
  Tensor dmask;  // dropout keep bits, consumed by the backward pass
  if (a.drop_thresh) {
    dmask = at::empty({(int64_t)a.B * a.H * a.Sq * a.mask_words}, q.options().dtype(at::kShort));
    a.dmask = (uint16_t*)dmask.data_ptr();
  } else {
    dmask = at::empty({0}, q.options().dtype(at::kShort));
  }
  check(apex::attn_fwd(a, dt_code(q.scalar_type()), cur_stream()), "attn_fwd");
  return {o, lse, dmask};
}

// returns true when the fp8 codes of dq / dk / dv were written (q8_* given and the single-kernel
// backward ran: Sk <= 128; longer key ranges compute dq in a separate kernel without codes)
bool flash_attn_bwd(Tensor dout, Tensor q, Tensor k, Tensor v, Tensor o, Tensor lse, Tensor dq,
                    Tensor dk, Tensor dv, bool causal, double scale, double p_drop, int64_t seed,
                    int64_t offset, const c10::optional<Tensor>& k_lens,
                    const c10::optional<Tensor>& dmask, const c10::optional<Tensor>& dsum, int64_t dbg,
                    const c10::optional<Tensor>& bias, const c10::optional<Tensor>& q8_dq,
                    const c10::optional<Tensor>& q8_dk, const c10::optional<Tensor>& q8_dv,
                    const c10::optional<Tensor>& q8_scale, const c10::optional<Tensor>& q8_amax, int64_t q8_fmt,
                    const c10::optional<Tensor>& dbias, bool q8_only) {
  apex::AttnArgs a = attn_common(q, k, v, causal, scale, p_drop, seed, offset, k_lens);
  a.dbg = (int)dbg;
  attn_set_bias(a, bias, q);
  if (dbias.has_value() && dbias->defined()) {
    // gradient of a trainable bias: a zeroed fp32 tensor with the bias's sizes, contiguous; the
    // kernels add dS into it (atomically where the bias broadcasts over batch, heads or queries)
    const Tensor& t = *dbias;
    TORCH_CHECK(a.bias, "flash_attn_bwd: dbias needs the bias");
    TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kFloat && t.is_contiguous() && t.dim() == 4 &&
                    t.sizes() == bias->sizes(),
                "flash_attn_bwd: dbias must be a zeroed contiguous fp32 tensor of the bias's sizes");
    a.dbias = t.data_ptr<float>();
    a.dbias_bs = t.size(0) == 1 ? 0 : t.stride(0);
    a.dbias_hs = t.size(1) == 1 ? 0 : t.stride(1);
    a.dbias_qs = t.size(2) == 1 ? 0 : t.stride(2);
    a.dbias_atomic = (t.size(0) == 1 && a.B > 1) || (t.size(1) == 1 && a.H > 1) || (t.size(2) == 1 && a.Sq > 1);
  }
  TORCH_CHECK(!(a.bias && dsum.has_value() && dsum->defined()), "flash_attn_bwd: dsum with a score bias is not supported");
  if (dsum.has_value() && dsum->defined()) {
    TORCH_CHECK(dsum->is_cuda() && dsum->scalar_type() == at::kFloat && dsum->is_contiguous() &&
                    dsum->numel() == (int64_t)a.B * 3 * a.H * a.D,
                "flash_attn_bwd: dsum must be a zeroed fp32 [B, 3, H, D] tensor");
    a.dsum = dsum->data_ptr<float>();
  }
  a.o = o.data_ptr();
  attn_set(a, o, a.o_bs, a.o_ss, a.o_hs);
  a.lse = lse.data_ptr<float>();
  attn_set(a, dout, a.do_bs, a.do_ss, a.do_hs);
  attn_set(a, dq, a.dq_bs, a.dq_ss, a.dq_hs);
  attn_set(a, dk, a.dk_bs, a.dk_ss, a.dk_hs);
  attn_set(a, dv, a.dv_bs, a.dv_ss, a.dv_hs);
  a.dq = dq.data_ptr();
  a.mask_words = 2 * (((int64_t)a.Sk + 31) / 32);
  if (a.drop_thresh) {
    TORCH_CHECK(dmask.has_value() && dmask->numel() == (int64_t)a.B * a.H * a.Sq * a.mask_words,
                "flash_attn_bwd: dropout mask from the forward pass is required");
    a.dmask = (uint16_t*)dmask->data_ptr();
  }
  const int64_t rows = (int64_t)a.B * a.H * a.Sq;
  Tensor delta_ws;  // rowsum(dO * O), one pre-pass kernel, read by the dK/dV and dQ kernels
  // fp32 (attention_f32.hip) always runs the delta pre-pass + dK/dV + dQ kernels
  const bool two_kernel = q.scalar_type() == at::kFloat || apex::attn_bwd_needs_dq_acc(a);
  if (two_kernel) delta_ws = at::empty({rows}, q.options().dtype(at::kFloat));
  bool q8 = false;
  if (!two_kernel && !apex::attn_bwd_split() && q8_dq.has_value() && q8_dq->defined()) {
    a.q8dq = attn_q8(q8_dq, dq, "flash_attn_bwd dq");
    a.q8dk = attn_q8(q8_dk, dk, "flash_attn_bwd dk");
    a.q8dv = attn_q8(q8_dv, dv, "flash_attn_bwd dv");
    TORCH_CHECK(a.q8dk && a.q8dv, "flash_attn_bwd: q8_dq, q8_dk and q8_dv go together");
    attn_q8_scale(a, q8_scale, q8_amax, q8_fmt, dq);
    a.q8only = q8_only ? 1 : 0;  // dq / dk / dv allocated, not written: the caller reads their codes alone
    q8 = true;
  }
  check(apex::attn_bwd(a, dout.data_ptr(), delta_ws.defined() ? delta_ws.data_ptr<float>() : nullptr,
                       dk.data_ptr(), dv.data_ptr(), dt_code(q.scalar_type()), cur_stream()),
        "attn_bwd");
  return q8;
}

// --------------------------------------------------------------------------
// fused elementwise (bias / act / dropout / residual / LN)
// --------------------------------------------------------------------------
std::pair<uint32_t, float> drop_params(double p) {
  if (p <= 0.0) return {0u, 1.f};
  TORCH_CHECK(p < 1.0, "dropout p must be < 1");
  uint32_t th = (uint32_t)std::lround(p * 65536.0);
  if (th == 0) th = 1;
  return {th, (float)(1.0 / (1.0 - th / 65536.0))};
}

int64_t cols_of(const Tensor& x) { return x.dim() ? x.size(-1) : 1; }

// optional caller-provided output (e.g. a parameter's slot in a DDP gradient bucket, so the
// gradient lands there with no copy); checked against the shape / dtype the op would allocate
Tensor out_or_empty(const c10::optional<Tensor>& out, at::IntArrayRef sizes, const at::TensorOptions& opt,
                    const char* what) {
  if (out.has_value() && out->defined()) {
    TORCH_CHECK(out->is_contiguous() && out->numel() == c10::multiply_integers(sizes) &&
                    out->scalar_type() == opt.dtype().toScalarType() && out->device() == opt.device(),
                what, ": out must be a contiguous tensor of the result's size, dtype and device");
    return *out;
  }
  return at::empty(sizes, opt);
}

Tensor k_bias_act_fwd(Tensor x, const c10::optional<Tensor>& b, int64_t act) {
  TORCH_CHECK(x.is_contiguous(), "bias_act: x must be contiguous");
  const int64_t cols = cols_of(x), rows = x.numel() / std::max<int64_t>(cols, 1);
  Tensor y = at::empty_like(x);
  const int bdt = b.has_value() && b->defined() ? dt_code(b->scalar_type()) : dt_code(x.scalar_type());
  check(apex::bias_act_fwd(x.data_ptr(), opt_vptr(b), y.data_ptr(), rows, (int)cols, (int)act,
                           dt_code(x.scalar_type()), bdt, cur_stream()),
        "bias_act_fwd");
  return y;
}

std::vector<Tensor> k_bias_act_bwd(Tensor dy, Tensor x, const c10::optional<Tensor>& b, int64_t act) {
  const int64_t cols = cols_of(x), rows = x.numel() / std::max<int64_t>(cols, 1);
  Tensor dyc = dy.contiguous();
  Tensor dx = at::empty_like(x);
  const bool hb = b.has_value() && b->defined();
  Tensor db = hb ? at::empty_like(*b) : Tensor();
  Tensor ws = hb ? at::empty({apex::colsum_parts(rows) * cols}, x.options().dtype(at::kFloat)) : Tensor();
  const int bdt = hb ? dt_code(b->scalar_type()) : dt_code(x.scalar_type());
  check(apex::bias_act_bwd(dyc.data_ptr(), x.data_ptr(), opt_vptr(b), dx.data_ptr(),
                           hb ? db.data_ptr() : nullptr, hb ? ws.data_ptr<float>() : nullptr, rows,
                           (int)cols, (int)act, dt_code(x.scalar_type()), bdt, cur_stream()),
        "bias_act_bwd");
  return {dx, db};
}

Tensor k_bda_fwd(Tensor x, const c10::optional<Tensor>& b, Tensor res, double p, int64_t seed,
                 int64_t offset) {
  TORCH_CHECK(x.is_contiguous() && res.is_contiguous() && x.sizes() == res.sizes(), "bias_dropout_add: shapes");
  const int64_t cols = cols_of(x), rows = x.numel() / std::max<int64_t>(cols, 1);
  Tensor y = at::empty_like(x);
  auto dp = drop_params(p);
  const int bdt = b.has_value() && b->defined() ? dt_code(b->scalar_type()) : dt_code(x.scalar_type());
  check(apex::bias_dropout_add_fwd(x.data_ptr(), opt_vptr(b), res.data_ptr(), y.data_ptr(), rows, (int)cols,
                                   (uint64_t)seed, (uint64_t)offset, dp.first, dp.second,
                                   dt_code(x.scalar_type()), bdt, cur_stream()),
        "bias_dropout_add_fwd");
  return y;
}

std::vector<Tensor> k_bda_bwd(Tensor dy, double p, int64_t seed, int64_t offset,
                              const c10::optional<Tensor>& bias_like, const c10::optional<Tensor>& dbias_out) {
  Tensor dyc = dy.contiguous();
  const int64_t cols = cols_of(dyc), rows = dyc.numel() / std::max<int64_t>(cols, 1);
  Tensor dx = at::empty_like(dyc);
  const bool hb = bias_like.has_value() && bias_like->defined();
  Tensor db = hb ? out_or_empty(dbias_out, bias_like->sizes(), bias_like->options(), "bias_dropout_add_bwd") : Tensor();
  Tensor ws = hb ? at::empty({apex::colsum_parts(rows) * cols}, dyc.options().dtype(at::kFloat)) : Tensor();
  auto dp = drop_params(p);
  check(apex::bias_dropout_add_bwd(dyc.data_ptr(), dx.data_ptr(), hb ? db.data_ptr() : nullptr,
                                   hb ? ws.data_ptr<float>() : nullptr, rows, (int)cols, (uint64_t)seed,
                                   (uint64_t)offset, dp.first, dp.second, dt_code(dyc.scalar_type()),
                                   hb ? dt_code(bias_like->scalar_type()) : dt_code(dyc.scalar_type()),
                                   cur_stream()),
        "bias_dropout_add_bwd");
  return {dx, db};
}

Tensor k_colsum(Tensor x, at::ScalarType out_dtype, const c10::optional<Tensor>& out_opt) {
  Tensor xc = x.contiguous();
  const int64_t cols = cols_of(xc), rows = xc.numel() / std::max<int64_t>(cols, 1);
  Tensor out = out_or_empty(out_opt, {cols}, xc.options().dtype(out_dtype), "colsum");
  Tensor ws = at::empty({apex::colsum_parts(rows) * cols}, xc.options().dtype(at::kFloat));
  check(apex::colsum(xc.data_ptr(), out.data_ptr(), ws.data_ptr<float>(), rows, (int)cols,
                     dt_code(xc.scalar_type()), dt_code(out_dtype), cur_stream()),
        "colsum");
  return out;
}

// split-K combine: slabs fp32 [S, ...] -> sum over S in out_dtype, shape slabs.shape[1:]
Tensor k_splitk_reduce(Tensor slabs, at::ScalarType out_dtype, const c10::optional<Tensor>& out_opt,
                       bool accumulate = false) {
  TORCH_CHECK(slabs.is_cuda() && slabs.scalar_type() == at::kFloat && slabs.dim() >= 2, "splitk_reduce: fp32 slabs");
  Tensor sc = slabs.contiguous();
  Tensor out = out_or_empty(out_opt, sc.sizes().slice(1), sc.options().dtype(out_dtype), "splitk_reduce");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(sc.data_ptr()) % 16 == 0 && (out.numel() % 4 == 0 || sc.size(0) == 1),
              "splitk_reduce: alignment");
  TORCH_CHECK(!accumulate || (out_opt.has_value() && out_dtype == at::kFloat),
              "splitk_reduce: accumulate needs an fp32 out");
  check(apex::splitk_reduce(sc.data_ptr<float>(), out.data_ptr(), out.numel(), (int)sc.size(0), dt_code(out_dtype),
                            cur_stream(), accumulate ? 1 : 0),
        "splitk_reduce");
  return out;
}

bool k_bdaln_supported(int64_t cols) { return apex::bdaln_supported((int)cols) != 0; }

// fp8 side output of a producer: codes uint8 like `like`, fp32 one-element scale / amax (device)
static apex::Q8Out q8_args(const c10::optional<Tensor>& out, const c10::optional<Tensor>& scale,
                           const c10::optional<Tensor>& amax, int64_t fmt, const Tensor& like, const char* what) {
  apex::Q8Out q;
  if (!out.has_value() || !out->defined()) return q;
  TORCH_CHECK(out->scalar_type() == at::kByte && out->is_contiguous() && out->numel() == like.numel() &&
                  out->device() == like.device(),
              what, ": q8_out must be a contiguous uint8 tensor like the output");
  TORCH_CHECK(scale.has_value() && amax.has_value() && scale->scalar_type() == at::kFloat &&
                  amax->scalar_type() == at::kFloat && scale->numel() >= 1 && amax->numel() >= 1 &&
                  scale->device() == like.device() && amax->device() == like.device(),
              what, ": q8_scale / q8_amax fp32 device tensors");
  TORCH_CHECK(fmt == 0 || fmt == 1, what, ": q8_fmt 0 (e4m3) or 1 (e5m2)");
  q.y = out->data_ptr<uint8_t>();
  q.scale = scale->data_ptr<float>();
  q.amax = amax->data_ptr<float>();
  q.fmt = (int)fmt;
  return q;
}
bool k_bdaln_wide_supported(int64_t cols) { return apex::bdaln_wide_supported((int)cols) != 0; }

// store_s = false (post-LN memory-efficient mode): the LN input s is not written (an empty tensor is
// returned); the backward rebuilds x-hat from y (k_bdaln_bwd with beta)
std::vector<Tensor> k_bdaln_fwd(Tensor x, const c10::optional<Tensor>& b, Tensor res, Tensor gamma,
                                Tensor beta, double eps, double p, int64_t seed, int64_t offset, bool store_s,
                                const c10::optional<Tensor>& q8_out, const c10::optional<Tensor>& q8_scale,
                                const c10::optional<Tensor>& q8_amax, int64_t q8_fmt, bool s_cond) {
  TORCH_CHECK(x.is_contiguous() && res.is_contiguous() && x.sizes() == res.sizes(), "bdaln: shapes");
  const int64_t cols = cols_of(x), rows = x.numel() / std::max<int64_t>(cols, 1);
  Tensor y = at::empty_like(x), s = store_s ? at::empty_like(x) : at::empty({0}, x.options());
  auto fo = x.options().dtype(at::kFloat);
  Tensor mean = at::empty({rows}, fo), rstd = at::empty({rows}, fo);
  auto dp = drop_params(p);
  check(apex::bdaln_fwd(x.data_ptr(), opt_vptr(b), res.data_ptr(), gamma.data_ptr(), beta.data_ptr(),
                        y.data_ptr(), store_s ? s.data_ptr() : nullptr, mean.data_ptr<float>(), rstd.data_ptr<float>(), rows,
                        (int)cols, (float)eps, (uint64_t)seed, (uint64_t)offset, dp.first, dp.second,
                        dt_code(x.scalar_type()), dt_code(gamma.scalar_type()), cur_stream(),
                        q8_args(q8_out, q8_scale, q8_amax, q8_fmt, y, "bdaln_fwd"), (store_s && s_cond) ? 1 : 0),
        "bdaln_fwd");
  return {y, s, mean, rstd};
}

std::vector<Tensor> k_bdaln_bwd(Tensor dy, Tensor s, Tensor gamma, Tensor mean, Tensor rstd, double p,
                                int64_t seed, int64_t offset, bool has_bias, const c10::optional<Tensor>& dgamma_out,
                                const c10::optional<Tensor>& dbeta_out, const c10::optional<Tensor>& dbias_out,
                                const c10::optional<Tensor>& ds_extra, const c10::optional<Tensor>& beta,
                                const c10::optional<Tensor>& q8_out, const c10::optional<Tensor>& q8_scale,
                                const c10::optional<Tensor>& q8_amax, int64_t q8_fmt,
                                const c10::optional<Tensor>& s_alt, bool q8_only) {
  // beta given: `s` is the LN output y of a store_s = false (or s_cond) forward (x-hat = (y - beta) /
  // gamma); s_alt: the s_cond forward's conditionally stored LN input, read instead when gamma has a 0
  Tensor dyc = dy.contiguous();
  const bool from_y = beta.has_value() && beta->defined();
  if (from_y)
    TORCH_CHECK(beta->is_contiguous() && beta->sizes() == gamma.sizes() && beta->scalar_type() == gamma.scalar_type() &&
                    s.is_contiguous(),
                "bdaln_bwd: beta like gamma, y contiguous");
  const int64_t cols = cols_of(s), rows = s.numel() / std::max<int64_t>(cols, 1);
  Tensor dse;
  if (ds_extra.has_value() && ds_extra->defined()) {
    dse = ds_extra->contiguous();
    TORCH_CHECK(dse.numel() == s.numel() && dse.scalar_type() == s.scalar_type(), "bdaln_bwd: ds_extra like s");
  }
  Tensor dres = at::empty_like(s), dx = at::empty_like(s);
  Tensor dgamma = out_or_empty(dgamma_out, gamma.sizes(), gamma.options(), "bdaln_bwd dgamma");
  Tensor dbeta = out_or_empty(dbeta_out, gamma.sizes(), gamma.options(), "bdaln_bwd dbeta");
  Tensor dbias = has_bias ? out_or_empty(dbias_out, gamma.sizes(), gamma.options(), "bdaln_bwd dbias") : Tensor();
  Tensor ws = at::empty({apex::bdaln_ws_floats(rows, (int)cols)}, s.options().dtype(at::kFloat));
  auto dp = drop_params(p);
  apex::Q8Out q8 = q8_args(q8_out, q8_scale, q8_amax, q8_fmt, dx, "bdaln_bwd");
  // q8_only: dx is allocated but not written (its consumers read the codes alone)
  TORCH_CHECK(!q8_only || q8.y, "bdaln_bwd: q8_only needs q8_out");
  q8.only = q8_only ? 1 : 0;
  check(apex::bdaln_bwd(dyc.data_ptr(), s.data_ptr(), gamma.data_ptr(), from_y ? beta->data_ptr() : nullptr,
                        mean.data_ptr<float>(),
                        rstd.data_ptr<float>(), dse.defined() ? dse.data_ptr() : nullptr, dres.data_ptr(),
                        dx.data_ptr(), dgamma.data_ptr(),
                        dbeta.data_ptr(), has_bias ? dbias.data_ptr() : nullptr, ws.data_ptr<float>(), rows,
                        (int)cols, (uint64_t)seed, (uint64_t)offset, dp.first, dp.second,
                        dt_code(s.scalar_type()), dt_code(gamma.scalar_type()), cur_stream(),
                        q8,
                        (from_y && s_alt.has_value() && s_alt->defined() && s_alt->numel() == s.numel())
                            ? s_alt->data_ptr() : nullptr),
        "bdaln_bwd");
  return {dres, dx, dgamma, dbeta, dbias};
}

// --------------------------------------------------------------------------
// BERT embeddings (fused_ops.hip): ids / tids int32 [B, S] (clamped by the caller)
// --------------------------------------------------------------------------
std::vector<Tensor> k_embed_ln_fwd(Tensor ids, const c10::optional<Tensor>& tids, Tensor Ww, Tensor Wp, Tensor Wt,
                                   Tensor gamma, Tensor beta, double eps, double p, int64_t seed, int64_t offset) {
  TORCH_CHECK(ids.is_cuda() && ids.dim() == 2 && ids.is_contiguous() && ids.scalar_type() == at::kInt,
              "embed_ln_fwd: ids int32 [B, S]");
  TORCH_CHECK(Ww.is_contiguous() && Wp.is_contiguous() && Wt.is_contiguous() && Ww.dim() == 2 &&
                  Wp.size(1) == Ww.size(1) && Wt.size(1) == Ww.size(1) && Wp.scalar_type() == Ww.scalar_type() &&
                  Wt.scalar_type() == Ww.scalar_type() && Wp.size(0) >= ids.size(1),
              "embed_ln_fwd: tables");
  const int* tp = nullptr;
  if (tids.has_value() && tids->defined()) {
    TORCH_CHECK(tids->sizes() == ids.sizes() && tids->is_contiguous() && tids->scalar_type() == at::kInt,
                "embed_ln_fwd: type ids int32 [B, S]");
    tp = tids->data_ptr<int>();
  }
  const int64_t B = ids.size(0), S = ids.size(1), H = Ww.size(1), rows = B * S;
  auto xo = Ww.options();
  Tensor y = at::empty({B, S, H}, xo), sv = at::empty({B, S, H}, xo);
  auto fo = xo.dtype(at::kFloat);
  Tensor mean = at::empty({rows}, fo), rstd = at::empty({rows}, fo);
  auto dp = drop_params(p);
  check(apex::embed_ln_fwd(ids.data_ptr<int>(), tp, Ww.data_ptr(), Wp.data_ptr(), Wt.data_ptr(), gamma.data_ptr(),
                           beta.data_ptr(), y.data_ptr(), sv.data_ptr(), mean.data_ptr<float>(), rstd.data_ptr<float>(),
                           rows, (int)H, (int)S, (float)eps, (uint64_t)seed, (uint64_t)offset, dp.first, dp.second,
                           dt_code(Ww.scalar_type()), dt_code(gamma.scalar_type()), cur_stream()),
        "embed_ln_fwd");
  return {y, sv, mean, rstd};
}

// -> {ds [B, S, H], dWp [npos, H] (rows >= S zero), dWt [tvocab, H], dgamma, dbeta}
std::vector<Tensor> k_embed_ln_bwd(Tensor dy, Tensor sv, Tensor gamma, Tensor mean, Tensor rstd,
                                   const c10::optional<Tensor>& tids, int64_t tvocab, int64_t npos, double p,
                                   int64_t seed, int64_t offset, const c10::optional<Tensor>& dwp_out,
                                   const c10::optional<Tensor>& dwt_out, const c10::optional<Tensor>& dgamma_out,
                                   const c10::optional<Tensor>& dbeta_out) {
  Tensor dyc = dy.contiguous();
  TORCH_CHECK(sv.dim() == 3 && dyc.sizes() == sv.sizes(), "embed_ln_bwd: shapes");
  const int64_t B = sv.size(0), S = sv.size(1), H = sv.size(2);
  TORCH_CHECK(npos >= S && tvocab >= 1 && tvocab <= 2, "embed_ln_bwd: table sizes");
  const int* tp = nullptr;
  if (tids.has_value() && tids->defined()) tp = tids->data_ptr<int>();
  Tensor ds = at::empty_like(sv);
  Tensor dWp = out_or_empty(dwp_out, {npos, H}, sv.options(), "embed_ln_bwd dWp");
  if (npos > S) dWp.view({npos, H}).narrow(0, S, npos - S).zero_();  // positions past S: no gradient
  Tensor dWt = out_or_empty(dwt_out, {tvocab, H}, sv.options(), "embed_ln_bwd dWt");
  Tensor dgamma = out_or_empty(dgamma_out, gamma.sizes(), gamma.options(), "embed_ln_bwd dgamma");
  Tensor dbeta = out_or_empty(dbeta_out, gamma.sizes(), gamma.options(), "embed_ln_bwd dbeta");
  const int nwt = apex::embed_nwt(B);
  auto fo = sv.options().dtype(at::kFloat);
  Tensor part_pos = at::empty({(int64_t)nwt * S * H}, fo);
  Tensor part_tg = at::empty({S * nwt * 4 * H}, fo);
  auto dp = drop_params(p);
  check(apex::embed_ln_bwd(dyc.data_ptr(), sv.data_ptr(), gamma.data_ptr(), mean.data_ptr<float>(),
                           rstd.data_ptr<float>(), tp, (int)tvocab, ds.data_ptr(), part_pos.data_ptr<float>(),
                           part_tg.data_ptr<float>(), dWp.data_ptr(), dWt.data_ptr(), dgamma.data_ptr(),
                           dbeta.data_ptr(), B, (int)H, (int)S, (uint64_t)seed, (uint64_t)offset, dp.first, dp.second,
                           dt_code(sv.scalar_type()), dt_code(gamma.scalar_type()), cur_stream()),
        "embed_ln_bwd");
  return {ds, dWp, dWt, dgamma, dbeta};
}

// dW [vocab, H]: zero rows, plus the ds rows of every token summed into its id's row
Tensor k_embed_segsum(Tensor ds, Tensor sorted_ids, Tensor perm, int64_t vocab, const c10::optional<Tensor>& out) {
  TORCH_CHECK(ds.is_contiguous() && sorted_ids.scalar_type() == at::kInt && perm.scalar_type() == at::kLong &&
                  sorted_ids.is_contiguous() && perm.is_contiguous() && sorted_ids.numel() == perm.numel(),
              "embed_segsum: int32 sorted ids, int64 permutation");
  const int64_t H = ds.size(-1), R = ds.numel() / H;
  TORCH_CHECK(sorted_ids.numel() == R, "embed_segsum: one id per ds row");
  Tensor dW = out_or_empty(out, {vocab, H}, ds.options(), "embed_segsum");
  dW.zero_();
  check(apex::embed_segsum(ds.data_ptr(), sorted_ids.data_ptr<int>(), perm.data_ptr<int64_t>(), dW.data_ptr(), R,
                           (int)H, dt_code(ds.scalar_type()), cur_stream()),
        "embed_segsum");
  return dW;
}

// --------------------------------------------------------------------------
// weight norm: v viewed as [R, C]; row_mode: one norm per row (dim=0), else per column
// --------------------------------------------------------------------------
std::vector<Tensor> k_wn_fwd(Tensor v, Tensor g, bool row_mode) {
  Tensor vc = v.contiguous();
  const int64_t R = row_mode ? vc.size(0) : vc.numel() / vc.size(-1);
  const int64_t C = vc.numel() / std::max<int64_t>(R, 1);
  Tensor w = at::empty_like(vc);
  Tensor norms = at::empty({row_mode ? R : C}, vc.options().dtype(at::kFloat));
  Tensor gc = g.contiguous();
  check(apex::weight_norm_fwd(vc.data_ptr(), gc.data_ptr(), w.data_ptr(), norms.data_ptr<float>(), R, C,
                              row_mode, dt_code(vc.scalar_type()), dt_code(gc.scalar_type()), cur_stream()),
        "weight_norm_fwd");
  return {w, norms};
}

std::vector<Tensor> k_wn_bwd(Tensor dw, Tensor v, Tensor g, Tensor norms, bool row_mode) {
  Tensor vc = v.contiguous(), dwc = dw.contiguous(), gc = g.contiguous();
  const int64_t R = row_mode ? vc.size(0) : vc.numel() / vc.size(-1);
  const int64_t C = vc.numel() / std::max<int64_t>(R, 1);
  Tensor dv = at::empty_like(vc), dg = at::empty_like(gc);
  check(apex::weight_norm_bwd(dwc.data_ptr(), vc.data_ptr(), gc.data_ptr(), norms.data_ptr<float>(),
                              dv.data_ptr(), dg.data_ptr(), R, C, row_mode, dt_code(vc.scalar_type()),
                              dt_code(gc.scalar_type()), cur_stream()),
        "weight_norm_bwd");
  return {dv, dg};
}

// --------------------------------------------------------------------------
// RNN cells (gates precomputed by GEMMs): PyTorch gate order
// --------------------------------------------------------------------------
std::vector<Tensor> k_lstm_fwd(Tensor ig, const c10::optional<Tensor>& hg, const c10::optional<Tensor>& bih,
                               const c10::optional<Tensor>& bhh, Tensor cx) {
  Tensor igc = ig.contiguous(), cxc = cx.contiguous();
  const int64_t B = cxc.size(0), H = cxc.size(1);
  Tensor hy = at::empty_like(cxc), cy = at::empty_like(cxc);
  Tensor ws = at::empty({B * 5 * H}, cxc.options().dtype(at::kFloat));
  c10::optional<Tensor> hgc = hg.has_value() && hg->defined() ? c10::optional<Tensor>(hg->contiguous()) : c10::nullopt;
  check(apex::lstm_cell_fwd(igc.data_ptr(), opt_vptr(hgc), opt_vptr(bih), opt_vptr(bhh), cxc.data_ptr(),
                            hy.data_ptr(), cy.data_ptr(), ws.data_ptr<float>(), B, H,
                            dt_code(cxc.scalar_type()), cur_stream()),
        "lstm_cell_fwd");
  return {hy, cy, ws};
}

std::vector<Tensor> k_lstm_bwd(const c10::optional<Tensor>& dhy, const c10::optional<Tensor>& dcy, Tensor cx,
                               Tensor ws) {
  Tensor cxc = cx.contiguous();
  const int64_t B = cxc.size(0), H = cxc.size(1);
  Tensor dg = at::empty({B, 4 * H}, cxc.options()), dcx = at::empty_like(cxc);
  c10::optional<Tensor> a = dhy.has_value() && dhy->defined() ? c10::optional<Tensor>(dhy->contiguous()) : c10::nullopt;
  c10::optional<Tensor> c = dcy.has_value() && dcy->defined() ? c10::optional<Tensor>(dcy->contiguous()) : c10::nullopt;
  check(apex::lstm_cell_bwd(opt_vptr(a), opt_vptr(c), cxc.data_ptr(), ws.data_ptr<float>(), dg.data_ptr(),
                            dcx.data_ptr(), B, H, dt_code(cxc.scalar_type()), cur_stream()),
        "lstm_cell_bwd");
  return {dg, dcx};
}

std::vector<Tensor> k_gru_fwd(Tensor ig, Tensor hg, const c10::optional<Tensor>& bih,
                              const c10::optional<Tensor>& bhh, Tensor hx) {
  Tensor igc = ig.contiguous(), hgc = hg.contiguous(), hxc = hx.contiguous();
  const int64_t B = hxc.size(0), H = hxc.size(1);
  Tensor hy = at::empty_like(hxc);
  Tensor ws = at::empty({B * 4 * H}, hxc.options().dtype(at::kFloat));
  check(apex::gru_cell_fwd(igc.data_ptr(), hgc.data_ptr(), opt_vptr(bih), opt_vptr(bhh), hxc.data_ptr(),
                           hy.data_ptr(), ws.data_ptr<float>(), B, H, dt_code(hxc.scalar_type()), cur_stream()),
        "gru_cell_fwd");
  return {hy, ws};
}

std::vector<Tensor> k_gru_bwd(Tensor dhy, Tensor hx, Tensor ws) {
  Tensor hxc = hx.contiguous(), d = dhy.contiguous();
  const int64_t B = hxc.size(0), H = hxc.size(1);
  Tensor dig = at::empty({B, 3 * H}, hxc.options()), dhg = at::empty({B, 3 * H}, hxc.options());
  Tensor dhx = at::empty_like(hxc);
  check(apex::gru_cell_bwd(d.data_ptr(), hxc.data_ptr(), ws.data_ptr<float>(), dig.data_ptr(), dhg.data_ptr(),
                           dhx.data_ptr(), B, H, dt_code(hxc.scalar_type()), cur_stream()),
        "gru_cell_bwd");
  return {dig, dhg, dhx};
}

// --------------------------------------------------------------------------
// SyncBatchNorm: x viewed as [N, C, S] (NCHW) or [N, S, C] (nhwc)
// --------------------------------------------------------------------------
std::vector<int64_t> bn_dims(const Tensor& x, bool nhwc) {
  const int64_t N = x.size(0);
  const int64_t C = nhwc ? x.size(-1) : x.size(1);
  const int64_t S = x.numel() / std::max<int64_t>(N * C, 1);
  return {N, C, S};
}

static Tensor bn_partials(const Tensor& x, bool nhwc, int* spo) {
  TORCH_CHECK(x.is_contiguous(), "syncbn: input must be contiguous in its layout");
  auto d = bn_dims(x, nhwc);
  const int sp = apex::bn_splits_for(d[0], d[1], d[2], nhwc, dt_code(x.scalar_type()));
  Tensor part = at::empty({d[1] * sp * 3}, x.options().dtype(at::kFloat));
  check(apex::bn_stats(x.data_ptr(), part.data_ptr<float>(), d[0], d[1], d[2], nhwc, dt_code(x.scalar_type()),
                       spo, cur_stream()),
        "bn_stats");
  return part;
}

static void check_running(const c10::optional<Tensor>& rm, const c10::optional<Tensor>& rv, int64_t C) {
  TORCH_CHECK(rv.has_value() && rv->defined() && rm->scalar_type() == at::kFloat && rv->scalar_type() == at::kFloat &&
                  rm->is_contiguous() && rv->is_contiguous() && rm->numel() == C && rv->numel() == C,
              "syncbn: fp32 contiguous [C] running statistics");
}

// local per-channel (mean, m2, count) triples [C, 3], written by the combine kernel itself
Tensor k_bn_local_stats(Tensor x, bool nhwc) {
  int spo = 0;
  Tensor part = bn_partials(x, nhwc, &spo);
  const int64_t C = bn_dims(x, nhwc)[1];
  Tensor out = at::empty({C, 3}, x.options().dtype(at::kFloat));
  check(apex::bn_combine(part.data_ptr<float>(), spo, C, 0, nullptr, nullptr, nullptr, cur_stream(), nullptr, 0.f,
                         nullptr, nullptr, 0.f, out.data_ptr<float>()),
        "bn_combine");
  return out;
}

// Single-process statistics in two launches: partial Welford reduce, then one combine that writes
// mean / biased var / count / invstd, updates the fp32 running statistics (unbiased variance) and
// bumps num_batches_tracked — the whole forward prologue of a BatchNorm layer.
std::vector<Tensor> k_bn_stats(Tensor x, bool nhwc, double eps, const c10::optional<Tensor>& running_mean,
                               const c10::optional<Tensor>& running_var, double momentum,
                               const c10::optional<Tensor>& num_batches_tracked) {
  int spo = 0;
  Tensor part = bn_partials(x, nhwc, &spo);
  const int64_t C = bn_dims(x, nhwc)[1];
  auto fo = x.options().dtype(at::kFloat);
  Tensor mean = at::empty({C}, fo), var = at::empty({C}, fo), cnt = at::empty({C}, fo), inv = at::empty({C}, fo);
  const bool upd = running_mean.has_value() && running_mean->defined();
  if (upd) check_running(running_mean, running_var, C);
  int64_t* nt = nullptr;
  if (num_batches_tracked.has_value() && num_batches_tracked->defined()) {
    TORCH_CHECK(num_batches_tracked->scalar_type() == at::kLong && num_batches_tracked->numel() == 1 &&
                    num_batches_tracked->device() == x.device(),
                "syncbn: num_batches_tracked must be a one-element int64 tensor on the input's device");
    nt = num_batches_tracked->data_ptr<int64_t>();
  }
  check(apex::bn_combine(part.data_ptr<float>(), spo, C, 0, mean.data_ptr<float>(), var.data_ptr<float>(),
                         cnt.data_ptr<float>(), cur_stream(), inv.data_ptr<float>(), (float)eps,
                         upd ? running_mean->data_ptr<float>() : nullptr,
                         upd ? running_var->data_ptr<float>() : nullptr, (float)momentum, nullptr, nt),
        "bn_combine");
  return {mean, var, cnt, inv};
}

// gathered [G, C, 3] -> (mean, biased var, count)
// eps >= 0: also return invstd; running_mean / running_var (fp32, contiguous): updated in place with
// `momentum` by the same kernel (one launch for the whole post-combine tail of a BatchNorm layer)
std::vector<Tensor> k_bn_combine(Tensor gathered, double eps, const c10::optional<Tensor>& running_mean,
                                 const c10::optional<Tensor>& running_var, double momentum) {
  Tensor g = gathered.contiguous();
  const int groups = (int)g.size(0);
  const int64_t C = g.size(1);
  auto fo = g.options().dtype(at::kFloat);
  Tensor mean = at::empty({C}, fo), var = at::empty({C}, fo), cnt = at::empty({C}, fo);
  Tensor invstd = eps >= 0.0 ? at::empty({C}, fo) : Tensor();
  const bool upd = running_mean.has_value() && running_mean->defined();
  if (upd) check_running(running_mean, running_var, C);
  check(apex::bn_combine(g.data_ptr<float>(), groups, C, 1, mean.data_ptr<float>(), var.data_ptr<float>(),
                         cnt.data_ptr<float>(), cur_stream(), invstd.defined() ? invstd.data_ptr<float>() : nullptr,
                         (float)std::max(eps, 0.0), upd ? running_mean->data_ptr<float>() : nullptr,
                         upd ? running_var->data_ptr<float>() : nullptr, (float)momentum),
        "bn_combine");
  return {mean, var, cnt, invstd};
}

// z: optional residual added after the affine, before the ReLU (same shape / layout as x)
Tensor k_bn_elemt(Tensor x, Tensor mean, Tensor invstd, const c10::optional<Tensor>& w,
                  const c10::optional<Tensor>& b, bool nhwc, bool relu, const c10::optional<Tensor>& z) {
  auto d = bn_dims(x, nhwc);
  Tensor zc;
  if (z.has_value() && z->defined()) {
    zc = z->contiguous();
    TORCH_CHECK(zc.sizes() == x.sizes() && zc.scalar_type() == x.scalar_type(), "bn_elemt: z like x");
  }
  Tensor y = at::empty_like(x);
  const int wdt = w.has_value() && w->defined() ? dt_code(w->scalar_type()) : apex::kF32Code;
  Tensor coef = at::empty({2 * d[1] + 4}, x.options().dtype(at::kFloat));
  check(apex::bn_elemt(x.data_ptr(), mean.data_ptr<float>(), invstd.data_ptr<float>(), opt_vptr(w), opt_vptr(b),
                       zc.defined() ? zc.data_ptr() : nullptr, y.data_ptr(), d[0], d[1], d[2], nhwc, relu, dt_code(x.scalar_type()), wdt,
                       coef.data_ptr<float>(), cur_stream()),
        "bn_elemt");
  return y;
}

// local (sum_dy, sum_dy_xmu) -> [2, C]
// ym: optional forward output of a fused-ReLU bn_elemt (the gradient counts only where ym > 0)
Tensor k_bn_bwd_reduce(Tensor dy, Tensor x, Tensor mean, bool nhwc, const c10::optional<Tensor>& ym) {
  auto d = bn_dims(x, nhwc);
  Tensor dyc = dy.contiguous();
  Tensor yc;
  if (ym.has_value() && ym->defined()) {
    yc = ym->contiguous();
    TORCH_CHECK(yc.sizes() == x.sizes() && yc.scalar_type() == x.scalar_type(), "bn_bwd_reduce: ym like x");
  }
  const int sp = apex::bn_splits_for(d[0], d[1], d[2], nhwc, dt_code(x.scalar_type()));
  auto fo = x.options().dtype(at::kFloat);
  Tensor part = at::empty({d[1] * sp * 2}, fo);
  Tensor out = at::empty({2, d[1]}, fo);
  check(apex::bn_bwd_reduce(dyc.data_ptr(), x.data_ptr(), yc.defined() ? yc.data_ptr() : nullptr,
                            mean.data_ptr<float>(), part.data_ptr<float>(),
                            out.data_ptr<float>(), out.data_ptr<float>() + d[1], d[0], d[1], d[2], nhwc,
                            dt_code(x.scalar_type()), cur_stream()),
        "bn_bwd_reduce");
  return out;
}

// ym: as k_bn_bwd_reduce; with_dz: also return the masked gradient (the fused residual's gradient)
std::vector<Tensor> k_bn_bwd_elemt(Tensor dy, Tensor x, Tensor mean, Tensor invstd, const c10::optional<Tensor>& w,
                                   Tensor sums, Tensor count, bool nhwc, const c10::optional<Tensor>& ym,
                                   bool with_dz) {
  auto d = bn_dims(x, nhwc);
  TORCH_CHECK(count.is_cuda() && count.scalar_type() == at::kFloat && count.numel() == d[1] && count.is_contiguous(),
              "bn_bwd_elemt: count must be the fp32 [C] device tensor from bn_combine");
  Tensor dyc = dy.contiguous();
  Tensor dx = at::empty_like(x);
  Tensor sc = sums.contiguous();
  Tensor yc, dz;
  if (ym.has_value() && ym->defined()) {
    yc = ym->contiguous();
    TORCH_CHECK(yc.sizes() == x.sizes() && yc.scalar_type() == x.scalar_type(), "bn_bwd_elemt: ym like x");
  }
  TORCH_CHECK(!with_dz || yc.defined(), "bn_bwd_elemt: with_dz needs ym");
  if (with_dz) dz = at::empty_like(x);
  Tensor coef = at::empty({3 * d[1] + 4}, x.options().dtype(at::kFloat));
  const int wdt = w.has_value() && w->defined() ? dt_code(w->scalar_type()) : apex::kF32Code;
  check(apex::bn_bwd_elemt(dyc.data_ptr(), x.data_ptr(), mean.data_ptr<float>(), invstd.data_ptr<float>(),
                           opt_vptr(w), sc.data_ptr<float>(), sc.data_ptr<float>() + d[1],
                           count.data_ptr<float>(), yc.defined() ? yc.data_ptr() : nullptr,
                           with_dz ? dz.data_ptr() : nullptr, dx.data_ptr(), d[0], d[1], d[2], nhwc,
                           dt_code(x.scalar_type()), wdt, coef.data_ptr<float>(), cur_stream()),
        "bn_bwd_elemt");
  return {dx, dz};
}

// --------------------------------------------------------------------------
// fused scale-mask softmax: x [..., sq, sk] (batch*heads flattened), mask uint8 [B, 1|H, sq, sk]
// --------------------------------------------------------------------------
bool k_smx_supported(int64_t cols) { return apex::scaled_softmax_supported((int)cols) != 0; }

Tensor k_smx_fwd(Tensor x, const c10::optional<Tensor>& mask, double scale, int64_t mode, int64_t heads) {
  TORCH_CHECK(x.is_contiguous() && x.dim() >= 2, "scaled_masked_softmax: contiguous input");
  const int64_t cols = x.size(-1), sq = x.size(-2);
  const int64_t rows = x.numel() / cols;
  Tensor y = at::empty_like(x);
  const uint8_t* mp = nullptr;
  int mask_heads = 1;
  if (mode == 1) {
    TORCH_CHECK(mask.has_value() && mask->defined() && mask->is_contiguous(), "mask required");
    TORCH_CHECK(mask->size(-1) == cols && mask->size(-2) == sq, "mask shape mismatch");
    mp = (const uint8_t*)mask->data_ptr();
    mask_heads = (int)mask->size(1);
  }
  check(apex::scaled_masked_softmax_fwd(x.data_ptr(), mp, y.data_ptr(), rows, (int)cols, (int)sq, (int)heads,
                                        mask_heads, (float)scale, (int)mode, dt_code(x.scalar_type()),
                                        cur_stream()),
        "scaled_masked_softmax_fwd");
  return y;
}

Tensor k_smx_bwd(Tensor dy, Tensor y, double scale) {
  Tensor dyc = dy.contiguous();
  const int64_t cols = y.size(-1), rows = y.numel() / cols;
  Tensor dx = at::empty_like(y);
  check(apex::scaled_masked_softmax_bwd(dyc.data_ptr(), y.data_ptr(), dx.data_ptr(), rows, (int)cols,
                                        (float)scale, dt_code(y.scalar_type()), cur_stream()),
        "scaled_masked_softmax_bwd");
  return dx;
}

// context parallelism: fused log-sum-exp merge of one ring-attention block into the fp32 accumulator
// acc_o [B, Sa, H, D] / acc_lse [B, H, Sa] fp32 contiguous; the block o [B, S, H, D] / lse [B, H, S]
// merges into accumulator rows s0 .. s0 + S
void k_lse_merge(Tensor acc_o, Tensor acc_lse, Tensor o, Tensor lse, bool first, int64_t s0) {
  TORCH_CHECK(acc_o.is_cuda() && acc_o.scalar_type() == at::kFloat && acc_o.is_contiguous() && acc_o.dim() == 4,
              "lse_merge: acc_o fp32 [B,S,H,D] contiguous");
  TORCH_CHECK(acc_lse.scalar_type() == at::kFloat && acc_lse.is_contiguous() && lse.scalar_type() == at::kFloat &&
                  lse.is_contiguous(),
              "lse_merge: fp32 contiguous lse");
  TORCH_CHECK(o.is_contiguous() && o.dim() == 4 && o.size(0) == acc_o.size(0) && o.size(2) == acc_o.size(2) &&
                  o.size(3) == acc_o.size(3) && s0 >= 0 && s0 + o.size(1) <= acc_o.size(1),
              "lse_merge: o [B, S, H, D] contiguous, rows s0 .. s0 + S of acc_o");
  const int64_t B = o.size(0), S = o.size(1), H = o.size(2), D = o.size(3), Sa = acc_o.size(1);
  TORCH_CHECK(acc_lse.numel() == B * H * Sa && lse.numel() == B * H * S, "lse_merge: lse [B,H,S]");
  check(apex::lse_merge(acc_o.data_ptr<float>(), acc_lse.data_ptr<float>(), o.data_ptr(), lse.data_ptr<float>(), B,
                        (int)S, (int)H, (int)D, first ? 1 : 0, dt_code(o.scalar_type()), cur_stream(), (int)Sa,
                        (int)s0),
        "lse_merge");
}

Tensor flash_dropout_mask(int64_t B, int64_t H, int64_t Sq, int64_t Sk, double p_drop, int64_t seed,
                          int64_t offset, at::Device dev) {
  Tensor out = at::empty({B, H, Sq, Sk}, at::TensorOptions().dtype(at::kByte).device(dev));
  const uint32_t th = apex::attn_drop_thresh(p_drop);
  check(apex::attn_dropout_mask(out.data_ptr<uint8_t>(), B * H, (int)Sq, (int)Sk, (uint64_t)seed,
                                (uint64_t)offset, th, cur_stream()),
        "attn_dropout_mask");
  return out;
}

// --------------------------------------------------------------------------
// K-09 input normalisation: x uint8 [B,H,W,C] (nhwc_in) or [B,C,H,W]; returns the normalised
// tensor in `out_dtype`, NCHW-contiguous (channels_last=false) or channels_last.
// --------------------------------------------------------------------------
Tensor k_input_normalize(Tensor x, std::vector<double> mean, std::vector<double> stdv, bool nhwc_in,
                         bool channels_last, at::ScalarType out_dtype) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kByte && x.dim() == 4, "input_normalize: uint8 4-D cuda");
  Tensor xc = x.contiguous();
  const int64_t B = xc.size(0);
  const int64_t C = nhwc_in ? xc.size(3) : xc.size(1);
  const int64_t H = nhwc_in ? xc.size(1) : xc.size(2), W = nhwc_in ? xc.size(2) : xc.size(3);
  TORCH_CHECK((int64_t)mean.size() == C && (int64_t)stdv.size() == C, "mean/std need one value per channel");
  TORCH_CHECK(!(channels_last && !nhwc_in), "NCHW uint8 input -> channels_last output is not supported");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(xc.data_ptr()) % 16 == 0, "input must be 16-byte aligned");
  auto opts = xc.options().dtype(out_dtype);
  Tensor y = channels_last ? at::empty({B, C, H, W}, opts.memory_format(at::MemoryFormat::ChannelsLast))
                           : at::empty({B, C, H, W}, opts);
  float m[4], sd[4];
  for (int64_t c = 0; c < C && c < 4; ++c) {
    m[c] = (float)mean[c];
    sd[c] = (float)stdv[c];
  }
  const int layout = nhwc_in ? (channels_last ? 0 : 1) : 2;
  const int rc = apex::input_normalize((const uint8_t*)xc.data_ptr(), y.data_ptr(), B, C, H * W, layout, m, sd,
                                       dt_code(out_dtype), cur_stream());
  TORCH_CHECK(rc != 1, "input_normalize: unsupported geometry (C<=4; NHWC->NCHW needs H*W % 8 == 0)");
  check(rc, "input_normalize");
  return y;
}

// ---------------------------------------------------------------------------
// MFMA GEMM (gemm.hip): C = epi(A[M,K] . B[N,K]^T). Returns [C, H] (H: pre-activation for
// EPI_BIAS_GELU, gelu'(H) for EPI_BIAS_GELU_D) or [C, dbias] (EPI_DGELU, EPI_MUL). A may be any [..., K] view with a unit inner stride.
// ---------------------------------------------------------------------------
bool k_gemm_supported(Tensor a, Tensor b) {
  if (!a.is_cuda() || a.dim() < 2 || b.dim() != 2 || a.scalar_type() != b.scalar_type()) return false;
  if (a.scalar_type() != at::kBFloat16 && a.scalar_type() != at::kHalf) return false;
  if (a.stride(-1) != 1 || b.stride(1) != 1) return false;
  const int64_t K = a.size(-1), N = b.size(0);
  const int64_t M = a.numel() / std::max<int64_t>(K, 1);
  if (b.size(1) != K || M >= (1ll << 31) || N >= (1ll << 31)) return false;
  // rows of A must be evenly strided when A is viewed as [M, K]
  if (a.dim() > 2 && !a.is_contiguous()) return false;
  const int64_t lda = a.dim() == 2 ? a.stride(0) : K;
  auto al = [](const Tensor& t) { return reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0; };
  return al(a) && al(b) && apex::gemm_supported((int)M, (int)N, (int)K, lda, b.stride(0), N);
}

std::vector<Tensor> k_gemm(Tensor a, Tensor b, int64_t epi, const c10::optional<Tensor>& bias,
                           const c10::optional<Tensor>& aux, c10::optional<at::ScalarType> bias_grad_dtype,
                           const c10::optional<Tensor>& bias_grad_out) {
  TORCH_CHECK(k_gemm_supported(a, b), "gemm: unsupported operands (bf16/fp16, K % 64 == 0, N % 8 == 0, "
              "16-byte aligned, unit inner stride)");
  const int64_t K = a.size(-1), N = b.size(0), M = a.numel() / K;
  const int64_t lda = a.dim() == 2 ? a.stride(0) : K;
  std::vector<int64_t> osz(a.sizes().begin(), a.sizes().end());
  osz.back() = N;
  Tensor c = at::empty(osz, a.options());
  apex::GemmArgs g{};
  g.A = a.data_ptr();
  g.B = b.data_ptr();
  g.C = c.data_ptr();
  g.M = (int)M;
  g.N = (int)N;
  g.K = (int)K;
  g.lda = lda;
  g.ldb = b.stride(0);
  g.ldc = N;
  g.epi = (int)epi;
  Tensor extra;
  const bool gelu_fwd = epi == apex::EPI_BIAS_GELU || epi == apex::EPI_BIAS_GELU_TANH ||
                        epi == apex::EPI_BIAS_GELU_D || epi == apex::EPI_BIAS_GELU_TANH_D;
  const bool dgelu = epi == apex::EPI_DGELU || epi == apex::EPI_DGELU_TANH || epi == apex::EPI_MUL;
  TORCH_CHECK(epi >= 0 && epi <= apex::EPI_MUL && epi != apex::EPI_F32, "gemm: bad epilogue ", epi);
  if (epi == apex::EPI_BIAS || gelu_fwd) {
    TORCH_CHECK(bias.has_value() && bias->defined() && bias->is_contiguous() && bias->numel() == N &&
                    bias->scalar_type() == a.scalar_type(),
                "gemm: bias must be a contiguous [N] tensor of the operand dtype");
    g.bias = bias->data_ptr();
  }
  if (gelu_fwd) {
    extra = at::empty(osz, a.options());
    g.aux_out = extra.data_ptr();
  }
  Tensor part;
  if (dgelu || epi == apex::EPI_RESID) {
    TORCH_CHECK(aux.has_value() && aux->defined() && aux->scalar_type() == a.scalar_type() &&
                    aux->numel() == M * N && aux->stride(-1) == 1 && aux->is_contiguous(),
                "gemm: aux must be a contiguous [M, N] tensor of the operand dtype");
    g.aux = aux->data_ptr();
    g.ldaux = N;
  }
  if (dgelu) {
    part = at::empty({apex::gemm_part_rows((int)M), N}, a.options().dtype(at::kFloat));
    g.part = part.data_ptr<float>();
  }
  check(apex::gemm_nt(g, dt_code(a.scalar_type()), cur_stream()), "gemm");
  if (dgelu && bias_grad_dtype.has_value()) {
    extra = out_or_empty(bias_grad_out, {N}, a.options().dtype(*bias_grad_dtype), "gemm bias grad");
    check(apex::gemm_bias_grad(part.data_ptr<float>(), (int)part.size(0), (int)N, extra.data_ptr(),
                               dt_code(*bias_grad_dtype), cur_stream()),
          "gemm_bias_grad");
  }
  return {c, extra};
}

// ---------------------------------------------------------------------------
// FP8 (gemm.hip fp8 path + fp8.hip): a8 [..., K] / b8 [N, K] uint8 e4m3|e5m2 codes, alpha_a /
// alpha_b fp32 device scalars (the inverse quantisation scales); output in out_dtype
// ---------------------------------------------------------------------------
void f8_check_scalar(const Tensor& t, const char* what) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kFloat && t.numel() >= 1, what, " must be an fp32 device scalar");
}

bool k_gemm_f8_supported(Tensor a, Tensor b) {
  if (!a.is_cuda() || a.dim() < 2 || b.dim() != 2 || a.scalar_type() != at::kByte || b.scalar_type() != at::kByte)
    return false;
  if (a.stride(-1) != 1 || b.stride(1) != 1) return false;
  const int64_t K = a.size(-1), N = b.size(0);
  const int64_t M = a.numel() / std::max<int64_t>(K, 1);
  if (b.size(1) != K || M >= (1ll << 31) || N >= (1ll << 31)) return false;
  if (a.dim() > 2 && !a.is_contiguous()) return false;
  const int64_t lda = a.dim() == 2 ? a.stride(0) : K;
  auto al = [](const Tensor& t) { return reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0; };
  return al(a) && al(b) && apex::gemm_f8_supported((int)M, (int)N, (int)K, lda, b.stride(0), N);
}

std::vector<Tensor> k_gemm_f8(Tensor a, Tensor b, Tensor alpha_a, Tensor alpha_b, int64_t fmt_a, int64_t epi,
                              const c10::optional<Tensor>& bias, const c10::optional<Tensor>& aux,
                              c10::optional<at::ScalarType> bias_grad_dtype, at::ScalarType out_dtype,
                              const c10::optional<Tensor>& q8_out, const c10::optional<Tensor>& q8_scale,
                              const c10::optional<Tensor>& q8_amax, int64_t q8_fmt, bool q8_only) {
  TORCH_CHECK(k_gemm_f8_supported(a, b), "gemm_f8: unsupported operands (uint8 codes, K % 128 == 0, N % 8 == 0, "
              "16-byte aligned, unit inner stride)");
  TORCH_CHECK(out_dtype == at::kBFloat16 || out_dtype == at::kHalf, "gemm_f8: bf16 / fp16 output");
  f8_check_scalar(alpha_a, "alpha_a");
  f8_check_scalar(alpha_b, "alpha_b");
  const int64_t K = a.size(-1), N = b.size(0), M = a.numel() / K;
  std::vector<int64_t> osz(a.sizes().begin(), a.sizes().end());
  osz.back() = N;
  auto oopt = a.options().dtype(out_dtype);
  Tensor c = at::empty(osz, oopt);
  apex::GemmArgs g{};
  g.A = a.data_ptr();
  g.B = b.data_ptr();
  g.C = c.data_ptr();
  g.M = (int)M;
  g.N = (int)N;
  g.K = (int)K;
  g.lda = a.dim() == 2 ? a.stride(0) : K;
  g.ldb = b.stride(0);
  g.ldc = N;
  g.epi = (int)epi;
  g.alpha_a = alpha_a.data_ptr<float>();
  g.alpha_b = alpha_b.data_ptr<float>();
  Tensor extra, part;
  const bool gelu_fwd = epi == apex::EPI_BIAS_GELU || epi == apex::EPI_BIAS_GELU_TANH ||
                        epi == apex::EPI_BIAS_GELU_D || epi == apex::EPI_BIAS_GELU_TANH_D;
  const bool mul = epi == apex::EPI_DGELU || epi == apex::EPI_DGELU_TANH || epi == apex::EPI_MUL;
  TORCH_CHECK(epi >= 0 && epi <= apex::EPI_MUL && epi != apex::EPI_F32, "gemm_f8: bad epilogue ", epi);
  if (epi == apex::EPI_BIAS || gelu_fwd) {
    TORCH_CHECK(bias.has_value() && bias->defined() && bias->is_contiguous() && bias->numel() == N &&
                    bias->scalar_type() == out_dtype, "gemm_f8: bias must be a contiguous [N] tensor of out_dtype");
    g.bias = bias->data_ptr();
  }
  if (gelu_fwd) {
    extra = at::empty(osz, oopt);
    g.aux_out = extra.data_ptr();
  }
  if (mul || epi == apex::EPI_RESID) {
    TORCH_CHECK(aux.has_value() && aux->defined() && aux->scalar_type() == out_dtype && aux->numel() == M * N &&
                    aux->is_contiguous(), "gemm_f8: aux must be a contiguous [M, N] tensor of out_dtype");
    g.aux = aux->data_ptr();
    g.ldaux = N;
  }
  if (mul) {
    part = at::empty({apex::gemm_part_rows((int)M), N}, a.options().dtype(at::kFloat));
    g.part = part.data_ptr<float>();
  }
  g.q8 = q8_args(q8_out, q8_scale, q8_amax, q8_fmt, c, "gemm_f8");
  TORCH_CHECK(!g.q8.y || gelu_fwd || mul, "gemm_f8: q8_out needs a GELU / dGELU / MUL epilogue");
  // q8_only: the returned C is allocated but (on the kernels that honour it: bias+GELU+derivative and
  // multiply, full 256x256 tiles) never written — the caller promises that only the codes are read
  TORCH_CHECK(!q8_only || g.q8.y, "gemm_f8: q8_only needs q8_out");
  g.q8.only = q8_only ? 1 : 0;
  check(apex::gemm_nt_f8(g, (int)fmt_a, 0, dt_code(out_dtype), cur_stream()), "gemm_f8");
  if (mul && bias_grad_dtype.has_value()) {
    extra = at::empty({N}, a.options().dtype(*bias_grad_dtype));
    check(apex::gemm_bias_grad(part.data_ptr<float>(), (int)part.size(0), (int)N, extra.data_ptr(),
                               dt_code(*bias_grad_dtype), cur_stream()), "gemm_bias_grad");
  }
  return {c, extra};
}

struct F8Opt {
  float* amax = nullptr;
  const float* cur = nullptr;
  float* scale_inv = nullptr;
};

F8Opt f8_opts(const c10::optional<Tensor>& amax, const c10::optional<Tensor>& cur_amax,
              const c10::optional<Tensor>& scale_inv, double smax) {
  F8Opt o;
  if (amax.has_value() && amax->defined()) {
    f8_check_scalar(*amax, "amax");
    o.amax = amax->data_ptr<float>();
  }
  if (cur_amax.has_value() && cur_amax->defined()) {
    f8_check_scalar(*cur_amax, "cur_amax");
    TORCH_CHECK(scale_inv.has_value() && scale_inv->defined() && smax > 0,
                "fp8 current scaling needs scale_inv and smax > 0");
    o.cur = cur_amax->data_ptr<float>();
  }
  if (scale_inv.has_value() && scale_inv->defined()) {
    f8_check_scalar(*scale_inv, "scale_inv");
    o.scale_inv = scale_inv->data_ptr<float>();
  }
  return o;
}

// delayed scaling: quantise with scale (and fold max|x| into amax); current scaling: cur_amax holds
// max|x| already, scale / scale_inv are written (= smax / cur_amax and its inverse)
Tensor k_fp8_quantize(Tensor x, int64_t fmt, Tensor scale, const c10::optional<Tensor>& amax,
                      const c10::optional<Tensor>& cur_amax, const c10::optional<Tensor>& scale_inv, double smax) {
  TORCH_CHECK(x.is_cuda() && x.is_contiguous(), "fp8_quantize: contiguous device tensor");
  f8_check_scalar(scale, "scale");
  const F8Opt o = f8_opts(amax, cur_amax, scale_inv, smax);
  Tensor y = at::empty(x.sizes(), x.options().dtype(at::kByte));
  check(apex::fp8_quantize(x.data_ptr(), y.data_ptr<uint8_t>(), x.numel(), dt_code(x.scalar_type()), (int)fmt,
                           scale.data_ptr<float>(), o.scale_inv, o.amax, o.cur, (float)smax, cur_stream()),
        "fp8_quantize");
  return y;
}

Tensor k_fp8_quantize_t(Tensor x, int64_t fmt, Tensor scale, const c10::optional<Tensor>& amax,
                        const c10::optional<Tensor>& cur_amax, const c10::optional<Tensor>& scale_inv, double smax) {
  TORCH_CHECK(x.is_cuda() && x.is_contiguous() && x.dim() == 2, "fp8_quantize_t: contiguous 2-D device tensor");
  f8_check_scalar(scale, "scale");
  const F8Opt o = f8_opts(amax, cur_amax, scale_inv, smax);
  Tensor y = at::empty({x.size(1), x.size(0)}, x.options().dtype(at::kByte));
  check(apex::fp8_quantize_t(x.data_ptr(), y.data_ptr<uint8_t>(), (int)x.size(0), (int)x.size(1),
                             dt_code(x.scalar_type()), (int)fmt, scale.data_ptr<float>(), o.scale_inv, o.amax, o.cur,
                             (float)smax, cur_stream()),
        "fp8_quantize_t");
  return y;
}

// one step's weights through the batched current-scaling quantiser: per weight the e4m3 codes
// of W and (want_t) of W^T, scale / scale_inv / amax written at its slot -> [y0, yt0, y1, yt1, ...]
// (yt empty when not wanted)
std::vector<Tensor> k_fp8_quantize_weights(const std::vector<Tensor>& ws, const std::vector<int64_t>& slots,
                                           const std::vector<bool>& want_t, int64_t fmt, Tensor scale,
                                           Tensor scale_inv, Tensor amax, double smax) {
  const size_t n = ws.size();
  TORCH_CHECK(slots.size() == n && want_t.size() == n, "fp8_quantize_weights: one slot / flag per weight");
  TORCH_CHECK(scale.is_cuda() && scale.scalar_type() == at::kFloat && scale_inv.scalar_type() == at::kFloat &&
                  amax.scalar_type() == at::kFloat && scale.is_contiguous() && scale_inv.is_contiguous() &&
                  amax.is_contiguous(),
              "fp8_quantize_weights: fp32 contiguous slot buffers");
  std::vector<Tensor> out;
  out.reserve(2 * n);
  if (n == 0) return out;
  Tensor host = at::empty({(int64_t)(n * sizeof(apex::WqDesc))}, at::TensorOptions().dtype(at::kByte).pinned_memory(true));
  auto* d = reinterpret_cast<apex::WqDesc*>(host.data_ptr<uint8_t>());
  int64_t ab = 0, qb = 0;
  const int dt = dt_code(ws[0].scalar_type());
  for (size_t i = 0; i < n; ++i) {
    const Tensor& w = ws[i];
    TORCH_CHECK(w.is_cuda() && w.dim() == 2 && w.is_contiguous() && dt_code(w.scalar_type()) == dt &&
                    w.device() == scale.device(),
                "fp8_quantize_weights: contiguous 2-D device weights of one dtype");
    TORCH_CHECK(slots[i] >= 0 && slots[i] < scale.numel() && slots[i] < scale_inv.numel() && slots[i] < amax.numel(),
                "fp8_quantize_weights: slot out of range");
    const int64_t R = w.size(0), C = w.size(1);
    TORCH_CHECK(R > 0 && C > 0 && R < (1 << 30) && C < (1 << 30), "fp8_quantize_weights: weight shape");
    Tensor y = at::empty({R, C}, w.options().dtype(at::kByte));
    Tensor yt = want_t[i] ? at::empty({C, R}, w.options().dtype(at::kByte)) : at::empty({0}, w.options().dtype(at::kByte));
    d[i] = apex::WqDesc{w.data_ptr(), y.data_ptr<uint8_t>(), want_t[i] ? yt.data_ptr<uint8_t>() : nullptr, (int)R, (int)C,
                        (int)slots[i], 0, ab, qb};
    ab += (R * C + 65535) / 65536;
    qb += ((R + 63) / 64) * ((C + 63) / 64);
    out.push_back(y);
    out.push_back(yt);
  }
  Tensor dev = host.to(scale.device(), /*non_blocking=*/true);
  check(apex::fp8_quantize_weights(reinterpret_cast<const apex::WqDesc*>(dev.data_ptr<uint8_t>()), (int)n, ab, qb, dt,
                                   (int)fmt, scale.data_ptr<float>(), scale_inv.data_ptr<float>(), amax.data_ptr<float>(),
                                   (float)smax, cur_stream()),
        "fp8_quantize_weights");
  return out;
}

void k_fp8_amax(Tensor x, Tensor amax) {
  TORCH_CHECK(x.is_cuda() && x.is_contiguous(), "fp8_amax: contiguous device tensor");
  f8_check_scalar(amax, "amax");
  check(apex::fp8_amax(x.data_ptr(), x.numel(), dt_code(x.scalar_type()), amax.data_ptr<float>(), cur_stream()),
        "fp8_amax");
}

void k_fp8_update_scales(Tensor hist, Tensor amax_cur, Tensor scale, Tensor scale_inv, Tensor fmt_max, int64_t n_slots,
                         int64_t idx, double margin_scale) {
  TORCH_CHECK(hist.is_cuda() && hist.dim() == 2 && hist.is_contiguous() && hist.scalar_type() == at::kFloat,
              "fp8_update_scales: hist fp32 [slots, history]");
  TORCH_CHECK(n_slots <= hist.size(0) && idx >= 0 && idx < hist.size(1), "fp8_update_scales: bad slot count / index");
  check(apex::fp8_update_scales(hist.data_ptr<float>(), amax_cur.data_ptr<float>(), scale.data_ptr<float>(),
                                scale_inv.data_ptr<float>(), fmt_max.data_ptr<float>(), (int)n_slots,
                                (int)hist.size(1), (int)idx, (float)margin_scale, cur_stream()),
        "fp8_update_scales");
}

// weight gradient: out[P, Q] = a^T b for a [R, P], b [R, Q] (contraction over the R rows, split
// into `splits` slices whose fp32 partials are combined by splitk_reduce)
bool k_gemm_tt_supported(Tensor a, Tensor b, int64_t splits) {
  if (!a.is_cuda() || a.dim() != 2 || b.dim() != 2 || a.scalar_type() != b.scalar_type()) return false;
  if (a.scalar_type() != at::kBFloat16 && a.scalar_type() != at::kHalf) return false;
  if (!a.is_contiguous() || !b.is_contiguous() || a.size(0) != b.size(0)) return false;
  auto al = [](const Tensor& t) { return reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0; };
  return al(a) && al(b) && splits >= 1 &&
         apex::gemm_tt_supported((int)a.size(1), (int)b.size(1), (int)a.size(0), (int)splits, a.size(1), b.size(1));
}

Tensor k_gemm_tt(Tensor a, Tensor b, int64_t splits, at::ScalarType out_dtype, const c10::optional<Tensor>& out_opt) {
  TORCH_CHECK(k_gemm_tt_supported(a, b, splits), "gemm_tt: unsupported operands");
  const int64_t R = a.size(0), P = a.size(1), Q = b.size(1);
  apex::GemmArgs g{};
  g.A = a.data_ptr();
  g.B = b.data_ptr();
  g.M = (int)P;
  g.N = (int)Q;
  g.K = (int)R;  // all contraction rows: the kernel cuts them into `splits` slices of whole K-tiles
  g.lda = P;
  g.ldb = Q;
  g.ldc = Q;
  g.splits = (int)splits;
  Tensor out;
  if (splits == 1 && out_dtype == a.scalar_type() && !out_opt) {
    out = at::empty({P, Q}, a.options());
    g.C = out.data_ptr();
    g.epi = apex::EPI_NONE;
    check(apex::gemm_tt(g, dt_code(a.scalar_type()), cur_stream()), "gemm_tt");
    return out;
  }
  Tensor slabs = at::empty({splits, P, Q}, a.options().dtype(at::kFloat));
  g.part = slabs.data_ptr<float>();
  g.epi = apex::EPI_F32;
  check(apex::gemm_tt(g, dt_code(a.scalar_type()), cur_stream()), "gemm_tt");
  // (out given: the reduction writes the parameter's gradient-bucket slot directly)
  return k_splitk_reduce(slabs, out_dtype, out_opt);
}

// fp8 weight gradient: out[P, Q] = alpha_a alpha_b a^T b over uint8 codes a [R, P] (format fmt_a),
// b [R, Q] (fmt_b) — the codes the forward / backward GEMMs already consumed — split into `splits`
// slices of fp32 partials, combined (and rounded to out_dtype) by splitk_reduce
bool k_gemm_tt_f8_supported(Tensor a, Tensor b, int64_t splits) {
  if (!a.is_cuda() || a.dim() != 2 || b.dim() != 2 || a.scalar_type() != at::kByte || b.scalar_type() != at::kByte)
    return false;
  if (!a.is_contiguous() || !b.is_contiguous() || a.size(0) != b.size(0)) return false;
  auto al = [](const Tensor& t) { return reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0; };
  return al(a) && al(b) && splits >= 1 &&
         apex::gemm_tt_f8_supported((int)a.size(1), (int)b.size(1), (int)a.size(0), (int)splits, a.size(1), b.size(1));
}

Tensor k_gemm_tt_f8(Tensor a, Tensor b, Tensor alpha_a, Tensor alpha_b, int64_t fmt_a, int64_t fmt_b, int64_t splits,
                    at::ScalarType out_dtype, const c10::optional<Tensor>& out_opt) {
  TORCH_CHECK(k_gemm_tt_f8_supported(a, b, splits), "gemm_tt_f8: unsupported operands");
  TORCH_CHECK(alpha_a.is_cuda() && alpha_a.scalar_type() == at::kFloat && alpha_a.numel() >= 1 && alpha_b.is_cuda() &&
                  alpha_b.scalar_type() == at::kFloat && alpha_b.numel() >= 1,
              "gemm_tt_f8: alpha_a / alpha_b must be fp32 device scalars");
  const int64_t R = a.size(0), P = a.size(1), Q = b.size(1);
  apex::GemmArgs g{};
  g.A = a.data_ptr();
  g.B = b.data_ptr();
  g.M = (int)P;
  g.N = (int)Q;
  g.K = (int)R;  // all contraction rows: the kernel cuts them into `splits` slices of whole K-tiles
  g.lda = P;
  g.ldb = Q;
  g.ldc = Q;
  g.splits = (int)splits;
  g.alpha_a = alpha_a.data_ptr<float>();
  g.alpha_b = alpha_b.data_ptr<float>();
  Tensor slabs = at::empty({splits, P, Q}, a.options().dtype(at::kFloat));
  g.part = slabs.data_ptr<float>();
  g.epi = apex::EPI_F32;
  check(apex::gemm_tt_f8(g, (int)fmt_a, (int)fmt_b, cur_stream()), "gemm_tt_f8");
  return k_splitk_reduce(slabs, out_dtype, out_opt);
}

// out[P, Q] += a^T b in fp32 (a [R, P], b [R, Q] 16-bit, out fp32 contiguous): the weight gradient
// accumulated straight into an fp32 main_grad by the transposed-read MFMA kernel's
// read-modify-write epilogue — one launch, no slab, no 16-bit rounding of the micro-batch dW
void k_gemm_tt_acc(Tensor a, Tensor b, Tensor out) {
  TORCH_CHECK(k_gemm_tt_supported(a, b, 1), "gemm_tt_acc: unsupported operands");
  const int64_t P = a.size(1), Q = b.size(1);
  TORCH_CHECK(out.is_cuda() && out.scalar_type() == at::kFloat && out.is_contiguous() && out.dim() == 2 &&
                  out.size(0) == P && out.size(1) == Q && reinterpret_cast<uintptr_t>(out.data_ptr()) % 16 == 0,
              "gemm_tt_acc: out must be a contiguous fp32 [P, Q] tensor");
  apex::GemmArgs g{};
  g.A = a.data_ptr();
  g.B = b.data_ptr();
  g.M = (int)P;
  g.N = (int)Q;
  g.K = (int)a.size(0);
  g.lda = P;
  g.ldb = Q;
  g.ldc = Q;
  g.splits = 1;
  g.part = out.data_ptr<float>();
  g.epi = apex::EPI_F32_ACC;
  check(apex::gemm_tt(g, dt_code(a.scalar_type()), cur_stream()), "gemm_tt_acc");
}

// sum the rows of an fp32 [P, N] partials tensor -> [N] in out_dtype
Tensor k_partial_colsum(Tensor part, at::ScalarType out_dtype, const c10::optional<Tensor>& out_opt) {
  TORCH_CHECK(part.is_cuda() && part.scalar_type() == at::kFloat && part.dim() == 2 && part.is_contiguous(),
              "partial_colsum: contiguous fp32 [P, N]");
  Tensor out = out_or_empty(out_opt, {part.size(1)}, part.options().dtype(out_dtype), "partial_colsum");
  check(apex::gemm_bias_grad(part.data_ptr<float>(), (int)part.size(0), (int)part.size(1), out.data_ptr(),
                             dt_code(out_dtype), cur_stream()),
        "partial_colsum");
  return out;
}

Tensor k_transpose(Tensor x) {
  TORCH_CHECK(x.is_cuda() && x.dim() == 2, "transpose: 2-D device tensor");
  Tensor xc = x.contiguous();
  if (reinterpret_cast<uintptr_t>(xc.data_ptr()) % 16 != 0) xc = xc.clone();
  Tensor out = at::empty({xc.size(1), xc.size(0)}, xc.options());
  check(apex::transpose_2d(xc.data_ptr(), out.data_ptr(), (int)xc.size(0), (int)xc.size(1),
                           dt_code(xc.scalar_type()), cur_stream()),
        "transpose");
  return out;
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
  m.def("ln_bwd", &ln_bwd, py::arg("dy"), py::arg("x"), py::arg("cols"), py::arg("gamma"), py::arg("beta"),
        py::arg("mean"), py::arg("rstd"), py::arg("rms"), py::arg("dgamma_out") = py::none(),
        py::arg("dbeta_out") = py::none());
  m.def("xent_fwd", &xent_fwd);
  m.def("xent_bwd", &xent_bwd);
  m.def("gemm_f8_supported", &k_gemm_f8_supported);
  m.def("gemm_f8", &k_gemm_f8, py::arg("a"), py::arg("b"), py::arg("alpha_a"), py::arg("alpha_b"), py::arg("fmt_a"),
        py::arg("epi"), py::arg("bias") = py::none(), py::arg("aux") = py::none(),
        py::arg("bias_grad_dtype") = py::none(), py::arg("out_dtype") = at::kBFloat16, py::arg("q8_out") = py::none(),
        py::arg("q8_scale") = py::none(), py::arg("q8_amax") = py::none(), py::arg("q8_fmt") = 0,
        py::arg("q8_only") = false);
  m.def("fp8_quantize_weights", &k_fp8_quantize_weights, py::arg("weights"), py::arg("slots"), py::arg("want_t"),
        py::arg("fmt"), py::arg("scale"), py::arg("scale_inv"), py::arg("amax"), py::arg("smax"));
  m.def("fp8_quantize", &k_fp8_quantize, py::arg("x"), py::arg("fmt"), py::arg("scale"), py::arg("amax") = py::none(),
        py::arg("cur_amax") = py::none(), py::arg("scale_inv") = py::none(), py::arg("smax") = 0.0);
  m.def("fp8_quantize_t", &k_fp8_quantize_t, py::arg("x"), py::arg("fmt"), py::arg("scale"),
        py::arg("amax") = py::none(), py::arg("cur_amax") = py::none(), py::arg("scale_inv") = py::none(),
        py::arg("smax") = 0.0);
  m.def("fp8_amax", &k_fp8_amax);
  m.def("fp8_update_scales", &k_fp8_update_scales);
  m.def("flash_attn_fwd", &flash_attn_fwd, py::arg("q"), py::arg("k"), py::arg("v"), py::arg("causal"),
        py::arg("scale"), py::arg("p_drop"), py::arg("seed"), py::arg("offset"), py::arg("k_lens"),
        py::arg("bias") = py::none(), py::arg("q8_out") = py::none(), py::arg("q8_scale") = py::none(),
        py::arg("q8_amax") = py::none(), py::arg("q8_fmt") = 0);
  m.def("gemm_set_dbg", [](int64_t v) { check(apex::gemm_set_dbg((int)v), "gemm_set_dbg"); });
  // which = 0: 16-bit persistent GEMM, 1: fp8 persistent GEMM; v = 1 / 0 forces it on / off, -1 restores
  // the APEX_GEMM_PERSIST(_F8) choice; returns the previous forced value
  m.def("set_gemm_persist", [](int64_t which, int64_t v) { return (int64_t)apex::gemm_set_persist((int)which, (int)v); },
        py::arg("which"), py::arg("v"));
  m.def("flash_attn_bwd", &flash_attn_bwd, py::arg("dout"), py::arg("q"), py::arg("k"), py::arg("v"),
        py::arg("o"), py::arg("lse"), py::arg("dq"), py::arg("dk"), py::arg("dv"), py::arg("causal"),
        py::arg("scale"), py::arg("p_drop"), py::arg("seed"), py::arg("offset"), py::arg("k_lens"),
        py::arg("dmask"), py::arg("dsum") = py::none(), py::arg("dbg") = 0, py::arg("bias") = py::none(),
        py::arg("q8_dq") = py::none(), py::arg("q8_dk") = py::none(), py::arg("q8_dv") = py::none(),
        py::arg("q8_scale") = py::none(), py::arg("q8_amax") = py::none(), py::arg("q8_fmt") = 0,
        py::arg("dbias") = py::none(), py::arg("q8_only") = false);
  m.def("partial_colsum", &k_partial_colsum, py::arg("part"), py::arg("out_dtype"), py::arg("out") = py::none());
  m.def("flash_dropout_mask", &flash_dropout_mask);
  m.def("lse_merge", &k_lse_merge, py::arg("acc_o"), py::arg("acc_lse"), py::arg("o"), py::arg("lse"),
        py::arg("first"), py::arg("s0") = 0);
  m.def("weight_norm_fwd", &k_wn_fwd);
  m.def("weight_norm_bwd", &k_wn_bwd);
  m.def("lstm_cell_fwd", &k_lstm_fwd);
  m.def("lstm_cell_bwd", &k_lstm_bwd);
  m.def("gru_cell_fwd", &k_gru_fwd);
  m.def("gru_cell_bwd", &k_gru_bwd);
  m.def("bn_local_stats", &k_bn_local_stats);
  m.def("bn_stats", &k_bn_stats, py::arg("x"), py::arg("nhwc"), py::arg("eps"), py::arg("running_mean") = py::none(),
        py::arg("running_var") = py::none(), py::arg("momentum") = 0.0, py::arg("num_batches_tracked") = py::none());
  m.def("bn_combine", &k_bn_combine, py::arg("gathered"), py::arg("eps") = -1.0, py::arg("running_mean") = py::none(),
        py::arg("running_var") = py::none(), py::arg("momentum") = 0.0);
  m.def("bn_elemt", &k_bn_elemt, py::arg("x"), py::arg("mean"), py::arg("invstd"), py::arg("w"), py::arg("b"),
        py::arg("nhwc"), py::arg("relu"), py::arg("z") = py::none());
  m.def("bn_bwd_reduce", &k_bn_bwd_reduce, py::arg("dy"), py::arg("x"), py::arg("mean"), py::arg("nhwc"),
        py::arg("ym") = py::none());
  m.def("bn_bwd_elemt", &k_bn_bwd_elemt, py::arg("dy"), py::arg("x"), py::arg("mean"), py::arg("invstd"),
        py::arg("w"), py::arg("sums"), py::arg("count"), py::arg("nhwc"), py::arg("ym") = py::none(),
        py::arg("with_dz") = false);
  m.def("scaled_softmax_supported", &k_smx_supported);
  m.def("scaled_masked_softmax_fwd", &k_smx_fwd);
  m.def("scaled_masked_softmax_bwd", &k_smx_bwd);
  m.def("bias_act_fwd", &k_bias_act_fwd);
  m.def("bias_act_bwd", &k_bias_act_bwd);
  m.def("bias_dropout_add_fwd", &k_bda_fwd);
  m.def("bias_dropout_add_bwd", &k_bda_bwd, py::arg("dy"), py::arg("p"), py::arg("seed"), py::arg("offset"),
        py::arg("bias_like"), py::arg("dbias_out") = py::none());
  m.def("colsum", &k_colsum, py::arg("x"), py::arg("out_dtype"), py::arg("out") = py::none());
  m.def("splitk_reduce", &k_splitk_reduce, py::arg("slabs"), py::arg("out_dtype"), py::arg("out") = py::none(),
        py::arg("accumulate") = false);
  m.def("bdaln_supported", &k_bdaln_supported);
  m.def("bdaln_wide_supported", &k_bdaln_wide_supported);
  m.def("bdaln_fwd", &k_bdaln_fwd, py::arg("x"), py::arg("b"), py::arg("res"), py::arg("gamma"), py::arg("beta"),
        py::arg("eps"), py::arg("p"), py::arg("seed"), py::arg("offset"), py::arg("store_s") = true, py::arg("q8_out") = py::none(), py::arg("q8_scale") = py::none(),
        py::arg("q8_amax") = py::none(), py::arg("q8_fmt") = 0, py::arg("s_cond") = false);
  m.def("embed_ln_fwd", &k_embed_ln_fwd);
  m.def("embed_ln_bwd", &k_embed_ln_bwd, py::arg("dy"), py::arg("s"), py::arg("gamma"), py::arg("mean"),
        py::arg("rstd"), py::arg("tids"), py::arg("tvocab"), py::arg("npos"), py::arg("p"), py::arg("seed"),
        py::arg("offset"), py::arg("dwp_out") = py::none(), py::arg("dwt_out") = py::none(),
        py::arg("dgamma_out") = py::none(), py::arg("dbeta_out") = py::none());
  m.def("embed_segsum", &k_embed_segsum, py::arg("ds"), py::arg("sorted_ids"), py::arg("perm"), py::arg("vocab"),
        py::arg("out") = py::none());
  m.def("bdaln_bwd", &k_bdaln_bwd, py::arg("dy"), py::arg("s"), py::arg("gamma"), py::arg("mean"), py::arg("rstd"),
        py::arg("p"), py::arg("seed"), py::arg("offset"), py::arg("has_bias"), py::arg("dgamma_out") = py::none(),
        py::arg("dbeta_out") = py::none(), py::arg("dbias_out") = py::none(), py::arg("ds_extra") = py::none(),
        py::arg("beta") = py::none(), py::arg("q8_out") = py::none(), py::arg("q8_scale") = py::none(),
        py::arg("q8_amax") = py::none(), py::arg("q8_fmt") = 0, py::arg("s_alt") = py::none(),
        py::arg("q8_only") = false);
  m.def("input_normalize", &k_input_normalize);
  m.def("gemm_supported", &k_gemm_supported);
  m.def("gemm", &k_gemm, py::arg("a"), py::arg("b"), py::arg("epi") = 0, py::arg("bias") = py::none(),
        py::arg("aux") = py::none(), py::arg("bias_grad_dtype") = py::none(), py::arg("bias_grad_out") = py::none());
  m.def("transpose", &k_transpose);
  m.def("gemm_tt_supported", &k_gemm_tt_supported);
  m.def("gemm_tt", &k_gemm_tt, py::arg("a"), py::arg("b"), py::arg("splits"), py::arg("out_dtype"),
        py::arg("out") = py::none());
  m.def("gemm_tt_acc", &k_gemm_tt_acc);
  m.def("gemm_tt_f8_supported", &k_gemm_tt_f8_supported);
  m.def("gemm_tt_f8", &k_gemm_tt_f8, py::arg("a"), py::arg("b"), py::arg("alpha_a"), py::arg("alpha_b"),
        py::arg("fmt_a"), py::arg("fmt_b"), py::arg("splits"), py::arg("out_dtype"), py::arg("out") = py::none());
  m.attr("EPI_NONE") = (int)apex::EPI_NONE;
  m.attr("EPI_BIAS") = (int)apex::EPI_BIAS;
  m.attr("EPI_BIAS_GELU") = (int)apex::EPI_BIAS_GELU;
  m.attr("EPI_DGELU") = (int)apex::EPI_DGELU;
  m.attr("EPI_RESID") = (int)apex::EPI_RESID;
  m.attr("EPI_BIAS_GELU_TANH") = (int)apex::EPI_BIAS_GELU_TANH;
  m.attr("EPI_DGELU_TANH") = (int)apex::EPI_DGELU_TANH;
  m.attr("EPI_BIAS_GELU_D") = (int)apex::EPI_BIAS_GELU_D;
  m.attr("EPI_BIAS_GELU_TANH_D") = (int)apex::EPI_BIAS_GELU_TANH_D;
  m.attr("EPI_MUL") = (int)apex::EPI_MUL;
}
