// Host-callable launchers for every apex HIP kernel. The .hip translation units
// include only HIP headers (fast, torch-free compiles); bindings.cpp adapts
// at::Tensor arguments onto these raw-pointer entry points.
// Every launcher returns 0 on success or a hipError_t / -1 (bad dtype) code.
#pragma once
#include <hip/hip_runtime_api.h>
#include <stdint.h>

#include "multi_tensor.h"

namespace apex {

// dtype codes (same values as common.h DType)
constexpr int kF32Code = 0, kF16Code = 1, kBF16Code = 2;

// ----------------------------- multi-tensor --------------------------------
struct SgdArgs {
  float lr, momentum, dampening, wd;
  int nesterov, first_run, wd_after_momentum;
  float grad_scale;
  const float* grad_scale_ptr;
  const int* noop;
};

struct AdamArgs {
  float lr, beta1, beta2, eps, wd, bc1, bc2;
  int adamw;
  float grad_scale;
  const float* grad_scale_ptr;
  const int* noop;
};

struct LambArgs {
  float lr, beta1, beta2, eps, wd, max_grad_norm;
  int adamw, bias_correction, grad_averaging, use_nvlamb;
  float grad_scale;
  const float* grad_scale_ptr;
  const int* noop;
  int* overflow_out;
  const float* gnorm_in;  // optional precomputed (unscaled) global grad norm
};

struct LarcArgs {
  float trust_coefficient, eps, lr, wd;
  int clip;
};

int mt_scale(const MTMeta& m, int in_dt, int out_dt, const float* sp, float sv, int* overflow,
             hipStream_t s);
int mt_axpby(const MTMeta& m, int x_dt, int y_dt, int o_dt, float a, float b, int check,
             int* overflow, hipStream_t s);
int mt_l2norm(const MTMeta& m, int list, int dt, float* partial, float* out_tensor,
              float* out_global, const float* sp, float sv, int* overflow, hipStream_t s);
int mt_sgd(const MTMeta& m, int g_dt, int p_dt, int c_dt, const SgdArgs& a, hipStream_t s);
int mt_adam(const MTMeta& m, int g_dt, int p_dt, int c_dt, const AdamArgs& a, hipStream_t s);
int mt_lamb(const MTMeta& m, int g_dt, int p_dt, int c_dt, const LambArgs& a, float* ws, int* step,
            hipStream_t s);
int mt_larc(const MTMeta& m, int g_dt, int p_dt, const LarcArgs& a, float* ws, hipStream_t s);
int amp_update_scale(float* scale, int* tracker, const int* overflow, float growth, float backoff,
                     int interval, float min_scale, float max_scale, hipStream_t s);

// ----------------------------- normalization -------------------------------
// rows x cols, x/y dtype xdt, gamma/beta dtype wdt (may be null). mean/rstd fp32 [rows].
int layer_norm_fwd(const void* x, const void* gamma, const void* beta, void* y, float* mean,
                   float* rstd, int64_t rows, int cols, float eps, int xdt, int wdt, int rms,
                   hipStream_t s);
// dgamma/dbeta computed through fp32 partial buffer `ws` of size [ceil(rows/rows_per_part)][2*cols]
int layer_norm_bwd(const void* dy, const void* x, const void* gamma, const float* mean,
                   const float* rstd, void* dx, void* dgamma, void* dbeta, float* ws,
                   int64_t rows, int cols, int xdt, int wdt, int rms, hipStream_t s);
int64_t layer_norm_bwd_ws_floats(int64_t rows, int cols);

// ----------------------------- softmax cross-entropy -----------------------
int xentropy_fwd(const void* logits, const int64_t* labels, float* losses, float* lse, int64_t rows,
                 int V, float smoothing, int64_t ignore_index, int dt, hipStream_t s);
int xentropy_bwd(const void* dloss, int64_t dloss_stride, int dloss_dt, const void* logits,
                 const float* lse, const int64_t* labels, void* dlogits, int64_t rows, int V,
                 float smoothing, int64_t ignore_index, int dt, hipStream_t s);

}  // namespace apex
