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
  int* first_run_dev;  // optional device flag: nonzero until the first NON-skipped step ran
};

struct AdamArgs {
  float lr, beta1, beta2, eps, wd, bc1, bc2;
  int adamw;
  float grad_scale;
  const float* grad_scale_ptr;
  const int* noop;
  int* step;           // optional device step counter, advanced only by non-skipped steps;
  int bias_correction; // with `step`, bc1/bc2 are computed on the device from it
  float* scal;         // 2-float workspace for the device bias corrections
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

// ----------------------------- flash attention ------------------------------
// Tensors are [B, S, H, D] views; *_bs / *_ss / *_hs are batch / seq / head strides in
// elements (the D dimension must be contiguous and 16-byte aligned).
struct AttnArgs {
  const void* q;
  const void* k;
  const void* v;
  void* o;
  float* lse;  // [B*H, Sq] natural-log sum-exp
  void* dq;
  int64_t q_bs, q_ss, q_hs, k_bs, k_ss, k_hs, v_bs, v_ss, v_hs, o_bs, o_ss, o_hs;
  int64_t do_bs, do_ss, do_hs, dq_bs, dq_ss, dq_hs, dk_bs, dk_ss, dk_hs, dv_bs, dv_ss, dv_hs;
  int B, H, Sq, Sk, D;
  int causal;
  float scale, scale_log2;
  uint32_t drop_thresh;  // keep iff 8-bit uniform >= drop_thresh (0 = no dropout)
  float drop_scale;      // 256 / (256 - drop_thresh)
  uint64_t seed, offset;
  const int* k_lens;     // optional per-batch valid key length
  uint16_t* dmask;       // dropout keep bits [B*H, Sq, mask_words] (fwd writes, bwd reads): one
                         // 32-bit word per (row, 32-key block), bit k <-> key 32 blk + k
  int64_t mask_words;    // 2 * ceil(Sk / 32) (uint16 units)
  int dbg;               // unused by the kernels (the runtime section-skip branches forced accumulator copies)
  float* dsum;           // optional, zeroed [B][3][H][D]: bwd adds the column sums (over positions)
                         // of dq, dk, dv — the packed-QKV projection's bias gradient, per batch
  const void* bias;      // optional additive score bias (input dtype), element (b, h, q, key) at
  int64_t bias_bs, bias_hs, bias_qs;  // b*bias_bs + h*bias_hs + q*bias_qs + key (0 = broadcast)
  // optional gradient of a trainable bias (backward): fp32, element (b, h, q, key) at
  // b*dbias_bs + h*dbias_hs + q*dbias_qs + key; the score gradient dS (natural domain, before the
  // softmax scale) is stored there, or atomically added when a dimension is broadcast (dbias_atomic)
  float* dbias;
  int64_t dbias_bs, dbias_hs, dbias_qs;
  int dbias_atomic;
  // fp8 producer-side codes (apex.fp8): the kernels also write fp8 codes of what they store, for the
  // GEMM that consumes it next (no standalone quantise pass): forward -> O (the attention-out GEMM's
  // e4m3 operand), backward -> dq / dk / dv (the QKV input-gradient GEMM's e5m2 operand). Each code
  // array has its tensor's element layout (same strides); codes = sat(value * q8_scale[0]), max|value|
  // folded into q8_amax[0]. Null: off.
  uint8_t* q8o;
  uint8_t* q8dq;
  uint8_t* q8dk;
  uint8_t* q8dv;
  const float* q8_scale;
  float* q8_amax;
  int q8_fmt;  // 0 = e4m3, 1 = e5m2
  // backward with q8dq..: dq / dk / dv are NOT stored, only their codes (their consumers, the QKV
  // input-gradient GEMM and weight gradient, read codes alone: apex.fp8 codes_only_ok)
  int q8only;
};
inline uint32_t attn_drop_thresh(double p) {  // 8-bit keep threshold in [1, 255], 0 = off
  if (p <= 0.0) return 0u;
  long t = (long)(p * 256.0 + 0.5);
  return (uint32_t)(t < 1 ? 1 : t > 255 ? 255 : t);
}
int attn_fwd(const AttnArgs& a, int dt, hipStream_t s);
bool attn_bwd_needs_dq_acc(const AttnArgs& a);
bool attn_bwd_split();
// delta_ws: [B*H*Sq] fp32 workspace when attn_bwd_needs_dq_acc (two-kernel backward)
int attn_bwd(const AttnArgs& a, const void* dout, float* delta_ws, void* dk, void* dv, int dt,
             hipStream_t s);
// context parallelism: acc (fp32 [B,S,H,D] + lse [B,H,S]) <- exact log-sum-exp merge with one block's
// (o [B,S,H,D] in dt, lse [B,H,S]); first = 1 initialises the accumulator from the block
int lse_merge(float* acc_o, float* acc_lse, const void* o, const float* lse, int64_t B, int S, int H, int D,
              int first, int dt, hipStream_t s, int Sa = 0, int s0 = 0);
int attn_dropout_mask(uint8_t* out, int64_t BH, int Sq, int Sk, uint64_t seed, uint64_t offset,
                      uint32_t thresh, hipStream_t s);

// ----------------------------- fused elementwise ---------------------------
// act: 0 gelu(erf), 1 gelu(tanh), 2 relu, 3 identity. cols % 8 == 0.
int bias_act_fwd(const void* x, const void* b, void* y, int64_t rows, int cols, int act, int xdt,
                 int bdt, hipStream_t s);
// ws: >= colsum_parts(rows) * cols floats
int bias_act_bwd(const void* dy, const void* x, const void* b, void* dx, void* db, float* ws,
                 int64_t rows, int cols, int act, int xdt, int bdt, hipStream_t s);
int bias_dropout_add_fwd(const void* x, const void* b, const void* res, void* y, int64_t rows, int cols,
                         uint64_t seed, uint64_t offset, uint32_t thresh, float scale, int xdt, int bdt,
                         hipStream_t s);
int bias_dropout_add_bwd(const void* dy, void* dx, void* db, float* ws, int64_t rows, int cols,
                         uint64_t seed, uint64_t offset, uint32_t thresh, float scale, int xdt, int bdt,
                         hipStream_t s);
int colsum(const void* x, void* out, float* ws, int64_t rows, int cols, int xdt, int odt, hipStream_t s);
int splitk_reduce(const float* slabs, void* out, int64_t n, int nsplit, int odt, hipStream_t s,
                  int accumulate = 0);
int64_t colsum_parts(int64_t rows);
// fp8 side output of a producer kernel (delayed scaling: codes = sat(v * scale[0]), max|v| folded
// into amax[0] for the next scale update; fmt 0 = e4m3, 1 = e5m2). y == nullptr: none.
struct Q8Out {
  uint8_t* y = nullptr;
  const float* scale = nullptr;
  float* amax = nullptr;
  int fmt = 0;
  int only = 0;  // GEMM producers: the codes are the output's only consumer-visible form (C not stored)
};
int bdaln_supported(int cols);
int bdaln_wide_supported(int cols);  // 2056..4096 columns (bdaln fwd/bwd only, not the embedding block)
int bdaln_fwd(const void* x, const void* b, const void* res, const void* gamma, const void* beta, void* y,
              void* s_out, float* mean, float* rstd, int64_t rows, int cols, float eps, uint64_t seed,
              uint64_t offset, uint32_t thresh, float scale, int xdt, int wdt, hipStream_t s,
              Q8Out q8 = Q8Out{},  // q8: fp8 codes of y (narrow rows only)
              int s_cond = 0);      // 1: s_out written only when gamma has a zero entry (post-LN mem mode)
// BERT embeddings: s = Ww[id] + Wp[row % S] + Wt[type]; y = dropout(LN(s)); backward -> ds, dWp, dWt
// (type vocab <= 2), dgamma, dbeta; embed_segsum: word rows from the id-sorted token list
int embed_ln_fwd(const int* ids, const int* tids, const void* Ww, const void* Wp, const void* Wt, const void* gamma,
                 const void* beta, void* y, void* s_out, float* mean, float* rstd, int64_t rows, int cols, int S,
                 float eps, uint64_t seed, uint64_t offset, uint32_t thresh, float scale, int xdt, int wdt,
                 hipStream_t s);
int embed_nwt(int64_t B);
int embed_ln_bwd(const void* dy, const void* s_in, const void* gamma, const float* mean, const float* rstd,
                 const int* tids, int tvocab, void* ds_out, float* part_pos, float* part_tg, void* dWp, void* dWt,
                 void* dgamma, void* dbeta, int64_t B, int cols, int S, uint64_t seed, uint64_t offset,
                 uint32_t thresh, float scale, int xdt, int wdt, hipStream_t s);
int embed_segsum(const void* ds, const int* sorted, const int64_t* perm, void* dW, int64_t R, int cols, int xdt,
                 hipStream_t s);
int64_t bdaln_ws_floats(int64_t rows, int cols);
// dse (nullable): extra gradient of s from its other consumers (pre-LN residual stream), added to ds
int bdaln_bwd(const void* dy, const void* s_in, const void* gamma, const void* beta, const float* mean,
              const float* rstd, const void* dse, void* dres, void* dx, void* dgamma, void* dbeta, void* dbias,
              float* ws, int64_t rows, int cols, uint64_t seed, uint64_t offset, uint32_t thresh, float scale,
              int xdt, int wdt, hipStream_t s,  // beta != nullptr: s_in is the LN output y (post-LN, narrow)
              Q8Out q8 = Q8Out{},  // q8: fp8 codes of dx (narrow rows only)
              const void* s_alt = nullptr);  // beta given: the s of an s_cond forward (zero-gamma fallback)

// ----------------------------- weight norm / RNN cells / SyncBN ------------
int weight_norm_fwd(const void* v, const void* g, void* w, float* norms, int64_t R, int64_t C, int row_mode,
                    int vdt, int gdt, hipStream_t s);
int weight_norm_bwd(const void* dw, const void* v, const void* g, const float* norms, void* dv, void* dg,
                    int64_t R, int64_t C, int row_mode, int vdt, int gdt, hipStream_t s);
int lstm_cell_fwd(const void* ig, const void* hg, const void* bih, const void* bhh, const void* cx, void* hy,
                  void* cy, float* ws, int64_t B, int64_t H, int dt, hipStream_t s);
int lstm_cell_bwd(const void* dhy, const void* dcy, const void* cx, const float* ws, void* dgates, void* dcx,
                  int64_t B, int64_t H, int dt, hipStream_t s);
int gru_cell_fwd(const void* ig, const void* hg, const void* bih, const void* bhh, const void* hx, void* hy,
                 float* ws, int64_t B, int64_t H, int dt, hipStream_t s);
int gru_cell_bwd(const void* dhy, const void* hx, const float* ws, void* dig, void* dhg, void* dhx, int64_t B,
                 int64_t H, int dt, hipStream_t s);
int bn_splits_for(int64_t N, int64_t C, int64_t S, int nhwc, int dt);
int bn_stats(const void* x, float* part, int64_t N, int64_t C, int64_t S, int nhwc, int dt, int* splits_out,
             hipStream_t s);
// invstd (nullable): rsqrt(var + eps); rmean / rvar (nullable, fp32): running-statistics momentum update
int bn_combine(const float* in, int groups, int64_t C, int gmajor, float* mean, float* var, float* count,
               hipStream_t s, float* invstd = nullptr, float eps = 0.f, float* rmean = nullptr,
               float* rvar = nullptr, float momentum = 0.f, float* triple = nullptr,
               int64_t* ntrack = nullptr);
// Fused residual + ReLU (ResNet blocks): bn_elemt adds z (nullable, x's layout) after the affine
// and before the ReLU; the backward kernels take the forward output ym (nullable) and pass the
// gradient only where ym > 0; bn_bwd_elemt also writes that masked gradient to dz (z's gradient).
int bn_elemt(const void* x, const float* mean, const float* invstd, const void* w, const void* b, const void* z,
             void* y, int64_t N, int64_t C, int64_t S, int nhwc, int relu, int dt, int wdt, float* coef,
             hipStream_t s);
int bn_bwd_reduce(const void* dy, const void* x, const void* ym, const float* mean, float* part, float* sum_dy,
                  float* sum_dy_xmu, int64_t N, int64_t C, int64_t S, int nhwc, int dt, hipStream_t s);
int bn_bwd_elemt(const void* dy, const void* x, const float* mean, const float* invstd, const void* w,
                 const float* sum_dy, const float* sum_dy_xmu, const float* count, const void* ym, void* dz,
                 void* dx, int64_t N, int64_t C, int64_t S, int nhwc, int dt, int wdt, float* coef, hipStream_t s);

// ----------------------------- fused scale-mask softmax --------------------
// mode 0: scale only, 1: byte mask [B, mask_heads, sq, cols] (nonzero masked), 2: causal
int scaled_softmax_supported(int cols);
int scaled_masked_softmax_fwd(const void* x, const uint8_t* mask, void* y, int64_t rows, int cols, int sq,
                              int heads, int mask_heads, float scale, int mode, int dt, hipStream_t s);
int scaled_masked_softmax_bwd(const void* dy, const void* y, void* dx, int64_t rows, int cols, float scale, int dt,
                              hipStream_t s);

// ----------------------------- softmax cross-entropy -----------------------
int xentropy_fwd(const void* logits, const int64_t* labels, float* losses, float* lse, int64_t rows,
                 int V, float smoothing, int64_t ignore_index, int dt, hipStream_t s);
int xentropy_bwd(const void* dloss, int64_t dloss_stride, int dloss_dt, const void* logits,
                 const float* lse, const int64_t* labels, void* dlogits, int64_t rows, int V,
                 float smoothing, int64_t ignore_index, int dt, hipStream_t s);

// ----------------------------- MFMA GEMM (gemm.hip) ------------------------
enum GemmEpi : int { EPI_NONE = 0, EPI_BIAS = 1, EPI_BIAS_GELU = 2, EPI_DGELU = 3, EPI_RESID = 4, EPI_F32 = 5,
                     EPI_BIAS_GELU_TANH = 6, EPI_DGELU_TANH = 7,
                     // forward GELU that stores gelu'(h) instead of h, and its backward: C = acc * aux
                     EPI_BIAS_GELU_D = 8, EPI_BIAS_GELU_TANH_D = 9, EPI_MUL = 10,
                     // fp32 read-modify-write: part[m, n] += acc (the weight gradient accumulated
                     // straight into an fp32 main_grad, one K slice)
                     EPI_F32_ACC = 11 };
struct GemmArgs {
  const void* A;  // [M, K] row-major, lda
  const void* B;  // [N, K] row-major, ldb
  void* C;        // [M, N] row-major, ldc
  int M, N, K;
  int64_t lda, ldb, ldc;
  const void* bias;  // [N]            EPI_BIAS, EPI_BIAS_GELU
  const void* aux;   // [M, N], ldaux  EPI_DGELU (pre-activation H), EPI_RESID (residual), EPI_MUL (gelu'(H))
  int64_t ldaux;
  void* aux_out;     // [M, N], ldc    EPI_BIAS_GELU (pre-activation H), EPI_BIAS_GELU_D (gelu'(H))
  float* part;       // [gemm_part_rows(M), N] fp32  EPI_DGELU / EPI_MUL (bias-grad partials)
  int epi;
  int splits;        // gemm_tt: split-K slices (blockIdx.y)
  const float* alpha_a = nullptr;  // fp8: dequantisation scales (1 / quantisation scale) of A and B,
  const float* alpha_b = nullptr;  // device scalars; C = epi(alpha_a * alpha_b * A8 . B8^T)
  Q8Out q8{};  // fp8 GEMM, GELU / dGELU / MUL epilogues: also write fp8 codes of C (ldc bytes per row)
};
bool gemm_supported(int M, int N, int K, int64_t lda, int64_t ldb, int64_t ldc);
int64_t gemm_part_rows(int M);
int gemm_nt(const GemmArgs& g, int dt, hipStream_t s);
// FP8 operands (uint8 storage; fmt 0 = e4m3, 1 = e5m2; B must be e4m3): K % 128 == 0
bool gemm_f8_supported(int M, int N, int K, int64_t lda, int64_t ldb, int64_t ldc);
int gemm_nt_f8(const GemmArgs& g, int fmt_a, int fmt_b, int out_dt, hipStream_t s);
// fp8.hip: per-tensor scaled quantisation + delayed-scaling bookkeeping (fmt 0 = e4m3, 1 = e5m2)
// delayed scaling: scale read, amax (optional) accumulated; current scaling (cur != null): scale /
// scale_inv WRITTEN from smax / cur[0]
int fp8_quantize(const void* x, uint8_t* y, int64_t n, int dt, int fmt, float* scale, float* scale_inv, float* amax,
                 const float* cur, float smax, hipStream_t s);
int fp8_quantize_t(const void* x, uint8_t* y, int R, int C, int dt, int fmt, float* scale, float* scale_inv,
                   float* amax, const float* cur, float smax, hipStream_t s);
int fp8_amax(const void* x, int64_t n, int dt, float* amax, hipStream_t s);
// one step's weights (batched current-scaling quantisation): W [R, C] -> codes y [R, C] and, when
// yt != null, y^T [C, R]; slot = the weight's scale / scale_inv / amax index; ablock0 / qblock0 =
// prefix of the amax (64 K-element spans) / quantise (64 x 64 tiles) block counts
struct WqDesc {
  const void* w;
  uint8_t* y;
  uint8_t* yt;
  int R, C;
  int slot;
  int pad;
  int64_t ablock0, qblock0;
};
int fp8_quantize_weights(const WqDesc* d, int nd, int64_t ablocks, int64_t qblocks, int dt, int fmt, float* scale,
                         float* scale_inv, float* amax, float smax, hipStream_t s);
int fp8_update_scales(float* hist, float* amax_cur, float* scale, float* scale_inv, const float* fmt_max,
                      int n_slots, int hist_len, int idx, float margin_scale, hipStream_t s);
int gemm_set_dbg(int v);  // diagnostics: 2 = skip the epilogue
int gemm_set_persist(int which, int v);  // force the persistent GEMM on / off (tests); returns the previous value
// weight-gradient form: C[P, Q] = A^T B with A [R, P], B [R, Q] row-major (contraction over rows)
bool gemm_tt_supported(int P, int Q, int R, int splits, int64_t lda, int64_t ldb);
int gemm_tt(const GemmArgs& g, int dt, hipStream_t s);
bool gemm_tt_f8_supported(int P, int Q, int R, int splits, int64_t lda, int64_t ldb);
int gemm_tt_f8(const GemmArgs& g, int fmt_a, int fmt_b, hipStream_t s);
int gemm_bias_grad(const float* part, int parts, int N, void* out, int odt, hipStream_t s);
int transpose_2d(const void* in, void* out, int R, int C, int dt, hipStream_t s);

// ----------------------------- input pipeline (K-09) -----------------------
// layout: 0 NHWC->NHWC, 1 NHWC->NCHW (hw % 8 == 0, C in {1,3,4}), 2 NCHW->NCHW. Returns 1 if
// the geometry is unsupported.
int input_normalize(const uint8_t* x, void* y, int64_t B, int64_t C, int64_t hw, int layout, const float* mean,
                    const float* stdv, int ydt, hipStream_t s);

}  // namespace apex
