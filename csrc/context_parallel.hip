// Context parallelism (apex.transformer.context_parallel): the exact log-sum-exp merge of ring
// attention's per-block partial outputs, fused into one pass.
//
// Ring attention computes, for each query chunk, one flash-attention block per visible key chunk,
// each with its own normalisation: (o_j [B, S, H, D] in the input dtype, lse_j [B, H, S] fp32,
// natural log, +inf for rows with no visible key). The exact result is
//   lse = log(sum_j exp(lse_j)),   o = sum_j exp(lse_j - lse) o_j
// accumulated block by block into an fp32 (acc_o, acc_lse). Round 3 did this with eight torch ops
// over the whole [B, S, H, D] fp32 accumulator per block (logaddexp, two exps, two broadcast
// multiplies, an add, two where): each a full read + write of the accumulator. Here one kernel
// reads acc_o and o once and writes acc_o once; `first` initialises the accumulator from the first
// block (no zero fill, no exp).
//
// One thread per 8 consecutive elements of a (b, s, h) row (16-byte loads of o, 2 x 16-byte fp32 of
// acc_o); D % 8 == 0 and D <= 256, so a row's D / 8 threads sit in one wave and the lane that
// writes acc_lse reads it in the same instruction as its row mates.
#include "common.h"
#include "kernels.h"

#include <math.h>

namespace apex {

// The accumulator may cover more rows than the block: acc_o [B, Sa, H, D] / acc_lse [B, H, Sa] with
// the block's rows at s0 .. s0 + S (a zigzag ring step that sees only this rank's late chunk
// merges into that half of the accumulator in place, no chunk copies).
template <typename T>
__global__ void __launch_bounds__(256) lse_merge_kernel(float* __restrict__ acc_o, float* __restrict__ acc_lse,
                                                        const T* __restrict__ o, const float* __restrict__ lse,
                                                        int64_t rows, int S, int H, int D, int first, int Sa,
                                                        int s0) {
  const int cpr = D >> 3;
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t row = idx / cpr;
  if (row >= rows) return;
  const int c = (int)(idx - row * cpr);
  const int64_t h = row % H, bs = row / H, s = bs % S, b = bs / S;
  const int64_t li = (b * H + h) * S + s;
  const int64_t lai = (b * H + h) * Sa + s0 + s;
  float ln = lse[li];
  if (ln == INFINITY) ln = -INFINITY;  // the flash kernels mark a row with no visible key +inf
  const int64_t e = row * D + c * 8;
  const int64_t ea = ((b * Sa + s0 + s) * H + h) * D + c * 8;
  float x[8];
  load_f<T, 8>(o + e, x);
  if (first) {
    store_f<float, 8>(acc_o + ea, x);
    if (c == 0) acc_lse[lai] = ln;
    return;
  }
  const float la = acc_lse[lai];
  const float mx = fmaxf(la, ln);
  float nw, wo, wn;
  if (mx == -INFINITY) {  // neither side has a visible key yet
    nw = -INFINITY;
    wo = 0.f;
    wn = 0.f;
  } else {
    wo = __expf(la - mx);
    wn = __expf(ln - mx);
    const float sum = wo + wn;
    nw = mx + __logf(sum);
    const float inv = 1.f / sum;
    wo *= inv;
    wn *= inv;
  }
  float a[8];
  load_f<float, 8>(acc_o + ea, a);
#pragma unroll
  for (int k = 0; k < 8; ++k) a[k] = fmaf(a[k], wo, x[k] * wn);
  store_f<float, 8>(acc_o + ea, a);
  if (c == 0) acc_lse[lai] = nw;
}

int lse_merge(float* acc_o, float* acc_lse, const void* o, const float* lse, int64_t B, int S, int H, int D,
              int first, int dt, hipStream_t s, int Sa, int s0) {
  if (D % 8 || D > 256 || D <= 0) return -2;
  if (Sa <= 0) Sa = S;
  if (s0 < 0 || s0 + S > Sa) return -3;
  const int64_t rows = B * (int64_t)S * H;
  if (rows == 0) return 0;
  const int64_t n = rows * (D / 8);
  const dim3 grid((unsigned)((n + 255) / 256));
  if (dt == kBF16)
    hipLaunchKernelGGL(lse_merge_kernel<bf16>, grid, dim3(256), 0, s, acc_o, acc_lse, (const bf16*)o, lse, rows, S,
                       H, D, first, Sa, s0);
  else if (dt == kF16)
    hipLaunchKernelGGL(lse_merge_kernel<f16>, grid, dim3(256), 0, s, acc_o, acc_lse, (const f16*)o, lse, rows, S, H,
                       D, first, Sa, s0);
  else
    hipLaunchKernelGGL(lse_merge_kernel<float>, grid, dim3(256), 0, s, acc_o, acc_lse, (const float*)o, lse, rows,
                       S, H, D, first, Sa, s0);
  return (int)hipGetLastError();
}

}  // namespace apex
