// FP8 support kernels for the fp8 GEMM path (amp fp8 option, apex/fp8): per-tensor scaled
// quantisation to OCP e4m3 / e5m2 (gfx950's native FP8 encodings) and the delayed-scaling
// bookkeeping — every quantisation records the amax of its input on the device, and one launch
// per step folds those amaxes into a rolling history and recomputes every scale. No host sync.
//
//   quantize      y8 = sat(x * scale[slot])           + amax_cur[slot] = max |x|
//                 (current scaling: scale = fmt_max * 2^-margin / amax measured just before)
//   quantize_t    y8[c][r] = sat(x[r][c] * scale)     (weights for the dgrad GEMM: W^T, K-contiguous)
//   amax          amax_cur[slot] = max |x|             (first use of a slot: current scaling)
//   update        hist[slot][idx] = amax_cur; a = max(hist[slot]); scale = fmt_max / a / 2^margin;
//                 scale_inv = 1 / scale; amax_cur = 0
// The conversions are the hardware v_cvt_pk_fp8_f32 / v_cvt_pk_bf8_f32 (round to nearest even); x
// is clamped to the format's finite range first (e4m3fn has no infinity).
#include "common.h"
#include "kernels.h"
#include "fp8_pack.h"

namespace apex {

namespace {

template <int FMT>
__device__ __forceinline__ uint32_t pack4(float a, float b, float c, float d) {
  return f8_pack4<FMT>(a, b, c, d);
}

__device__ __forceinline__ float wave_max(float v) { return f8_wave_max(v); }
__device__ __forceinline__ void block_amax(float mx, float* amax) { f8_block_amax(mx, amax); }

// Scale source of one quantisation. Delayed: s = scale[0] (from the history), the input's amax
// is folded into amax[0] for the next update. Current (cur != null, amax already measured by
// amax_kernel): s = smax / cur[0], written back to scale[0] / scale_inv[0] by the first block.
struct QScale {
  float* scale;
  float* scale_inv;
  float* amax;
  const float* cur;
  float smax;
};

__device__ __forceinline__ float q_scale(const QScale& q, bool first_block) {
  if (!q.cur) return q.scale[0];
  const float a = q.cur[0];
  const float s = (a > 0.f && isfinite(a)) ? q.smax / a : 1.f;
  if (first_block && threadIdx.x == 0) {
    q.scale[0] = s;
    q.scale_inv[0] = 1.f / s;
  }
  return s;
}

// 8 elements per lane per iteration (16-byte loads of 16-bit inputs, 8-byte stores)
template <typename T, int FMT>
__global__ void __launch_bounds__(256) quantize_kernel(const T* __restrict__ x, uint8_t* __restrict__ y, int64_t n,
                                                       QScale q) {
  const float s = q_scale(q, blockIdx.x == 0);
  float* amax = q.amax;
  float mx = 0.f;
  const int64_t nv = n / 8;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < nv; i += (int64_t)gridDim.x * 256) {
    float v[8];
    load_f<T, 8>(x + i * 8, v);
#pragma unroll
    for (int k = 0; k < 8; ++k) mx = fmaxf(mx, fabsf(v[k]));
    uint2 w;
    w.x = pack4<FMT>(v[0] * s, v[1] * s, v[2] * s, v[3] * s);
    w.y = pack4<FMT>(v[4] * s, v[5] * s, v[6] * s, v[7] * s);
    *reinterpret_cast<uint2*>(y + i * 8) = w;
  }
  for (int64_t i = nv * 8 + (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const float v = to_f(x[i]);
    mx = fmaxf(mx, fabsf(v));
    y[i] = (uint8_t)(pack4<FMT>(v * s, 0.f, 0.f, 0.f) & 0xff);
  }
  if (amax) block_amax(mx, amax);
}

template <typename T>
__global__ void __launch_bounds__(256) amax_kernel(const T* __restrict__ x, int64_t n, float* __restrict__ amax) {
  float mx = 0.f;
  const int64_t nv = n / 8;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < nv; i += (int64_t)gridDim.x * 256) {
    float v[8];
    load_f<T, 8>(x + i * 8, v);
#pragma unroll
    for (int k = 0; k < 8; ++k) mx = fmaxf(mx, fabsf(v[k]));
  }
  for (int64_t i = nv * 8 + (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    mx = fmaxf(mx, fabsf(to_f(x[i])));
  block_amax(mx, amax);
}

// y[C][R] = quant(x[R][C]): 64 x 64 tiles through LDS, 8 elements (one 8-byte store) per lane
template <typename T, int FMT>
__global__ void __launch_bounds__(256) quantize_t_kernel(const T* __restrict__ x, uint8_t* __restrict__ y, int R,
                                                         int C, QScale q) {
  __shared__ float tile[64][65];
  const float s = q_scale(q, blockIdx.x == 0 && blockIdx.y == 0);
  float* amax = q.amax;
  const int r0 = blockIdx.y * 64, c0 = blockIdx.x * 64;
  float mx = 0.f;
  for (int idx = threadIdx.x; idx < 64 * 64; idx += 256) {
    const int rr = idx / 64, cc = idx % 64;
    const int r = r0 + rr, c = c0 + cc;
    const float v = (r < R && c < C) ? to_f(x[(int64_t)r * C + c]) : 0.f;
    mx = fmaxf(mx, fabsf(v));
    tile[rr][cc] = v * s;
  }
  __syncthreads();
  // thread -> (output row c, 8 consecutive r)
  for (int idx = threadIdx.x; idx < 64 * 8; idx += 256) {
    const int cc = idx / 8, rg = (idx % 8) * 8;
    const int c = c0 + cc, r = r0 + rg;
    if (c >= C) continue;
    const float* t = &tile[0][0];
    float v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = t[(rg + k) * 65 + cc];
    if (r + 8 <= R) {
      uint2 w;
      w.x = pack4<FMT>(v[0], v[1], v[2], v[3]);
      w.y = pack4<FMT>(v[4], v[5], v[6], v[7]);
      *reinterpret_cast<uint2*>(y + (int64_t)c * R + r) = w;
    } else {
      for (int k = 0; k < 8 && r + k < R; ++k) y[(int64_t)c * R + r + k] = (uint8_t)(pack4<FMT>(v[k], 0.f, 0.f, 0.f) & 0xff);
    }
  }
  if (amax) block_amax(mx, amax);
}

// one thread per slot
__global__ void update_scales_kernel(float* __restrict__ hist, float* __restrict__ amax_cur, float* __restrict__ scale,
                                     float* __restrict__ scale_inv, const float* __restrict__ fmt_max, int n_slots,
                                     int hist_len, int idx, float margin_scale) {
  const int sl = blockIdx.x * blockDim.x + threadIdx.x;
  if (sl >= n_slots) return;
  float* h = hist + (int64_t)sl * hist_len;
  const float cur = amax_cur[sl];
  h[idx] = isfinite(cur) ? cur : 0.f;  // an overflowed (skipped) step does not poison the window
  float a = 0.f;
  for (int k = 0; k < hist_len; ++k) a = fmaxf(a, h[k]);
  if (a > 0.f && isfinite(a)) {
    const float sc = fmt_max[sl] / a * margin_scale;
    scale[sl] = sc;
    scale_inv[sl] = 1.f / sc;
  }
  amax_cur[sl] = 0.f;
}

// ---- batched weight quantisation (one optimizer step's weights in three launches) ----------------
// The fp8 GEMMs quantise every weight once per step with current scaling: exact amax, then the
// e4m3 codes of W (forward) and of W^T (input-gradient GEMM). Per weight that was an amax, a
// quantise and a transposing quantise launch (~300 launches of ~10 us for BERT-Large's 96 GEMM
// weights, mostly launch-bound); here every weight of the step goes through one zeroing, one amax
// and one quantise launch, the last reading each 64 x 64 tile once for both outputs.
// Work lists: amax blocks walk 64 K-element spans, quantise blocks 64 x 64 tiles; block -> weight
// by binary search over the descriptors' first-block prefix.
__global__ void wq_zero_kernel(const WqDesc* __restrict__ d, int nd, float* __restrict__ amax) {
  for (int i = threadIdx.x; i < nd; i += blockDim.x) amax[d[i].slot] = 0.f;
}

__device__ __forceinline__ int wq_find(const WqDesc* __restrict__ d, int nd, int64_t b, bool quant) {
  int lo = 0, hi = nd - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if ((quant ? d[mid].qblock0 : d[mid].ablock0) <= b) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

constexpr int kWqSpan = 65536;  // elements per amax block

template <typename T>
__global__ void __launch_bounds__(256) wq_amax_kernel(const WqDesc* __restrict__ d, int nd, float* __restrict__ amax) {
  const WqDesc w = d[wq_find(d, nd, blockIdx.x, false)];
  const int64_t n = (int64_t)w.R * w.C;
  const int64_t e0 = (int64_t)(blockIdx.x - w.ablock0) * kWqSpan;
  const int64_t e1 = e0 + kWqSpan < n ? e0 + kWqSpan : n;
  const T* x = (const T*)w.w;
  float mx = 0.f;
  if ((n & 7) == 0) {
    for (int64_t i = e0 + threadIdx.x * 8; i < e1; i += 256 * 8) {
      float v[8];
      load_f<T, 8>(x + i, v);
#pragma unroll
      for (int k = 0; k < 8; ++k) mx = fmaxf(mx, fabsf(v[k]));
    }
  } else {
    for (int64_t i = e0 + threadIdx.x; i < e1; i += 256) mx = fmaxf(mx, fabsf(to_f(x[i])));
  }
  block_amax(mx, amax + w.slot);
}

template <typename T, int FMT>
__global__ void __launch_bounds__(256) wq_quant_kernel(const WqDesc* __restrict__ d, int nd, float* __restrict__ scale,
                                                       float* __restrict__ scale_inv, const float* __restrict__ amax,
                                                       float smax) {
  __shared__ float tile[64][65];
  const WqDesc w = d[wq_find(d, nd, blockIdx.x, true)];
  const int tb = blockIdx.x - w.qblock0;
  const int tiles_c = (w.C + 63) / 64;
  const int r0 = (tb / tiles_c) * 64, c0 = (tb % tiles_c) * 64;
  const float a = amax[w.slot];
  const float s = (a > 0.f && isfinite(a)) ? smax / a : 1.f;
  if (tb == 0 && threadIdx.x == 0) {
    scale[w.slot] = s;
    scale_inv[w.slot] = 1.f / s;
  }
  const T* x = (const T*)w.w;
  // load: thread -> (row rr, 8 consecutive columns); the row-major codes go out straight away
  for (int idx = threadIdx.x; idx < 64 * 8; idx += 256) {
    const int rr = idx / 8, cg = (idx % 8) * 8;
    const int r = r0 + rr, c = c0 + cg;
    float v[8];
    if (r < w.R && c + 8 <= w.C && (w.C & 7) == 0) {
      load_f<T, 8>(x + (int64_t)r * w.C + c, v);
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] *= s;
      uint2 q;
      q.x = pack4<FMT>(v[0], v[1], v[2], v[3]);
      q.y = pack4<FMT>(v[4], v[5], v[6], v[7]);
      *reinterpret_cast<uint2*>(w.y + (int64_t)r * w.C + c) = q;
    } else {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        v[k] = (r < w.R && c + k < w.C) ? to_f(x[(int64_t)r * w.C + c + k]) * s : 0.f;
        if (r < w.R && c + k < w.C) w.y[(int64_t)r * w.C + c + k] = (uint8_t)(pack4<FMT>(v[k], 0.f, 0.f, 0.f) & 0xff);
      }
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) tile[rr][cg + k] = v[k];
  }
  if (!w.yt) return;  // (block-uniform)
  __syncthreads();
  // transposed codes: thread -> (output row c, 8 consecutive r)
  for (int idx = threadIdx.x; idx < 64 * 8; idx += 256) {
    const int cc = idx / 8, rg = (idx % 8) * 8;
    const int c = c0 + cc, r = r0 + rg;
    if (c >= w.C) continue;
    float v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = tile[rg + k][cc];
    if (r + 8 <= w.R && (w.R & 7) == 0) {
      uint2 q;
      q.x = pack4<FMT>(v[0], v[1], v[2], v[3]);
      q.y = pack4<FMT>(v[4], v[5], v[6], v[7]);
      *reinterpret_cast<uint2*>(w.yt + (int64_t)c * w.R + r) = q;
    } else {
      for (int k = 0; k < 8 && r + k < w.R; ++k)
        w.yt[(int64_t)c * w.R + r + k] = (uint8_t)(pack4<FMT>(v[k], 0.f, 0.f, 0.f) & 0xff);
    }
  }
}

inline int grid_for(int64_t n8) {
  int64_t g = (n8 + 255) / 256;
  return (int)(g < 1 ? 1 : g > 1024 ? 1024 : g);  // 4 blocks / CU, grid-stride beyond
}

}  // namespace

#define FP8_DT(DT, T, ...)                                  \
  switch (DT) {                                             \
    case kF32: { using T = float; __VA_ARGS__; } break;     \
    case kF16: { using T = f16; __VA_ARGS__; } break;       \
    case kBF16: { using T = bf16; __VA_ARGS__; } break;     \
    default: return -1;                                     \
  }

int fp8_quantize(const void* x, uint8_t* y, int64_t n, int dt, int fmt, float* scale, float* scale_inv, float* amax,
                 const float* cur, float smax, hipStream_t s) {
  if (n == 0) return 0;
  if (cur && (!scale_inv || smax <= 0.f)) return -2;
  const QScale q{scale, scale_inv, amax, cur, smax};
  const int g = grid_for((n + 7) / 8);
  if (fmt == 0) {
    FP8_DT(dt, T, hipLaunchKernelGGL((quantize_kernel<T, 0>), dim3(g), dim3(256), 0, s, (const T*)x, y, n, q));
  } else {
    FP8_DT(dt, T, hipLaunchKernelGGL((quantize_kernel<T, 1>), dim3(g), dim3(256), 0, s, (const T*)x, y, n, q));
  }
  return (int)hipGetLastError();
}

int fp8_quantize_t(const void* x, uint8_t* y, int R, int C, int dt, int fmt, float* scale, float* scale_inv,
                   float* amax, const float* cur, float smax, hipStream_t s) {
  if (R == 0 || C == 0) return 0;
  if (cur && (!scale_inv || smax <= 0.f)) return -2;
  const QScale q{scale, scale_inv, amax, cur, smax};
  dim3 grid((C + 63) / 64, (R + 63) / 64);
  if (fmt == 0) {
    FP8_DT(dt, T, hipLaunchKernelGGL((quantize_t_kernel<T, 0>), grid, dim3(256), 0, s, (const T*)x, y, R, C, q));
  } else {
    FP8_DT(dt, T, hipLaunchKernelGGL((quantize_t_kernel<T, 1>), grid, dim3(256), 0, s, (const T*)x, y, R, C, q));
  }
  return (int)hipGetLastError();
}

int fp8_amax(const void* x, int64_t n, int dt, float* amax, hipStream_t s) {
  if (n == 0) return 0;
  FP8_DT(dt, T, hipLaunchKernelGGL((amax_kernel<T>), dim3(grid_for((n + 7) / 8)), dim3(256), 0, s, (const T*)x, n, amax));
  return (int)hipGetLastError();
}

int fp8_quantize_weights(const WqDesc* d, int nd, int64_t ablocks, int64_t qblocks, int dt, int fmt, float* scale,
                         float* scale_inv, float* amax, float smax, hipStream_t s) {
  if (nd == 0) return 0;
  if (ablocks <= 0 || qblocks <= 0 || ablocks >= (1ll << 31) || qblocks >= (1ll << 31)) return -2;
  hipLaunchKernelGGL(wq_zero_kernel, dim3(1), dim3(256), 0, s, d, nd, amax);
  FP8_DT(dt, T, hipLaunchKernelGGL((wq_amax_kernel<T>), dim3((int)ablocks), dim3(256), 0, s, d, nd, amax));
  if (fmt == 0) {
    FP8_DT(dt, T, hipLaunchKernelGGL((wq_quant_kernel<T, 0>), dim3((int)qblocks), dim3(256), 0, s, d, nd, scale, scale_inv,
                                     amax, smax));
  } else {
    FP8_DT(dt, T, hipLaunchKernelGGL((wq_quant_kernel<T, 1>), dim3((int)qblocks), dim3(256), 0, s, d, nd, scale, scale_inv,
                                     amax, smax));
  }
  return (int)hipGetLastError();
}

int fp8_update_scales(float* hist, float* amax_cur, float* scale, float* scale_inv, const float* fmt_max,
                      int n_slots, int hist_len, int idx, float margin_scale, hipStream_t s) {
  if (n_slots == 0) return 0;
  hipLaunchKernelGGL(update_scales_kernel, dim3((n_slots + 255) / 256), dim3(256), 0, s, hist, amax_cur, scale,
                     scale_inv, fmt_max, n_slots, hist_len, idx, margin_scale);
  return (int)hipGetLastError();
}

}  // namespace apex
