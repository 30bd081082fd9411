// Fused scale + mask + softmax forward/backward (apex.transformer.functional
// FusedScaleMaskSoftmax; the Megatron "scaled_masked_softmax" / "scaled_upper_triang_masked_
// softmax" kernels re-designed for wave64).
//
// One wave64 per row while the row fits in registers (cols <= 64 * 8 * KPL), 16-byte loads,
// fp32 max/sum via xor-shuffles; mask modes: none, byte mask [B, 1|H, Sq, Sk] (nonzero =
// masked -> -10000 like the reference kernels), causal (key > query masked).
// Backward: dx = scale * y * (dy - sum(dy * y)), one wave per row.
#include "common.h"
#include "kernels.h"

namespace apex {

template <typename T, int KPL, int MODE>
__global__ void __launch_bounds__(256) smx_fwd_kernel(const T* __restrict__ x, const uint8_t* __restrict__ mask,
                                                     T* __restrict__ y, int64_t rows, int cols, int sq,
                                                     int heads, int mask_heads, float scale) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int q = (int)(row % sq);
  const int64_t bh = row / sq;
  const uint8_t* mrow = nullptr;
  if (MODE == 1) {
    const int64_t b = bh / heads, h = bh % heads;
    mrow = mask + ((b * mask_heads + (mask_heads == 1 ? 0 : h)) * sq + q) * (int64_t)cols;
  }
  const T* xr = x + row * cols;
  float v[KPL][8];
  float mx = -INFINITY;
#pragma unroll
  for (int j = 0; j < KPL; ++j) {
    const int c0 = (j * 64 + lane) * 8;
    if (c0 < cols) {
      load_f<T, 8>(xr + c0, v[j]);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        float t = v[j][k] * scale;
        if (MODE == 1 && mrow[c0 + k]) t = -10000.f;
        if (MODE == 2 && c0 + k > q) t = -INFINITY;
        v[j][k] = t;
        mx = fmaxf(mx, t);
      }
    } else {
#pragma unroll
      for (int k = 0; k < 8; ++k) v[j][k] = -INFINITY;
    }
  }
  mx = wave_max(mx);
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < KPL; ++j)
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float e = v[j][k] == -INFINITY ? 0.f : __expf(v[j][k] - mx);
      v[j][k] = e;
      s += e;
    }
  s = wave_sum(s);
  const float inv = s > 0.f ? 1.f / s : 0.f;
  T* yr = y + row * cols;
#pragma unroll
  for (int j = 0; j < KPL; ++j) {
    const int c0 = (j * 64 + lane) * 8;
    if (c0 < cols) {
      float o[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) o[k] = v[j][k] * inv;
      store_f<T, 8>(yr + c0, o);
    }
  }
}

template <typename T, int KPL>
__global__ void __launch_bounds__(256) smx_bwd_kernel(const T* __restrict__ dy, const T* __restrict__ y,
                                                     T* __restrict__ dx, int64_t rows, int cols, float scale) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  float a[KPL][8], b[KPL][8];
  float dot = 0.f;
#pragma unroll
  for (int j = 0; j < KPL; ++j) {
    const int c0 = (j * 64 + lane) * 8;
    if (c0 < cols) {
      load_f<T, 8>(dy + row * cols + c0, a[j]);
      load_f<T, 8>(y + row * cols + c0, b[j]);
#pragma unroll
      for (int k = 0; k < 8; ++k) dot += a[j][k] * b[j][k];
    }
  }
  dot = wave_sum(dot);
#pragma unroll
  for (int j = 0; j < KPL; ++j) {
    const int c0 = (j * 64 + lane) * 8;
    if (c0 < cols) {
      float o[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) o[k] = scale * b[j][k] * (a[j][k] - dot);
      store_f<T, 8>(dx + row * cols + c0, o);
    }
  }
}

#define SMX_DISPATCH(DT, T, ...)                            \
  switch (DT) {                                             \
    case kF32: { using T = float; __VA_ARGS__; } break;     \
    case kF16: { using T = f16; __VA_ARGS__; } break;       \
    case kBF16: { using T = bf16; __VA_ARGS__; } break;     \
    default: return -1;                                     \
  }
#define SMX_KPL(C, KPL, ...)                                \
  if ((C) <= 512) { constexpr int KPL = 1; __VA_ARGS__; }   \
  else if ((C) <= 1024) { constexpr int KPL = 2; __VA_ARGS__; } \
  else if ((C) <= 2048) { constexpr int KPL = 4; __VA_ARGS__; } \
  else if ((C) <= 4096) { constexpr int KPL = 8; __VA_ARGS__; } \
  else { return -2; }

int scaled_softmax_supported(int cols) { return cols % 8 == 0 && cols <= 4096; }

int scaled_masked_softmax_fwd(const void* x, const uint8_t* mask, void* y, int64_t rows, int cols, int sq,
                              int heads, int mask_heads, float scale, int mode, int dt, hipStream_t s) {
  if (rows == 0) return 0;
  if (!scaled_softmax_supported(cols)) return -2;
  const dim3 grid((unsigned)((rows + 3) / 4));
  SMX_DISPATCH(dt, T, SMX_KPL(cols, KPL, {
    if (mode == 0)
      hipLaunchKernelGGL((smx_fwd_kernel<T, KPL, 0>), grid, dim3(256), 0, s, (const T*)x, mask, (T*)y, rows, cols,
                         sq, heads, mask_heads, scale);
    else if (mode == 1)
      hipLaunchKernelGGL((smx_fwd_kernel<T, KPL, 1>), grid, dim3(256), 0, s, (const T*)x, mask, (T*)y, rows, cols,
                         sq, heads, mask_heads, scale);
    else
      hipLaunchKernelGGL((smx_fwd_kernel<T, KPL, 2>), grid, dim3(256), 0, s, (const T*)x, mask, (T*)y, rows, cols,
                         sq, heads, mask_heads, scale);
  }));
  return (int)hipGetLastError();
}

int scaled_masked_softmax_bwd(const void* dy, const void* y, void* dx, int64_t rows, int cols, float scale, int dt,
                              hipStream_t s) {
  if (rows == 0) return 0;
  if (!scaled_softmax_supported(cols)) return -2;
  const dim3 grid((unsigned)((rows + 3) / 4));
  SMX_DISPATCH(dt, T, SMX_KPL(cols, KPL,
      hipLaunchKernelGGL((smx_bwd_kernel<T, KPL>), grid, dim3(256), 0, s, (const T*)dy, (const T*)y, (T*)dx, rows,
                         cols, scale)));
  return (int)hipGetLastError();
}

}  // namespace apex
