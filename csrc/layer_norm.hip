// FusedLayerNorm / FusedRMSNorm forward + backward (NS-03).
//
// Fast path (cols % 8 == 0, cols <= 4096): one wave64 per row; each lane keeps
// VPT 16-byte vectors of the row in registers, so x is read from HBM exactly
// once in fwd and once in bwd (exact two-pass mean/var from registers).
// Backward fuses dgamma/dbeta: a lane always owns the same columns, so a wave
// accumulates them across all its rows in registers, the 4 waves of a block
// combine through LDS and write one fp32 partial row; a column-reduction kernel
// sums the partials (deterministic, no float atomics).
// Slow path (any cols): block-per-row kernels + column-tile dgamma kernel.
#include "common.h"
#include "kernels.h"

namespace apex {

constexpr int kLnBlock = 256;
constexpr int kMaxBwdParts = 768;  // 3 blocks per CU; rows per wave adapts to reach it

template <typename T, typename W, int VPT, bool RMS>
__global__ void __launch_bounds__(kLnBlock) ln_fwd_fast(const T* __restrict__ x,
                                                       const W* __restrict__ gamma,
                                                       const W* __restrict__ beta, T* __restrict__ y,
                                                       float* __restrict__ mean,
                                                       float* __restrict__ rstd, int64_t rows,
                                                       int cols, float eps) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * (kLnBlock / 64) + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int nvec = cols >> 3;
  const T* xr = x + row * cols;
  float v[VPT][8];
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < VPT; ++j) {
    const int vi = j * 64 + lane;
    if (vi < nvec) {
      load_f<T, 8>(xr + vi * 8, v[j]);
#pragma unroll
      for (int k = 0; k < 8; ++k) s += v[j][k];
    } else {
#pragma unroll
      for (int k = 0; k < 8; ++k) v[j][k] = 0.f;
    }
  }
  const float inv_n = 1.f / (float)cols;
  float mu = 0.f;
  if (!RMS) mu = wave_sum(s) * inv_n;
  float ss = 0.f;
#pragma unroll
  for (int j = 0; j < VPT; ++j) {
    const int vi = j * 64 + lane;
    if (vi < nvec) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float d = v[j][k] - mu;
        ss += d * d;
      }
    }
  }
  const float rs = rsqrtf(wave_sum(ss) * inv_n + eps);
  if (lane == 0) {
    if (mean) mean[row] = mu;
    rstd[row] = rs;
  }
  T* yr = y + row * cols;
#pragma unroll
  for (int j = 0; j < VPT; ++j) {
    const int vi = j * 64 + lane;
    if (vi < nvec) {
      float g[8], b[8], o[8];
      if (gamma) load_f<W, 8>(gamma + vi * 8, g);
      else {
#pragma unroll
        for (int k = 0; k < 8; ++k) g[k] = 1.f;
      }
      if (beta) load_f<W, 8>(beta + vi * 8, b);
      else {
#pragma unroll
        for (int k = 0; k < 8; ++k) b[k] = 0.f;
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) o[k] = (v[j][k] - mu) * rs * g[k] + b[k];
      store_f<T, 8>(yr + vi * 8, o);
    }
  }
}

// dx + per-block partial dgamma/dbeta. ws row p = [dgamma(cols) | dbeta(cols)]
template <typename T, typename W, int VPT, bool RMS>
__global__ void __launch_bounds__(kLnBlock) ln_bwd_fast(const T* __restrict__ dy,
                                                       const T* __restrict__ x,
                                                       const W* __restrict__ gamma,
                                                       const float* __restrict__ mean,
                                                       const float* __restrict__ rstd,
                                                       T* __restrict__ dx, float* __restrict__ ws,
                                                       int64_t rows, int cols, int rpw) {
  extern __shared__ __attribute__((aligned(16))) float lds[];  // [4 waves][2*cols]
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int nvec = cols >> 3;
  const float inv_n = 1.f / (float)cols;
  float dg[VPT][8], db[VPT][8], g[VPT][8];
#pragma unroll
  for (int j = 0; j < VPT; ++j) {
    const int vi = j * 64 + lane;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      dg[j][k] = 0.f;
      db[j][k] = 0.f;
      g[j][k] = 1.f;
    }
    if (gamma && vi < nvec) load_f<W, 8>(gamma + vi * 8, g[j]);
  }
  const int64_t rows_per_block = (int64_t)rpw * (kLnBlock / 64);
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
  // the next row's x / dy are loaded (raw 16-byte packs) before this row's reduction and stores:
  // two rows of loads in flight per wave (one row per wave left the kernel latency-bound at
  // ~3.9 TB/s, profiles/r2_pmc_bw_kernels.json)
  typedef Pack<T, 8> P8;
  P8 nx[VPT], nd[VPT];
  auto fetch = [&](int64_t row) {
#pragma unroll
    for (int j = 0; j < VPT; ++j) {
      const int vi = j * 64 + lane;
      if (vi < nvec && row < rows) {
        nx[j] = *reinterpret_cast<const P8*>(x + row * cols + vi * 8);
        nd[j] = *reinterpret_cast<const P8*>(dy + row * cols + vi * 8);
      }
    }
  };
  fetch(r0 + wid);
  for (int rr = 0; rr < rpw; ++rr) {
    const int64_t row = r0 + (int64_t)rr * (kLnBlock / 64) + wid;
    if (row >= rows) break;
    float xh[VPT][8], dv[VPT][8];
#pragma unroll
    for (int j = 0; j < VPT; ++j)
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        xh[j][k] = to_f(nx[j].v[k]);
        dv[j][k] = to_f(nd[j].v[k]);
      }
    if (rr + 1 < rpw) fetch(row + (kLnBlock / 64));
    const float mu = RMS ? 0.f : mean[row];
    const float rs = rstd[row];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int j = 0; j < VPT; ++j) {
      const int vi = j * 64 + lane;
      if (vi < nvec) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          xh[j][k] = (xh[j][k] - mu) * rs;
          const float dyg = dv[j][k] * g[j][k];
          s1 += dyg;
          s2 += dyg * xh[j][k];
          dg[j][k] += dv[j][k] * xh[j][k];
          db[j][k] += dv[j][k];
        }
      }
    }
    s2 = wave_sum(s2) * inv_n;
    if (!RMS) s1 = wave_sum(s1) * inv_n;
    T* dxr = dx + row * cols;
#pragma unroll
    for (int j = 0; j < VPT; ++j) {
      const int vi = j * 64 + lane;
      if (vi < nvec) {
        float o[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const float dyg = dv[j][k] * g[j][k];
          o[k] = RMS ? rs * (dyg - xh[j][k] * s2) : rs * (dyg - s1 - xh[j][k] * s2);
        }
        store_f<T, 8>(dxr + vi * 8, o);
      }
    }
  }
  // combine the 4 waves' column partials through LDS
  float* mine = lds + wid * 2 * cols;
#pragma unroll
  for (int j = 0; j < VPT; ++j) {
    const int vi = j * 64 + lane;
    if (vi < nvec) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        mine[vi * 8 + k] = dg[j][k];
        mine[cols + vi * 8 + k] = db[j][k];
      }
    }
  }
  __syncthreads();
  float* out = ws + (int64_t)blockIdx.x * 2 * cols;
  for (int c = threadIdx.x; c < 2 * cols; c += kLnBlock) {
    float a = 0.f;
#pragma unroll
    for (int w = 0; w < kLnBlock / 64; ++w) a += lds[w * 2 * cols + c];
    out[c] = a;
  }
}

// Wide rows (VPT 5..8 vectors per lane, e.g. Megatron's H = 2560 / 4096): the register-resident
// fast kernel would need 4 x VPT x 8 fp32 row/partial registers, so this one keeps only the
// dgamma / dbeta partials in registers and reads each row twice (the second pass hits L1/L2: a row
// is 5-8 KB), with gamma from cache. Same per-block partial rows as ln_bwd_fast (replaces the
// block-per-row dx kernel + strided column kernel of the slow path).
template <typename T, typename W, int VPT, bool RMS>
__global__ void __launch_bounds__(kLnBlock) ln_bwd_wide(const T* __restrict__ dy,
                                                       const T* __restrict__ x,
                                                       const W* __restrict__ gamma,
                                                       const float* __restrict__ mean,
                                                       const float* __restrict__ rstd,
                                                       T* __restrict__ dx, float* __restrict__ ws,
                                                       int64_t rows, int cols, int rpw) {
  extern __shared__ __attribute__((aligned(16))) float lds[];  // [4 waves][cols]
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int nvec = cols >> 3;
  const float inv_n = 1.f / (float)cols;
  float dg[VPT][8], db[VPT][8];
#pragma unroll
  for (int j = 0; j < VPT; ++j)
#pragma unroll
    for (int k = 0; k < 8; ++k) dg[j][k] = db[j][k] = 0.f;
  auto gam = [&](int vi, float (&g)[8]) {
    if (gamma) load_f<W, 8>(gamma + vi * 8, g);
    else {
#pragma unroll
      for (int k = 0; k < 8; ++k) g[k] = 1.f;
    }
  };
  const int64_t r0 = (int64_t)blockIdx.x * rpw * (kLnBlock / 64);
  for (int rr = 0; rr < rpw; ++rr) {
    const int64_t row = r0 + (int64_t)rr * (kLnBlock / 64) + wid;
    if (row >= rows) break;
    const float mu = RMS ? 0.f : mean[row];
    const float rs = rstd[row];
    const T* xr = x + row * cols;
    const T* dyr = dy + row * cols;
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int j = 0; j < VPT; ++j) {
      const int vi = j * 64 + lane;
      if (vi < nvec) {
        float xv[8], dv[8], g[8];
        load_f<T, 8>(xr + vi * 8, xv);
        load_f<T, 8>(dyr + vi * 8, dv);
        gam(vi, g);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const float xh = (xv[k] - mu) * rs;
          const float dyg = dv[k] * g[k];
          s1 += dyg;
          s2 += dyg * xh;
          dg[j][k] += dv[k] * xh;
          db[j][k] += dv[k];
        }
      }
    }
    s2 = wave_sum(s2) * inv_n;
    if (!RMS) s1 = wave_sum(s1) * inv_n;
    T* dxr = dx + row * cols;
#pragma unroll
    for (int j = 0; j < VPT; ++j) {
      const int vi = j * 64 + lane;
      if (vi < nvec) {
        float xv[8], dv[8], g[8], o[8];
        load_f<T, 8>(xr + vi * 8, xv);
        load_f<T, 8>(dyr + vi * 8, dv);
        gam(vi, g);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const float xh = (xv[k] - mu) * rs;
          const float dyg = dv[k] * g[k];
          o[k] = RMS ? rs * (dyg - xh * s2) : rs * (dyg - s1 - xh * s2);
        }
        store_f<T, 8>(dxr + vi * 8, o);
      }
    }
  }
  // combine the 4 waves' partials through LDS, dgamma then dbeta ([4 waves][cols] each: <= 64 KB)
  float* mine = lds + wid * cols;
  float* out = ws + (int64_t)blockIdx.x * 2 * cols;
#pragma unroll
  for (int half = 0; half < 2; ++half) {
    if (half) __syncthreads();
#pragma unroll
    for (int j = 0; j < VPT; ++j) {
      const int vi = j * 64 + lane;
      if (vi < nvec) {
#pragma unroll
        for (int k = 0; k < 8; ++k) mine[vi * 8 + k] = half ? db[j][k] : dg[j][k];
      }
    }
    __syncthreads();
    for (int c = threadIdx.x; c < cols; c += kLnBlock) {
      float a = 0.f;
#pragma unroll
      for (int w = 0; w < kLnBlock / 64; ++w) a += lds[w * cols + c];
      out[half * cols + c] = a;
    }
  }
}

// ------------------------------ slow path ----------------------------------
template <typename T, typename W, bool RMS>
__global__ void __launch_bounds__(kLnBlock) ln_fwd_slow(const T* __restrict__ x,
                                                       const W* __restrict__ gamma,
                                                       const W* __restrict__ beta, T* __restrict__ y,
                                                       float* __restrict__ mean,
                                                       float* __restrict__ rstd, int cols,
                                                       float eps) {
  __shared__ float red[kLnBlock / 64];
  const int64_t row = blockIdx.x;
  const T* xr = x + row * cols;
  float s = 0.f;
  for (int c = threadIdx.x; c < cols; c += kLnBlock) s += to_f(xr[c]);
  const float mu = RMS ? 0.f : block_sum(s, red) / cols;
  float ss = 0.f;
  for (int c = threadIdx.x; c < cols; c += kLnBlock) {
    const float d = to_f(xr[c]) - mu;
    ss += d * d;
  }
  const float rs = rsqrtf(block_sum(ss, red) / cols + eps);
  if (threadIdx.x == 0) {
    if (mean) mean[row] = mu;
    rstd[row] = rs;
  }
  T* yr = y + row * cols;
  for (int c = threadIdx.x; c < cols; c += kLnBlock) {
    const float g = gamma ? to_f(gamma[c]) : 1.f;
    const float b = beta ? to_f(beta[c]) : 0.f;
    yr[c] = from_f<T>((to_f(xr[c]) - mu) * rs * g + b);
  }
}

template <typename T, typename W, bool RMS>
__global__ void __launch_bounds__(kLnBlock) ln_bwd_dx_slow(const T* __restrict__ dy,
                                                          const T* __restrict__ x,
                                                          const W* __restrict__ gamma,
                                                          const float* __restrict__ mean,
                                                          const float* __restrict__ rstd,
                                                          T* __restrict__ dx, int cols) {
  __shared__ float red[kLnBlock / 64];
  const int64_t row = blockIdx.x;
  const float mu = RMS ? 0.f : mean[row];
  const float rs = rstd[row];
  const T* xr = x + row * cols;
  const T* dyr = dy + row * cols;
  float s1 = 0.f, s2 = 0.f;
  for (int c = threadIdx.x; c < cols; c += kLnBlock) {
    const float g = gamma ? to_f(gamma[c]) : 1.f;
    const float dyg = to_f(dyr[c]) * g;
    s1 += dyg;
    s2 += dyg * (to_f(xr[c]) - mu) * rs;
  }
  s1 = block_sum(s1, red) / cols;
  s2 = block_sum(s2, red) / cols;
  T* dxr = dx + row * cols;
  for (int c = threadIdx.x; c < cols; c += kLnBlock) {
    const float g = gamma ? to_f(gamma[c]) : 1.f;
    const float dyg = to_f(dyr[c]) * g;
    const float xh = (to_f(xr[c]) - mu) * rs;
    dxr[c] = from_f<T>(RMS ? rs * (dyg - xh * s2) : rs * (dyg - s1 - xh * s2));
  }
}

// grid (ceil(cols/256), parts): partial column sums over a row range.
template <typename T, bool RMS>
__global__ void __launch_bounds__(kLnBlock) ln_bwd_gb_slow(const T* __restrict__ dy,
                                                          const T* __restrict__ x,
                                                          const float* __restrict__ mean,
                                                          const float* __restrict__ rstd,
                                                          float* __restrict__ ws, int64_t rows,
                                                          int cols, int64_t rows_per_part) {
  const int c = blockIdx.x * kLnBlock + threadIdx.x;
  if (c >= cols) return;
  const int64_t r0 = (int64_t)blockIdx.y * rows_per_part;
  const int64_t r1 = r0 + rows_per_part < rows ? r0 + rows_per_part : rows;
  float dg = 0.f, db = 0.f;
  for (int64_t r = r0; r < r1; ++r) {
    const float mu = RMS ? 0.f : mean[r];
    const float d = to_f(dy[r * cols + c]);
    dg += d * (to_f(x[r * cols + c]) - mu) * rstd[r];
    db += d;
  }
  float* out = ws + (int64_t)blockIdx.y * 2 * cols;
  out[c] = dg;
  out[cols + c] = db;
}

static inline int ln_vpt(int cols) {
  if (cols % 8 != 0) return 0;
  const int nvec = cols / 8;
  if (nvec <= 64) return 1;
  if (nvec <= 128) return 2;
  if (nvec <= 256) return 4;
  if (nvec <= 512) return 8;
  return 0;
}

static inline bool ln_fast_ok(const void* a, const void* b, const void* c, const void* d, int cols) {
  auto al = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
  return ln_vpt(cols) > 0 && al(a) && al(b) && al(c) && al(d);
}

static inline int ln_bwd_rpw(int64_t rows) {
  const int64_t r = (rows + 4 * kMaxBwdParts - 1) / (4 * kMaxBwdParts);
  return r < 1 ? 1 : (int)r;
}

int64_t layer_norm_bwd_ws_floats(int64_t rows, int cols) {
  (void)rows;
  return (int64_t)kMaxBwdParts * 2 * (int64_t)cols;
}

#define LN_DISPATCH_T(DT, T, ...)                           \
  switch (DT) {                                             \
    case kF32: { using T = float; __VA_ARGS__; } break;     \
    case kF16: { using T = f16; __VA_ARGS__; } break;       \
    case kBF16: { using T = bf16; __VA_ARGS__; } break;     \
    default: return -1;                                     \
  }

#define LN_DISPATCH_VPT(V, VPT, ...)                        \
  switch (V) {                                              \
    case 1: { constexpr int VPT = 1; __VA_ARGS__; } break;  \
    case 2: { constexpr int VPT = 2; __VA_ARGS__; } break;  \
    case 4: { constexpr int VPT = 4; __VA_ARGS__; } break;  \
    case 8: { constexpr int VPT = 8; __VA_ARGS__; } break;  \
    default: return -1;                                     \
  }

#define LN_DISPATCH_RMS(R, RMS, ...)                        \
  if (R) { constexpr bool RMS = true; __VA_ARGS__; }        \
  else { constexpr bool RMS = false; __VA_ARGS__; }

int layer_norm_fwd(const void* x, const void* gamma, const void* beta, void* y, float* mean,
                   float* rstd, int64_t rows, int cols, float eps, int xdt, int wdt, int rms,
                   hipStream_t s) {
  if (rows == 0) return 0;
  if (!gamma && !beta) wdt = xdt;
  const bool fast = ln_fast_ok(x, y, gamma, beta, cols);
  LN_DISPATCH_T(xdt, T, LN_DISPATCH_T(wdt, W, LN_DISPATCH_RMS(rms, RMS, {
    if (fast) {
      const int vpt = ln_vpt(cols);
      const int64_t grid = (rows + 3) / 4;
      LN_DISPATCH_VPT(vpt, VPT,
          hipLaunchKernelGGL((ln_fwd_fast<T, W, VPT, RMS>), dim3((unsigned)grid), dim3(kLnBlock), 0,
                             s, (const T*)x, (const W*)gamma, (const W*)beta, (T*)y, mean, rstd,
                             rows, cols, eps));
    } else {
      hipLaunchKernelGGL((ln_fwd_slow<T, W, RMS>), dim3((unsigned)rows), dim3(kLnBlock), 0, s,
                         (const T*)x, (const W*)gamma, (const W*)beta, (T*)y, mean, rstd, cols, eps);
    }
  })));
  return (int)hipGetLastError();
}

int layer_norm_bwd(const void* dy, const void* x, const void* gamma, const float* mean,
                   const float* rstd, void* dx, void* dgamma, void* dbeta, float* ws, int64_t rows,
                   int cols, int xdt, int wdt, int rms, hipStream_t s) {
  if (rows == 0) return 0;
  if (!gamma) wdt = xdt;
  const bool fast = ln_fast_ok(x, dy, dx, gamma, cols) && ln_vpt(cols) <= 4;
  // wide rows: 5..8 16-byte vectors per lane (cols 2056 .. 4096)
  const int wvpt = (cols % 8 == 0 && cols / 8 > 256 && cols / 8 <= 512) ? (cols / 8 + 63) / 64 : 0;
  const bool wide = !fast && wvpt > 0 && ln_fast_ok(x, dy, dx, gamma, cols);
  const bool need_gb = dgamma || dbeta;
  LN_DISPATCH_T(xdt, T, LN_DISPATCH_T(wdt, W, LN_DISPATCH_RMS(rms, RMS, {
    int parts;
    if (fast) {
      const int vpt = ln_vpt(cols);
      const int rpw = ln_bwd_rpw(rows);
      const int64_t rpb = (int64_t)rpw * (kLnBlock / 64);
      parts = (int)((rows + rpb - 1) / rpb);
      const size_t lds = (size_t)4 * 2 * cols * sizeof(float);
      LN_DISPATCH_VPT(vpt, VPT,
          hipLaunchKernelGGL((ln_bwd_fast<T, W, VPT, RMS>), dim3(parts), dim3(kLnBlock), lds, s,
                             (const T*)dy, (const T*)x, (const W*)gamma, mean, rstd, (T*)dx, ws,
                             rows, cols, rpw));
    } else if (wide) {
      const int rpw = ln_bwd_rpw(rows);
      const int64_t rpb = (int64_t)rpw * (kLnBlock / 64);
      parts = (int)((rows + rpb - 1) / rpb);
      const size_t lds = (size_t)4 * cols * sizeof(float);
      switch (wvpt) {
        case 5: hipLaunchKernelGGL((ln_bwd_wide<T, W, 5, RMS>), dim3(parts), dim3(kLnBlock), lds, s, (const T*)dy,
                                   (const T*)x, (const W*)gamma, mean, rstd, (T*)dx, ws, rows, cols, rpw); break;
        case 6: hipLaunchKernelGGL((ln_bwd_wide<T, W, 6, RMS>), dim3(parts), dim3(kLnBlock), lds, s, (const T*)dy,
                                   (const T*)x, (const W*)gamma, mean, rstd, (T*)dx, ws, rows, cols, rpw); break;
        case 7: hipLaunchKernelGGL((ln_bwd_wide<T, W, 7, RMS>), dim3(parts), dim3(kLnBlock), lds, s, (const T*)dy,
                                   (const T*)x, (const W*)gamma, mean, rstd, (T*)dx, ws, rows, cols, rpw); break;
        default: hipLaunchKernelGGL((ln_bwd_wide<T, W, 8, RMS>), dim3(parts), dim3(kLnBlock), lds, s, (const T*)dy,
                                    (const T*)x, (const W*)gamma, mean, rstd, (T*)dx, ws, rows, cols, rpw); break;
      }
    } else {
      hipLaunchKernelGGL((ln_bwd_dx_slow<T, W, RMS>), dim3((unsigned)rows), dim3(kLnBlock), 0, s,
                         (const T*)dy, (const T*)x, (const W*)gamma, mean, rstd, (T*)dx, cols);
      parts = 256;
      if (need_gb) {
        const int64_t rpp = (rows + parts - 1) / parts;
        hipLaunchKernelGGL((ln_bwd_gb_slow<T, RMS>), dim3((cols + kLnBlock - 1) / kLnBlock, parts),
                           dim3(kLnBlock), 0, s, (const T*)dy, (const T*)x, mean, rstd, ws, rows,
                           cols, rpp);
      }
    }
    if (need_gb) {
      launch_partial_colsum3<W>(ws, parts, 2 * (int64_t)cols, cols, (W*)dgamma, (W*)dbeta, (W*)nullptr, s);
    }
  })));
  return (int)hipGetLastError();
}

}  // namespace apex
