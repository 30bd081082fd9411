// Fused softmax cross-entropy with label smoothing, forward + backward (NS-06).
//
// One 256-thread block per row. Forward makes ONE pass over the row with an online
// (max, sum-exp) merge per lane, also accumulating sum(x) for label smoothing;
// 16-byte loads. Backward recomputes softmax from the saved per-row log-sum-exp
// (no N x V probability tensor is ever stored) and writes dlogits in the input dtype.
//   loss = (1-s) * (lse - x_y) + s * (lse - mean(x))
//   dx   = dloss * (softmax(x) - (1-s) * onehot(y) - s / V)
#include "common.h"
#include "kernels.h"

namespace apex {

constexpr int kXeBlock = 256;

__device__ __forceinline__ void online_merge(float& m, float& s, float m2, float s2) {
  const float mn = fmaxf(m, m2);
  if (mn == -INFINITY) return;
  s = s * __expf(m - mn) + s2 * __expf(m2 - mn);
  m = mn;
}

template <typename T>
__global__ void __launch_bounds__(kXeBlock) xent_fwd_kernel(const T* __restrict__ x,
                                                           const int64_t* __restrict__ labels,
                                                           float* __restrict__ loss,
                                                           float* __restrict__ lse_out, int V,
                                                           float smoothing, int64_t ignore_index,
                                                           int vec) {
  __shared__ float sm[kXeBlock / 64], ss[kXeBlock / 64], sx[kXeBlock / 64];
  const int64_t row = blockIdx.x;
  const T* xr = x + row * (int64_t)V;
  float m = -INFINITY, s = 0.f, sumx = 0.f;
  if (vec) {
    for (int i = threadIdx.x * 8; i < V; i += kXeBlock * 8) {
      float v[8];
      load_f<T, 8>(xr + i, v);
      float lm = v[0];
#pragma unroll
      for (int k = 1; k < 8; ++k) lm = fmaxf(lm, v[k]);
      float ls = 0.f;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        ls += __expf(v[k] - lm);
        sumx += v[k];
      }
      online_merge(m, s, lm, ls);
    }
  } else {
    for (int i = threadIdx.x; i < V; i += kXeBlock) {
      const float v = to_f(xr[i]);
      online_merge(m, s, v, 1.f);
      sumx += v;
    }
  }
  // wave merge
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float m2 = __shfl_xor(m, o, 64), s2 = __shfl_xor(s, o, 64);
    online_merge(m, s, m2, s2);
    sumx += __shfl_xor(sumx, o, 64);
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) {
    sm[wid] = m;
    ss[wid] = s;
    sx[wid] = sumx;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float M = sm[0], S = ss[0], X = sx[0];
    for (int w = 1; w < kXeBlock / 64; ++w) {
      online_merge(M, S, sm[w], ss[w]);
      X += sx[w];
    }
    const float lse = M + __logf(S);
    const int64_t y = labels[row];
    lse_out[row] = lse;
    if (y == ignore_index || y < 0 || y >= V) {
      loss[row] = 0.f;
    } else {
      const float xy = to_f(xr[y]);
      loss[row] = (1.f - smoothing) * (lse - xy) + smoothing * (lse - X / (float)V);
    }
  }
}

template <typename T, typename G>
__global__ void __launch_bounds__(kXeBlock) xent_bwd_kernel(const G* __restrict__ dloss,
                                                           int64_t dloss_stride,
                                                           const T* __restrict__ x,
                                                           const float* __restrict__ lse,
                                                           const int64_t* __restrict__ labels,
                                                           T* __restrict__ dx, int V,
                                                           float smoothing, int64_t ignore_index,
                                                           int vec) {
  const int64_t row = blockIdx.x;
  const T* xr = x + row * (int64_t)V;
  T* dr = dx + row * (int64_t)V;
  const int64_t y = labels[row];
  const bool ign = (y == ignore_index || y < 0 || y >= V);
  const float g = ign ? 0.f : to_f(dloss[row * dloss_stride]);
  const float L = lse[row];
  const float sv = smoothing / (float)V;
  const float on = 1.f - smoothing;
  if (vec) {
    for (int i = threadIdx.x * 8; i < V; i += kXeBlock * 8) {
      float v[8];
      load_f<T, 8>(xr + i, v);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        float p = __expf(v[k] - L) - sv;
        if (i + k == y) p -= on;
        v[k] = g * p;
      }
      store_f<T, 8>(dr + i, v);
    }
  } else {
    for (int i = threadIdx.x; i < V; i += kXeBlock) {
      float p = __expf(to_f(xr[i]) - L) - sv;
      if (i == y) p -= on;
      dr[i] = from_f<T>(g * p);
    }
  }
}

#define XE_DISPATCH(DT, T, ...)                             \
  switch (DT) {                                             \
    case kF32: { using T = float; __VA_ARGS__; } break;     \
    case kF16: { using T = f16; __VA_ARGS__; } break;       \
    case kBF16: { using T = bf16; __VA_ARGS__; } break;     \
    default: return -1;                                     \
  }

int xentropy_fwd(const void* logits, const int64_t* labels, float* losses, float* lse, int64_t rows,
                 int V, float smoothing, int64_t ignore_index, int dt, hipStream_t s) {
  if (rows == 0) return 0;
  const int vec = (V % 8 == 0) && (((uintptr_t)logits & 15) == 0);
  XE_DISPATCH(dt, T,
      hipLaunchKernelGGL((xent_fwd_kernel<T>), dim3((unsigned)rows), dim3(kXeBlock), 0, s,
                         (const T*)logits, labels, losses, lse, V, smoothing, ignore_index, vec));
  return (int)hipGetLastError();
}

int xentropy_bwd(const void* dloss, int64_t dloss_stride, int dloss_dt, const void* logits,
                 const float* lse, const int64_t* labels, void* dlogits, int64_t rows, int V,
                 float smoothing, int64_t ignore_index, int dt, hipStream_t s) {
  if (rows == 0) return 0;
  const int vec = (V % 8 == 0) && (((uintptr_t)logits & 15) == 0) && (((uintptr_t)dlogits & 15) == 0);
  XE_DISPATCH(dt, T, XE_DISPATCH(dloss_dt, G,
      hipLaunchKernelGGL((xent_bwd_kernel<T, G>), dim3((unsigned)rows), dim3(kXeBlock), 0, s,
                         (const G*)dloss, dloss_stride, (const T*)logits, lse, labels, (T*)dlogits,
                         V, smoothing, ignore_index, vec)));
  return (int)hipGetLastError();
}

}  // namespace apex
