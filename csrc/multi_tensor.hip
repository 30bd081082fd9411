// Multi-tensor fused kernels: unscale+overflow (K-01), copy-cast (K-02), l2norm (K-07),
// axpby, and the fused optimizers SGD / Adam(W) / LAMB / NovoGrad-lite (NS-02).
//
// Reference behaviour being replaced:
//   apex/amp/scaler.py:6-18            per-param float(g.sum()) host sync + g.mul_
//   apex/fp16_utils/fp16util.py:93-129 master<->model copies
//   apex/parallel/LARC.py:79-82        per-param host-synced norms
// Design: one launch per op over a device-resident chunk table (multi_tensor.h).
// 256-thread blocks (4 x wave64), grid capped at 8 blocks/CU and grid-strided over chunks; the
// single-pass kernels (scale, l2norm, SGD, Adam, LAMB) sweep a chunk with stream_for (lane-
// contiguous 4-element groups, 4 in flight per lane, non-temporal state traffic), the rest with
// chunk_for (8 contiguous elements per lane).
#include <type_traits>

#include "common.h"
#include "kernels.h"
#include "multi_tensor.h"

namespace apex {

using I8 = std::integral_constant<int, 8>;
using I1 = std::integral_constant<int, 1>;

constexpr int kBlock = 256;
constexpr int kMaxGrid = 2048;

struct ChunkView {
  int t;
  int64_t start;
  int64_t n;
};

__device__ __forceinline__ ChunkView chunk_view(const MTMeta& m, int c) {
  const int64_t e = m.chunks[c];
  ChunkView v;
  v.t = (int)(e >> kChunkShift);
  v.start = (e & ((1LL << kChunkShift) - 1)) * (int64_t)m.chunk_size;
  const int64_t rem = m.numel[v.t] - v.start;
  v.n = rem < m.chunk_size ? rem : m.chunk_size;
  return v;
}

// Calls body(I8{}, i) for vector groups and body(I1{}, i) for the scalar tail.
template <typename Body>
__device__ __forceinline__ void chunk_for(const MTMeta& m, int64_t n, Body&& body) {
  const int64_t nv = m.aligned ? (n & ~int64_t(7)) : 0;
  for (int64_t i = threadIdx.x * 8; i < nv; i += (int64_t)blockDim.x * 8) body(I8{}, i);
  for (int64_t i = nv + threadIdx.x; i < n; i += blockDim.x) body(I1{}, i);
}

// Streaming sweep of one chunk for the single-pass optimizer / scaler kernels: each lane owns
// 4-element groups laid out lane-contiguously (one wave instruction = 1 KB of fp32 contiguous,
// not every other 16 B of a 2 KB span), kStreamU groups per lane per iteration with all their
// loads issued before any store (aliasing keeps the compiler from hoisting the next
// iteration's loads above this one's stores, so the in-flight bytes have to be explicit).
// body(IG<NG>, IG<NE>, j0, stride): NG groups of NE elements at j0 + g * stride, g < NG.
// tools/bwlab/adam_lab.hip: the Adam stream at 6.42 TB/s with nt loads/stores (= the read-only
// ceiling of the same four fp32 streams) vs 5.84 for the 8-contiguous-elements layout.
template <int G>
using IG = std::integral_constant<int, G>;
constexpr int kStreamU = 4;
constexpr int kGroup = 4;

template <typename Body>
__device__ __forceinline__ void stream_for(const MTMeta& m, int64_t n, Body&& body) {
  const int64_t nv = m.aligned ? (n & ~int64_t(kGroup - 1)) : 0;
  constexpr int64_t kStride = (int64_t)kBlock * kGroup;
  constexpr int64_t kStep = kStride * kStreamU;
  const int64_t t4 = (int64_t)threadIdx.x * kGroup;
  int64_t base = 0;
  for (; base + kStep <= nv; base += kStep) body(IG<kStreamU>{}, IG<kGroup>{}, base + t4, kStride);
  for (int64_t j = base + t4; j < nv; j += kStride) body(IG<1>{}, IG<kGroup>{}, j, 0);
  for (int64_t j = nv + threadIdx.x; j < n; j += kBlock) body(IG<1>{}, IG<1>{}, j, 0);
}

__device__ __forceinline__ float read_scale(const float* p, float v) { return p ? *p : v; }

static inline int grid_for(int nchunks) {
  return nchunks < kMaxGrid ? (nchunks > 0 ? nchunks : 1) : kMaxGrid;
}

// ---------------------------------------------------------------------------
// scale: out = in * s ; flag non-finite inputs.  (K-01 / K-02)
// ---------------------------------------------------------------------------
template <typename TI, typename TO>
__global__ void __launch_bounds__(kBlock) scale_kernel(MTMeta m, const float* sp, float sv,
                                                      int* overflow) {
  const float s = read_scale(sp, sv);
  bool bad = false;
  for (int c = blockIdx.x; c < m.nchunks; c += gridDim.x) {
    const ChunkView cv = chunk_view(m, c);
    const TI* in = (const TI*)m.ptr(0, cv.t) + cv.start;
    TO* out = (TO*)m.ptr(1, cv.t) + cv.start;
    stream_for(m, cv.n, [&](auto NGc, auto NEc, int64_t j0, int64_t st) {
      constexpr int NG = decltype(NGc)::value, NE = decltype(NEc)::value;
      float x[NG][NE];
#pragma unroll
      for (int u = 0; u < NG; ++u) load_f_nt<TI, NE>(in + j0 + u * st, x[u]);
#pragma unroll
      for (int u = 0; u < NG; ++u)
#pragma unroll
        for (int k = 0; k < NE; ++k) {
          bad |= !__builtin_isfinite(x[u][k]);
          x[u][k] *= s;
        }
#pragma unroll
      for (int u = 0; u < NG; ++u) store_f<TO, NE>(out + j0 + u * st, x[u]);
    });
  }
  if (bad && overflow) *overflow = 1;
}

// ---------------------------------------------------------------------------
// axpby: out = a*x + b*y ; check = -1 both, 0 x only, 1 y only
// ---------------------------------------------------------------------------
template <typename TX, typename TY, typename TO>
__global__ void __launch_bounds__(kBlock) axpby_kernel(MTMeta m, float a, float b, int check,
                                                      int* overflow) {
  bool bad = false;
  for (int c = blockIdx.x; c < m.nchunks; c += gridDim.x) {
    const ChunkView cv = chunk_view(m, c);
    const TX* x = (const TX*)m.ptr(0, cv.t) + cv.start;
    const TY* y = (const TY*)m.ptr(1, cv.t) + cv.start;
    TO* o = (TO*)m.ptr(2, cv.t) + cv.start;
    chunk_for(m, cv.n, [&](auto NC, int64_t i) {
      constexpr int N = decltype(NC)::value;
      float xv[N], yv[N], r[N];
      load_f<TX, N>(x + i, xv);
      load_f<TY, N>(y + i, yv);
#pragma unroll
      for (int k = 0; k < N; ++k) {
        if (check != 1) bad |= !__builtin_isfinite(xv[k]);
        if (check != 0) bad |= !__builtin_isfinite(yv[k]);
        r[k] = a * xv[k] + b * yv[k];
      }
      store_f<TO, N>(o + i, r);
    });
  }
  if (bad && overflow) *overflow = 1;
}

// ---------------------------------------------------------------------------
// l2norm partials: partial[c] = sum(x^2 * s^2) over chunk c  (+ overflow flag)
// ---------------------------------------------------------------------------
template <typename T>
__global__ void __launch_bounds__(kBlock) sumsq_kernel(MTMeta m, int list, float* partial,
                                                      int* overflow) {
  __shared__ float red[kBlock / kWave];
  bool bad = false;
  for (int c = blockIdx.x; c < m.nchunks; c += gridDim.x) {
    const ChunkView cv = chunk_view(m, c);
    const T* x = (const T*)m.ptr(list, cv.t) + cv.start;
    float acc = 0.f;
    stream_for(m, cv.n, [&](auto NGc, auto NEc, int64_t j0, int64_t st) {
      constexpr int NG = decltype(NGc)::value, NE = decltype(NEc)::value;
      float v[NG][NE];
#pragma unroll
      for (int u = 0; u < NG; ++u) load_f<T, NE>(x + j0 + u * st, v[u]);
#pragma unroll
      for (int u = 0; u < NG; ++u)
#pragma unroll
        for (int k = 0; k < NE; ++k) {
          bad |= !__builtin_isfinite(v[u][k]);
          acc += v[u][k] * v[u][k];
        }
    });
    acc = block_sum(acc, red);
    if (threadIdx.x == 0) partial[c] = acc;
  }
  if (bad && overflow) *overflow = 1;
}

// Reduce chunk partials: blocks [0, T) -> per-tensor norms; block T -> global norm.
// out_tensor[t] = sqrt(sum) * s ; out_global = sqrt(total) * s
__global__ void __launch_bounds__(kBlock) norm_finalize_kernel(MTMeta m, const float* partial,
                                                              float* out_tensor, float* out_global,
                                                              const float* sp, float sv) {
  __shared__ float red[kBlock / kWave];
  const float s = read_scale(sp, sv);
  const int b = blockIdx.x;
  if (b < m.ntensors) {
    if (!out_tensor) return;
    const int64_t c0 = m.chunk_off[b], c1 = m.chunk_off[b + 1];
    float acc = 0.f;
    for (int64_t c = c0 + threadIdx.x; c < c1; c += blockDim.x) acc += partial[c];
    acc = block_sum(acc, red);
    if (threadIdx.x == 0) out_tensor[b] = sqrtf(acc) * s;
  } else {
    if (!out_global) return;
    float acc = 0.f;
    for (int c = threadIdx.x; c < m.nchunks; c += blockDim.x) acc += partial[c];
    acc = block_sum(acc, red);
    if (threadIdx.x == 0) *out_global = sqrtf(acc) * s;
  }
}

// ---------------------------------------------------------------------------
// SGD (momentum / nesterov / weight decay), optional low-precision param copy.
// lists: g, p, mom, [copy]
// ---------------------------------------------------------------------------
template <typename G, typename P, typename C>
__global__ void __launch_bounds__(kBlock) sgd_kernel(MTMeta m, SgdArgs a) {
  if (a.noop && *a.noop) return;
  const float gs = read_scale(a.grad_scale_ptr, a.grad_scale);
  if (a.first_run_dev) a.first_run = *a.first_run_dev != 0;
  const bool has_copy = m.nlists > 3;
  for (int c = blockIdx.x; c < m.nchunks; c += gridDim.x) {
    const ChunkView cv = chunk_view(m, c);
    const G* g = (const G*)m.ptr(0, cv.t) + cv.start;
    P* p = (P*)m.ptr(1, cv.t) + cv.start;
    float* mom = a.momentum != 0.f ? (float*)m.ptr(2, cv.t) + cv.start : nullptr;
    C* cp = has_copy ? (C*)m.ptr(3, cv.t) + cv.start : nullptr;
    stream_for(m, cv.n, [&](auto NGc, auto NEc, int64_t j0, int64_t st) {
      constexpr int NG = decltype(NGc)::value, NE = decltype(NEc)::value;
      float gv[NG][NE], pv[NG][NE], mv[NG][NE];
#pragma unroll
      for (int u = 0; u < NG; ++u) {
        load_f_nt<G, NE>(g + j0 + u * st, gv[u]);
        load_f_nt<P, NE>(p + j0 + u * st, pv[u]);
        if (mom && !a.first_run) load_f_nt<float, NE>(mom + j0 + u * st, mv[u]);
      }
#pragma unroll
      for (int u = 0; u < NG; ++u)
#pragma unroll
        for (int k = 0; k < NE; ++k) {
          float gg = gv[u][k] * gs;
          if (a.wd != 0.f && !a.wd_after_momentum) gg += a.wd * pv[u][k];
          if (mom) {
            mv[u][k] = a.first_run ? gg : a.momentum * mv[u][k] + (1.f - a.dampening) * gg;
            gg = a.nesterov ? gg + a.momentum * mv[u][k] : mv[u][k];
          }
          if (a.wd != 0.f && a.wd_after_momentum) gg += a.wd * pv[u][k];
          pv[u][k] -= a.lr * gg;
        }
#pragma unroll
      for (int u = 0; u < NG; ++u) {
        store_f_nt<P, NE>(p + j0 + u * st, pv[u]);
        if (mom) store_f_nt<float, NE>(mom + j0 + u * st, mv[u]);
        if (cp) store_f_nt<C, NE>(cp + j0 + u * st, pv[u]);
      }
    });
  }
}

// After a (possibly skipped) step: a device flag/counter advances only when the step ran, so a
// dynamic-loss-scale overflow never consumes SGD's first-run momentum init or an Adam step.
__global__ void clear_flag_unless_noop_kernel(int* flag, const int* noop) {
  if (!(noop && *noop)) *flag = 0;
}

// Adam step counter and bias corrections on the device (1 thread, before the update kernel)
__global__ void adam_prep_kernel(int* step, const int* noop, float beta1, float beta2, int bias_correction,
                                 float* scal) {
  int st = *step;
  if (!(noop && *noop)) *step = ++st;
  scal[0] = bias_correction ? 1.f - powf(beta1, (float)st) : 1.f;
  scal[1] = bias_correction ? 1.f - powf(beta2, (float)st) : 1.f;
}

// ---------------------------------------------------------------------------
// Adam / AdamW. lists: g, p, m, v, [copy]
// ---------------------------------------------------------------------------
template <typename G, typename P, typename C>
__global__ void __launch_bounds__(kBlock) adam_kernel(MTMeta m, AdamArgs a) {
  if (a.noop && *a.noop) return;
  const float gs = read_scale(a.grad_scale_ptr, a.grad_scale);
  const bool has_copy = m.nlists > 4;
  const float b1 = a.beta1, b2 = a.beta2;
  const float rbc1 = 1.f / (a.step ? a.scal[0] : a.bc1), rbc2 = 1.f / (a.step ? a.scal[1] : a.bc2);
  for (int c = blockIdx.x; c < m.nchunks; c += gridDim.x) {
    const ChunkView cv = chunk_view(m, c);
    const G* g = (const G*)m.ptr(0, cv.t) + cv.start;
    P* p = (P*)m.ptr(1, cv.t) + cv.start;
    float* mm = (float*)m.ptr(2, cv.t) + cv.start;
    float* vv = (float*)m.ptr(3, cv.t) + cv.start;
    C* cp = has_copy ? (C*)m.ptr(4, cv.t) + cv.start : nullptr;
    stream_for(m, cv.n, [&](auto NGc, auto NEc, int64_t j0, int64_t st) {
      constexpr int NG = decltype(NGc)::value, NE = decltype(NEc)::value;
      float gv[NG][NE], pv[NG][NE], mv[NG][NE], vq[NG][NE];
#pragma unroll
      for (int u = 0; u < NG; ++u) {
        load_f_nt<G, NE>(g + j0 + u * st, gv[u]);
        load_f_nt<P, NE>(p + j0 + u * st, pv[u]);
        load_f_nt<float, NE>(mm + j0 + u * st, mv[u]);
        load_f_nt<float, NE>(vv + j0 + u * st, vq[u]);
      }
#pragma unroll
      for (int u = 0; u < NG; ++u)
#pragma unroll
        for (int k = 0; k < NE; ++k) {
          float gg = gv[u][k] * gs;
          if (!a.adamw && a.wd != 0.f) gg += a.wd * pv[u][k];
          mv[u][k] = b1 * mv[u][k] + (1.f - b1) * gg;
          vq[u][k] = b2 * vq[u][k] + (1.f - b2) * gg * gg;
          const float denom = sqrtf(vq[u][k] * rbc2) + a.eps;
          float upd = (mv[u][k] * rbc1) / denom;
          if (a.adamw && a.wd != 0.f) upd += a.wd * pv[u][k];
          pv[u][k] -= a.lr * upd;
        }
#pragma unroll
      for (int u = 0; u < NG; ++u) {
        store_f_nt<P, NE>(p + j0 + u * st, pv[u]);
        store_f_nt<float, NE>(mm + j0 + u * st, mv[u]);
        store_f_nt<float, NE>(vv + j0 + u * st, vq[u]);
        if (cp) store_f_nt<C, NE>(cp + j0 + u * st, pv[u]);
      }
    });
  }
}

// ---------------------------------------------------------------------------
// LAMB.
//  prep  (1 block): global grad norm -> clip divisor, device step++, bias corrections
//  stage1: m,v update; u = m^/(sqrt(v^)+eps) (+wd*p); partial sums of p^2 and u^2
//  finalize per-tensor norms (norm_finalize_kernel twice)
//  stage2: recompute u from the updated m, v and p (lamb_u, the same expression), then
//          p -= lr * trust * u ; optional low-precision copy
// u never reaches HBM: stage 1 writes m, v (8 B) instead of m, v, u (12 B) and stage 2 reads
// p, m, v (12 B) instead of p, u (8 B) — the same 40 B per parameter as a stored fp32 u, minus
// a parameter-sized fp32 scratch buffer (1.3 GB for BERT-Large) and its state-dict entry.
// scal layout: [0] grad norm, [1] clip divisor, [2] bc1, [3] bc2
// ---------------------------------------------------------------------------
__device__ __forceinline__ float lamb_u(float mv, float vv, float pv, float rbc1, float rbc2, const LambArgs& a) {
  float u = (mv * rbc1) / (sqrtf(vv * rbc2) + a.eps);
  if (a.adamw && a.wd != 0.f) u += a.wd * pv;
  return u;
}

__global__ void lamb_prep_kernel(const float* partial, int nchunks, LambArgs a, float* scal,
                                 int* step) {
  __shared__ float red[kBlock / kWave];
  float acc = 0.f;
  if (!a.gnorm_in)
    for (int c = threadIdx.x; c < nchunks; c += blockDim.x) acc += partial[c];
  acc = block_sum(acc, red);
  if (threadIdx.x == 0) {
    const float gs = read_scale(a.grad_scale_ptr, a.grad_scale);
    // external norm is already unscaled (computed over all param groups)
    const float gnorm = a.gnorm_in ? *a.gnorm_in : sqrtf(acc) * gs;
    float clip = 1.f;
    if (a.max_grad_norm > 0.f && gnorm > a.max_grad_norm) clip = gnorm / a.max_grad_norm;
    const bool skip = a.noop && *a.noop;
    int st = *step;
    if (!skip) {
      st += 1;
      *step = st;
    }
    float bc1 = 1.f, bc2 = 1.f;
    if (a.bias_correction) {
      bc1 = 1.f - powf(a.beta1, (float)st);
      bc2 = 1.f - powf(a.beta2, (float)st);
    }
    scal[0] = gnorm;
    scal[1] = clip;
    scal[2] = bc1;
    scal[3] = bc2;
  }
}

template <typename G, typename P>
__global__ void __launch_bounds__(kBlock) lamb_stage1_kernel(MTMeta m, LambArgs a, const float* scal,
                                                            float* part_p, float* part_u) {
  __shared__ float red[kBlock / kWave];
  if (a.noop && *a.noop) return;
  const float gs = read_scale(a.grad_scale_ptr, a.grad_scale) / scal[1];
  const float rbc1 = 1.f / scal[2], rbc2 = 1.f / scal[3];
  const float b1 = a.beta1, b2 = a.beta2, b3 = a.grad_averaging ? 1.f - a.beta1 : 1.f;
  // last chunk first: the grad-norm pass just read the gradients in ascending order, so the
  // chunks it read last may still sit in the 256 MB infinity cache
  for (int cc = blockIdx.x; cc < m.nchunks; cc += gridDim.x) {
    const int c = m.nchunks - 1 - cc;
    const ChunkView cv = chunk_view(m, c);
    const G* g = (const G*)m.ptr(0, cv.t) + cv.start;
    const P* p = (const P*)m.ptr(1, cv.t) + cv.start;
    float* mm = (float*)m.ptr(2, cv.t) + cv.start;
    float* vv = (float*)m.ptr(3, cv.t) + cv.start;
    float sp = 0.f, su = 0.f;
    stream_for(m, cv.n, [&](auto NGc, auto NEc, int64_t j0, int64_t st) {
      constexpr int NG = decltype(NGc)::value, NE = decltype(NEc)::value;
      float gv[NG][NE], pv[NG][NE], mv[NG][NE], vq[NG][NE];
#pragma unroll
      for (int u = 0; u < NG; ++u) {
        load_f_nt<G, NE>(g + j0 + u * st, gv[u]);
        load_f_nt<P, NE>(p + j0 + u * st, pv[u]);
        load_f_nt<float, NE>(mm + j0 + u * st, mv[u]);
        load_f_nt<float, NE>(vv + j0 + u * st, vq[u]);
      }
#pragma unroll
      for (int u = 0; u < NG; ++u)
#pragma unroll
        for (int k = 0; k < NE; ++k) {
          float gg = gv[u][k] * gs;
          if (!a.adamw && a.wd != 0.f) gg += a.wd * pv[u][k];
          mv[u][k] = b1 * mv[u][k] + b3 * gg;
          vq[u][k] = b2 * vq[u][k] + (1.f - b2) * gg * gg;
          const float uu = lamb_u(mv[u][k], vq[u][k], pv[u][k], rbc1, rbc2, a);
          sp += pv[u][k] * pv[u][k];
          su += uu * uu;
        }
#pragma unroll
      for (int u = 0; u < NG; ++u) {
        store_f_nt<float, NE>(mm + j0 + u * st, mv[u]);
        store_f_nt<float, NE>(vv + j0 + u * st, vq[u]);
      }
    });
    sp = block_sum(sp, red);
    su = block_sum(su, red);
    if (threadIdx.x == 0) {
      part_p[c] = sp;
      part_u[c] = su;
    }
  }
}

template <typename P, typename C>
__global__ void __launch_bounds__(kBlock) lamb_stage2_kernel(MTMeta m, LambArgs a, const float* scal,
                                                            const float* pnorm, const float* unorm) {
  if (a.noop && *a.noop) return;
  const bool has_copy = m.nlists > 4;
  const float rbc1 = 1.f / scal[2], rbc2 = 1.f / scal[3];
  for (int c = blockIdx.x; c < m.nchunks; c += gridDim.x) {
    const ChunkView cv = chunk_view(m, c);
    P* p = (P*)m.ptr(1, cv.t) + cv.start;
    const float* mm = (const float*)m.ptr(2, cv.t) + cv.start;
    const float* vv = (const float*)m.ptr(3, cv.t) + cv.start;
    C* cp = has_copy ? (C*)m.ptr(4, cv.t) + cv.start : nullptr;
    float ratio = a.lr;
    if (a.use_nvlamb || a.wd != 0.f) {
      const float pn = pnorm[cv.t], un = unorm[cv.t];
      if (pn != 0.f && un != 0.f) ratio = a.lr * (pn / un);
    }
    stream_for(m, cv.n, [&](auto NGc, auto NEc, int64_t j0, int64_t st) {
      constexpr int NG = decltype(NGc)::value, NE = decltype(NEc)::value;
      float pv[NG][NE], mv[NG][NE], vq[NG][NE];
#pragma unroll
      for (int u = 0; u < NG; ++u) {
        load_f_nt<P, NE>(p + j0 + u * st, pv[u]);
        load_f_nt<float, NE>(mm + j0 + u * st, mv[u]);
        load_f_nt<float, NE>(vv + j0 + u * st, vq[u]);
      }
#pragma unroll
      for (int u = 0; u < NG; ++u)
#pragma unroll
        for (int k = 0; k < NE; ++k) pv[u][k] -= ratio * lamb_u(mv[u][k], vq[u][k], pv[u][k], rbc1, rbc2, a);
#pragma unroll
      for (int u = 0; u < NG; ++u) {
        store_f_nt<P, NE>(p + j0 + u * st, pv[u]);
        if (cp) store_f_nt<C, NE>(cp + j0 + u * st, pv[u]);
      }
    });
  }
}

// ---------------------------------------------------------------------------
// Per-tensor scale (LARC trust ratio application): x[t] *= factor[t]
// lists: g, p ; g = (g*gs + wd*p) * adaptive_lr (computed from norms on device)
// ---------------------------------------------------------------------------
template <typename G, typename P>
__global__ void __launch_bounds__(kBlock) larc_kernel(MTMeta m, LarcArgs a, const float* pnorm,
                                                     const float* gnorm) {
  for (int c = blockIdx.x; c < m.nchunks; c += gridDim.x) {
    const ChunkView cv = chunk_view(m, c);
    G* g = (G*)m.ptr(0, cv.t) + cv.start;
    const P* p = (const P*)m.ptr(1, cv.t) + cv.start;
    const float pn = pnorm[cv.t], gn = gnorm[cv.t];
    // reference LARC.py:84-92: untouched grad when either norm is zero
    if (pn == 0.f || gn == 0.f) continue;
    float alr = a.trust_coefficient * pn / (gn + pn * a.wd + a.eps);
    if (a.clip) alr = fminf(alr / a.lr, 1.f);
    chunk_for(m, cv.n, [&](auto NC, int64_t i) {
      constexpr int N = decltype(NC)::value;
      float gv[N], pv[N];
      load_f<G, N>(g + i, gv);
      load_f<P, N>(p + i, pv);
#pragma unroll
      for (int k = 0; k < N; ++k) gv[k] = (gv[k] + a.wd * pv[k]) * alr;
      store_f<G, N>(g + i, gv);
    });
  }
}

// ---------------------------------------------------------------------------
// dtype dispatch
// ---------------------------------------------------------------------------
#define APEX_DISPATCH1(DT, T, ...)                          \
  switch (DT) {                                             \
    case kF32: { using T = float; __VA_ARGS__; } break;     \
    case kF16: { using T = f16; __VA_ARGS__; } break;       \
    case kBF16: { using T = bf16; __VA_ARGS__; } break;     \
    default: return -1;                                     \
  }

int mt_scale(const MTMeta& m, int in_dt, int out_dt, const float* sp, float sv, int* overflow,
             hipStream_t s) {
  if (m.nchunks == 0) return 0;
  APEX_DISPATCH1(in_dt, TI, APEX_DISPATCH1(out_dt, TO,
      hipLaunchKernelGGL((scale_kernel<TI, TO>), dim3(grid_for(m.nchunks)), dim3(kBlock), 0, s, m,
                         sp, sv, overflow)));
  return (int)hipGetLastError();
}

int mt_axpby(const MTMeta& m, int x_dt, int y_dt, int o_dt, float a, float b, int check,
             int* overflow, hipStream_t s) {
  if (m.nchunks == 0) return 0;
  APEX_DISPATCH1(x_dt, TX, APEX_DISPATCH1(y_dt, TY, APEX_DISPATCH1(o_dt, TO,
      hipLaunchKernelGGL((axpby_kernel<TX, TY, TO>), dim3(grid_for(m.nchunks)), dim3(kBlock), 0, s,
                         m, a, b, check, overflow))));
  return (int)hipGetLastError();
}

int mt_l2norm(const MTMeta& m, int list, int dt, float* partial, float* out_tensor,
              float* out_global, const float* sp, float sv, int* overflow, hipStream_t s) {
  if (m.nchunks == 0) return 0;
  APEX_DISPATCH1(dt, T,
      hipLaunchKernelGGL((sumsq_kernel<T>), dim3(grid_for(m.nchunks)), dim3(kBlock), 0, s, m, list,
                         partial, overflow));
  hipLaunchKernelGGL(norm_finalize_kernel, dim3(m.ntensors + 1), dim3(kBlock), 0, s, m, partial,
                     out_tensor, out_global, sp, sv);
  return (int)hipGetLastError();
}

int mt_sgd(const MTMeta& m, int g_dt, int p_dt, int c_dt, const SgdArgs& a, hipStream_t s) {
  if (m.nchunks == 0) return 0;
  if (m.nlists <= 3) c_dt = p_dt;
  APEX_DISPATCH1(g_dt, G, APEX_DISPATCH1(p_dt, P, APEX_DISPATCH1(c_dt, C,
      hipLaunchKernelGGL((sgd_kernel<G, P, C>), dim3(grid_for(m.nchunks)), dim3(kBlock), 0, s, m,
                         a))));
  if (a.first_run_dev)
    hipLaunchKernelGGL(clear_flag_unless_noop_kernel, dim3(1), dim3(1), 0, s, a.first_run_dev, a.noop);
  return (int)hipGetLastError();
}

int mt_adam(const MTMeta& m, int g_dt, int p_dt, int c_dt, const AdamArgs& a, hipStream_t s) {
  if (m.nchunks == 0) return 0;
  if (m.nlists <= 4) c_dt = p_dt;
  if (a.step)
    hipLaunchKernelGGL(adam_prep_kernel, dim3(1), dim3(1), 0, s, a.step, a.noop, a.beta1, a.beta2,
                       a.bias_correction, a.scal);
  APEX_DISPATCH1(g_dt, G, APEX_DISPATCH1(p_dt, P, APEX_DISPATCH1(c_dt, C,
      hipLaunchKernelGGL((adam_kernel<G, P, C>), dim3(grid_for(m.nchunks)), dim3(kBlock), 0, s, m,
                         a))));
  return (int)hipGetLastError();
}

int mt_lamb(const MTMeta& m, int g_dt, int p_dt, int c_dt, const LambArgs& a, float* ws,
            int* step, hipStream_t s) {
  // ws layout: [4 scal][C gpart][C ppart][C upart][T pnorm][T unorm]
  if (m.nchunks == 0) return 0;
  if (m.nlists <= 4) c_dt = p_dt;
  const int C = m.nchunks, T = m.ntensors;
  float* scal = ws;
  float* gpart = ws + 4;
  float* ppart = gpart + C;
  float* upart = ppart + C;
  float* pnorm = upart + C;
  float* unorm = pnorm + T;
  const int grid = grid_for(C);
  if (!a.gnorm_in) {
    APEX_DISPATCH1(g_dt, G,
        hipLaunchKernelGGL((sumsq_kernel<G>), dim3(grid), dim3(kBlock), 0, s, m, 0, gpart,
                           a.overflow_out));
  }
  hipLaunchKernelGGL(lamb_prep_kernel, dim3(1), dim3(kBlock), 0, s, gpart, C, a, scal, step);
  APEX_DISPATCH1(g_dt, G, APEX_DISPATCH1(p_dt, P,
      hipLaunchKernelGGL((lamb_stage1_kernel<G, P>), dim3(grid), dim3(kBlock), 0, s, m, a, scal,
                         ppart, upart)));
  hipLaunchKernelGGL(norm_finalize_kernel, dim3(T), dim3(kBlock), 0, s, m, ppart, pnorm,
                     (float*)nullptr, (const float*)nullptr, 1.f);
  hipLaunchKernelGGL(norm_finalize_kernel, dim3(T), dim3(kBlock), 0, s, m, upart, unorm,
                     (float*)nullptr, (const float*)nullptr, 1.f);
  APEX_DISPATCH1(p_dt, P, APEX_DISPATCH1(c_dt, C,
      hipLaunchKernelGGL((lamb_stage2_kernel<P, C>), dim3(grid), dim3(kBlock), 0, s, m, a, scal, pnorm,
                         unorm)));
  return (int)hipGetLastError();
}

int mt_larc(const MTMeta& m, int g_dt, int p_dt, const LarcArgs& a, float* ws, hipStream_t s) {
  // ws: [C part][T pnorm][T gnorm]
  if (m.nchunks == 0) return 0;
  const int C = m.nchunks, T = m.ntensors;
  float* part = ws;
  float* pnorm = ws + C;
  float* gnorm = pnorm + T;
  const int grid = grid_for(C);
  APEX_DISPATCH1(p_dt, P,
      hipLaunchKernelGGL((sumsq_kernel<P>), dim3(grid), dim3(kBlock), 0, s, m, 1, part,
                         (int*)nullptr));
  hipLaunchKernelGGL(norm_finalize_kernel, dim3(T), dim3(kBlock), 0, s, m, part, pnorm,
                     (float*)nullptr, (const float*)nullptr, 1.f);
  APEX_DISPATCH1(g_dt, G,
      hipLaunchKernelGGL((sumsq_kernel<G>), dim3(grid), dim3(kBlock), 0, s, m, 0, part,
                         (int*)nullptr));
  hipLaunchKernelGGL(norm_finalize_kernel, dim3(T), dim3(kBlock), 0, s, m, part, gnorm,
                     (float*)nullptr, (const float*)nullptr, 1.f);
  APEX_DISPATCH1(g_dt, G, APEX_DISPATCH1(p_dt, P,
      hipLaunchKernelGGL((larc_kernel<G, P>), dim3(grid), dim3(kBlock), 0, s, m, a, pnorm,
                         gnorm)));
  return (int)hipGetLastError();
}

// Device-side dynamic loss-scale update (no host sync):
//   overflow -> scale *= backoff, growth_tracker = 0
//   else     -> tracker += 1; if tracker == interval: scale *= growth, tracker = 0
__global__ void update_scale_kernel(float* scale, int* tracker, const int* overflow,
                                    float growth, float backoff, int interval, float min_scale,
                                    float max_scale) {
  if (*overflow) {
    *scale = fmaxf(*scale * backoff, min_scale);
    *tracker = 0;
  } else {
    int t = *tracker + 1;
    if (t >= interval) {
      *scale = fminf(*scale * growth, max_scale);
      t = 0;
    }
    *tracker = t;
  }
}

int amp_update_scale(float* scale, int* tracker, const int* overflow, float growth, float backoff,
                     int interval, float min_scale, float max_scale, hipStream_t s) {
  hipLaunchKernelGGL(update_scale_kernel, dim3(1), dim3(1), 0, s, scale, tracker, overflow, growth,
                     backoff, interval, min_scale, max_scale);
  return (int)hipGetLastError();
}

}  // namespace apex
