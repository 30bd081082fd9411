// OCP fp8 (e4m3 / e5m2) packing shared by the standalone quantisers (fp8.hip) and the producer
// kernels that emit fp8 codes of their own output (bias+dropout+residual+LayerNorm forward and
// backward in fused_ops.hip): saturating conversion on gfx950's v_cvt_pk_{fp8,bf8}_f32, 8 codes
// per 8-byte store, and the per-block max|x| folded into the slot's device amax.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kernels.h"  // Q8Out

namespace apex {

constexpr float kF8E4M3Max = 448.f;
constexpr float kF8E5M2Max = 57344.f;

template <int FMT>
__device__ __forceinline__ uint32_t f8_pack4(float a, float b, float c, float d) {
  // saturate with v_med3_f32: one instruction per value, and no NaN-canonicalising v_max_f32 x, x
  // that fminf / fmaxf insert before each clamp when the input's provenance is unknown
  const float m = FMT == 0 ? kF8E4M3Max : kF8E5M2Max;
  a = __builtin_amdgcn_fmed3f(a, -m, m);
  b = __builtin_amdgcn_fmed3f(b, -m, m);
  c = __builtin_amdgcn_fmed3f(c, -m, m);
  d = __builtin_amdgcn_fmed3f(d, -m, m);
  int w = 0;
  if constexpr (FMT == 0) {
    w = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, w, false);
    w = __builtin_amdgcn_cvt_pk_fp8_f32(c, d, w, true);
  } else {
    w = __builtin_amdgcn_cvt_pk_bf8_f32(a, b, w, false);
    w = __builtin_amdgcn_cvt_pk_bf8_f32(c, d, w, true);
  }
  return (uint32_t)w;
}

// 8 values * s -> 8 codes (one 8-byte store); fmt 0 = e4m3, 1 = e5m2 (wave-uniform)
__device__ __forceinline__ void f8_store8(uint8_t* p, const float (&v)[8], float s, int fmt) {
  uint2 w;
  if (fmt == 0) {
    w.x = f8_pack4<0>(v[0] * s, v[1] * s, v[2] * s, v[3] * s);
    w.y = f8_pack4<0>(v[4] * s, v[5] * s, v[6] * s, v[7] * s);
  } else {
    w.x = f8_pack4<1>(v[0] * s, v[1] * s, v[2] * s, v[3] * s);
    w.y = f8_pack4<1>(v[4] * s, v[5] * s, v[6] * s, v[7] * s);
  }
  *reinterpret_cast<uint2*>(p) = w;
}

// ---- producer-side codes of values a 16-bit store just wrote ---------------------------------------
// The codes must be those of the STORED (rounded) values, so they are taken from the packed 16-bit
// words themselves: bf16 -> f32 is a shift / mask (no second rounding convert), the running max|x|
// is one v_max3_f32 with |.| modifiers per two values, the scale one packed multiply per two.
typedef float f8_f2 __attribute__((ext_vector_type(2)));

template <typename T> __device__ __forceinline__ f8_f2 f8_unpack2(uint32_t w);
template <> __device__ __forceinline__ f8_f2 f8_unpack2<__bf16>(uint32_t w) {
  return f8_f2{__uint_as_float(w << 16), __uint_as_float(w & 0xffff0000u)};
}
template <> __device__ __forceinline__ f8_f2 f8_unpack2<_Float16>(uint32_t w) {
  typedef _Float16 h2 __attribute__((ext_vector_type(2)));
  const h2 h = __builtin_bit_cast(h2, w);
  return f8_f2{(float)h[0], (float)h[1]};
}

__device__ __forceinline__ void f8_amax2(float& mx, f8_f2 v) {
  asm("v_max3_f32 %0, |%1|, |%2|, %0" : "+v"(mx) : "v"(v[0]), "v"(v[1]));
}

// four codes of the 16-bit values in two packed words: sat(x * s); mx = max(mx, |x|)
template <int FMT, typename T>
__device__ __forceinline__ uint32_t f8_codes4(uint32_t w0, uint32_t w1, float s, float& mx) {
  const f8_f2 ab = f8_unpack2<T>(w0), cd = f8_unpack2<T>(w1);
  f8_amax2(mx, ab);
  f8_amax2(mx, cd);
  const f8_f2 p = ab * f8_f2{s, s}, q = cd * f8_f2{s, s};
  return f8_pack4<FMT>(p[0], p[1], q[0], q[1]);
}

// 8 values stored as 16-bit T (one 16-byte store) plus their codes (one 8-byte store); fmt
// wave-uniform. store_v = false (wave-uniform; codes-only outputs, Q8Out::only): the codes alone
template <typename T>
__device__ __forceinline__ void f8_store_with_codes8(T* dst, uint8_t* cdst, const float (&v)[8], float s, int fmt,
                                                     float& mx, bool store_v = true) {
  static_assert(sizeof(T) == 2, "16-bit stores");
  struct alignas(16) P8 {
    T v[8];
  } pk;
#pragma unroll
  for (int i = 0; i < 8; ++i) pk.v[i] = (T)v[i];
  if (store_v) *reinterpret_cast<P8*>(dst) = pk;
  const uint4 w = __builtin_bit_cast(uint4, pk);
  uint2 c;
  if (fmt == 0) {
    c.x = f8_codes4<0, T>(w.x, w.y, s, mx);
    c.y = f8_codes4<0, T>(w.z, w.w, s, mx);
  } else {
    c.x = f8_codes4<1, T>(w.x, w.y, s, mx);
    c.y = f8_codes4<1, T>(w.z, w.w, s, mx);
  }
  *reinterpret_cast<uint2*>(cdst) = c;
}

// non-negative floats order like their bit patterns: max via integer atomics
__device__ __forceinline__ void f8_atomic_max_pos(float* p, float v) {
  atomicMax(reinterpret_cast<unsigned int*>(p), __float_as_uint(v));
}

__device__ __forceinline__ float f8_wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// block max (256 threads) -> ONE atomic per block: thousands of same-address atomics serialise in
// L2 (one per wave made the standalone quantiser atomic-bound at ~0.19 ms regardless of size). The
// plain pre-read is only a filter: amax only grows, so a stale value costs an extra atomic, never a
// missed one. Every thread of the block must call it.
__device__ __forceinline__ void f8_block_amax(float mx, float* amax) {
  __shared__ float red[4];
  mx = f8_wave_max(mx);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = mx;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float m = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
    if (m > 0.f && m > *(volatile float*)amax) f8_atomic_max_pos(amax, m);
  }
}

// The filter value for the overload below, read at kernel START: an agent-scope atomic load (a
// vector load that reads L2; a plain load of this wave-uniform address becomes a scalar load whose
// cache keeps the launch's first value for every later workgroup on the CU).
__device__ __forceinline__ float f8_amax_seen(const float* amax) {
  return __hip_atomic_load(amax, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Two-stage filter: the block max is first compared with `seen` (f8_amax_seen at kernel start, its
// latency under the main loop); only a block that beats it re-reads amax at its end before the
// atomic. Once amax has grown, later workgroups skip the end-of-block read round trip; the
// workgroups that start while amax is still near 0 (it starts every step at 0) keep the exact
// re-read — with the start value alone they all issued same-address atomics (fp8 step: LayerNorm
// forward 136 -> 302 us, profiles/r6_bert_b768_fp8_step_kernels_stale_filter.txt).
__device__ __forceinline__ void f8_block_amax(float mx, float* amax, float seen) {
  __shared__ float red[4];
  mx = f8_wave_max(mx);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = mx;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float m = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
    if (m > 0.f && m > seen && m > *(volatile float*)amax) f8_atomic_max_pos(amax, m);
  }
}

}  // namespace apex
