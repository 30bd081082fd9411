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
  const float m = FMT == 0 ? kF8E4M3Max : kF8E5M2Max;
  a = fminf(fmaxf(a, -m), m);
  b = fminf(fmaxf(b, -m), m);
  c = fminf(fmaxf(c, -m), m);
  d = fminf(fmaxf(d, -m), m);
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

}  // namespace apex
