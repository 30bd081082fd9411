// Shared device helpers for every apex HIP kernel (CDNA4 / gfx950 only).
//
// Design notes (MI355X-first):
//  * wave64 everywhere: reductions are 6-step __shfl_xor butterflies over 64 lanes.
//  * bf16 is the clang-native __bf16 type: on gfx950 float->bf16 lowers to the
//    hardware v_cvt_pk_bf16_f32 (RNE), so no bit-twiddling conversion code.
//  * every memory-bound kernel moves 16 B per lane (8 x 16-bit or 4 x fp32);
//    Vec<T> below is the single abstraction for that.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace apex {

using bf16 = __bf16;
using f16 = _Float16;

// dtype codes shared with bindings.cpp / python
enum DType : int { kF32 = 0, kF16 = 1, kBF16 = 2 };

constexpr int kWave = 64;

__device__ __forceinline__ float to_f(float x) { return x; }
__device__ __forceinline__ float to_f(f16 x) { return (float)x; }
__device__ __forceinline__ float to_f(bf16 x) { return (float)x; }

template <typename T> __device__ __forceinline__ T from_f(float x);
template <> __device__ __forceinline__ float from_f<float>(float x) { return x; }
template <> __device__ __forceinline__ f16 from_f<f16>(float x) { return (f16)x; }
template <> __device__ __forceinline__ bf16 from_f<bf16>(float x) { return (bf16)x; }

// N elements of T packed so that one load is 16 bytes when N*sizeof(T)==16.
template <typename T, int N>
struct alignas(sizeof(T) * N) Pack {
  T v[N];
};

template <typename T, int N>
__device__ __forceinline__ void load_f(const T* __restrict__ p, float (&out)[N]) {
  Pack<T, N> pk = *reinterpret_cast<const Pack<T, N>*>(p);
#pragma unroll
  for (int i = 0; i < N; ++i) out[i] = to_f(pk.v[i]);
}

template <typename T, int N>
__device__ __forceinline__ void store_f(T* __restrict__ p, const float (&in)[N]) {
  Pack<T, N> pk;
#pragma unroll
  for (int i = 0; i < N; ++i) pk.v[i] = from_f<T>(in[i]);
  *reinterpret_cast<Pack<T, N>*>(p) = pk;
}

// Non-temporal variants for single-pass streams (optimizer states, gradients): the loads and
// stores carry the nt hint, so a multi-GB sweep does not churn the L2 / Infinity Cache lines
// the next kernel wants. Measured on the Adam stream (tools/bwlab/adam_lab.hip, 512 M params):
// nt loads + stores with 4 lane-contiguous 16-B groups in flight 6.42 TB/s vs 5.84 plain.
template <typename T, int N>
__device__ __forceinline__ void load_f_nt(const T* __restrict__ p, float (&out)[N]) {
  constexpr int B = (int)sizeof(T) * N;
  if constexpr (B == 16 || B == 8) {
    typedef unsigned V __attribute__((ext_vector_type(B / 4)));
    const V v = __builtin_nontemporal_load(reinterpret_cast<const V*>(p));
    Pack<T, N> pk;
    __builtin_memcpy(&pk, &v, B);
#pragma unroll
    for (int i = 0; i < N; ++i) out[i] = to_f(pk.v[i]);
  } else if constexpr (B == 4) {
    const unsigned v = __builtin_nontemporal_load(reinterpret_cast<const unsigned*>(p));
    Pack<T, N> pk;
    __builtin_memcpy(&pk, &v, 4);
#pragma unroll
    for (int i = 0; i < N; ++i) out[i] = to_f(pk.v[i]);
  } else {
    load_f<T, N>(p, out);
  }
}

template <typename T, int N>
__device__ __forceinline__ void store_f_nt(T* __restrict__ p, const float (&in)[N]) {
  constexpr int B = (int)sizeof(T) * N;
  Pack<T, N> pk;
#pragma unroll
  for (int i = 0; i < N; ++i) pk.v[i] = from_f<T>(in[i]);
  if constexpr (B == 16 || B == 8) {
    typedef unsigned V __attribute__((ext_vector_type(B / 4)));
    V v;
    __builtin_memcpy(&v, &pk, B);
    __builtin_nontemporal_store(v, reinterpret_cast<V*>(p));
  } else if constexpr (B == 4) {
    unsigned v;
    __builtin_memcpy(&v, &pk, 4);
    __builtin_nontemporal_store(v, reinterpret_cast<unsigned*>(p));
  } else {
    *reinterpret_cast<Pack<T, N>*>(p) = pk;
  }
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, kWave));
  return v;
}

// Block-wide sum; `red` must hold blockDim.x/64 floats. Result valid in all threads.
__device__ __forceinline__ float block_sum(float v, float* red) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  v = wave_sum(v);
  __syncthreads();
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float t = lane < nw ? red[lane] : 0.f;
  return wave_sum(t);
}

__device__ __forceinline__ float block_max(float v, float* red) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  v = wave_max(v);
  __syncthreads();
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float t = lane < nw ? red[lane] : -INFINITY;
  return wave_max(t);
}

// ---------------------------------------------------------------------------
// Column sum of fp32 partial rows: out[c] = sum_p part[p*ld + c]  (c < cols).
// Block = 256 threads = 16 columns x 16 part-groups: every thread issues parts/16
// loads of 64-byte row segments, the 16 groups combine in LDS. Launch with
// grid = ceil(cols / 16). Deterministic (fixed summation order).
// ---------------------------------------------------------------------------
// Up to 3 column sets of `cols` each, laid out consecutively in a partial row
// (e.g. [dgamma | dbeta | dbias]); set k is written to outs[k] (null -> skipped).
template <typename W>
struct ColsumOuts {
  W* o[3];
};

template <typename W>
__global__ void __launch_bounds__(256) partial_colsum_kernel(const float* __restrict__ part, int parts,
                                                            int64_t ld, int cols, int nsets,
                                                            ColsumOuts<W> outs) {
  __shared__ float red[16][17];
  const int cl = threadIdx.x & 15, grp = threadIdx.x >> 4;
  const int c = blockIdx.x * 16 + cl;  // over nsets * cols
  const int set = c / cols;
  const bool live = c < nsets * cols && outs.o[set < 3 ? set : 0] != nullptr;
  float a = 0.f;
  if (live) {
#pragma unroll 4
    for (int p = grp; p < parts; p += 16) a += part[(int64_t)p * ld + c];
  }
  red[grp][cl] = a;
  __syncthreads();
  if (grp == 0 && live) {
    float t = 0.f;
#pragma unroll
    for (int g = 0; g < 16; ++g) t += red[g][cl];
    outs.o[set][c - set * cols] = (W)t;
  }
}

template <typename W>
inline void launch_partial_colsum3(const float* part, int parts, int64_t ld, int cols, W* o0, W* o1,
                                   W* o2, hipStream_t s) {
  const int nsets = o2 ? 3 : (o1 ? 2 : 1);
  if (cols <= 0) return;
  ColsumOuts<W> outs{{o0, o1, o2}};
  hipLaunchKernelGGL((partial_colsum_kernel<W>), dim3((nsets * cols + 15) / 16), dim3(256), 0, s, part,
                     parts, ld, cols, nsets, outs);
}

template <typename W>
inline void launch_partial_colsum(const float* part, int parts, int64_t ld, int cols, W* out,
                                  hipStream_t s) {
  if (!out) return;
  launch_partial_colsum3<W>(part, parts, ld, cols, out, nullptr, nullptr, s);
}

// ---------------------------------------------------------------------------
// Philox-4x32-10 counter RNG (stateless: (seed, offset, subsequence) -> 4 u32).
// Dropout kernels derive the counter from the element index so fwd and bwd
// regenerate identical masks without storing them when asked to.
// ---------------------------------------------------------------------------
struct Philox {
  uint4 ctr;
  uint2 key;
  __device__ __forceinline__ Philox(uint64_t seed, uint64_t subseq, uint64_t offset) {
    key = make_uint2((uint32_t)seed, (uint32_t)(seed >> 32));
    ctr = make_uint4((uint32_t)offset, (uint32_t)(offset >> 32), (uint32_t)subseq,
                     (uint32_t)(subseq >> 32));
  }
  __device__ __forceinline__ static uint32_t mulhilo(uint32_t a, uint32_t b, uint32_t& hi) {
    uint64_t p = (uint64_t)a * b;
    hi = (uint32_t)(p >> 32);
    return (uint32_t)p;
  }
  // 7 rounds: Philox4x32-7 is the smallest round count the Random123 authors report as
  // passing BigCrush (10 is their safety margin). Dropout masks are the only consumer; inside
  // the attention forward the RNG is VALU work competing with the softmax, and 7 rounds cut
  // its cost by 30 %. Every kernel (forward, backward, mask-debug) uses this same generator.
  static constexpr int kRounds = 7;
  __device__ __forceinline__ uint4 next() {
    uint4 c = ctr;
    uint2 k = key;
#pragma unroll
    for (int r = 0; r < kRounds; ++r) {
      uint32_t hi0, hi1;
      uint32_t lo0 = mulhilo(0xD2511F53u, c.x, hi0);
      uint32_t lo1 = mulhilo(0xCD9E8D57u, c.z, hi1);
      c = make_uint4(hi1 ^ c.y ^ k.x, lo1, hi0 ^ c.w ^ k.y, lo0);
      k.x += 0x9E3779B9u;
      k.y += 0xBB67AE85u;
    }
    if (++ctr.x == 0) ++ctr.y;
    return c;
  }
};

__device__ __forceinline__ float u32_to_unit(uint32_t x) {
  // (0, 1]
  return (float)(x >> 8) * (1.0f / 16777216.0f) + (0.5f / 16777216.0f);
}

}  // namespace apex

#define APEX_HIP_CHECK(expr)                                                    \
  do {                                                                          \
    hipError_t _e = (expr);                                                     \
    if (_e != hipSuccess) return (int)_e;                                       \
  } while (0)
