// Fused transformer elementwise kernels (bias / activation / dropout / residual / LayerNorm)
// with the bias gradient folded into the backward pass.
//
//   bias_act      y = act(x + b)                         bwd: dx = dy*act'(x+b), db = colsum(dx)
//   bias_drop_add y = res + dropout(x + b)               bwd: dres = dy, dx = dy*mask/(1-p), db
//   bdaln         s = res + dropout(x + b); y = LN(s)     bwd: LN bwd -> ds; dres = ds; dx; db,
//                                                              dgamma, dbeta
// Dropout masks are never stored: element e keeps iff 16-bit chunk (e & 7) of
// Philox(seed, 0, offset + e/8) >= thresh, regenerated identically in backward.
// Column sums (bias / gamma / beta grads) are accumulated per thread in registers over a
// row block, written as fp32 partial rows and reduced by colsum_reduce (deterministic).
#include "common.h"
#include "kernels.h"
#include "fp8_pack.h"

#include <type_traits>

namespace apex {

constexpr int kEwBlock = 256;

__device__ __forceinline__ float gelu_erf(float x) { return 0.5f * x * (1.f + erff(x * 0.70710678118654752f)); }
__device__ __forceinline__ float gelu_erf_grad(float x) {
  const float cdf = 0.5f * (1.f + erff(x * 0.70710678118654752f));
  const float pdf = 0.3989422804014327f * __expf(-0.5f * x * x);
  return cdf + x * pdf;
}
__device__ __forceinline__ float gelu_tanh(float x) {
  const float u = 0.7978845608028654f * (x + 0.044715f * x * x * x);
  return 0.5f * x * (1.f + tanhf(u));
}
__device__ __forceinline__ float gelu_tanh_grad(float x) {
  const float u = 0.7978845608028654f * (x + 0.044715f * x * x * x);
  const float t = tanhf(u);
  return 0.5f * (1.f + t) + 0.5f * x * (1.f - t * t) * 0.7978845608028654f * (1.f + 3.f * 0.044715f * x * x);
}

template <int ACT>
__device__ __forceinline__ float act_f(float x) {
  if (ACT == 0) return gelu_erf(x);
  if (ACT == 1) return gelu_tanh(x);
  if (ACT == 2) return fmaxf(x, 0.f);
  return x;  // identity
}
template <int ACT>
__device__ __forceinline__ float act_g(float x) {
  if (ACT == 0) return gelu_erf_grad(x);
  if (ACT == 1) return gelu_tanh_grad(x);
  if (ACT == 2) return x > 0.f ? 1.f : 0.f;
  return 1.f;
}

// 8 keep flags for elements [e8*8, e8*8+8)
__device__ __forceinline__ void drop_mask8(uint64_t seed, uint64_t offset, int64_t e8, uint32_t thresh,
                                           bool (&keep)[8]) {
  Philox ph(seed, 0, offset + (uint64_t)e8);
  const uint4 r = ph.next();
  const uint32_t w[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const uint32_t v = (k & 1) ? (w[k >> 1] >> 16) : (w[k >> 1] & 0xffffu);
    keep[k] = v >= thresh;
  }
}

// Geometry shared by the column-chunk kernels: block = 256 threads x 8 columns = 2048
// columns; grid.x = column chunks, grid.y = row blocks of `rpb` rows.
struct ColGeom {
  int64_t rows;
  int cols;
  int rpb;
};

// ------------------------------- bias + activation -------------------------
template <typename T, typename W, int ACT>
__global__ void __launch_bounds__(kEwBlock) bias_act_fwd_kernel(const T* __restrict__ x,
                                                               const W* __restrict__ b,
                                                               T* __restrict__ y, ColGeom g) {
  const int c = (blockIdx.x * kEwBlock + threadIdx.x) * 8;
  if (c >= g.cols) return;
  float bv[8];
  if (b) load_f<W, 8>(b + c, bv);
  else {
#pragma unroll
    for (int k = 0; k < 8; ++k) bv[k] = 0.f;
  }
  const int64_t r0 = (int64_t)blockIdx.y * g.rpb;
  const int64_t r1 = min(r0 + g.rpb, g.rows);
  for (int64_t r = r0; r < r1; ++r) {
    float v[8];
    load_f<T, 8>(x + r * g.cols + c, v);
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = act_f<ACT>(v[k] + bv[k]);
    store_f<T, 8>(y + r * g.cols + c, v);
  }
}

template <typename T, typename W, int ACT>
__global__ void __launch_bounds__(kEwBlock) bias_act_bwd_kernel(const T* __restrict__ dy,
                                                               const T* __restrict__ x,
                                                               const W* __restrict__ b,
                                                               T* __restrict__ dx,
                                                               float* __restrict__ part, ColGeom g) {
  const int c = (blockIdx.x * kEwBlock + threadIdx.x) * 8;
  if (c >= g.cols) return;
  float bv[8], acc[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) acc[k] = 0.f;
  if (b) load_f<W, 8>(b + c, bv);
  else {
#pragma unroll
    for (int k = 0; k < 8; ++k) bv[k] = 0.f;
  }
  const int64_t r0 = (int64_t)blockIdx.y * g.rpb;
  const int64_t r1 = min(r0 + g.rpb, g.rows);
  for (int64_t r = r0; r < r1; ++r) {
    float v[8], d[8];
    load_f<T, 8>(x + r * g.cols + c, v);
    load_f<T, 8>(dy + r * g.cols + c, d);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      d[k] *= act_g<ACT>(v[k] + bv[k]);
      acc[k] += d[k];
    }
    store_f<T, 8>(dx + r * g.cols + c, d);
  }
  if (part) store_f<float, 8>(part + (int64_t)blockIdx.y * g.cols + c, acc);
}

// ----------------------------- bias + dropout + residual ---------------------
template <typename T, typename W, bool DROP>
__global__ void __launch_bounds__(kEwBlock) bda_fwd_kernel(const T* __restrict__ x, const W* __restrict__ b,
                                                          const T* __restrict__ res, T* __restrict__ y,
                                                          ColGeom g, uint64_t seed, uint64_t offset,
                                                          uint32_t thresh, float scale) {
  const int c = (blockIdx.x * kEwBlock + threadIdx.x) * 8;
  if (c >= g.cols) return;
  float bv[8];
  if (b) load_f<W, 8>(b + c, bv);
  else {
#pragma unroll
    for (int k = 0; k < 8; ++k) bv[k] = 0.f;
  }
  const int64_t r0 = (int64_t)blockIdx.y * g.rpb;
  const int64_t r1 = min(r0 + g.rpb, g.rows);
  for (int64_t r = r0; r < r1; ++r) {
    const int64_t e = r * g.cols + c;
    float v[8], rv[8];
    load_f<T, 8>(x + e, v);
    load_f<T, 8>(res + e, rv);
    bool keep[8];
    if (DROP) drop_mask8(seed, offset, e >> 3, thresh, keep);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      float t = v[k] + bv[k];
      if (DROP) t = keep[k] ? t * scale : 0.f;
      v[k] = rv[k] + t;
    }
    store_f<T, 8>(y + e, v);
  }
}

template <typename T, bool DROP>
__global__ void __launch_bounds__(kEwBlock) bda_bwd_kernel(const T* __restrict__ dy, T* __restrict__ dx,
                                                          float* __restrict__ part, ColGeom g,
                                                          uint64_t seed, uint64_t offset,
                                                          uint32_t thresh, float scale) {
  const int c = (blockIdx.x * kEwBlock + threadIdx.x) * 8;
  if (c >= g.cols) return;
  float acc[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) acc[k] = 0.f;
  const int64_t r0 = (int64_t)blockIdx.y * g.rpb;
  const int64_t r1 = min(r0 + g.rpb, g.rows);
  for (int64_t r = r0; r < r1; ++r) {
    const int64_t e = r * g.cols + c;
    float d[8];
    load_f<T, 8>(dy + e, d);
    bool keep[8];
    if (DROP) drop_mask8(seed, offset, e >> 3, thresh, keep);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      if (DROP) d[k] = keep[k] ? d[k] * scale : 0.f;
      acc[k] += d[k];
    }
    if (dx) store_f<T, 8>(dx + e, d);
  }
  if (part) store_f<float, 8>(part + (int64_t)blockIdx.y * g.cols + c, acc);
}

// ------------------------- bias + dropout + residual + LayerNorm ------------
// one wave per row (cols % 8 == 0, cols <= 512*VPT... VPT vectors of 8 per lane)
template <typename T, typename W, int VPT, bool DROP>
__global__ void __launch_bounds__(kEwBlock) bdaln_fwd_kernel(const T* __restrict__ x, const W* __restrict__ b,
                                                            const T* __restrict__ res,
                                                            const W* __restrict__ gamma,
                                                            const W* __restrict__ beta, T* __restrict__ y,
                                                            T* __restrict__ s_out, float* __restrict__ mean,
                                                            float* __restrict__ rstd, int64_t rows, int cols,
                                                            float eps, uint64_t seed, uint64_t offset,
                                                            uint32_t thresh, float scale, Q8Out q8, int s_cond) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  // fp8 scale and amax filter value read up front (not behind the row's reductions)
  const float qs = q8.y ? q8.scale[0] : 0.f, q8seen = q8.y ? f8_amax_seen(q8.amax) : 0.f;
  if (row >= rows) {
    if (q8.y) f8_block_amax(0.f, q8.amax, q8seen);  // the block reduction needs every wave
    return;
  }
  const int nvec = cols >> 3;
  float v[VPT][8];
  float sum = 0.f;
#pragma unroll
  for (int j = 0; j < VPT; ++j) {
    const int vi = j * 64 + lane;
    if (vi < nvec) {
      const int64_t e = row * cols + vi * 8;
      float xv[8], rv[8], bv[8];
      load_f<T, 8>(x + e, xv);
      load_f<T, 8>(res + e, rv);
      if (b) load_f<W, 8>(b + vi * 8, bv);
      else {
#pragma unroll
        for (int k = 0; k < 8; ++k) bv[k] = 0.f;
      }
      bool keep[8];
      if (DROP) drop_mask8(seed, offset, e >> 3, thresh, keep);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        float t = xv[k] + bv[k];
        if (DROP) t = keep[k] ? t * scale : 0.f;
        v[j][k] = rv[k] + t;
      }
      // the LN input is stored at the activation precision and normalised from that value,
      // so backward (which reads s_out) sees exactly what forward normalised; s_out == nullptr:
      // not stored (post-LN memory-efficient mode: the backward rebuilds x-hat from y)
      if (s_out && !s_cond) store_f<T, 8>(s_out + e, v[j]);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        v[j][k] = to_f(from_f<T>(v[j][k]));
        sum += v[j][k];
      }
    } else {
#pragma unroll
      for (int k = 0; k < 8; ++k) v[j][k] = 0.f;
    }
  }
  const float inv_n = 1.f / (float)cols;
  const float mu = wave_sum(sum) * inv_n;
  float ss = 0.f;
#pragma unroll
  for (int j = 0; j < VPT; ++j) {
    if (j * 64 + lane < nvec) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float d = v[j][k] - mu;
        ss += d * d;
      }
    }
  }
  const float rs = rsqrtf(wave_sum(ss) * inv_n + eps);
  if (lane == 0) {
    mean[row] = mu;
    rstd[row] = rs;
  }
  float mx = 0.f;
  bool gz = false;  // a gamma entry of exactly 0 (s_cond: the backward cannot rebuild x-hat from y)
#pragma unroll
  for (int j = 0; j < VPT; ++j) {
    const int vi = j * 64 + lane;
    if (vi < nvec) {
      float gv[8], bb[8], o[8];
      load_f<W, 8>(gamma + vi * 8, gv);
      load_f<W, 8>(beta + vi * 8, bb);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        o[k] = (v[j][k] - mu) * rs * gv[k] + bb[k];
        gz |= gv[k] == 0.f;
      }
      if (q8.y) {
        // with the fp8 codes of the output as stored (rounded to T): the next GEMM's operand
        // without a standalone quantise pass re-reading y from HBM
        if constexpr (sizeof(T) == 2) {
          f8_store_with_codes8<T>(y + row * cols + vi * 8, q8.y + row * cols + vi * 8, o, qs, q8.fmt, mx);
        } else {
          store_f<T, 8>(y + row * cols + vi * 8, o);
#pragma unroll
          for (int k = 0; k < 8; ++k) mx = fmaxf(mx, fabsf(o[k]));
          f8_store8(q8.y + row * cols + vi * 8, o, qs, q8.fmt);
        }
      } else {
        store_f<T, 8>(y + row * cols + vi * 8, o);
      }
    }
  }
  if (q8.y) f8_block_amax(mx, q8.amax, q8seen);
  // s_cond (memory-efficient post-LN): s is stored only when gamma has a zero entry — every wave
  // holds the whole gamma row, so the decision is the same for every row of the launch, and the
  // backward (bdaln_bwd_kernel FROMY) makes the same test to read s instead of rebuilding x-hat.
  // v still holds s rounded to T, i.e. exactly what the unconditional store writes.
  if (s_out && s_cond && __any(gz)) {
#pragma unroll
    for (int j = 0; j < VPT; ++j) {
      const int vi = j * 64 + lane;
      if (vi < nvec) store_f<T, 8>(s_out + row * cols + vi * 8, v[j]);
    }
  }
}

// part rows: [dgamma | dbeta | dbias] (3*cols floats) per block.
// Each wave walks `rows_per_wave` rows (4 waves interleaved per block); the NEXT row's s / dy are
// loaded into registers (raw 16-byte packs) before the current row's reduction and stores, so every
// wave keeps two rows of loads in flight — with one row per wave the kernel was latency-bound at
// ~4.2 TB/s (rocprofv3 FETCH/WRITE_SIZE, profiles/r2_pmc_bw_kernels.json).
// EXTRA (pre-LN residual streams, GPT): s also feeds the next residual add, so its gradient is
// LN_bwd(dy) + dse — dse is added here instead of by a separate autograd accumulate pass.
// FROMY (post-LN, memory-efficient): `s` points at the LN OUTPUT y and x-hat = (y - beta) / gamma,
// so the forward need not store s at all (one [rows, cols] write less per sublayer; y is saved
// anyway as the next GEMM's input). dgamma accumulates dy * (y - beta) and is divided by gamma once.
// Q8: also write fp8 codes of dx (template flag: the runtime branch cost the plain kernel its third
// wave per SIMD, 168 -> 170 VGPRs; the Q8 variant is held to 3 waves per SIMD explicitly — at 2 it
// ran 210 vs 145 us at the BERT shape)
template <typename T, typename W, int VPT, bool DROP, bool EXTRA, bool FROMY, bool Q8>
__device__ __forceinline__ void bdaln_bwd_body(const T* __restrict__ dy, const T* __restrict__ s,
                                                            const W* __restrict__ gamma,
                                                            const W* __restrict__ beta,
                                                            const float* __restrict__ mean,
                                                            const float* __restrict__ rstd,
                                                            const T* __restrict__ dse,
                                                            T* __restrict__ dres, T* __restrict__ dx,
                                                            float* __restrict__ part, int64_t rows, int cols,
                                                            int rows_per_wave, uint64_t seed,
                                                            uint64_t offset, uint32_t thresh, float scale,
                                                            Q8Out q8) {
  extern __shared__ __attribute__((aligned(16))) float lds[];  // [4][3*cols]
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int nvec = cols >> 3;
  const float inv_n = 1.f / (float)cols;
  float qs = 0.f, q8seen = 0.f, mx = 0.f;
  if constexpr (Q8) {
    qs = q8.scale[0];
    q8seen = f8_amax_seen(q8.amax);
  }
  float dg[VPT][8], dbt[VPT][8], dbi[VPT][8], g[VPT][8];
#pragma unroll
  for (int j = 0; j < VPT; ++j) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      dg[j][k] = dbt[j][k] = dbi[j][k] = 0.f;
      g[j][k] = 1.f;
    }
    if (j * 64 + lane < nvec) load_f<W, 8>(gamma + (j * 64 + lane) * 8, g[j]);
  }
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_wave * 4;
  typedef Pack<T, 8> P8;
  P8 ns[VPT], nd[VPT], ne[EXTRA ? VPT : 1];
  auto fetch = [&](int64_t row) {
#pragma unroll
    for (int j = 0; j < VPT; ++j) {
      const int vi = j * 64 + lane;
      if (vi < nvec && row < rows) {
        ns[j] = *reinterpret_cast<const P8*>(s + row * cols + vi * 8);
        nd[j] = *reinterpret_cast<const P8*>(dy + row * cols + vi * 8);
        if constexpr (EXTRA) ne[j] = *reinterpret_cast<const P8*>(dse + row * cols + vi * 8);
      }
    }
  };
  fetch(r0 + wid);
  if constexpr (FROMY) {
    // beta and 1/gamma (fp32) staged once in the head of the partial-combine LDS buffer (free until
    // the row loop ends): per row they come back as 16-byte LDS reads — a register copy took the
    // kernel from 3 to 2 waves per SIMD, per-row global reads put an L2 round trip on every row
    for (int c = threadIdx.x; c < cols; c += kEwBlock) {
      lds[c] = to_f(beta[c]);
      lds[cols + c] = 1.f / to_f(gamma[c]);
    }
    __syncthreads();
  }
  for (int rr = 0; rr < rows_per_wave; ++rr) {
    const int64_t row = r0 + (int64_t)rr * 4 + wid;
    if (row >= rows) break;
    float xh[VPT][8], dv[VPT][8], ev[EXTRA ? VPT : 1][8];
#pragma unroll
    for (int j = 0; j < VPT; ++j)
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        xh[j][k] = to_f(ns[j].v[k]);
        dv[j][k] = to_f(nd[j].v[k]);
        if constexpr (EXTRA) ev[j][k] = to_f(ne[j].v[k]);
      }
    if (rr + 1 < rows_per_wave) fetch(row + 4);
    const float mu = FROMY ? 0.f : mean[row], rs = rstd[row];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int j = 0; j < VPT; ++j) {
      const int vi = j * 64 + lane;
      if (vi < nvec) {
        float bt[8], ig[8];
        if constexpr (FROMY) {
          *reinterpret_cast<float4*>(bt) = *reinterpret_cast<const float4*>(lds + vi * 8);
          *reinterpret_cast<float4*>(bt + 4) = *reinterpret_cast<const float4*>(lds + vi * 8 + 4);
          *reinterpret_cast<float4*>(ig) = *reinterpret_cast<const float4*>(lds + cols + vi * 8);
          *reinterpret_cast<float4*>(ig + 4) = *reinterpret_cast<const float4*>(lds + cols + vi * 8 + 4);
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const float dyg = dv[j][k] * g[j][k];
          s1 += dyg;
          if constexpr (FROMY) {
            const float yc = xh[j][k] - bt[k];  // = x-hat * gamma
            s2 += dv[j][k] * yc;
            dg[j][k] += dv[j][k] * yc;  // / gamma at the end
            xh[j][k] = yc * ig[k];
          } else {
            xh[j][k] = (xh[j][k] - mu) * rs;
            s2 += dyg * xh[j][k];
            dg[j][k] += dv[j][k] * xh[j][k];
          }
          dbt[j][k] += dv[j][k];
        }
      }
    }
    s1 = wave_sum(s1) * inv_n;
    s2 = wave_sum(s2) * inv_n;
#pragma unroll
    for (int j = 0; j < VPT; ++j) {
      const int vi = j * 64 + lane;
      if (vi < nvec) {
        const int64_t e = row * cols + vi * 8;
        float ds[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          ds[k] = rs * (dv[j][k] * g[j][k] - s1 - xh[j][k] * s2);
          if constexpr (EXTRA) ds[k] += ev[j][k];
        }
        store_f<T, 8>(dres + e, ds);
        bool keep[8];
        if (DROP) drop_mask8(seed, offset, e >> 3, thresh, keep);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          if (DROP) ds[k] = keep[k] ? ds[k] * scale : 0.f;
          dbi[j][k] += ds[k];
        }
        if constexpr (Q8 && sizeof(T) == 2) {  // with the fp8 codes of dx as stored (the dgrad GEMM's operand)
          // (q8.only: dx's consumers read the codes alone — apex.fp8 codes_only_ok — dx is not stored)
          f8_store_with_codes8<T>(dx + e, q8.y + e, ds, qs, q8.fmt, mx, !q8.only);
        } else {
          if (!(Q8 && q8.only)) store_f<T, 8>(dx + e, ds);
          if constexpr (Q8) {
#pragma unroll
            for (int k = 0; k < 8; ++k) mx = fmaxf(mx, fabsf(ds[k]));
            f8_store8(q8.y + e, ds, qs, q8.fmt);
          }
        }
      }
    }
  }
  if constexpr (Q8) f8_block_amax(mx, q8.amax, q8seen);
  if constexpr (FROMY) __syncthreads();  // every wave is done with the staged beta / 1/gamma
  float* mine = lds + wid * 3 * cols;
#pragma unroll
  for (int j = 0; j < VPT; ++j) {
    const int vi = j * 64 + lane;
    if (vi < nvec) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        mine[vi * 8 + k] = FROMY ? dg[j][k] / g[j][k] : dg[j][k];
        mine[cols + vi * 8 + k] = dbt[j][k];
        mine[2 * cols + vi * 8 + k] = dbi[j][k];
      }
    }
  }
  __syncthreads();
  float* out = part + (int64_t)blockIdx.x * 3 * cols;
  for (int c = threadIdx.x; c < 3 * cols; c += kEwBlock)
    out[c] = lds[c] + lds[3 * cols + c] + lds[6 * cols + c] + lds[9 * cols + c];
}

// s_alt (FROMY only): the conditionally stored LN input of an s_cond forward. A gamma entry of exactly
// 0 makes x-hat = (y - beta) / gamma unrecoverable for its column; the forward then stored s, and
// the launch (gamma is the same for every wave: the test agrees across the grid) runs the
// stored-input body on it instead — exact gradients, no 0 * inf NaNs.
template <typename T, typename W, int VPT, bool DROP, bool EXTRA = false, bool FROMY = false, bool Q8 = false>
__global__ void __launch_bounds__(kEwBlock) __attribute__((amdgpu_waves_per_eu(Q8 ? 3 : 1))) bdaln_bwd_kernel(const T* __restrict__ dy, const T* __restrict__ s,
                                                            const W* __restrict__ gamma,
                                                            const W* __restrict__ beta,
                                                            const float* __restrict__ mean,
                                                            const float* __restrict__ rstd,
                                                            const T* __restrict__ dse,
                                                            T* __restrict__ dres, T* __restrict__ dx,
                                                            float* __restrict__ part, int64_t rows, int cols,
                                                            int rows_per_wave, uint64_t seed,
                                                            uint64_t offset, uint32_t thresh, float scale,
                                                            Q8Out q8, const T* __restrict__ s_alt) {
  if constexpr (FROMY) {
    if (s_alt) {
      const int lane = threadIdx.x & 63, nvec = cols >> 3;
      bool gz = false;
#pragma unroll
      for (int j = 0; j < VPT; ++j) {
        if (j * 64 + lane < nvec) {
          float gv[8];
          load_f<W, 8>(gamma + (j * 64 + lane) * 8, gv);
#pragma unroll
          for (int k = 0; k < 8; ++k) gz |= gv[k] == 0.f;
        }
      }
      if (__any(gz)) {
        bdaln_bwd_body<T, W, VPT, DROP, EXTRA, false, Q8>(dy, s_alt, gamma, nullptr, mean, rstd, dse, dres, dx, part,
                                                           rows, cols, rows_per_wave, seed, offset, thresh, scale, q8);
        return;
      }
    }
  }
  bdaln_bwd_body<T, W, VPT, DROP, EXTRA, FROMY, Q8>(dy, s, gamma, beta, mean, rstd, dse, dres, dx, part, rows, cols,
                                                     rows_per_wave, seed, offset, thresh, scale, q8);
}

// Wide rows (2056..4096 cols, VPT 5..8 vectors per lane: Megatron H = 2560): the fast kernel's
// register-resident rows + gamma + three partial rows would spill, so this variant keeps only the
// dgamma / dbeta / dbias partials in registers and reads each row twice (second pass from L1/L2;
// a row is 5-8 KB), gamma from cache; the partials combine through LDS one third at a time
// ([4 waves][cols] floats <= 64 KB). Same ws layout as bdaln_bwd_kernel.
template <typename T, typename W, int VPT, bool DROP, bool EXTRA>
__global__ void __launch_bounds__(kEwBlock) bdaln_bwd_wide_kernel(const T* __restrict__ dy, const T* __restrict__ s,
                                                                 const W* __restrict__ gamma,
                                                                 const float* __restrict__ mean,
                                                                 const float* __restrict__ rstd,
                                                                 const T* __restrict__ dse, T* __restrict__ dres,
                                                                 T* __restrict__ dx, float* __restrict__ part,
                                                                 int64_t rows, int cols, int rows_per_wave,
                                                                 uint64_t seed, uint64_t offset, uint32_t thresh,
                                                                 float scale) {
  extern __shared__ __attribute__((aligned(16))) float lds[];  // [4][cols]
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int nvec = cols >> 3;
  const float inv_n = 1.f / (float)cols;
  float dg[VPT][8], dbt[VPT][8], dbi[VPT][8];
#pragma unroll
  for (int j = 0; j < VPT; ++j)
#pragma unroll
    for (int k = 0; k < 8; ++k) dg[j][k] = dbt[j][k] = dbi[j][k] = 0.f;
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_wave * 4;
  for (int rr = 0; rr < rows_per_wave; ++rr) {
    const int64_t row = r0 + (int64_t)rr * 4 + wid;
    if (row >= rows) break;
    const float mu = mean[row], rs = rstd[row];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int j = 0; j < VPT; ++j) {
      const int vi = j * 64 + lane;
      if (vi < nvec) {
        const int64_t e = row * cols + vi * 8;
        float xv[8], dv[8], g[8];
        load_f<T, 8>(s + e, xv);
        load_f<T, 8>(dy + e, dv);
        load_f<W, 8>(gamma + vi * 8, g);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const float xh = (xv[k] - mu) * rs;
          const float dyg = dv[k] * g[k];
          s1 += dyg;
          s2 += dyg * xh;
          dg[j][k] += dv[k] * xh;
          dbt[j][k] += dv[k];
        }
      }
    }
    s1 = wave_sum(s1) * inv_n;
    s2 = wave_sum(s2) * inv_n;
#pragma unroll
    for (int j = 0; j < VPT; ++j) {
      const int vi = j * 64 + lane;
      if (vi < nvec) {
        const int64_t e = row * cols + vi * 8;
        float xv[8], dv[8], g[8], ev[8], ds[8];
        load_f<T, 8>(s + e, xv);
        load_f<T, 8>(dy + e, dv);
        load_f<W, 8>(gamma + vi * 8, g);
        if constexpr (EXTRA) load_f<T, 8>(dse + e, ev);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          ds[k] = rs * (dv[k] * g[k] - s1 - (xv[k] - mu) * rs * s2);
          if constexpr (EXTRA) ds[k] += ev[k];
        }
        store_f<T, 8>(dres + e, ds);
        bool keep[8];
        if (DROP) drop_mask8(seed, offset, e >> 3, thresh, keep);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          if (DROP) ds[k] = keep[k] ? ds[k] * scale : 0.f;
          dbi[j][k] += ds[k];
        }
        store_f<T, 8>(dx + e, ds);
      }
    }
  }
  float* mine = lds + wid * cols;
  float* out = part + (int64_t)blockIdx.x * 3 * cols;
#pragma unroll
  for (int t = 0; t < 3; ++t) {
    if (t) __syncthreads();
#pragma unroll
    for (int j = 0; j < VPT; ++j) {
      const int vi = j * 64 + lane;
      if (vi < nvec) {
#pragma unroll
        for (int k = 0; k < 8; ++k) mine[vi * 8 + k] = t == 0 ? dg[j][k] : t == 1 ? dbt[j][k] : dbi[j][k];
      }
    }
    __syncthreads();
    for (int c = threadIdx.x; c < cols; c += kEwBlock)
      out[t * cols + c] = lds[c] + lds[cols + c] + lds[2 * cols + c] + lds[3 * cols + c];
  }
}

// ------------------------- BERT embeddings (gather-sum + LayerNorm + dropout) -------------
// forward, one wave per token row (row = b*S + pos):
//   s = Ww[id] + Wp[pos] + Wt[type]; y = dropout(LN(s))     (s stored for the backward)
// The word / type ids are int32, clamped to the table by the caller (apex.ops.fused).
template <typename T, typename W, int VPT, bool DROP>
__global__ void __launch_bounds__(kEwBlock) embed_ln_fwd_kernel(const int* __restrict__ ids, const int* __restrict__ tids,
                                                               const T* __restrict__ Ww, const T* __restrict__ Wp,
                                                               const T* __restrict__ Wt, const W* __restrict__ gamma,
                                                               const W* __restrict__ beta, T* __restrict__ y,
                                                               T* __restrict__ s_out, float* __restrict__ mean,
                                                               float* __restrict__ rstd, int64_t rows, int cols, int S,
                                                               float eps, uint64_t seed, uint64_t offset,
                                                               uint32_t thresh, float scale) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int nvec = cols >> 3;
  const int pos = (int)(row % S);
  const T* wr = Ww + (int64_t)ids[row] * cols;
  const T* pr = Wp + (int64_t)pos * cols;
  const T* tr = tids ? Wt + (int64_t)tids[row] * cols : Wt;
  float v[VPT][8];
  float sum = 0.f;
#pragma unroll
  for (int j = 0; j < VPT; ++j) {
    const int vi = j * 64 + lane;
    if (vi < nvec) {
      float a[8], b[8], c[8];
      load_f<T, 8>(wr + vi * 8, a);
      load_f<T, 8>(pr + vi * 8, b);
      load_f<T, 8>(tr + vi * 8, c);
#pragma unroll
      for (int k = 0; k < 8; ++k) v[j][k] = a[k] + b[k] + c[k];
      store_f<T, 8>(s_out + row * cols + vi * 8, v[j]);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        v[j][k] = to_f(from_f<T>(v[j][k]));  // normalise exactly what the backward reads
        sum += v[j][k];
      }
    } else {
#pragma unroll
      for (int k = 0; k < 8; ++k) v[j][k] = 0.f;
    }
  }
  const float inv_n = 1.f / (float)cols;
  const float mu = wave_sum(sum) * inv_n;
  float ss = 0.f;
#pragma unroll
  for (int j = 0; j < VPT; ++j)
    if (j * 64 + lane < nvec)
#pragma unroll
      for (int k = 0; k < 8; ++k) ss += (v[j][k] - mu) * (v[j][k] - mu);
  const float rs = rsqrtf(wave_sum(ss) * inv_n + eps);
  if (lane == 0) {
    mean[row] = mu;
    rstd[row] = rs;
  }
#pragma unroll
  for (int j = 0; j < VPT; ++j) {
    const int vi = j * 64 + lane;
    if (vi < nvec) {
      const int64_t e = row * cols + vi * 8;
      float gv[8], bb[8], o[8];
      load_f<W, 8>(gamma + vi * 8, gv);
      load_f<W, 8>(beta + vi * 8, bb);
      bool keep[8];
      if (DROP) drop_mask8(seed, offset, e >> 3, thresh, keep);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        o[k] = (v[j][k] - mu) * rs * gv[k] + bb[k];
        if (DROP) o[k] = keep[k] ? o[k] * scale : 0.f;
      }
      store_f<T, 8>(y + e, o);
    }
  }
}

// backward: grid (S, NWT / 4); wave (pos = blockIdx.x, w) walks the batch rows b = w, w + NWT, ...
// of one position: dropout-backward + LayerNorm-backward -> ds (the gradient of the sum, stored for
// the word-embedding segment sum), and in registers the position row's gradient, the type rows'
// (type vocab <= 2) and dgamma / dbeta, written as fp32 partial rows:
//   part_pos [NWT][S][cols], part_tg [S * NWT][4][cols] = {dgamma, dbeta, dtype0, dtype1}
template <typename T, typename W, int VPT, bool DROP>
__global__ void __launch_bounds__(kEwBlock) embed_ln_bwd_kernel(const T* __restrict__ dy, const T* __restrict__ s,
                                                               const W* __restrict__ gamma, const float* __restrict__ mean,
                                                               const float* __restrict__ rstd, const int* __restrict__ tids,
                                                               T* __restrict__ ds_out, float* __restrict__ part_pos,
                                                               float* __restrict__ part_tg, int64_t B, int cols, int S,
                                                               int nwt, uint64_t seed, uint64_t offset, uint32_t thresh,
                                                               float scale) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int pos = blockIdx.x;
  const int w = blockIdx.y * 4 + wid;
  const int nvec = cols >> 3;
  const float inv_n = 1.f / (float)cols;
  float g[VPT][8], dgm[VPT][8], dbt[VPT][8], dps[VPT][8], dt0[VPT][8], dt1[VPT][8];
#pragma unroll
  for (int j = 0; j < VPT; ++j) {
#pragma unroll
    for (int k = 0; k < 8; ++k) g[j][k] = dgm[j][k] = dbt[j][k] = dps[j][k] = dt0[j][k] = dt1[j][k] = 0.f;
    if (j * 64 + lane < nvec) load_f<W, 8>(gamma + (j * 64 + lane) * 8, g[j]);
  }
  typedef Pack<T, 8> P8;
  P8 ns[VPT], nd[VPT];
  auto fetch = [&](int64_t b) {
    const int64_t row = b * S + pos;
#pragma unroll
    for (int j = 0; j < VPT; ++j) {
      const int vi = j * 64 + lane;
      if (vi < nvec && b < B) {
        ns[j] = *reinterpret_cast<const P8*>(s + row * cols + vi * 8);
        nd[j] = *reinterpret_cast<const P8*>(dy + row * cols + vi * 8);
      }
    }
  };
  if (w < nwt) {
    fetch(w);
    for (int64_t b = w; b < B; b += nwt) {
      const int64_t row = b * S + pos;
      float xh[VPT][8], dv[VPT][8];
#pragma unroll
      for (int j = 0; j < VPT; ++j)
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          xh[j][k] = to_f(ns[j].v[k]);
          dv[j][k] = to_f(nd[j].v[k]);
        }
      if (b + nwt < B) fetch(b + nwt);
      const float mu = mean[row], rs = rstd[row];
      const int tt = tids ? tids[row] : 0;
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int j = 0; j < VPT; ++j) {
        const int vi = j * 64 + lane;
        if (vi < nvec) {
          bool keep[8];
          if (DROP) drop_mask8(seed, offset, (row * cols + vi * 8) >> 3, thresh, keep);
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            if (DROP) dv[j][k] = keep[k] ? dv[j][k] * scale : 0.f;
            xh[j][k] = (xh[j][k] - mu) * rs;
            const float dyg = dv[j][k] * g[j][k];
            s1 += dyg;
            s2 += dyg * xh[j][k];
            dgm[j][k] += dv[j][k] * xh[j][k];
            dbt[j][k] += dv[j][k];
          }
        }
      }
      s1 = wave_sum(s1) * inv_n;
      s2 = wave_sum(s2) * inv_n;
#pragma unroll
      for (int j = 0; j < VPT; ++j) {
        const int vi = j * 64 + lane;
        if (vi < nvec) {
          float d[8];
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            d[k] = rs * (dv[j][k] * g[j][k] - s1 - xh[j][k] * s2);
            dps[j][k] += d[k];
            if (tt == 0) dt0[j][k] += d[k];
            else dt1[j][k] += d[k];
          }
          store_f<T, 8>(ds_out + row * cols + vi * 8, d);
        }
      }
    }
  }
  if (w >= nwt) return;
  float* pp = part_pos + ((int64_t)w * S + pos) * cols;
  float* pt = part_tg + ((int64_t)pos * nwt + w) * 4 * cols;
#pragma unroll
  for (int j = 0; j < VPT; ++j) {
    const int vi = j * 64 + lane;
    if (vi < nvec) {
      store_f<float, 8>(pp + vi * 8, dps[j]);
      store_f<float, 8>(pt + vi * 8, dgm[j]);
      store_f<float, 8>(pt + cols + vi * 8, dbt[j]);
      store_f<float, 8>(pt + 2 * cols + vi * 8, dt0[j]);
      store_f<float, 8>(pt + 3 * cols + vi * 8, dt1[j]);
    }
  }
}

// word-embedding gradient: one wave per position of the id-sorted token list; the head of each
// run of equal ids sums the ds rows of that run (fixed order: deterministic) into dW[id]
template <typename T, int VPT>
__global__ void __launch_bounds__(kEwBlock) embed_segsum_kernel(const T* __restrict__ ds, const int* __restrict__ sorted,
                                                               const int64_t* __restrict__ perm, T* __restrict__ dW,
                                                               int64_t R, int cols) {
  const int lane = threadIdx.x & 63;
  const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i >= R) return;
  const int id = sorted[i];
  if (i > 0 && sorted[i - 1] == id) return;
  const int nvec = cols >> 3;
  float acc[VPT][8];
#pragma unroll
  for (int j = 0; j < VPT; ++j)
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[j][k] = 0.f;
  for (int64_t t = i; t < R && sorted[t] == id; ++t) {
    const T* r = ds + perm[t] * cols;
#pragma unroll
    for (int j = 0; j < VPT; ++j) {
      const int vi = j * 64 + lane;
      if (vi < nvec) {
        float v[8];
        load_f<T, 8>(r + vi * 8, v);
#pragma unroll
        for (int k = 0; k < 8; ++k) acc[j][k] += v[k];
      }
    }
  }
#pragma unroll
  for (int j = 0; j < VPT; ++j) {
    const int vi = j * 64 + lane;
    if (vi < nvec) store_f<T, 8>(dW + (int64_t)id * cols + vi * 8, acc[j]);
  }
}

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
#define EW_DISPATCH(DT, T, ...)                             \
  switch (DT) {                                             \
    case kF32: { using T = float; __VA_ARGS__; } break;     \
    case kF16: { using T = f16; __VA_ARGS__; } break;       \
    case kBF16: { using T = bf16; __VA_ARGS__; } break;     \
    default: return -1;                                     \
  }
#define EW_ACT(A, ACT, ...)                                 \
  switch (A) {                                              \
    case 0: { constexpr int ACT = 0; __VA_ARGS__; } break;  \
    case 1: { constexpr int ACT = 1; __VA_ARGS__; } break;  \
    case 2: { constexpr int ACT = 2; __VA_ARGS__; } break;  \
    case 3: { constexpr int ACT = 3; __VA_ARGS__; } break;  \
    default: return -1;                                     \
  }

static inline ColGeom col_geom(int64_t rows, int cols, int target_parts) {
  ColGeom g;
  g.rows = rows;
  g.cols = cols;
  const int chunks = (cols + 2047) / 2048;
  // aim for ~target_parts * chunks blocks, >= 16 rows per block
  int64_t rpb = (rows + target_parts - 1) / target_parts;
  if (rpb < 16) rpb = 16;
  g.rpb = (int)rpb;
  (void)chunks;
  return g;
}

int64_t colsum_parts(int64_t rows) {
  int64_t p = (rows + 15) / 16;
  return p < 512 ? p : 512;
}

int bias_act_fwd(const void* x, const void* b, void* y, int64_t rows, int cols, int act, int xdt,
                 int bdt, hipStream_t s) {
  if (rows == 0) return 0;
  if (cols % 8) return -2;
  ColGeom g = col_geom(rows, cols, 512);
  dim3 grid((cols / 8 + kEwBlock - 1) / kEwBlock, (unsigned)((rows + g.rpb - 1) / g.rpb));
  if (!b) bdt = xdt;
  EW_DISPATCH(xdt, T, EW_DISPATCH(bdt, W, EW_ACT(act, ACT,
      hipLaunchKernelGGL((bias_act_fwd_kernel<T, W, ACT>), grid, dim3(kEwBlock), 0, s, (const T*)x,
                         (const W*)b, (T*)y, g))));
  return (int)hipGetLastError();
}

int bias_act_bwd(const void* dy, const void* x, const void* b, void* dx, void* db, float* ws,
                 int64_t rows, int cols, int act, int xdt, int bdt, hipStream_t s) {
  if (rows == 0) return 0;
  if (cols % 8) return -2;
  ColGeom g = col_geom(rows, cols, 512);
  const int parts = (int)((rows + g.rpb - 1) / g.rpb);
  dim3 grid((cols / 8 + kEwBlock - 1) / kEwBlock, parts);
  if (!b) bdt = xdt;
  EW_DISPATCH(xdt, T, EW_DISPATCH(bdt, W, EW_ACT(act, ACT, {
    hipLaunchKernelGGL((bias_act_bwd_kernel<T, W, ACT>), grid, dim3(kEwBlock), 0, s, (const T*)dy,
                       (const T*)x, (const W*)b, (T*)dx, db ? ws : nullptr, g);
    if (db)
      launch_partial_colsum<W>(ws, parts, (int64_t)cols, cols, (W*)db, s);
  })));
  return (int)hipGetLastError();
}

int bias_dropout_add_fwd(const void* x, const void* b, const void* res, void* y, int64_t rows, int cols,
                         uint64_t seed, uint64_t offset, uint32_t thresh, float scale, int xdt, int bdt,
                         hipStream_t s) {
  if (rows == 0) return 0;
  if (cols % 8) return -2;
  ColGeom g = col_geom(rows, cols, 512);
  dim3 grid((cols / 8 + kEwBlock - 1) / kEwBlock, (unsigned)((rows + g.rpb - 1) / g.rpb));
  if (!b) bdt = xdt;
  EW_DISPATCH(xdt, T, EW_DISPATCH(bdt, W, {
    if (thresh)
      hipLaunchKernelGGL((bda_fwd_kernel<T, W, true>), grid, dim3(kEwBlock), 0, s, (const T*)x,
                         (const W*)b, (const T*)res, (T*)y, g, seed, offset, thresh, scale);
    else
      hipLaunchKernelGGL((bda_fwd_kernel<T, W, false>), grid, dim3(kEwBlock), 0, s, (const T*)x,
                         (const W*)b, (const T*)res, (T*)y, g, seed, offset, thresh, scale);
  }));
  return (int)hipGetLastError();
}

int bias_dropout_add_bwd(const void* dy, void* dx, void* db, float* ws, int64_t rows, int cols,
                         uint64_t seed, uint64_t offset, uint32_t thresh, float scale, int xdt, int bdt,
                         hipStream_t s) {
  if (rows == 0) return 0;
  if (cols % 8) return -2;
  ColGeom g = col_geom(rows, cols, 512);
  const int parts = (int)((rows + g.rpb - 1) / g.rpb);
  dim3 grid((cols / 8 + kEwBlock - 1) / kEwBlock, parts);
  EW_DISPATCH(xdt, T, EW_DISPATCH(bdt, W, {
    if (thresh)
      hipLaunchKernelGGL((bda_bwd_kernel<T, true>), grid, dim3(kEwBlock), 0, s, (const T*)dy, (T*)dx,
                         db ? ws : nullptr, g, seed, offset, thresh, scale);
    else
      hipLaunchKernelGGL((bda_bwd_kernel<T, false>), grid, dim3(kEwBlock), 0, s, (const T*)dy, (T*)dx,
                         db ? ws : nullptr, g, seed, offset, thresh, scale);
    if (db)
      launch_partial_colsum<W>(ws, parts, (int64_t)cols, cols, (W*)db, s);
  }));
  return (int)hipGetLastError();
}

int colsum(const void* x, void* out, float* ws, int64_t rows, int cols, int xdt, int odt, hipStream_t s) {
  return bias_dropout_add_bwd(x, nullptr, out, ws, rows, cols, 0, 0, 0, 1.f, xdt, odt, s);
}

// ---------------------------------------------------------------------------
// split-K combine for the weight-gradient GEMMs: out[n] = sum_s slabs[s][n] (fp32 slabs from
// a batched GEMM over K slices) written once in the output dtype. 8 elements per lane, slabs
// walked with independent loads (no dependency between slices).
// ---------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const float* __restrict__ slabs, T* __restrict__ out,
                                                            int64_t n, int nsplit, int accumulate) {
  // accumulate (fp32 out only): out += sum of the slabs — the weight gradient of one micro-batch
  // added into an fp32 main_grad without a separate add pass
  const int64_t i = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 8;
  if (i >= n) return;
  if (i + 8 <= n) {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if constexpr (sizeof(T) == 4) {
      if (accumulate) {
        float a[4], b[4];
        load_f<float, 4>(reinterpret_cast<const float*>(out) + i, a);
        load_f<float, 4>(reinterpret_cast<const float*>(out) + i + 4, b);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          acc[e] = a[e];
          acc[4 + e] = b[e];
        }
      }
    }
    for (int s = 0; s < nsplit; ++s) {
      float a[4], b[4];
      load_f<float, 4>(slabs + (int64_t)s * n + i, a);
      load_f<float, 4>(slabs + (int64_t)s * n + i + 4, b);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        acc[e] += a[e];
        acc[4 + e] += b[e];
      }
    }
    if constexpr (sizeof(T) == 4) {
      float lo[4] = {acc[0], acc[1], acc[2], acc[3]}, hi[4] = {acc[4], acc[5], acc[6], acc[7]};
      store_f<T, 4>(out + i, lo);
      store_f<T, 4>(out + i + 4, hi);
    } else {
      store_f<T, 8>(out + i, acc);
    }
  } else {
    for (int64_t j = i; j < n; ++j) {
      float acc = (sizeof(T) == 4 && accumulate) ? to_f(out[j]) : 0.f;
      for (int s = 0; s < nsplit; ++s) acc += slabs[(int64_t)s * n + j];
      out[j] = from_f<T>(acc);
    }
  }
}

int splitk_reduce(const float* slabs, void* out, int64_t n, int nsplit, int odt, hipStream_t s, int accumulate) {
  if (n == 0) return 0;
  if (accumulate && odt != kF32) return -2;
  const unsigned grid = (unsigned)((n / 8 + 256) / 256);
  if (odt == kF32)
    hipLaunchKernelGGL((splitk_reduce_kernel<float>), dim3(grid), dim3(256), 0, s, slabs, (float*)out, n, nsplit,
                       accumulate);
  else if (odt == kF16)
    hipLaunchKernelGGL((splitk_reduce_kernel<f16>), dim3(grid), dim3(256), 0, s, slabs, (f16*)out, n, nsplit, 0);
  else
    hipLaunchKernelGGL((splitk_reduce_kernel<bf16>), dim3(grid), dim3(256), 0, s, slabs, (bf16*)out, n, nsplit, 0);
  return (int)hipGetLastError();
}

static inline int bdaln_vpt(int cols) {
  if (cols % 8) return 0;
  const int nvec = cols / 8;
  if (nvec <= 64) return 1;
  if (nvec <= 128) return 2;
  if (nvec <= 256) return 4;
  return 0;
}

int bdaln_supported(int cols) { return bdaln_vpt(cols) > 0; }

// 2056..4096 columns: forward with 5..8 vectors per lane, backward through bdaln_bwd_wide_kernel
static inline int bdaln_wide_vpt(int cols) {
  if (cols % 8) return 0;
  const int nvec = cols / 8;
  return (nvec > 256 && nvec <= 512) ? (nvec + 63) / 64 : 0;
}
int bdaln_wide_supported(int cols) { return bdaln_wide_vpt(cols) > 0; }

#define EW_VPT_WIDE(V, VPT, ...)                            \
  switch (V) {                                              \
    case 5: { constexpr int VPT = 5; __VA_ARGS__; } break;  \
    case 6: { constexpr int VPT = 6; __VA_ARGS__; } break;  \
    case 7: { constexpr int VPT = 7; __VA_ARGS__; } break;  \
    case 8: { constexpr int VPT = 8; __VA_ARGS__; } break;  \
    default: return -2;                                     \
  }

#define EW_VPT(V, VPT, ...)                                 \
  switch (V) {                                              \
    case 1: { constexpr int VPT = 1; __VA_ARGS__; } break;  \
    case 2: { constexpr int VPT = 2; __VA_ARGS__; } break;  \
    case 4: { constexpr int VPT = 4; __VA_ARGS__; } break;  \
    default: return -2;                                     \
  }

int bdaln_fwd(const void* x, const void* b, const void* res, const void* gamma, const void* beta, void* y,
              void* s_out, float* mean, float* rstd, int64_t rows, int cols, float eps, uint64_t seed,
              uint64_t offset, uint32_t thresh, float scale, int xdt, int wdt, hipStream_t s, Q8Out q8,
              int s_cond) {
  if (rows == 0) return 0;
  const int vpt = bdaln_vpt(cols);
  const dim3 grid((unsigned)((rows + 3) / 4));
  if (!vpt) {
    const int wv = bdaln_wide_vpt(cols);
    EW_DISPATCH(xdt, T, EW_DISPATCH(wdt, W, EW_VPT_WIDE(wv, VPT, {
      if (thresh)
        hipLaunchKernelGGL((bdaln_fwd_kernel<T, W, VPT, true>), grid, dim3(kEwBlock), 0, s, (const T*)x,
                           (const W*)b, (const T*)res, (const W*)gamma, (const W*)beta, (T*)y, (T*)s_out,
                           mean, rstd, rows, cols, eps, seed, offset, thresh, scale, q8, s_cond);
      else
        hipLaunchKernelGGL((bdaln_fwd_kernel<T, W, VPT, false>), grid, dim3(kEwBlock), 0, s, (const T*)x,
                           (const W*)b, (const T*)res, (const W*)gamma, (const W*)beta, (T*)y, (T*)s_out,
                           mean, rstd, rows, cols, eps, seed, offset, thresh, scale, q8, s_cond);
    })));
    return (int)hipGetLastError();
  }
  EW_DISPATCH(xdt, T, EW_DISPATCH(wdt, W, EW_VPT(vpt, VPT, {
    if (thresh)
      hipLaunchKernelGGL((bdaln_fwd_kernel<T, W, VPT, true>), grid, dim3(kEwBlock), 0, s, (const T*)x,
                         (const W*)b, (const T*)res, (const W*)gamma, (const W*)beta, (T*)y, (T*)s_out,
                         mean, rstd, rows, cols, eps, seed, offset, thresh, scale, q8, s_cond);
    else
      hipLaunchKernelGGL((bdaln_fwd_kernel<T, W, VPT, false>), grid, dim3(kEwBlock), 0, s, (const T*)x,
                         (const W*)b, (const T*)res, (const W*)gamma, (const W*)beta, (T*)y, (T*)s_out,
                         mean, rstd, rows, cols, eps, seed, offset, thresh, scale, q8, s_cond);
  })));
  return (int)hipGetLastError();
}

// 768 blocks = 3 per CU (the 48 KB combine buffer at cols 1024 allows 3): 12 waves per CU, each
// with two rows of loads in flight
constexpr int kBdalnMaxParts = 768;
static inline int bdaln_rpw(int64_t rows) {
  const int64_t r = (rows + 4 * kBdalnMaxParts - 1) / (4 * kBdalnMaxParts);
  return r < 1 ? 1 : (int)r;
}

int64_t bdaln_ws_floats(int64_t rows, int cols) {
  (void)rows;
  return (int64_t)kBdalnMaxParts * 3 * (int64_t)cols;
}

int bdaln_bwd(const void* dy, const void* s_in, const void* gamma, const void* beta, const float* mean,
              const float* rstd, const void* dse, void* dres, void* dx, void* dgamma, void* dbeta, void* dbias,
              float* ws, int64_t rows, int cols, uint64_t seed, uint64_t offset, uint32_t thresh, float scale,
              int xdt, int wdt, hipStream_t s, Q8Out q8, const void* s_alt) {
  if (rows == 0) return 0;
  const int vpt = bdaln_vpt(cols);
  const int rpw = bdaln_rpw(rows);
  const int parts = (int)((rows + 4 * rpw - 1) / (4 * rpw));
  if (beta && (!vpt || dse)) return -3;  // FROMY: post-LN (no ds_extra), narrow rows only
  if (q8.y && (!vpt || dse)) return -3;  // fp8 side output: narrow rows, no ds_extra
  if (!vpt) {
    const int wv = bdaln_wide_vpt(cols);
    const size_t wlds = (size_t)4 * cols * sizeof(float);
    EW_DISPATCH(xdt, T, EW_DISPATCH(wdt, W, EW_VPT_WIDE(wv, VPT, {
      auto launch = [&](auto drop_tag, auto extra_tag) {
        hipLaunchKernelGGL((bdaln_bwd_wide_kernel<T, W, VPT, decltype(drop_tag)::value, decltype(extra_tag)::value>),
                           dim3(parts), dim3(kEwBlock), wlds, s, (const T*)dy, (const T*)s_in, (const W*)gamma,
                           mean, rstd, (const T*)dse, (T*)dres, (T*)dx, ws, rows, cols, rpw, seed, offset, thresh,
                           scale);
      };
      if (thresh) {
        if (dse) launch(std::true_type{}, std::true_type{});
        else launch(std::true_type{}, std::false_type{});
      } else {
        if (dse) launch(std::false_type{}, std::true_type{});
        else launch(std::false_type{}, std::false_type{});
      }
      launch_partial_colsum3<W>(ws, parts, 3 * (int64_t)cols, cols, (W*)dgamma, (W*)dbeta, (W*)dbias, s);
    })));
    return (int)hipGetLastError();
  }
  const size_t lds = (size_t)4 * 3 * cols * sizeof(float);
  EW_DISPATCH(xdt, T, EW_DISPATCH(wdt, W, EW_VPT(vpt, VPT, {
    auto launch = [&](auto drop_tag, auto extra_tag) {
      constexpr bool D = decltype(drop_tag)::value, E = decltype(extra_tag)::value;
      if (q8.y && !E)
        hipLaunchKernelGGL((bdaln_bwd_kernel<T, W, VPT, D, false, false, true>), dim3(parts), dim3(kEwBlock), lds, s,
                           (const T*)dy, (const T*)s_in, (const W*)gamma, (const W*)nullptr, mean, rstd,
                           (const T*)dse, (T*)dres, (T*)dx, ws, rows, cols, rpw, seed, offset, thresh, scale, q8, (const T*)nullptr);
      else
        hipLaunchKernelGGL((bdaln_bwd_kernel<T, W, VPT, D, E>), dim3(parts), dim3(kEwBlock), lds, s, (const T*)dy,
                           (const T*)s_in, (const W*)gamma, (const W*)nullptr, mean, rstd, (const T*)dse, (T*)dres,
                           (T*)dx, ws, rows, cols, rpw, seed, offset, thresh, scale, q8, (const T*)nullptr);
    };
    if (beta) {
      auto launch_y = [&](auto drop_tag) {
        constexpr bool D = decltype(drop_tag)::value;
        if (q8.y)
          hipLaunchKernelGGL((bdaln_bwd_kernel<T, W, VPT, D, false, true, true>), dim3(parts), dim3(kEwBlock), lds,
                             s, (const T*)dy, (const T*)s_in, (const W*)gamma, (const W*)beta, mean, rstd,
                             (const T*)nullptr, (T*)dres, (T*)dx, ws, rows, cols, rpw, seed, offset, thresh, scale,
                             q8, (const T*)s_alt);
        else
          hipLaunchKernelGGL((bdaln_bwd_kernel<T, W, VPT, D, false, true>), dim3(parts), dim3(kEwBlock), lds, s,
                             (const T*)dy, (const T*)s_in, (const W*)gamma, (const W*)beta, mean, rstd,
                             (const T*)nullptr, (T*)dres, (T*)dx, ws, rows, cols, rpw, seed, offset, thresh, scale,
                             q8, (const T*)s_alt);
      };
      if (thresh) launch_y(std::true_type{});
      else launch_y(std::false_type{});
    } else if (thresh) {
      if (dse) launch(std::true_type{}, std::true_type{});
      else launch(std::true_type{}, std::false_type{});
    } else {
      if (dse) launch(std::false_type{}, std::true_type{});
      else launch(std::false_type{}, std::false_type{});
    }
    const int64_t ld = 3 * (int64_t)cols;
    launch_partial_colsum3<W>(ws, parts, ld, cols, (W*)dgamma, (W*)dbeta, (W*)dbias, s);
  })));
  return (int)hipGetLastError();
}

int embed_ln_fwd(const int* ids, const int* tids, const void* Ww, const void* Wp, const void* Wt, const void* gamma,
                 const void* beta, void* y, void* s_out, float* mean, float* rstd, int64_t rows, int cols, int S,
                 float eps, uint64_t seed, uint64_t offset, uint32_t thresh, float scale, int xdt, int wdt,
                 hipStream_t s) {
  if (rows == 0) return 0;
  const int vpt = bdaln_vpt(cols);
  const dim3 grid((unsigned)((rows + 3) / 4));
  EW_DISPATCH(xdt, T, EW_DISPATCH(wdt, W, EW_VPT(vpt, VPT, {
    if (thresh)
      hipLaunchKernelGGL((embed_ln_fwd_kernel<T, W, VPT, true>), grid, dim3(kEwBlock), 0, s, ids, tids, (const T*)Ww,
                         (const T*)Wp, (const T*)Wt, (const W*)gamma, (const W*)beta, (T*)y, (T*)s_out, mean, rstd,
                         rows, cols, S, eps, seed, offset, thresh, scale);
    else
      hipLaunchKernelGGL((embed_ln_fwd_kernel<T, W, VPT, false>), grid, dim3(kEwBlock), 0, s, ids, tids, (const T*)Ww,
                         (const T*)Wp, (const T*)Wt, (const W*)gamma, (const W*)beta, (T*)y, (T*)s_out, mean, rstd,
                         rows, cols, S, eps, seed, offset, thresh, scale);
  })));
  return (int)hipGetLastError();
}

int embed_nwt(int64_t B) { return B >= 16 ? 16 : (int)((B + 3) / 4 * 4); }

int embed_ln_bwd(const void* dy, const void* s_in, const void* gamma, const float* mean, const float* rstd,
                 const int* tids, int tvocab, void* ds_out, float* part_pos, float* part_tg, void* dWp, void* dWt,
                 void* dgamma, void* dbeta, int64_t B, int cols, int S, uint64_t seed, uint64_t offset,
                 uint32_t thresh, float scale, int xdt, int wdt, hipStream_t s) {
  if (B == 0) return 0;
  if (tvocab < 1 || tvocab > 2) return -3;
  const int vpt = bdaln_vpt(cols);
  const int nwt = embed_nwt(B);
  const dim3 grid((unsigned)S, (unsigned)(nwt / 4));
  EW_DISPATCH(xdt, T, EW_DISPATCH(wdt, W, EW_VPT(vpt, VPT, {
    if (thresh)
      hipLaunchKernelGGL((embed_ln_bwd_kernel<T, W, VPT, true>), grid, dim3(kEwBlock), 0, s, (const T*)dy,
                         (const T*)s_in, (const W*)gamma, mean, rstd, tids, (T*)ds_out, part_pos, part_tg, B, cols, S,
                         nwt, seed, offset, thresh, scale);
    else
      hipLaunchKernelGGL((embed_ln_bwd_kernel<T, W, VPT, false>), grid, dim3(kEwBlock), 0, s, (const T*)dy,
                         (const T*)s_in, (const W*)gamma, mean, rstd, tids, (T*)ds_out, part_pos, part_tg, B, cols, S,
                         nwt, seed, offset, thresh, scale);
    // position rows: sum over the nwt wave partials; gamma / beta and the two type rows over S * nwt
    launch_partial_colsum3<T>(part_pos, nwt, (int64_t)S * cols, S * cols, (T*)dWp, (T*)nullptr, (T*)nullptr, s);
    launch_partial_colsum3<W>(part_tg, S * nwt, 4 * (int64_t)cols, cols, (W*)dgamma, (W*)dbeta, (W*)nullptr, s);
    launch_partial_colsum3<T>(part_tg + 2 * cols, S * nwt, 4 * (int64_t)cols, tvocab * cols, (T*)dWt, (T*)nullptr,
                              (T*)nullptr, s);
  })));
  return (int)hipGetLastError();
}

int embed_segsum(const void* ds, const int* sorted, const int64_t* perm, void* dW, int64_t R, int cols, int xdt,
                 hipStream_t s) {
  if (R == 0) return 0;
  const int vpt = bdaln_vpt(cols);
  const dim3 grid((unsigned)((R + 3) / 4));
  EW_DISPATCH(xdt, T, EW_VPT(vpt, VPT,
      hipLaunchKernelGGL((embed_segsum_kernel<T, VPT>), grid, dim3(kEwBlock), 0, s, (const T*)ds, sorted, perm, (T*)dW,
                         R, cols)));
  return (int)hipGetLastError();
}

}  // namespace apex
