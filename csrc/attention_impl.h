// Flash attention forward + backward on CDNA4 MFMA (NS-05; apex.contrib.multihead_attn core).
//
// Layout: q/k/v/o are [B, S, H, D] views with arbitrary batch / seq strides (so the packed
// QKV projection output [B, S, 3, H, D] is consumed in place, no split/transposes).
// D in {32, 64, 128, 256} (other head dims are zero-padded to the next one by the caller);
// bf16 / fp16 in, fp32 accumulate; optional causal mask, per-batch key lengths, an additive
// score bias (BIAS: [B|1, H|1, Sq|1, Sk] in the input dtype — attention masks as -inf, ALiBi /
// relative-position biases) and Philox dropout regenerated identically in backward.
//
// This header holds the kernel templates; attention_d{32,64,128,256}.hip instantiate one head
// dim each (parallel compilation), attention.hip dispatches.
//
// Forward (one workgroup = 4 wave64 = 128 query rows, 32 per wave; K/V streamed in 64-key
// tiles through LDS):
//   S^T = K . Q^T with v_mfma_f32_32x32x16 — the swapped product puts ONE query per lane
//   (16 keys in registers, the other 16 in lane^32), so row max / row sum need a single
//   cross-half exchange and the rescale factor is lane-local;
//   O^T += V^T . P^T reuses the S^T accumulator registers directly as the B operand
//   (k-order permuted to match, no LDS round trip for P); the V^T operand comes from the
//   row-major V tile with ds_read_b64_tr_b16 (hardware transpose read).
// Backward (one workgroup = 4 waves x 32 keys = 128 keys; loop over 32-query blocks):
//   S = Q.K^T and dP = dO.V^T with K, V rows held in registers; dV += P^T.dO and
//   dK += dS^T.Q use the accumulators as A operands with tr-read B operands from the
//   Q/dO tiles in LDS; dQ = dS.K goes through LDS (dS) and, when several workgroups
//   share a query block (Sk > 128), fp32 atomics.
#pragma once
#include "common.h"
#include "fp8_pack.h"
#include "kernels.h"

#include <cstdlib>
#include <type_traits>

namespace apex {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <typename T> struct MfmaT;
template <> struct MfmaT<bf16> {
  using V8 = bf16x8;
  __device__ static __forceinline__ f32x16 mma(V8 a, V8 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
  }
};
template <> struct MfmaT<f16> {
  using V8 = f16x8;
  __device__ static __forceinline__ f32x16 mma(V8 a, V8 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
  }
};

// 16x16x32 products (the backward's dQ tiles): lane l holds C[4 (l >> 4) + i][l & 15]
template <typename T> struct Mfma16T;
template <> struct Mfma16T<bf16> {
  __device__ static __forceinline__ f32x4 mma(bf16x8 a, bf16x8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
  }
};
template <> struct Mfma16T<f16> {
  __device__ static __forceinline__ f32x4 mma(f16x8 a, f16x8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
  }
};

constexpr float kLog2e = 1.4426950408889634f;
constexpr float kLn2 = 0.6931471805599453f;

// transposed LDS read: 4 rows x 16 cols block, lane i of each 16-lane group gets column i
__device__ __forceinline__ s16x4 lds_tr16(const void* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) s16x4*)(p));
}

// LDS row strides (elements) of the 16-bit tiles, by how a tile is read. Bank model of
// MI355X_MICROARCH.md (LDS table): 16-byte row reads (ds_read_b128) are conflict-free at D + 8;
// transposed reads (ds_read_b64_tr_b16: 4 rows x 64 B per 32-lane group) need the rows 64 B apart
// modulo 256 B, i.e. D + 32; a tile read both ways is best at D + 8 (D = 64) / D + 24 (D >= 128),
// 2-way on the transposed reads. The uniform D + 8 made V's transposed reads 2-way (D = 64) and
// 4-way (D >= 128) conflicted: 22-48 % of all LDS cycles by rocprofv3 (profiles/r2_pmc_attn.json).
// (An XOR chunk swizzle makes the both-ways case conflict-free too, but its per-access address
// arithmetic cost registers — spills at D = 128 — in these VALU-bound loops.)
template <int D> constexpr int ld_rows() { return D + 8; }
template <int D> constexpr int ld_tr() { return D == 32 ? D : D + 32; }
template <int D> constexpr int ld_both() { return D >= 128 ? D + 24 : D + 8; }

// Workgroup barrier ordering LDS traffic only: the fences are restricted to the "local"
// address space, so outstanding global loads (register prefetches) are NOT drained at the
// barrier the way __syncthreads()'s full workgroup fence drains them.
__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// Cross-lane exchanges without an LDS round trip (__shfl_xor lowers to ds_bpermute + a wait):
// the lane ^ 32 partner through gfx950's v_permlane32_swap, and sums over aligned groups of
// 4 / 8 / 16 lanes through DPP (quad_perm, row_half_mirror, row_mirror).
__device__ __forceinline__ uint32_t xor32_u(uint32_t v) {
  const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
  return (__lane_id() & 32) ? r[0] : r[1];
}
__device__ __forceinline__ float xor32_f(float v) { return __uint_as_float(xor32_u(__float_as_uint(v))); }
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
template <int N>  // every lane of each aligned N-lane group ends with the group's sum
__device__ __forceinline__ float group_sum(float v) {
  static_assert(N == 1 || N == 2 || N == 4 || N == 8 || N == 16 || N == 32, "group size");
  if constexpr (N >= 2) v += dpp_f<0xB1>(v);   // quad_perm [1,0,3,2]: lane ^ 1
  if constexpr (N >= 4) v += dpp_f<0x4E>(v);   // quad_perm [2,3,0,1]: lane ^ 2
  if constexpr (N >= 8) v += dpp_f<0x141>(v);  // row_half_mirror: the other quad of the 8
  if constexpr (N >= 16) v += dpp_f<0x140>(v); // row_mirror: the other 8 of the row
  if constexpr (N >= 32) v += __shfl_xor(v, 16, 64);
  return v;
}

template <typename V8>
__device__ __forceinline__ V8 join4(s16x4 lo, s16x4 hi) {
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  s16x8 r = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(V8, r);
}

template <typename T, typename V8>
__device__ __forceinline__ V8 pack8(const float* x) {
  typedef T t8 __attribute__((ext_vector_type(8)));
  t8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = (T)x[j];
  return __builtin_bit_cast(V8, r);
}

// Attention dropout keep bits: 8-bit uniforms (keep iff u8 >= thresh), 16 per (row, 16-key half of a
// 32-key block). Each (row, half) is one stream: ONE Philox4x32-7 call (counter offset + hl,
// subsequence bh * Sq + row) seeds a xorshift128 state, and every 32-key block then takes the
// stream's next four 32-bit words, in block order. Round 3 drew one Philox call per block and half:
// its 14 64-bit integer multiplies (quarter-rate v_mad_u64_u32) per call were ~30 % of the BERT-shape
// forward (fwd 72.7 us with p = 0.1 vs 56.1 at p = 0, b256 s128, tools/attn_bench.py); a xorshift128
// step is six full-rate shift/xor ops. Dropout masks need uniform, uncorrelated bytes, not
// cryptographic strength; the Philox seeding keeps streams of different rows / heads / launches
// independent, and tests/test_attention_gpu.py checks the keep rate and the mask's decorrelation.
// The four words are compared against the threshold four bytes at a time (SWAR: the carry out of
// u + (256 - thresh) in each byte is the keep bit — u & 0x7f.. plus the low 7 bits of the addend,
// then the majority of the three top bits), and the carries are shifted into the natural bit order:
// the returned 16 bits land at positions 4 hl + {0..3, 8..11, 16..19, 24..27}, i.e. bit k of the OR
// of both halves is key k of the block (random word j = k & 3 of half hl = (k >> 2) & 1, byte k >> 3).
struct DropStream {
  uint32_t x, y, z, w, thresh;
  __device__ __forceinline__ DropStream(uint64_t seed, uint64_t offset, uint32_t thr, int64_t bh, int64_t row,
                                        int hl, int64_t Sq) {
    Philox ph(seed, (uint64_t)(bh * Sq + row), offset + (uint64_t)hl);
    const uint4 r = ph.next();
    x = r.x;
    y = r.y;
    z = r.z;
    w = r.w | (uint32_t)((r.x | r.y | r.z | r.w) == 0u);  // xorshift128's state must not be all zero
    thresh = thr;
  }
  __device__ __forceinline__ uint32_t next() {
    const uint32_t t = x ^ (x << 11);
    x = y;
    y = z;
    z = w;
    w = w ^ (w >> 19) ^ t ^ (t >> 8);
    return w;
  }
  // the next block's 16 keep bits of this half (bits 4 hl + {0-3, 8-11, 16-19, 24-27})
  __device__ __forceinline__ uint32_t half_bits(int hl) {
    const uint32_t C = (256u - thresh) * 0x01010101u;
    const uint32_t C7 = C & 0x7f7f7f7fu;
    uint32_t out = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t u = next();
      const uint32_t s7 = (u & 0x7f7f7f7fu) + C7;
      const uint32_t carry = ((u & C) | ((u | C) & s7)) & 0x80808080u;  // bit 8b+7: keep of byte b
      out |= carry >> (7 - j);                                           // -> bit 8b + j
    }
    return out << (4 * hl);
  }
  // half_bits plus the same decisions as byte masks for the P operand: byte b of bm[j] is 0xFF
  // iff element 4 b + j of the lane's 16 (key j + 8 b + 4 hl of the block) is kept. The forward
  // ANDs them into the packed bf16 P words (drop_pack): one v_perm + one v_and per pair of
  // probabilities instead of a bit test, compare and select per element on the fp32 values (which
  // also split the v_cvt_pk pairs: BERT-shape forward, 19 VALU instructions per score).
  __device__ __forceinline__ uint32_t half_masks(int hl, uint32_t (&bm)[4]) {
    const uint32_t C = (256u - thresh) * 0x01010101u;
    const uint32_t C7 = C & 0x7f7f7f7fu;
    uint32_t out = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t u = next();
      const uint32_t s7 = (u & 0x7f7f7f7fu) + C7;
      const uint32_t carry = ((u & C) | ((u | C) & s7)) & 0x80808080u;
      out |= carry >> (7 - j);
      bm[j] = carry | (carry - (carry >> 7));  // 0x80 -> 0xFF per kept byte (no borrow across bytes)
    }
    return out << (4 * hl);
  }
};

// Dropout on 8 packed 16-bit probabilities (elements 8 s2 .. 8 s2 + 7 of a lane's 16, word w =
// elements 2w, 2w + 1): word w &= the byte masks of its two elements, gathered by v_perm_b32
// (bytes 0-1 <- byte b of bm[j], bytes 2-3 <- byte b of bm[j + 1], b = (8 s2 + 2w) >> 2)
template <typename V8>
__device__ __forceinline__ V8 drop_pack(V8 pf, const uint32_t (&bm)[4], int s2) {
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  u32x4 w = __builtin_bit_cast(u32x4, pf);
#pragma unroll
  for (int ww = 0; ww < 4; ++ww) {
    const uint32_t b = 2 * s2 + (ww >> 1), j = 2 * (ww & 1);
    const uint32_t sel = b | (b << 8) | ((4 + b) << 16) | ((4 + b) << 24);
    w[ww] &= __builtin_amdgcn_perm(bm[j + 1], bm[j], sel);
  }
  return __builtin_bit_cast(V8, w);
}

// keep bits of block `blk` (bit k <-> key 32 blk + k) for one row, both halves (debug / test kernel)
__device__ __forceinline__ uint32_t drop_block_bits(uint64_t seed, uint64_t offset, uint32_t thresh, int64_t bh,
                                                    int64_t row, int64_t blk, int64_t Sq) {
  uint32_t out = 0;
  for (int hl = 0; hl < 2; ++hl) {
    DropStream st(seed, offset, thresh, bh, row, hl, Sq);
    uint32_t hb = 0;
    for (int64_t b = 0; b <= blk; ++b) hb = st.half_bits(hl);
    out |= hb;
  }
  return out;
}

// Additive score bias for this lane's query row and 4 consecutive keys key .. key+3 (8-byte load
// when all four are inside the row; keys >= Sk read 0 — they are masked anyway).
template <typename T>
__device__ __forceinline__ void bias4(const T* brow, int key, int Sk, float (&v)[4]) {
  if (key + 3 < Sk) {
    Pack<T, 4> pk = *reinterpret_cast<const Pack<T, 4>*>(brow + key);
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = to_f(pk.v[e]);
  } else {
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = key + e < Sk ? to_f(brow[key + e]) : 0.f;
  }
}

template <typename T>
__device__ __forceinline__ const T* bias_row(const AttnArgs& a, int b, int h, int q) {
  return (const T*)a.bias + b * a.bias_bs + h * a.bias_hs + (int64_t)min(q, a.Sq - 1) * a.bias_qs;
}

constexpr int kFwdWaves = 4;
constexpr int kFwdBQ = 32 * kFwdWaves;  // 128 query rows per workgroup
constexpr int kFwdKB = 64;              // keys per tile

// SHORT (D = 64, Sk <= 128, no dropout: BERT-shape inference): the whole key range is staged into LDS once (36 KB)
// and no register copy of K/V is live during the math, which brings the kernel to 128 VGPRs:
// 4 workgroups (16 waves, 144 KB of LDS) per CU instead of 2 for a kernel that is one
// load -> math -> store pass per workgroup, so the other workgroups' loads hide the HBM latency.
// DB (long key ranges): K/V tiles double-buffered in LDS with ONE barrier per tile — tile kt + 1
// (in registers since the middle of tile kt - 1) is written to the other buffer in the middle of
// tile kt's math, right after the S products, and tile kt + 2's global loads are issued then
// (cdna_hip_programming.md T14 "async-STAGE split"); the single-buffer loop pays two barriers per
// tile (previous tile consumed / this tile staged).
template <typename T, int D, bool CAUSAL, bool DROPOUT, bool SHORT, bool BIAS, bool DB = false, bool W4 = false>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(SHORT ? (DROPOUT ? (W4 ? 4 : 3) : 4) : (D > 128 ? 1 : (DB && D <= 64 && !DROPOUT ? 3 : 2)))))
attn_fwd_kernel(AttnArgs a) {
  static_assert(!SHORT || D == 64, "SHORT is the D = 64 single-pass variant");
  static_assert(!(SHORT && DB), "SHORT stages the whole key range once");
  using M = MfmaT<T>;
  using V8 = typename M::V8;
  constexpr int LDR = ld_rows<D>();  // K: row reads
  // V: transposed reads (SHORT keeps D + 8: the wider stride would take its two-tile LDS image to
  // 43 KB and the variant from 4 to 3 workgroups per CU)
  constexpr int LDV = SHORT ? ld_rows<D>() : ld_tr<D>();
  constexpr int NBUF = SHORT || DB ? 2 : 1;
  __shared__ __attribute__((aligned(16))) T lds_k[NBUF * kFwdKB * LDR];
  __shared__ __attribute__((aligned(16))) T lds_v[NBUF * kFwdKB * LDV];

  // wid through readfirstlane: wave-uniform in SGPRs, so tile-level conditions become scalar branches
  const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int r = lane & 31, hl = lane >> 5;
  const int bh = blockIdx.x;  // grid (B*H, query blocks): see attn_fwd_impl
  const int b = bh / a.H, h = bh % a.H;
  const int q0 = (CAUSAL ? gridDim.y - 1 - blockIdx.y : blockIdx.y) * kFwdBQ;
  const int qrow = q0 + 32 * wid + r;
  const int Sk = a.k_lens ? min(a.k_lens[b], a.Sk) : a.Sk;
  // BIAS: scores are taken to the natural domain s' = s * scale + bias, so the exp2 factor is log2(e)
  const float sl2 = BIAS ? kLog2e : a.scale_log2;

  const T* qp = (const T*)a.q + b * a.q_bs + h * a.q_hs;
  const T* kp = (const T*)a.k + b * a.k_bs + h * a.k_hs;
  const T* vp = (const T*)a.v + b * a.v_bs + h * a.v_hs;
  const T* brow = BIAS ? bias_row<T>(a, b, h, qrow) : nullptr;
  // fp8 codes of O: scale and the amax filter value read here, their latency under the main loop
  const float q8s = a.q8o ? a.q8_scale[0] : 0.f, q8seen = a.q8o ? f8_amax_seen(a.q8_amax) : 0.f;

  // Q^T fragments (B operand): lane (q=r, hl) holds Q[q][16s + 8hl .. +7]
  V8 qf[D / 16];
#pragma unroll
  for (int s = 0; s < D / 16; ++s) {
    if (qrow < a.Sq) qf[s] = *(const V8*)(qp + (int64_t)qrow * a.q_ss + 16 * s + 8 * hl);
    else qf[s] = V8{};
  }

  f32x16 o[D / 32];
#pragma unroll
  for (int i = 0; i < D / 32; ++i) o[i] = f32x16{};
  float m = -INFINITY, l = 0.f;

  int kend = Sk;
  if (CAUSAL) kend = min(kend, q0 + kFwdBQ);
  const int ntiles = (kend + kFwdKB - 1) / kFwdKB;

  // tile loader: 64 x D elements, 16B chunks, CH chunks per thread
  constexpr int CPR = D / 8;               // chunks per row
  constexpr int CH = kFwdKB * CPR / 256;   // chunks per thread per tensor
  // K/V tiles of the tile TWO ahead are loaded into registers while the current tile computes
  // (two register sets, loop unrolled by two) at D <= 64; one ahead at D >= 128 (register budget)
  constexpr bool KV2 = D <= 64 && !DB;
  constexpr int AHEAD = KV2 ? 2 : 1;
  struct KV {
    uint4 k[CH], v[CH];
  };
  KV kva, kvb;
  // dropout: each lane draws the keep bits of its own 16 keys of every 32-key block in the
  // loop, in block order, from its (row, half) stream (DropStream::half_bits), and the two lane
  // halves' words are combined and stored for the backward kernels
  uint32_t* mrow =
      DROPOUT && qrow < a.Sq ? (uint32_t*)(a.dmask + ((int64_t)bh * a.Sq + qrow) * a.mask_words) : nullptr;
  DropStream dg(a.seed, a.offset, DROPOUT ? a.drop_thresh : 0u, bh, qrow, hl, a.Sq);
  auto gload = [&](KV& R, int kt) {
    uint4 (&kreg)[CH] = R.k;
    uint4 (&vreg)[CH] = R.v;
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const int idx = threadIdx.x + 256 * c;
      const int row = idx / CPR, col = (idx % CPR) * 8;
      const int key = kt * kFwdKB + row;
      if (key < Sk) {
        kreg[c] = *(const uint4*)(kp + (int64_t)key * a.k_ss + col);
        vreg[c] = *(const uint4*)(vp + (int64_t)key * a.v_ss + col);
      } else {
        kreg[c] = make_uint4(0, 0, 0, 0);
        vreg[c] = make_uint4(0, 0, 0, 0);
      }
    }
  };
  auto lstore = [&](KV& R, const int rowoff) {
    uint4 (&kreg)[CH] = R.k;
    uint4 (&vreg)[CH] = R.v;
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const int idx = threadIdx.x + 256 * c;
      const int row = rowoff + idx / CPR, col = (idx % CPR) * 8;
      *(uint4*)(lds_k + row * LDR + col) = kreg[c];
      *(uint4*)(lds_v + row * LDV + col) = vreg[c];
    }
  };

  if (ntiles > 0) gload(kva, 0);
  if (KV2 && ntiles > 1) gload(kvb, 1);
  // math of key tile kt, read from LDS rows lr0 ..; mid() runs right after the S products (DB)
  auto compute = [&](const int kt, auto&& mid) {
    const int lr0 = SHORT ? kt * kFwdKB : DB ? (kt & 1) * kFwdKB : 0;
    uint32_t bm[2][4];
    if (DROPOUT) {
#pragma unroll
      for (int sb = 0; sb < 2; ++sb) {
        const int blk = (kt * kFwdKB >> 5) + sb;
        const uint32_t hb = dg.half_masks(hl, bm[sb]);  // block blk's bits at 4 hl + {0-3, 8-11, ..}
        const uint32_t word = hb | xor32_u(hb);
        if (hl == 0 && mrow && blk * 32 < a.Sk) mrow[blk] = word;
      }
    }
    const int kb = kt * kFwdKB;

    // ---- S^T for two 32-key sub-blocks
    // all K fragments of the tile are read before the MFMA chain (one LDS latency per tile
    // instead of one per MFMA); D = 256 reads one sub-block at a time (register budget)
    f32x16 st[2];
    if constexpr (D <= 128) {
      V8 kf[2][D / 16];
#pragma unroll
      for (int sb = 0; sb < 2; ++sb)
#pragma unroll
        for (int s = 0; s < D / 16; ++s) kf[sb][s] = *(const V8*)(lds_k + (lr0 + 32 * sb + r) * LDR + 16 * s + 8 * hl);
      __builtin_amdgcn_sched_group_barrier(0x100, 2 * (D / 16), 0);  // DS reads first
      __builtin_amdgcn_sched_group_barrier(0x008, 2 * (D / 16), 0);  // then the MFMAs
#pragma unroll
      for (int sb = 0; sb < 2; ++sb) {
        st[sb] = f32x16{};
#pragma unroll
        for (int s = 0; s < D / 16; ++s) st[sb] = M::mma(kf[sb][s], qf[s], st[sb]);
      }
    } else {
#pragma unroll
      for (int sb = 0; sb < 2; ++sb) {
        st[sb] = f32x16{};
#pragma unroll
        for (int s = 0; s < D / 16; ++s)
          st[sb] = M::mma(*(const V8*)(lds_k + (lr0 + 32 * sb + r) * LDR + 16 * s + 8 * hl), qf[s], st[sb]);
      }
    }
    mid();
    if constexpr (BIAS) {
      // element i of sub-block sb <-> key kb + 32 sb + (i & 3) + 8 (i >> 2) + 4 hl
#pragma unroll
      for (int sb = 0; sb < 2; ++sb)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          float bv[4];
          bias4<T>(brow, kb + 32 * sb + 8 * g + 4 * hl, a.Sk, bv);
#pragma unroll
          for (int e = 0; e < 4; ++e) st[sb][4 * g + e] = fmaf(st[sb][4 * g + e], a.scale, bv[e]);
        }
    }
    // D = 64: the V^T fragments of the PV product are read now, their LDS latency hidden
    // behind the softmax (D = 128 would not fit in the register budget of 2 workgroups/CU)
    constexpr bool HOIST_V = D == 64;
    V8 vt[2][2][HOIST_V ? D / 32 : 1];
    if constexpr (HOIST_V) {
#pragma unroll
      for (int sb = 0; sb < 2; ++sb)
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
          for (int db = 0; db < D / 32; ++db) {
            const int k0 = lr0 + 32 * sb + 16 * s2 + 4 * hl + ((lane & 15) >> 2);
            const int c0 = 32 * db + 16 * ((lane >> 4) & 1) + 4 * (lane & 3);
            vt[sb][s2][db] = join4<V8>(lds_tr16(lds_v + k0 * LDV + c0), lds_tr16(lds_v + (k0 + 8) * LDV + c0));
          }
    }
    // ---- mask (boundary tiles only) + running max on the RAW scores; the softmax scale is
    // folded into the exp2 argument (one FMA per element) and exp2 is the bare v_exp_f32
    // (no denormal range reduction: underflow to 0 is what softmax wants).
    const bool interior = (kb + kFwdKB <= Sk) && (!CAUSAL || kb + kFwdKB - 1 <= q0 + 32 * wid);
    if (!interior) {
      // keys valid for this lane's query: key < lim (one compare + select per element)
      const int lim = CAUSAL ? min(Sk, qrow + 1) : Sk;
#pragma unroll
      for (int sb = 0; sb < 2; ++sb) {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int key = kb + 32 * sb + (i & 3) + 8 * (i >> 2) + 4 * hl;
          if (key >= lim) st[sb][i] = -INFINITY;
        }
      }
    }
    float tmax = -INFINITY;
#pragma unroll
    for (int sb = 0; sb < 2; ++sb)
#pragma unroll
      for (int i = 0; i < 16; ++i) tmax = fmaxf(tmax, st[sb][i]);
    tmax = fmaxf(tmax, xor32_f(tmax));
    const float mnew = fmaxf(m, tmax);
    const float muse = mnew == -INFINITY ? 0.f : mnew;
    const float alpha = __builtin_amdgcn_exp2f((m - muse) * sl2);
    const float mscaled = -muse * sl2;
    m = mnew;
    float psum = 0.f;
#pragma unroll
    for (int sb = 0; sb < 2; ++sb) {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const float p = __builtin_amdgcn_exp2f(fmaf(st[sb][i], sl2, mscaled));
        psum += p;
        // dropout is applied to the packed P operand below (drop_pack); the 1/(1-p) rescale once
        // in the epilogue
        st[sb][i] = p;
      }
    }
    l = l * alpha + psum;
#pragma unroll
    for (int db = 0; db < D / 32; ++db)
#pragma unroll
      for (int i = 0; i < 16; ++i) o[db][i] *= alpha;
    // ---- O^T += V^T . P^T
#pragma unroll
    for (int sb = 0; sb < 2; ++sb) {
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        float pv[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) pv[j] = st[sb][8 * s2 + j];
        V8 pf = pack8<T, V8>(pv);
        if constexpr (DROPOUT) pf = drop_pack(pf, bm[sb], s2);
        const int k0 = lr0 + 32 * sb + 16 * s2 + 4 * hl + ((lane & 15) >> 2);
#pragma unroll
        for (int db = 0; db < D / 32; ++db) {
          if constexpr (HOIST_V) {
            o[db] = M::mma(vt[sb][s2][db], pf, o[db]);
          } else {
            const int c0 = 32 * db + 16 * ((lane >> 4) & 1) + 4 * (lane & 3);
            const s16x4 lo = lds_tr16(lds_v + k0 * LDV + c0);
            const s16x4 hi = lds_tr16(lds_v + (k0 + 8) * LDV + c0);
            o[db] = M::mma(join4<V8>(lo, hi), pf, o[db]);
          }
        }
      }
    }
  };
  auto nomid = [] {};
  auto tile = [&](KV& R, const int kt) {
    lds_barrier();  // previous tile fully consumed
    lstore(R, 0);
    lds_barrier();
    if (kt + AHEAD < ntiles) gload(R, kt + AHEAD);
    compute(kt, nomid);
  };
  if constexpr (SHORT) {
    // both (<= 2) tiles were loaded above: one LDS stage, then the math with no K/V registers live
    if (ntiles > 0) lstore(kva, 0);
    if (ntiles > 1) lstore(kvb, kFwdKB);
    lds_barrier();
    if (ntiles > 0) compute(0, nomid);
    if (ntiles > 1) compute(1, nomid);
  } else if constexpr (DB) {
    // tile 0 staged, tile 1 in registers; then per tile: barrier, S products, stage tile kt + 1
    // into the other buffer + issue tile kt + 2's loads, softmax, PV
    if (ntiles > 0) lstore(kva, 0);
    if (ntiles > 1) gload(kva, 1);
    for (int kt = 0; kt < ntiles; ++kt) {
      lds_barrier();  // tile kt's buffer complete; the other buffer's last readers (tile kt - 1) done
      compute(kt, [&] {
        if (kt + 1 < ntiles) {
          lstore(kva, ((kt + 1) & 1) * kFwdKB);
          if (kt + 2 < ntiles) gload(kva, kt + 2);
        }
      });
    }
  } else if constexpr (KV2) {
    for (int kt = 0; kt < ntiles; kt += 2) {
      tile(kva, kt);
      if (kt + 1 < ntiles) tile(kvb, kt + 1);
    }
  } else {
    for (int kt = 0; kt < ntiles; ++kt) tile(kva, kt);
  }
  // ---- epilogue
  const float ltot = l + xor32_f(l);
  float q8mx = 0.f;
  const float inv = ltot > 0.f ? (DROPOUT ? a.drop_scale : 1.f) / ltot : 0.f;
  // O rows packed to 16-bit: lane (r, hl) holds columns 32 db + 8 g + 4 hl .. + 3 of row qrow
  typedef T t4 __attribute__((ext_vector_type(4)));
  uint2 wv[D / 32][4];
#pragma unroll
  for (int db = 0; db < D / 32; ++db)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      t4 w;
#pragma unroll
      for (int e = 0; e < 4; ++e) w[e] = (T)(o[db][4 * g + e] * inv);
      wv[db][g] = __builtin_bit_cast(uint2, w);
    }
  // 16-byte row stores (cdna_hip_programming.md T21): for each column-group pair (g, g + 1) one
  // v_permlane32_swap per dword gives the lower half-wave columns 8 g .. 8 g + 7 of its row and the
  // upper half 8 g + 8 .. 8 g + 15 — half the store instructions of the 8-byte row-per-lane-pair
  // stores, same bytes (the store tail of a short-lived workgroup is issue-bound). The swaps run on
  // every lane, ahead of the row-validity branch.
  uint4 wide[D / 32][2];
#pragma unroll
  for (int db = 0; db < D / 32; ++db)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const auto rx = __builtin_amdgcn_permlane32_swap(wv[db][2 * j].x, wv[db][2 * j + 1].x, false, false);
      const auto ry = __builtin_amdgcn_permlane32_swap(wv[db][2 * j].y, wv[db][2 * j + 1].y, false, false);
      wide[db][j] = make_uint4(rx[0], ry[0], rx[1], ry[1]);
    }
  if (qrow < a.Sq) {
    const int64_t ooff = b * a.o_bs + h * a.o_hs + (int64_t)qrow * a.o_ss;
    T* op = (T*)a.o + ooff;
#pragma unroll
    for (int db = 0; db < D / 32; ++db)
#pragma unroll
      for (int j = 0; j < 2; ++j) *(uint4*)(op + 32 * db + 16 * j + 8 * hl) = wide[db][j];
    // Q8 (0: none, 1: e4m3, 2: e5m2) hoisted out of the store loop: fp8 codes of the stored
    // (rounded) values, the attention-out GEMM's operand, from the regrouped words: wide[db][j]
    // holds columns 32 db + 16 j + 8 hl .. + 7, so one more v_permlane32_swap per dword (the upper
    // half-wave's j = 0 codes for the lower half's j = 1 codes) gives the lower half columns
    // 32 db .. + 15 and the upper half 32 db + 16 .. + 31: one 16-byte code store per lane and
    // 32 columns (it was two 8-byte stores; the store tail of these short workgroups is issue-bound)
    auto store_q8 = [&](auto Q8c) {
      constexpr int Q8 = decltype(Q8c)::value;
#pragma unroll
      for (int db = 0; db < D / 32; ++db) {
        uint32_t c[2][2];
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          c[j][0] = f8_codes4<Q8 - 1, T>(wide[db][j].x, wide[db][j].y, q8s, q8mx);
          c[j][1] = f8_codes4<Q8 - 1, T>(wide[db][j].z, wide[db][j].w, q8s, q8mx);
        }
        const auto s0 = __builtin_amdgcn_permlane32_swap(c[0][0], c[1][0], false, false);
        const auto s1 = __builtin_amdgcn_permlane32_swap(c[0][1], c[1][1], false, false);
        *(uint4*)(a.q8o + ooff + 32 * db + 16 * hl) = make_uint4(s0[0], s1[0], s0[1], s1[1]);
      }
    };
    if (a.q8o) {
      if (a.q8_fmt == 0) store_q8(std::integral_constant<int, 1>{});
      else store_q8(std::integral_constant<int, 2>{});
    }
    if (hl == 0 && a.lse)
      a.lse[(int64_t)bh * a.Sq + qrow] = ltot > 0.f ? (m * sl2 + log2f(ltot)) * kLn2 : INFINITY;
  }
  if (a.q8o) f8_block_amax(q8mx, a.q8_amax, q8seen);  // every thread of the block reaches this
}

// ---------------------------------------------------------------------------
// Backward
// ---------------------------------------------------------------------------
constexpr int kBwdWaves = 4;
constexpr int kBwdBK = 32 * kBwdWaves;  // 128 keys per workgroup
constexpr int kBwdBQ = 32;              // queries per inner step

// delta = rowsum(dO * O) per query row, once (attn_bwd_delta_kernel), for the two-kernel backward:
// every dK/dV workgroup of a query block used to recompute it from O (a third 32 x D tile load,
// its unpack and a shuffle reduction per step, Sk / 128 times per row).
template <typename T, int D>
__global__ void __launch_bounds__(256) attn_bwd_delta_kernel(AttnArgs a, const void* dout, float* delta) {
  constexpr int CPR = D / 8;  // 16-byte chunks per row (4..32 lanes, a power of two)
  const int bh = blockIdx.y;
  const int b = bh / a.H, h = bh % a.H;
  const int idx = blockIdx.x * 256 + threadIdx.x;
  const int q = idx / CPR, col = (idx % CPR) * 8;
  float part = 0.f;
  if (q < a.Sq) {
    float ov[8], dov[8];
    load_f<T, 8>((const T*)a.o + b * a.o_bs + h * a.o_hs + (int64_t)q * a.o_ss + col, ov);
    load_f<T, 8>((const T*)dout + b * a.do_bs + h * a.do_hs + (int64_t)q * a.do_ss + col, dov);
#pragma unroll
    for (int e = 0; e < 8; ++e) part += ov[e] * dov[e];
  }
  part = group_sum<CPR>(part);
  if (q < a.Sq && (idx % CPR) == 0) delta[(int64_t)bh * a.Sq + q] = part;
}

// DQ = true (Sk <= 128: the workgroup holds every key, so it is the sole owner of dQ for its
// query rows and writes it directly; delta is computed here from O). DQ = false (longer key
// ranges): dK/dV only, delta read from attn_bwd_delta_kernel's output, and attn_bwd_dq_kernel
// computes dQ from a query-stationary loop (no cross-workgroup fp32 atomics; see the kernel below).
template <typename T, int D, bool CAUSAL, bool DROPOUT, bool DSUM, bool DQ, bool BIAS>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(D <= 64 ? 2 : 1, D <= 64 ? 2 : 1))) attn_bwd_kernel(AttnArgs a, const void* dout, const float* delta_in,
                                                         void* dk_out, void* dv_out) {
  using M = MfmaT<T>;
  using V8 = typename M::V8;
  constexpr int LDR = D + 8;          // dK / dV emit staging in lds_k (row reads)
  constexpr int LDQ = ld_both<D>();  // Q / dO: row and transposed reads
  // dS^T [key][q] (bf16): each lane writes its 16 query values of one key as 4 x ds_write_b64 (4
  // consecutive queries each; row stride 36 elements = 18 dwords: the 16 rows of a lane group land
  // on distinct bank pairs), the dQ product reads it back with ds_read_b64_tr_b16. Round 3 wrote
  // [q][key] with 16 ds_write_b16 per lane and step.
  // D = 64: dS^T unpadded, 8-byte piece c of key row k at c ^ ((k >> 1) & 7): the ds_write_b64 stores
  // and the dQ product's transposed reads both conflict-free (tools/lds_banks.py; 36: reads 2-way)
#ifndef APEX_ATT_DS_SWZ
#define APEX_ATT_DS_SWZ 1
#endif
  constexpr bool DSW = D == 64 && APEX_ATT_DS_SWZ;
  constexpr int LDT = DSW ? kBwdBQ : kBwdBQ + 4;
  auto dso = [](int row, int col) -> int {
    if constexpr (DSW) return row * LDT + (col ^ (((row >> 1) & 7) << 2));
    else return row * LDT + col;
  };
  // K^T row stride (elements); K^T shares lds_k. 144: the dQ product's 16-byte K^T row reads are
  // conflict-free (136: 2-way; tools/lds_banks.py)
  constexpr int KT_LD = kBwdBK + 16;
  constexpr int LDSK = D * KT_LD > kBwdBK * LDR ? D * KT_LD : kBwdBK * LDR;
  __shared__ __attribute__((aligned(16))) T lds_q[kBwdBQ * LDQ];
  __shared__ __attribute__((aligned(16))) T lds_do[kBwdBQ * LDQ];
  __shared__ __attribute__((aligned(16))) T lds_k[LDSK];
  __shared__ __attribute__((aligned(16))) T lds_ds[kBwdBK * LDT];
  __shared__ __attribute__((aligned(16))) float lds_lse[kBwdBQ], lds_delta[kBwdBQ];
  __shared__ __attribute__((aligned(16))) uint32_t lds_mask[4 * kBwdBQ];  // [wave's 32-key block][q]: bit k <-> key 32 wid + k

  // wid through readfirstlane: wave-uniform in SGPRs, so tile-level conditions become scalar branches
  const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int r = lane & 31, hl = lane >> 5;
  const int bh = blockIdx.x;  // grid (B*H, key blocks): key block 0 (the most queries when causal) first
  const int b = bh / a.H, h = bh % a.H;
  const int k0 = blockIdx.y * kBwdBK;
  const int Sk = a.k_lens ? min(a.k_lens[b], a.Sk) : a.Sk;
  const int mykey = k0 + 32 * wid + r;  // key row this lane holds as K/V operand

  const T* qp = (const T*)a.q + b * a.q_bs + h * a.q_hs;
  const T* kp = (const T*)a.k + b * a.k_bs + h * a.k_hs;
  const T* vp = (const T*)a.v + b * a.v_bs + h * a.v_hs;
  const T* dop = (const T*)dout + b * a.do_bs + h * a.do_hs;
  const T* op = (const T*)a.o + b * a.o_bs + h * a.o_hs;
  const float* lsep = a.lse + (int64_t)bh * a.Sq;
  const float* dlp = DQ ? nullptr : delta_in + (int64_t)bh * a.Sq;
  // BIAS: this lane's key column of the bias, bcol[q * bias_qs]
  const T* bcol = BIAS ? (const T*)a.bias + b * a.bias_bs + h * a.bias_hs + min(mykey, a.Sk - 1) : nullptr;

  // accumulators: dK, dV  [key x dim]: C rows = keys (regs), cols = dim (lanes)
  f32x16 dk[D / 32], dv[D / 32];
#pragma unroll
  for (int i = 0; i < D / 32; ++i) {
    dk[i] = f32x16{};
    dv[i] = f32x16{};
  }

  int qstart = 0;
  if (CAUSAL) qstart = (k0 / kBwdBQ) * kBwdBQ;
  const int nq = a.Sq;
  const float rkeep = a.drop_scale;

  // Q / dO / O tiles (32 x D), lse and the dropout words of the query block TWO steps ahead
  // are loaded into registers while the current block computes (two register sets, the loop
  // unrolled by two, so every global load has two steps of compute to land in); the barriers
  // below only wait for LDS traffic so these global loads stay in flight across them.
  constexpr int CPR = D / 8;
  constexpr int NCHK = kBwdBQ * CPR;                // 16-byte chunks per 32-row tile
  constexpr int NLD = NCHK >= 256 ? NCHK / 256 : 1;  // per thread (D = 32: half the threads)
  struct Pf {
    uint4 q[NLD], d[NLD], o[DQ ? NLD : 1];
    float lse, dl;
    uint32_t mask;
  };
  // two register sets where they fit (dK/dV-only kernel at D = 64); one set (prefetch one step
  // ahead) for the fused single-key-block kernel and D = 128, which would spill
  constexpr bool DEPTH2 = !DQ && D <= 64;
  constexpr int AHEAD = DEPTH2 ? 2 : 1;
  Pf pfa, pfb;
  auto fetch = [&](Pf& P, int qb) {
    uint4 (&pf_q)[NLD] = P.q;
    uint4 (&pf_do)[NLD] = P.d;
    float& pf_lse = P.lse;
    uint32_t& pf_mask = P.mask;
    pf_lse = INFINITY;
    pf_mask = 0u;
    // block base pointers are wave-uniform (scalar 64-bit math); the per-lane part is a 32-bit
    // offset (row < 32 rows of one block) that the compiler hoists out of the loop
    const T* qbase = qp + (int64_t)qb * a.q_ss;
    const T* dbase = dop + (int64_t)qb * a.do_ss;
#pragma unroll
    for (int c = 0; c < NLD; ++c) {
      const int idx = threadIdx.x + 256 * c;
      const int row = idx / CPR, col = (idx % CPR) * 8;
      const int q = qb + row;
      if (q < nq && idx < NCHK) {
        pf_q[c] = *(const uint4*)(qbase + (row * (int)a.q_ss + col));
        pf_do[c] = *(const uint4*)(dbase + (row * (int)a.do_ss + col));
        if constexpr (DQ) P.o[c] = *(const uint4*)(op + (int64_t)q * a.o_ss + col);
      } else {
        pf_q[c] = pf_do[c] = make_uint4(0, 0, 0, 0);
        if constexpr (DQ) P.o[c] = make_uint4(0, 0, 0, 0);
      }
    }
    // raw values only: any arithmetic on a loaded value here would make the compiler wait for
    // the whole prefetch (s_waitcnt vmcnt(0)) instead of letting it land during the next step
    if (threadIdx.x < kBwdBQ) {
      const int q = qb + threadIdx.x;
      if (q < nq) pf_lse = lsep[q];  // natural log; x log2(e) at staging
    }
    if (!DQ && threadIdx.x >= 128 && threadIdx.x < 128 + kBwdBQ) {
      const int q = qb + threadIdx.x - 128;
      P.dl = q < nq ? dlp[q] : 0.f;
    }
    if (DROPOUT && threadIdx.x < 4 * kBwdBQ) {
      // dropout words written by the forward: one per (query, 32-key block), bit k <-> key k
      const int qi = threadIdx.x & (kBwdBQ - 1), w = threadIdx.x / kBwdBQ;
      const int q = qb + qi, blk = (k0 >> 5) + w;
      if (q < nq && blk * 32 < a.Sk) pf_mask = ((const uint32_t*)(a.dmask + ((int64_t)bh * a.Sq + q) * a.mask_words))[blk];
    }
  };
  V8 kf[D / 16], vf[D / 16];
  auto load_kv = [&]() {
  // K and V rows for this wave's 32 keys as B operands: lane (key=r, hl) holds X[key][16s+8hl..]
#pragma unroll
  for (int s = 0; s < D / 16; ++s) {
    if (mykey < Sk) {
      kf[s] = *(const V8*)(kp + (int64_t)mykey * a.k_ss + 16 * s + 8 * hl);
      vf[s] = *(const V8*)(vp + (int64_t)mykey * a.v_ss + 16 * s + 8 * hl);
    } else {
      kf[s] = V8{};
      vf[s] = V8{};
    }
  }
  // whole K block to LDS transposed, K^T [D][KT_LD] (the A operand of dQ^T = K^T . dS^T, read as
  // 16-byte rows), written once per workgroup from the K rows just loaded as B operands (kf: key
  // mykey, dims 16s + 8hl .. +7; zero past Sk): each 2-byte store instruction writes one dim row, 32
  // consecutive keys per half-wave — conflict-free, and no second global read of K. (Round 5 staged
  // it from a fresh 16-byte-per-lane load of K with 8 dims x 8 keys per half-wave: 8-way conflicts,
  // half of the kernel's conflict cycles; a conflict-free re-load needed strided global loads.)
  if constexpr (DQ) {
#pragma unroll
    for (int s = 0; s < D / 16; ++s) {
      const T* e = (const T*)&kf[s];
#pragma unroll
      for (int j = 0; j < 8; ++j) lds_k[(16 * s + 8 * hl + j) * KT_LD + 32 * wid + r] = e[j];
    }
  }
  };
  // D <= 64: the K/V loads are issued after the first query-block fetch, so both latencies
  // overlap (at D >= 128 that order spills registers)
  if (D >= 128) load_kv();
  if (qstart < nq) fetch(pfa, qstart);
  if (DEPTH2 && qstart + kBwdBQ < nq) fetch(pfb, qstart + kBwdBQ);
  if (D < 128) load_kv();

  float dqcs[D / 32][4] = {};  // DSUM: this lane's dq dims (see the dQ section) summed over queries
  // fp8 producer-side codes of dq / dk / dv (AttnArgs::q8dq..): running max|value| of this lane
  float q8mx = 0.f;
  const float q8s = a.q8dq ? a.q8_scale[0] : 0.f, q8seen = a.q8dq ? f8_amax_seen(a.q8_amax) : 0.f;
  auto body = [&](Pf& P, const int qb) {
    uint4 (&pf_q)[NLD] = P.q;
    uint4 (&pf_do)[NLD] = P.d;
    if constexpr (D >= 128) {
      // keep dK / dV in AGPRs across the step (else the allocator parks two of them in VGPRs while
      // the S / dP products use their AGPRs: 64 accvgpr moves per step)
#pragma unroll
      for (int i = 0; i < D / 32; ++i) asm volatile("" : "+a"(dk[i]), "+a"(dv[i]));
    }
    lds_barrier();
    // stage the prefetched tiles; delta = rowsum(dO * O) is computed here from O
    // (CPR consecutive threads own one row -> xor-shuffle reduce), no separate pass.
#pragma unroll
    for (int c = 0; c < NLD; ++c) {
      const int idx = threadIdx.x + 256 * c;
      if (NCHK < 256 && idx >= NCHK) break;  // (wave-uniform: D = 32 leaves waves 2, 3 out)
      const int row = idx / CPR, col = (idx % CPR) * 8;
      if constexpr (DQ) {
        float ov[8], dov[8];
        load_f<T, 8>((const T*)&P.o[c], ov);
        load_f<T, 8>((const T*)&pf_do[c], dov);
        float part = 0.f;
#pragma unroll
        for (int e = 0; e < 8; ++e) part += ov[e] * dov[e];
        part = group_sum<CPR>(part);
        if ((idx % CPR) == 0) lds_delta[row] = part;
      }
      *(uint4*)(lds_q + row * LDQ + col) = pf_q[c];
      *(uint4*)(lds_do + row * LDQ + col) = pf_do[c];
    }
    if (threadIdx.x < kBwdBQ) lds_lse[threadIdx.x] = P.lse * kLog2e;  // +inf stays +inf
    if (!DQ && threadIdx.x >= 128 && threadIdx.x < 128 + kBwdBQ) lds_delta[threadIdx.x - 128] = P.dl;
    if (DROPOUT && threadIdx.x < 4 * kBwdBQ) lds_mask[threadIdx.x] = P.mask;
    if (qb + AHEAD * kBwdBQ < nq) fetch(P, qb + AHEAD * kBwdBQ);
    lds_barrier();

    // D >= 128 (one wave per SIMD): lse / delta / dropout words of this lane's 16 query rows
    // (8g + 4hl + e, e = 0..3) as 16-byte LDS reads issued ahead of the S / dP products, so their
    // latency hides behind the MFMAs (a scalar read + wait per element exposed ~16 LDS round trips
    // per step with no partner wave to cover them). D <= 64 runs two waves per SIMD and has no
    // 48 spare VGPRs: it reads the scalars in the elementwise loop.
    constexpr bool VROWS = D >= 128;
    f32x4 lse4[4], del4[4];
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    u32x4 msk4[4];
    if constexpr (VROWS) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        lse4[g] = *(const f32x4*)(lds_lse + 8 * g + 4 * hl);
        del4[g] = *(const f32x4*)(lds_delta + 8 * g + 4 * hl);
        if (DROPOUT) msk4[g] = *(const u32x4*)(lds_mask + wid * kBwdBQ + 8 * g + 4 * hl);
      }
    }

    // S = Q . K^T  [32 q x 32 keys]: A = Q rows (LDS), B = K rows (regs)
    f32x16 sacc = f32x16{}, dpacc = f32x16{};
#pragma unroll
    for (int s = 0; s < D / 16; ++s) {
      const V8 qa = *(const V8*)(lds_q + r * LDQ + 16 * s + 8 * hl);
      const V8 da = *(const V8*)(lds_do + r * LDQ + 16 * s + 8 * hl);
      sacc = M::mma(qa, kf[s], sacc);
      dpacc = M::mma(da, vf[s], dpacc);
    }
    // element i: q = qb + (i&3) + 8(i>>2) + 4hl, key = mykey.
    // pd = P * keep (the 1/(1-p) factor of dV is applied once, in the epilogue),
    // ds = P * (dP * keep / (1-p) - delta) (the softmax scale of dK / dQ likewise).
    float pd[16], ds[16];
    const bool interior = (k0 + 32 * wid + 31 < Sk) && (qb + kBwdBQ <= nq) && (!CAUSAL || k0 + 32 * wid + 31 <= qb);
    // exp2 is the bare v_exp_f32 (no denormal range reduction). One wave-uniform branch picks the
    // boundary variant for the whole tile (a per-element branch split the section into 16 blocks
    // the scheduler could not interleave).
    auto elementwise = [&](auto bound_tag) {
      constexpr bool BOUND = decltype(bound_tag)::value;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        // this lane's 4 query rows 8g + 4hl + e of lse / delta / dropout words: one 16-byte LDS read
        // each (round 3 read them as 48 scalar ds_read_b32 per step at D <= 64)
        f32x4 lg4, dg4;
        u32x4 mg4;
        if constexpr (VROWS) {
          lg4 = lse4[g];
          dg4 = del4[g];
          if constexpr (DROPOUT) mg4 = msk4[g];
        } else {
          lg4 = *(const f32x4*)(lds_lse + 8 * g + 4 * hl);
          dg4 = *(const f32x4*)(lds_delta + 8 * g + 4 * hl);
          if constexpr (DROPOUT) mg4 = *(const u32x4*)(lds_mask + wid * kBwdBQ + 8 * g + 4 * hl);
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int i = 4 * g + e;
          const int qi = 8 * g + 4 * hl + e;
          float lterm = -lg4[e];
          if constexpr (BIAS) {
            const int q = qb + qi;
            if (q < nq && mykey < Sk) lterm = fmaf(to_f(bcol[(int64_t)q * a.bias_qs]), kLog2e, lterm);
          }
          float p = __builtin_amdgcn_exp2f(fmaf(sacc[i], a.scale_log2, lterm));
          if constexpr (BOUND) {
            const int q = qb + qi;
            const bool valid = (mykey < Sk) && (q < nq) && !(CAUSAL && mykey > q);
            p = valid ? p : 0.f;
          }
          float dpv = dpacc[i];
          float pk = p;
          if constexpr (DROPOUT) {
            const int m = __builtin_amdgcn_sbfe((int)mg4[e], r, 1);
            pk = __builtin_bit_cast(float, __builtin_bit_cast(int, p) & m);
            dpv = __builtin_bit_cast(float, __builtin_bit_cast(int, dpv) & m);
          }
          pd[i] = pk;
          ds[i] = p * fmaf(dpv, rkeep, -dg4[e]);
        }
      }
    };
    if (interior)
      elementwise(std::false_type{});
    else
      elementwise(std::true_type{});
    if constexpr (BIAS) {
      // trainable bias: its gradient is dS (natural domain, before the softmax scale). Lanes of a
      // half hold 32 consecutive keys of one query row per element: coalesced 128-B runs.
      if (a.dbias && mykey < a.Sk) {
        float* dcol = a.dbias + b * a.dbias_bs + h * a.dbias_hs + mykey;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int q = qb + 8 * (i >> 2) + 4 * hl + (i & 3);
          if (q < nq) {
            float* dst = dcol + (int64_t)q * a.dbias_qs;
            if (a.dbias_atomic) atomicAdd(dst, ds[i]);
            else *dst = ds[i];
          }
        }
      }
    }
    // dV += P^T . dO : accumulator-as-A (contraction over q = rows), B = dO via tr reads
    // dK += dS^T . Q : same with Q
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      const V8 pa = pack8<T, V8>(pd + 8 * s2);
      const V8 sa = pack8<T, V8>(ds + 8 * s2);
      const int kq = 16 * s2 + 4 * hl + ((lane & 15) >> 2);
#pragma unroll
      for (int db = 0; db < D / 32; ++db) {
        const int c0 = 32 * db + 16 * ((lane >> 4) & 1) + 4 * (lane & 3);
        const V8 dob = join4<V8>(lds_tr16(lds_do + kq * LDQ + c0), lds_tr16(lds_do + (kq + 8) * LDQ + c0));
        const V8 qbf = join4<V8>(lds_tr16(lds_q + kq * LDQ + c0), lds_tr16(lds_q + (kq + 8) * LDQ + c0));
        dv[db] = M::mma(pa, dob, dv[db]);
        dk[db] = M::mma(sa, qbf, dk[db]);
      }
    }
    if constexpr (DQ) {
    // dS to LDS as [q][key] (bf16) for dQ = dS . K
#pragma unroll
    for (int g4 = 0; g4 < 4; ++g4) {
      typedef T t4 __attribute__((ext_vector_type(4)));
      t4 w;
#pragma unroll
      for (int e = 0; e < 4; ++e) w[e] = (T)ds[4 * g4 + e];  // queries 8 g4 + 4 hl + e
      *(t4*)(lds_ds + dso(32 * wid + r, 8 * g4 + 4 * hl)) = w;
    }
    lds_barrier();
    // dQ^T [D x 32 q] = K^T . dS^T on 16x16x32 MFMAs over the full 128-key contraction: wave
    // w owns query tile qt = w & 1 (16 queries) and D/32 dim tiles of 16 from (w >> 1) D/32;
    // A = K^T rows, B = dS rows (16-byte LDS reads); each lane ends with 4 consecutive dims of
    // one query (8-byte stores). No cross-wave reduction, no scattered 2-byte stores.
    {
      constexpr int NT = D / 32;
      const int qt = wid & 1, dt0 = (wid >> 1) * NT;
      const int lq = lane & 15, lg = lane >> 4;
      f32x4 acc[NT];
#pragma unroll
      for (int t = 0; t < NT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < kBwdBK; kk += 32) {
        // B = dS [8 keys x 16 queries]: two transposed 4-key blocks of dS^T (lane 4q'+p of the
        // group addresses key row kk + 8 lg + q', queries 16 qt + 4p; lane lq receives query 16 qt + lq)
        const int dr = kk + 8 * lg + ((lane & 15) >> 2), dc = 16 * qt + 4 * (lane & 3);
        const V8 bb = join4<V8>(lds_tr16(lds_ds + dso(dr, dc)), lds_tr16(lds_ds + dso(dr + 4, dc)));
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          const V8 aa = *(const V8*)(lds_k + ((dt0 + t) * 16 + lq) * KT_LD + kk + 8 * lg);
          acc[t] = Mfma16T<T>::mma(aa, bb, acc[t]);
        }
      }
      // this workgroup is the sole writer of these query rows (single key block): final dtype
      const int q = qb + 16 * qt + lq;
      typedef T t4 __attribute__((ext_vector_type(4)));
      uint2 wq[NT];
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        t4 w;
#pragma unroll
        for (int i = 0; i < 4; ++i) w[i] = (T)(acc[t][i] * a.scale);
        wq[t] = __builtin_bit_cast(uint2, w);
      }
      // 16-byte stores (as the forward's O, T21): lanes of 16-lane rows lg and lg + 1 hold 4 dims each
      // of the same query for dim tiles t and t + 1; one v_permlane16_swap per dword gives the even
      // rows dims 4 lg .. 4 lg + 7 of tile t and the odd rows those of tile t + 1 (every lane, ahead
      // of the row-validity branch)
      constexpr bool WIDE = NT % 2 == 0;
      uint4 wd[WIDE ? NT / 2 : 1];
      if constexpr (WIDE) {
#pragma unroll
        for (int t = 0; t < NT; t += 2) {
          const auto rx = __builtin_amdgcn_permlane16_swap(wq[t].x, wq[t + 1].x, false, false);
          const auto ry = __builtin_amdgcn_permlane16_swap(wq[t].y, wq[t + 1].y, false, false);
          wd[t / 2] = make_uint4(rx[0], ry[0], rx[1], ry[1]);
        }
      }
      if (q < nq) {
        const int64_t qoff = b * a.dq_bs + h * a.dq_hs + (int64_t)q * a.dq_ss;
        T* dqp = (T*)a.dq + qoff;
        if constexpr (WIDE) {
          if (!a.q8only) {
#pragma unroll
            for (int t = 0; t < NT; t += 2)
              *(uint4*)(dqp + (dt0 + t + (lg & 1)) * 16 + 8 * (lg >> 1)) = wd[t / 2];
          }
        }
        if (a.q8dq) {  // fp8 codes of dq as stored (the QKV input-gradient GEMM's operand)
          uint32_t cq[NT];
#pragma unroll
          for (int t = 0; t < NT; ++t)
            cq[t] = a.q8_fmt == 0 ? f8_codes4<0, T>(wq[t].x, wq[t].y, q8s, q8mx) : f8_codes4<1, T>(wq[t].x, wq[t].y, q8s, q8mx);
          if constexpr (WIDE) {  // the same regrouping: 8-byte stores (rows lg, lg + 1 share the query)
#pragma unroll
            for (int t = 0; t < NT; t += 2) {
              const auto rc = __builtin_amdgcn_permlane16_swap(cq[t], cq[t + 1], false, false);
              *(uint2*)(a.q8dq + qoff + (dt0 + t + (lg & 1)) * 16 + 8 * (lg >> 1)) = make_uint2(rc[0], rc[1]);
            }
          } else {
#pragma unroll
            for (int t = 0; t < NT; ++t) *(uint32_t*)(a.q8dq + qoff + (dt0 + t) * 16 + 4 * lg) = cq[t];
          }
        }
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          if constexpr (!WIDE) {
            if (!a.q8only) *(uint2*)(dqp + (dt0 + t) * 16 + 4 * lg) = wq[t];
          }
          if constexpr (DSUM) {
            const t4 w = __builtin_bit_cast(t4, wq[t]);
#pragma unroll
            for (int i = 0; i < 4; ++i) dqcs[t][i] += (float)w[i];
          }
        }
      }
    }
    }  // DQ
  };
  if constexpr (DEPTH2) {
    for (int qb = qstart; qb < nq; qb += 2 * kBwdBQ) {
      body(pfa, qb);
      if (qb + kBwdBQ < nq) body(pfb, qb + kBwdBQ);
    }
  } else {
    for (int qb = qstart; qb < nq; qb += kBwdBQ) body(pfa, qb);
  }
  // write dK, dV: element i of block db -> key = k0 + 32wid + (i&3)+8(i>>2)+4hl, dim = 32db + r
  T* dkp = (T*)dk_out + b * a.dk_bs + h * a.dk_hs;
  T* dvp = (T*)dv_out + b * a.dv_bs + h * a.dv_hs;
  // optional bias-gradient partials: column sums of the stored dq / dk / dv over positions
  float* dsum = DSUM ? a.dsum + ((int64_t)b * 3 * a.H + h) * D : nullptr;
  if (DSUM && DQ) {  // reduce over the 16 query lanes; both query-tile waves add their partials
    const int lq = lane & 15, lg = lane >> 4, dt0 = (wid >> 1) * (D / 32);
#pragma unroll
    for (int t = 0; t < D / 32; ++t) {
      float v[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        v[i] = dqcs[t][i];
        v[i] = group_sum<16>(v[i]);  // all 16 lanes hold the sum
      }
      // lane lq < 4 of each group adds dim 4 lg + lq: one atomic instruction (16 lanes) per tile
      // (atomics cost per instruction, so 4 single-lane instructions would cost 4x)
      const float x = lq == 0 ? v[0] : lq == 1 ? v[1] : lq == 2 ? v[2] : v[3];
      if (lq < 4) atomicAdd(dsum + (dt0 + t) * 16 + 4 * lg + lq, x);
    }
  }
  // dK then dV staged through LDS so the global stores are 16-byte row chunks. The staging image is
  // [D][keys] (row stride 132 elements = 66 dwords: the 16 rows of a lane group's ds_write_b64 land
  // on distinct bank pairs): each lane writes 4 consecutive keys of one dim per 8-byte store (8 per
  // tensor instead of round 3's 32 ds_write_b16 into a [key][D] image), and the store loop reads
  // 8 dims of one key with two ds_read_b64_tr_b16 (every lane active: the tr read gathers across
  // lanes).
  lds_barrier();  // every wave is done reading lds_k (dQ products)
  constexpr int LDE = kBwdBK + 4;
  static_assert(D * LDE <= LDSK, "dK/dV staging fits lds_k");
  auto emit = [&](const f32x16 (&acc)[D / 32], const float mul, T* dst, const int64_t ss, float* dsum_t,
                  uint8_t* q8dst) {
    typedef T t4 __attribute__((ext_vector_type(4)));
#pragma unroll
    for (int db = 0; db < D / 32; ++db) {
      float sum = 0.f;
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const int kl0 = 32 * wid + 8 * g4 + 4 * hl;  // keys kl0 .. kl0 + 3
        t4 w;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          w[e] = (T)(acc[db][4 * g4 + e] * mul);
          if constexpr (DSUM) sum += (k0 + kl0 + e < a.Sk) ? (float)w[e] : 0.f;
        }
        *(t4*)(lds_k + (32 * db + r) * LDE + kl0) = w;
      }
      if constexpr (DSUM) {
        sum += xor32_f(sum);
        if (hl == 0) atomicAdd(dsum_t + 32 * db + r, sum);
      }
    }
    lds_barrier();
    // 16-lane group tasks: (8-dim block, 16-key block); a wave's 4 groups take 4 consecutive dim
    // blocks of the same keys (64 contiguous bytes of each key row per store instruction)
    constexpr int NDB = D / 8, NTASK = NDB * (kBwdBK / 16);
    static_assert(NTASK % 16 == 0, "tasks per workgroup");
    // fp8 codes of the stored values (the same element offset in the code array), 16 bytes per
    // lane: the 16-lane groups g (even) and g + 1 hold adjacent 8-dim blocks of the same keys, so
    // for iterations it and it + 1 one v_permlane16_swap per dword gives the even groups 16 dims of
    // their iteration-it key and the odd groups 16 dims of their iteration-(it + 1) key — half the
    // code store instructions
    constexpr bool CPAIR = (NTASK / 16) % 2 == 0 && NDB % 2 == 0;
    uint2 cprev = make_uint2(0u, 0u);
    int kprev = 0, dprev = 0;
#pragma unroll
    for (int it = 0; it < NTASK / 16; ++it) {
      const int t = it * 16 + wid * 4 + (lane >> 4);
      const int d0 = (t % NDB) * 8, kb = (t / NDB) * 16;
      const T* src = lds_k + (d0 + ((lane & 15) >> 2)) * LDE + kb + 4 * (lane & 3);
      const s16x4 lo = lds_tr16(src), hi = lds_tr16(src + 4 * LDE);
      const int key = k0 + kb + (lane & 15);
      const V8 x = join4<V8>(lo, hi);
      if (key < a.Sk && !a.q8only) *(V8*)(dst + (int64_t)key * ss + d0) = x;
      if (q8dst) {
        const uint4 ww = __builtin_bit_cast(uint4, x);
        uint2 c;
        float mx = 0.f;  // only keys in range feed the amax
        if (a.q8_fmt == 0) {
          c.x = f8_codes4<0, T>(ww.x, ww.y, q8s, mx);
          c.y = f8_codes4<0, T>(ww.z, ww.w, q8s, mx);
        } else {
          c.x = f8_codes4<1, T>(ww.x, ww.y, q8s, mx);
          c.y = f8_codes4<1, T>(ww.z, ww.w, q8s, mx);
        }
        if (key < a.Sk) q8mx = fmaxf(q8mx, mx);
        if constexpr (CPAIR) {
          if (it & 1) {  // every lane swaps (outside the key branch)
            const auto sx = __builtin_amdgcn_permlane16_swap(cprev.x, c.x, false, false);
            const auto sy = __builtin_amdgcn_permlane16_swap(cprev.y, c.y, false, false);
            const bool odd = (lane >> 4) & 1;
            const int kk = odd ? key : kprev, dd = odd ? d0 - 8 : dprev;
            if (kk < a.Sk) *(uint4*)(q8dst + (int64_t)kk * ss + dd) = make_uint4(sx[0], sy[0], sx[1], sy[1]);
          } else {
            cprev = c;
            kprev = key;
            dprev = d0;
          }
        } else if (key < a.Sk) {
          *(uint2*)(q8dst + (int64_t)key * ss + d0) = c;
        }
      }
    }
    lds_barrier();
  };
  emit(dk, a.scale, dkp, a.dk_ss, DSUM ? dsum + (int64_t)a.H * D : nullptr,
       a.q8dk ? a.q8dk + b * a.dk_bs + h * a.dk_hs : nullptr);
  emit(dv, rkeep, dvp, a.dv_ss, DSUM ? dsum + (int64_t)2 * a.H * D : nullptr,
       a.q8dv ? a.q8dv + b * a.dv_bs + h * a.dv_hs : nullptr);
  if (a.q8dq) f8_block_amax(q8mx, a.q8_amax, q8seen);  // every thread of the block reaches this
}

// dQ for key ranges longer than one backward key block: query-stationary, the forward's
// structure (one workgroup = 4 waves x 32 query rows, K/V streamed in 64-key tiles):
//   S^T = K . Q^T and dP^T = V . dO^T (32x32x16, one query per lane, so lse and delta are
//   lane-local scalars), dS^T = P^T * (dP^T * keep - delta) in registers, and
//   dQ^T += K^T . dS^T with the dS^T accumulators reused directly as the B operand (the same
//   register reuse as O^T += V^T . P^T in the forward). Every dQ row has exactly one writer:
//   no fp32 atomics, no accumulator buffer, no conversion pass. The extra S / dP products (vs
//   the fused single-kernel backward) cost less than the fp32 atomic traffic they replace.
template <typename T, int D, bool CAUSAL, bool DROPOUT, bool DSUM, bool BIAS>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(D <= 64 ? 2 : 1, D <= 64 ? 2 : 1))) attn_bwd_dq_kernel(AttnArgs a, const void* dout, const float* delta_in) {
  using M = MfmaT<T>;
  using V8 = typename M::V8;
  constexpr int LDR = ld_rows<D>();  // V: row reads
  constexpr int LDK = ld_both<D>();  // K: row and transposed reads
  __shared__ __attribute__((aligned(16))) T lds_k[kFwdKB * LDK];
  __shared__ __attribute__((aligned(16))) T lds_v[kFwdKB * LDR];

  // wid through readfirstlane: wave-uniform in SGPRs, so tile-level conditions become scalar branches
  const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int r = lane & 31, hl = lane >> 5;
  const int bh = blockIdx.x;  // grid (B*H, query blocks), heaviest (causal: last) query blocks first
  const int b = bh / a.H, h = bh % a.H;
  const int q0 = (CAUSAL ? gridDim.y - 1 - blockIdx.y : blockIdx.y) * kFwdBQ;
  const int qrow = q0 + 32 * wid + r;
  const int Sk = a.k_lens ? min(a.k_lens[b], a.Sk) : a.Sk;

  const T* qp = (const T*)a.q + b * a.q_bs + h * a.q_hs;
  const T* dop = (const T*)dout + b * a.do_bs + h * a.do_hs;
  const T* kp = (const T*)a.k + b * a.k_bs + h * a.k_hs;
  const T* vp = (const T*)a.v + b * a.v_bs + h * a.v_hs;
  const T* brow = BIAS ? bias_row<T>(a, b, h, qrow) : nullptr;

  // Q^T and dO^T fragments (B operands): lane (q=r, hl) holds X[q][16s + 8hl .. +7]
  V8 qf[D / 16], df[D / 16];
#pragma unroll
  for (int s = 0; s < D / 16; ++s) {
    if (qrow < a.Sq) {
      qf[s] = *(const V8*)(qp + (int64_t)qrow * a.q_ss + 16 * s + 8 * hl);
      df[s] = *(const V8*)(dop + (int64_t)qrow * a.do_ss + 16 * s + 8 * hl);
    } else {
      qf[s] = V8{};
      df[s] = V8{};
    }
  }
  // log2-domain lse (+inf for padding rows and fully masked rows: P = 0) and delta
  const float lse2 = qrow < a.Sq ? a.lse[(int64_t)bh * a.Sq + qrow] * kLog2e : INFINITY;
  const float delta = qrow < a.Sq ? delta_in[(int64_t)bh * a.Sq + qrow] : 0.f;

  f32x16 dq[D / 32];
#pragma unroll
  for (int i = 0; i < D / 32; ++i) dq[i] = f32x16{};

  int kend = Sk;
  if (CAUSAL) kend = min(kend, q0 + kFwdBQ);
  const int ntiles = (kend + kFwdKB - 1) / kFwdKB;

  constexpr int CPR = D / 8;
  constexpr int CH = kFwdKB * CPR / 256;
  // K/V tiles of the tile TWO ahead are loaded into registers while the current tile computes
  // (two register sets, loop unrolled by two) at D <= 64; one ahead at D >= 128 (register budget)
  constexpr bool KV2 = D <= 64;
  constexpr int AHEAD = KV2 ? 2 : 1;
  struct KV {
    uint4 k[CH], v[CH];
    uint32_t m[2];
  };
  KV kva, kvb;
  const uint32_t* mrow =
      DROPOUT && qrow < a.Sq ? (const uint32_t*)(a.dmask + ((int64_t)bh * a.Sq + qrow) * a.mask_words) : nullptr;
  auto gload = [&](KV& R, int kt) {
    uint4 (&kreg)[CH] = R.k;
    uint4 (&vreg)[CH] = R.v;
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const int idx = threadIdx.x + 256 * c;
      const int row = idx / CPR, col = (idx % CPR) * 8;
      const int key = kt * kFwdKB + row;
      if (key < Sk) {
        kreg[c] = *(const uint4*)(kp + (int64_t)key * a.k_ss + col);
        vreg[c] = *(const uint4*)(vp + (int64_t)key * a.v_ss + col);
      } else {
        kreg[c] = make_uint4(0, 0, 0, 0);
        vreg[c] = make_uint4(0, 0, 0, 0);
      }
    }
    if (DROPOUT) {
      // the forward's keep bits for this lane's 16 keys of each 32-key block (same layout)
#pragma unroll
      for (int sb = 0; sb < 2; ++sb) {
        const int blk = (kt * kFwdKB >> 5) + sb;
        R.m[sb] = 0u;
        if (mrow && blk * 32 < a.Sk) R.m[sb] = mrow[blk];  // raw: shifted at use (no wait here)
      }
    }
  };
  auto lstore = [&](KV& R) {
    uint4 (&kreg)[CH] = R.k;
    uint4 (&vreg)[CH] = R.v;
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const int idx = threadIdx.x + 256 * c;
      const int row = idx / CPR, col = (idx % CPR) * 8;
      *(uint4*)(lds_k + row * LDK + col) = kreg[c];
      *(uint4*)(lds_v + row * LDR + col) = vreg[c];
    }
  };

  const float rkeep = a.drop_scale;
  if (ntiles > 0) gload(kva, 0);
  if (KV2 && ntiles > 1) gload(kvb, 1);
  auto tile = [&](KV& R, const int kt) {
    if constexpr (D >= 128) {
      // pin the dQ accumulators to AGPRs at the tile boundary: without it the allocator copied all
      // 64 of them to VGPRs and back every tile so the S / dP products could use their AGPRs
#pragma unroll
      for (int i = 0; i < D / 32; ++i) asm volatile("" : "+a"(dq[i]));
    }
    lds_barrier();  // previous tile fully consumed
    lstore(R);
    const uint32_t mcur[2] = {R.m[0] >> (4 * hl), R.m[1] >> (4 * hl)};
    lds_barrier();
    if (kt + AHEAD < ntiles) gload(R, kt + AHEAD);
    const int kb = kt * kFwdKB;

    f32x16 st[2], dpt[2];
#pragma unroll
    for (int sb = 0; sb < 2; ++sb) {
      V8 kf[D / 16], vf[D / 16];
#pragma unroll
      for (int s = 0; s < D / 16; ++s) {
        kf[s] = *(const V8*)(lds_k + (32 * sb + r) * LDK + 16 * s + 8 * hl);
        vf[s] = *(const V8*)(lds_v + (32 * sb + r) * LDR + 16 * s + 8 * hl);
      }
      __builtin_amdgcn_sched_group_barrier(0x100, 2 * (D / 16), 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 2 * (D / 16), 0);
      st[sb] = f32x16{};
      dpt[sb] = f32x16{};
#pragma unroll
      for (int s = 0; s < D / 16; ++s) {
        st[sb] = M::mma(kf[s], qf[s], st[sb]);
        dpt[sb] = M::mma(vf[s], df[s], dpt[sb]);
      }
    }
    const bool interior = (kb + kFwdKB <= Sk) && (!CAUSAL || kb + kFwdKB - 1 <= q0 + 32 * wid);
    const int lim = CAUSAL ? min(Sk, qrow + 1) : Sk;
    float bl2[2][16];  // BIAS: bias x log2(e) of element (sb, i)
    if constexpr (BIAS) {
#pragma unroll
      for (int sb = 0; sb < 2; ++sb)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          float bv[4];
          bias4<T>(brow, kb + 32 * sb + 8 * g + 4 * hl, a.Sk, bv);
#pragma unroll
          for (int e = 0; e < 4; ++e) bl2[sb][4 * g + e] = bv[e] * kLog2e;
        }
    }
#pragma unroll
    for (int sb = 0; sb < 2; ++sb) {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        float p = __builtin_amdgcn_exp2f(fmaf(st[sb][i], a.scale_log2, BIAS ? bl2[sb][i] - lse2 : -lse2));
        if (!interior) {
          const int key = kb + 32 * sb + (i & 3) + 8 * (i >> 2) + 4 * hl;
          if (key >= lim) p = 0.f;
        }
        float dp = dpt[sb][i];
        if (DROPOUT)
          dp = __builtin_bit_cast(float, __builtin_bit_cast(int, dp) & __builtin_amdgcn_sbfe((int)mcur[sb], (i & 3) + 8 * (i >> 2), 1));
        st[sb][i] = p * fmaf(dp, rkeep, -delta);  // dS^T (the softmax scale is applied once, at the end)
      }
    }
    // dQ^T += K^T . dS^T
#pragma unroll
    for (int sb = 0; sb < 2; ++sb) {
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        float sv[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) sv[j] = st[sb][8 * s2 + j];
        const V8 sf = pack8<T, V8>(sv);
        const int k0 = 32 * sb + 16 * s2 + 4 * hl + ((lane & 15) >> 2);
#pragma unroll
        for (int db = 0; db < D / 32; ++db) {
          const int c0 = 32 * db + 16 * ((lane >> 4) & 1) + 4 * (lane & 3);
          const s16x4 lo = lds_tr16(lds_k + k0 * LDK + c0);
          const s16x4 hi = lds_tr16(lds_k + (k0 + 8) * LDK + c0);
          dq[db] = M::mma(join4<V8>(lo, hi), sf, dq[db]);
        }
      }
    }
  };
  if constexpr (KV2) {
    for (int kt = 0; kt < ntiles; kt += 2) {
      tile(kva, kt);
      if (kt + 1 < ntiles) tile(kvb, kt + 1);
    }
  } else {
    for (int kt = 0; kt < ntiles; ++kt) tile(kva, kt);
  }
  // ---- epilogue: element 4g+e of block db -> dim 32db + 8g + 4hl + e of query qrow; 16-byte
  // stores through one v_permlane32_swap per dword and column-group pair (as the forward's O)
  float* dsum = DSUM ? a.dsum + ((int64_t)b * 3 * a.H + h) * D : nullptr;
  T* dqrow = (T*)a.dq + b * a.dq_bs + h * a.dq_hs + (int64_t)qrow * a.dq_ss;
#pragma unroll
  for (int db = 0; db < D / 32; ++db) {
    typedef T t4 __attribute__((ext_vector_type(4)));
    uint2 wv[4];
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      t4 w;
#pragma unroll
      for (int e = 0; e < 4; ++e) w[e] = (T)(dq[db][4 * g + e] * a.scale);
      wv[g] = __builtin_bit_cast(uint2, w);
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const auto rx = __builtin_amdgcn_permlane32_swap(wv[2 * j].x, wv[2 * j + 1].x, false, false);
      const auto ry = __builtin_amdgcn_permlane32_swap(wv[2 * j].y, wv[2 * j + 1].y, false, false);
      if (qrow < a.Sq) *(uint4*)(dqrow + 32 * db + 16 * j + 8 * hl) = make_uint4(rx[0], ry[0], rx[1], ry[1]);
    }
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const t4 w = __builtin_bit_cast(t4, wv[g]);
      if constexpr (DSUM) {
        // column sums of the stored values over this wave's 32 query rows (lanes r), then one
        // atomic per dim per wave
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float t = qrow < a.Sq ? (float)w[e] : 0.f;
          t = group_sum<32>(t);
          if (r == 0) atomicAdd(dsum + 32 * db + 8 * g + 4 * hl + e, t);
        }
      }
    }
  }
}


// ---------------------------------------------------------------------------
// per-head-dim launchers (instantiated by attention_d<D>.hip)
// ---------------------------------------------------------------------------
#define ATTN_DISPATCH(DT, T, ...)                         \
  switch (DT) {                                             \
    case kF16: { using T = f16; __VA_ARGS__; } break;       \
    case kBF16: { using T = bf16; __VA_ARGS__; } break;     \
    default: return -1;                                     \
  }
#define ATTN_DISPATCH_B(X, NAME, ...)                       \
  if (X) { constexpr bool NAME = true; __VA_ARGS__; }       \
  else { constexpr bool NAME = false; __VA_ARGS__; }

// double-buffered forward for key ranges > 128 (APEX_ATTN_FWD_DB=0 selects the two-barrier loop)
inline bool attn_fwd_db() {
  static const bool on = [] {
    const char* e = getenv("APEX_ATTN_FWD_DB");
    return !(e && e[0] == '0');
  }();
  return on;
}

// Dropout variants now that the keep bits are cheap (DropStream): the single-pass SHORT kernel
// (Sk <= 128) with dropout is the default (BERT-Large b768 s128 p = 0.1 forward 262-264 -> 253 us,
// profiles/r4_attn_stream_ab.jsonl; APEX_ATTN_FWD_SHORT_DROP=0 restores the two-barrier loop); the
// double-buffered loop with dropout stays off (GPT-2 s1024 p = 0.1 forward 87 -> 96 us;
// APEX_ATTN_FWD_DB_DROP=1 turns it on)
inline bool attn_env_on(const char* name, bool dflt) {
  const char* e = getenv(name);
  return e ? e[0] != '0' : dflt;
}
inline bool attn_fwd_short_drop() {
  static const bool on = attn_env_on("APEX_ATTN_FWD_SHORT_DROP", true);
  return on;
}
inline bool attn_fwd_db_drop() {
  static const bool on = attn_env_on("APEX_ATTN_FWD_DB_DROP", false);
  return on;
}

template <int D>
int attn_fwd_impl(const AttnArgs& a, int dt, hipStream_t s) {
  // grid (B*H, query blocks), dispatched x-fastest: every head's block of one query range goes out
  // together, and with a causal mask the heaviest ranges (the last query blocks, which see the most
  // keys) go first, so the short blocks fill the tail (longest-first list scheduling)
  dim3 grid(a.B * a.H, (a.Sq + kFwdBQ - 1) / kFwdBQ);
  const bool drop = a.drop_thresh > 0;
  // SHORT: single LDS stage (k_lens <= Sk). Without dropout only: measured at the BERT shape
  // (tools/attn_bench.py, b256 s128 h16) p = 0 fwd 61.1 -> 56.1 us, but p = 0.1 72.7 -> 73.8 us:
  // with dropout the kernel is bound by the Philox integer multiplies, not by load latency.
  // Re-measured with the dropout variant at 128 VGPRs / 4 workgroups per CU (round 2): 75.3-76.5
  // vs 74.0-75.7 us — the same; p = 0 at 56 us is within ~10 % of its HBM floor (276 MB moved).
  if constexpr (D == 64) {
    if (a.Sk <= 2 * kFwdKB && (!drop || attn_fwd_short_drop()) && !a.bias) {
      // W4: the dropout variant at 128 VGPRs / 4 workgroups per CU (APEX_ATTN_SHORT_W4, A/B knob):
      // 4 VGPRs spill there and it measured slower, b768 p = 0.1 245-247 -> 272-273 us
      // (profiles/r4_attn_short_w4_ab.jsonl, same box), so 3 workgroups per CU stays the default
      if (drop && attn_env_on("APEX_ATTN_SHORT_W4", false)) {
        ATTN_DISPATCH(dt, T, ATTN_DISPATCH_B(a.causal, C,
            hipLaunchKernelGGL((attn_fwd_kernel<T, 64, C, true, true, false, false, true>), grid, dim3(256), 0, s, a)));
        return (int)hipGetLastError();
      }
      ATTN_DISPATCH(dt, T, ATTN_DISPATCH_B(a.causal, C, ATTN_DISPATCH_B(drop, DR,
          hipLaunchKernelGGL((attn_fwd_kernel<T, 64, C, DR, true, false>), grid, dim3(256), 0, s, a))));
      return (int)hipGetLastError();
    }
  }
  // double-buffered loop where it measured faster (profiles/r2_attn_fwd_db_ab.txt, same box): D >= 128
  // (Megatron s2048 d128: 213 -> 195 us p = 0, 279 -> 269 p = 0.1) and D = 64 without dropout at 3
  // waves/SIMD (GPT-2 s1024: 104 -> 90 us); D = 64 with dropout keeps the two-barrier loop (the
  // Philox temporaries spill at 168 VGPRs: 145 -> 187 us, and at 2 waves/SIMD DB is 3 % slower)
  if (attn_fwd_db() && a.Sk > 2 * kFwdKB && (D >= 128 || (D == 64 && (!drop || attn_fwd_db_drop())))) {
    ATTN_DISPATCH(dt, T, ATTN_DISPATCH_B(a.causal, C, ATTN_DISPATCH_B(drop, DR, ATTN_DISPATCH_B(a.bias != nullptr, BI,
        hipLaunchKernelGGL((attn_fwd_kernel<T, D, C, DR, false, BI, true>), grid, dim3(256), 0, s, a)))));
    return (int)hipGetLastError();
  }
  ATTN_DISPATCH(dt, T, ATTN_DISPATCH_B(a.causal, C, ATTN_DISPATCH_B(drop, DR, ATTN_DISPATCH_B(a.bias != nullptr, BI,
      hipLaunchKernelGGL((attn_fwd_kernel<T, D, C, DR, false, BI>), grid, dim3(256), 0, s, a)))));
  return (int)hipGetLastError();
}

template <int D>
int attn_bwd_impl(const AttnArgs& a, const void* dout, float* delta_ws, void* dk, void* dv, int dt,
                  hipStream_t s) {
  const bool drop = a.drop_thresh > 0;
  const bool multi = attn_bwd_needs_dq_acc(a);
  if (multi && !delta_ws) return -4;
  if (a.bias && a.dsum) return -5;  // (not instantiated: the packed-QKV bias-grad fusion runs without a score bias)
  // (B*H, blocks) grids, heaviest blocks first under a causal mask (see attn_fwd_impl)
  dim3 grid(a.B * a.H, (a.Sk + kBwdBK - 1) / kBwdBK);
  dim3 qgrid(a.B * a.H, (a.Sq + kFwdBQ - 1) / kFwdBQ);
  if (multi) {
    dim3 dgrid((a.Sq * (D / 8) + 255) / 256, a.B * a.H);
    ATTN_DISPATCH(dt, T, hipLaunchKernelGGL((attn_bwd_delta_kernel<T, D>), dgrid, dim3(256), 0, s, a, dout, delta_ws));
  }
  ATTN_DISPATCH(dt, T, ATTN_DISPATCH_B(a.causal, C, ATTN_DISPATCH_B(drop, DR, {
    if (a.bias) {
      if (multi) {
        hipLaunchKernelGGL((attn_bwd_kernel<T, D, C, DR, false, false, true>), grid, dim3(256), 0, s, a, dout,
                           delta_ws, dk, dv);
        hipLaunchKernelGGL((attn_bwd_dq_kernel<T, D, C, DR, false, true>), qgrid, dim3(256), 0, s, a, dout,
                           (const float*)delta_ws);
      } else {
        hipLaunchKernelGGL((attn_bwd_kernel<T, D, C, DR, false, true, true>), grid, dim3(256), 0, s, a, dout,
                           nullptr, dk, dv);
      }
    } else {
      ATTN_DISPATCH_B(a.dsum != nullptr, DS, {
        if (multi) {
          hipLaunchKernelGGL((attn_bwd_kernel<T, D, C, DR, DS, false, false>), grid, dim3(256), 0, s, a, dout,
                             delta_ws, dk, dv);
          hipLaunchKernelGGL((attn_bwd_dq_kernel<T, D, C, DR, DS, false>), qgrid, dim3(256), 0, s, a, dout,
                             (const float*)delta_ws);
        } else {
          hipLaunchKernelGGL((attn_bwd_kernel<T, D, C, DR, DS, true, false>), grid, dim3(256), 0, s, a, dout,
                             nullptr, dk, dv);
        }
      });
    }
  })));
  return (int)hipGetLastError();
}

// entry points, one translation unit per head dim
int attn_fwd_d32(const AttnArgs& a, int dt, hipStream_t s);
int attn_fwd_d64(const AttnArgs& a, int dt, hipStream_t s);
int attn_fwd_d128(const AttnArgs& a, int dt, hipStream_t s);
int attn_fwd_d256(const AttnArgs& a, int dt, hipStream_t s);
int attn_bwd_d32(const AttnArgs& a, const void* dout, float* delta_ws, void* dk, void* dv, int dt, hipStream_t s);
int attn_bwd_d64(const AttnArgs& a, const void* dout, float* delta_ws, void* dk, void* dv, int dt, hipStream_t s);
int attn_bwd_d128(const AttnArgs& a, const void* dout, float* delta_ws, void* dk, void* dv, int dt, hipStream_t s);
int attn_bwd_d256(const AttnArgs& a, const void* dout, float* delta_ws, void* dk, void* dv, int dt, hipStream_t s);
// fp32 inputs (attention_f32.hip: f32 MFMA), head dims 32 / 64 / 128
int attn_fwd_f32(const AttnArgs& a, hipStream_t s);
int attn_bwd_f32(const AttnArgs& a, const void* dout, float* delta_ws, void* dk, void* dv, hipStream_t s);

}  // namespace apex
