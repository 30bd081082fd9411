// Flash attention for fp32 inputs on the exact f32 MFMA (v_mfma_f32_32x32x2_f32: f32 in, f32
// accumulate, bit-for-bit an fmaf chain; 1/16 of the bf16 matrix rate, the same as the f32 VALU
// peak but one VGPR per operand and the VALU left free for the softmax).
//
// Rounds 1-3 ran fp32 attention as torch compositions (the dense matmul -> softmax -> dropout ->
// matmul reference at training lengths, a query-blocked recomputation beyond): every [B, h, S, S]
// intermediate makes a round trip through HBM, ~3 elementwise passes each way. Here the scores
// never leave registers (same semantics as the bf16 kernels in attention_impl.h: causal mask
// key > query, per-batch key lengths, an additive [B|1, H|1, Sq|1, Sk] score bias, Philox-seeded
// dropout with the keep bits stored for backward; fp32 log-sum-exp, natural log, +inf for a row
// with no visible key). Head dims 32 / 64 / 128 (the Python side pads others up to 128).
//
// Layouts (cdna_hip_programming.md §3, 32x32x2 f32: lane l supplies A[i = l & 31][k = l >> 5] and
// B[k = l >> 5][j = l & 31]; the accumulator holds column j = l & 31, rows
// (r & 3) + 8 (r >> 2) + 4 (l >> 5) in registers r = 0..15):
//  * forward (per wave 32 queries): S^T = K . Q^T with the contraction permuted so MFMA s takes
//    d = s + (l >> 5) D / 2 — every lane reads its operand as float4 runs — leaving lane
//    (query, half) with 16 keys kappa(i, half) = (i & 3) + 8 (i >> 2) + 4 half of its query; the
//    next product O^T = V^T . P^T sums over exactly that row index, so P^T is the B operand as it
//    stands (no transpose, no LDS round trip) and V^T is staged transposed [D][32 + 4];
//  * dK/dV (key-stationary, per wave 32 keys): S = Q . K^T and dP = dO . V^T leave lane
//    (key, half) with 16 queries; dV^T = dO^T . P and dK^T = Q^T . dS take them as B operands, dO^T
//    and Q^T staged transposed;
//  * dQ (query-stationary, per wave 32 queries): S^T and dP^T as in the forward, then
//    dQ^T = K^T . dS^T (K^T staged transposed): each workgroup owns its dQ rows, no atomics.
// The softmax scale is folded into Q once (the forward's and the dQ kernel's Q registers, the
// dK/dV kernel's staged Q tile — which makes dK = dS^T (scale Q) with no epilogue multiply).
// Reference: apex/contrib/csrc/multihead_attn (fp32 softmax inside the fused MHA kernels) —
// /root/reference/apex/contrib/csrc/multihead_attn/softmax.cuh.
#include "attention_impl.h"

namespace apex {
namespace {

constexpr int kF32Waves = 4;
constexpr int kF32Tile = 32;                 // keys per forward / dQ tile, queries per dK/dV step
constexpr int kF32Rows = 32 * kF32Waves;     // queries (forward, dQ) or keys (dK/dV) per workgroup
constexpr int kF32LdT = kF32Tile + 4;        // transposed tiles [D][32 + 4]: 144-byte rows

__device__ __forceinline__ f32x16 mfma_f32(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

// 32 rows x D fp32 tile through registers: global float4 runs -> LDS row-major [32][D + 4]
// (16-byte rows offsets 272 B apart for D = 64: an 8-lane ds_read_b128 phase hits 8 distinct bank
// quads) and / or transposed [D][36]. Rows >= nrows load as zeros (a NaN there would survive
// P = 0 in the products).
template <int D>
struct Tile32 {
  static constexpr int CPR = D / 4;
  static constexpr int CH = kF32Tile * CPR / 256;
  static_assert(CH >= 1 && kF32Tile * CPR % 256 == 0, "tile must split evenly over 256 threads");
  float4 v[CH];
  __device__ __forceinline__ void load(const float* base, int64_t rs, int row0, int nrows, float mul = 1.f) {
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const int idx = threadIdx.x + 256 * c;
      const int row = row0 + idx / CPR, col = (idx % CPR) * 4;
      if (row < nrows) {
        v[c] = *(const float4*)(base + (int64_t)row * rs + col);
        v[c].x *= mul;
        v[c].y *= mul;
        v[c].z *= mul;
        v[c].w *= mul;
      } else {
        v[c] = make_float4(0.f, 0.f, 0.f, 0.f);
      }
    }
  }
  __device__ __forceinline__ void rows(float* lds) const {
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const int idx = threadIdx.x + 256 * c;
      *(float4*)(lds + (idx / CPR) * (D + 4) + (idx % CPR) * 4) = v[c];
    }
  }
  __device__ __forceinline__ void cols(float* ldt) const {
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const int idx = threadIdx.x + 256 * c;
      const int row = idx / CPR, col = (idx % CPR) * 4;
      ldt[(col + 0) * kF32LdT + row] = v[c].x;
      ldt[(col + 1) * kF32LdT + row] = v[c].y;
      ldt[(col + 2) * kF32LdT + row] = v[c].z;
      ldt[(col + 3) * kF32LdT + row] = v[c].w;
    }
  }
};

// acc (+)= A . B over D with A read as float4 runs from an LDS row (this lane's row, the half's
// D / 2 columns) and B from registers in the same permuted contraction order
template <int D>
__device__ __forceinline__ f32x16 mm_rows(const float* arow, const float (&b)[D / 2], f32x16 acc) {
#pragma unroll
  for (int c = 0; c < D / 8; ++c) {
    const float4 x = *(const float4*)(arow + 4 * c);
    acc = mfma_f32(x.x, b[4 * c + 0], acc);
    acc = mfma_f32(x.y, b[4 * c + 1], acc);
    acc = mfma_f32(x.z, b[4 * c + 2], acc);
    acc = mfma_f32(x.w, b[4 * c + 3], acc);
  }
  return acc;
}

// acc[db] += T^T . X where X is an accumulator tile (element j of lane (col, half) = row
// kappa(j, half)) and T^T rows are read from a transposed LDS tile [D][36] at this lane's d
template <int D>
__device__ __forceinline__ void mm_acc(const float* ldt, int r, int hl, const f32x16& x, f32x16 (&acc)[D / 32]) {
#pragma unroll
  for (int g = 0; g < 4; ++g)
#pragma unroll
    for (int db = 0; db < D / 32; ++db) {
      const float4 t = *(const float4*)(ldt + (32 * db + r) * kF32LdT + 8 * g + 4 * hl);
      acc[db] = mfma_f32(t.x, x[4 * g + 0], acc[db]);
      acc[db] = mfma_f32(t.y, x[4 * g + 1], acc[db]);
      acc[db] = mfma_f32(t.z, x[4 * g + 2], acc[db]);
      acc[db] = mfma_f32(t.w, x[4 * g + 3], acc[db]);
    }
}

// this lane's half of a row, D / 2 floats in the permuted contraction order, times mul
template <int D>
__device__ __forceinline__ void row_regs(const float* p, bool ok, int hl, float mul, float (&f)[D / 2]) {
#pragma unroll
  for (int c = 0; c < D / 8; ++c) {
    float4 t = ok ? *(const float4*)(p + hl * (D / 2) + 4 * c) : make_float4(0.f, 0.f, 0.f, 0.f);
    f[4 * c + 0] = t.x * mul;
    f[4 * c + 1] = t.y * mul;
    f[4 * c + 2] = t.z * mul;
    f[4 * c + 3] = t.w * mul;
  }
}

// store the accumulator tiles acc[db] (lane column = one output row, register rows = d) as float4
// runs of that row, times mul
template <int D>
__device__ __forceinline__ void store_rows(float* p, int hl, const f32x16 (&acc)[D / 32], float mul) {
#pragma unroll
  for (int db = 0; db < D / 32; ++db)
#pragma unroll
    for (int g = 0; g < 4; ++g)
      *(float4*)(p + 32 * db + 8 * g + 4 * hl) =
          make_float4(acc[db][4 * g] * mul, acc[db][4 * g + 1] * mul, acc[db][4 * g + 2] * mul, acc[db][4 * g + 3] * mul);
}

__device__ __forceinline__ int kappa(int i, int hl) { return (i & 3) + 8 * (i >> 2) + 4 * hl; }

// ---------------------------------------------------------------------------------------------
// forward: grid (B*H, query blocks of 128), heaviest (causal: last) blocks first; 4 waves x 32 queries
// ---------------------------------------------------------------------------------------------
template <int D, bool CAUSAL, bool DROPOUT, bool BIAS>
__global__ void __launch_bounds__(256) attn_f32_fwd_kernel(AttnArgs a) {
  constexpr int LDR = D + 4;
  __shared__ __attribute__((aligned(16))) float lds_k[kF32Tile * LDR];
  __shared__ __attribute__((aligned(16))) float lds_vt[D * kF32LdT];
  const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int r = lane & 31, hl = lane >> 5;
  const int bh = blockIdx.x, b = bh / a.H, h = bh % a.H;
  const int q0 = (CAUSAL ? gridDim.y - 1 - blockIdx.y : blockIdx.y) * kF32Rows;
  const int qw = q0 + 32 * wid;  // this wave's first query
  const int qrow = qw + r;
  const int Sk = a.k_lens ? min(a.k_lens[b], a.Sk) : a.Sk;
  const float* kp = (const float*)a.k + b * a.k_bs + h * a.k_hs;
  const float* vp = (const float*)a.v + b * a.v_bs + h * a.v_hs;
  const float* brow = BIAS ? bias_row<float>(a, b, h, qrow) : nullptr;

  float qf[D / 2];  // scale * Q[qrow][d(s, half)]
  row_regs<D>((const float*)a.q + b * a.q_bs + h * a.q_hs + (int64_t)qrow * a.q_ss, qrow < a.Sq, hl, a.scale, qf);
  f32x16 o[D / 32];
#pragma unroll
  for (int i = 0; i < D / 32; ++i) o[i] = f32x16{};
  float m = -INFINITY, l = 0.f;

  const int kend = CAUSAL ? min(Sk, q0 + kF32Rows) : Sk;
  const int ntiles = (kend + kF32Tile - 1) / kF32Tile;
  uint32_t* mrow =
      DROPOUT && qrow < a.Sq ? (uint32_t*)(a.dmask + ((int64_t)bh * a.Sq + qrow) * a.mask_words) : nullptr;
  DropStream dg(a.seed, a.offset, DROPOUT ? a.drop_thresh : 0u, bh, qrow, hl, a.Sq);

  Tile32<D> kt_r, vt_r;
  if (ntiles > 0) {
    kt_r.load(kp, a.k_ss, 0, Sk);
    vt_r.load(vp, a.v_ss, 0, Sk);
  }
  for (int kt = 0; kt < ntiles; ++kt) {
    lds_barrier();  // previous tile consumed
    kt_r.rows(lds_k);
    vt_r.cols(lds_vt);
    lds_barrier();
    if (kt + 1 < ntiles) {
      kt_r.load(kp, a.k_ss, (kt + 1) * kF32Tile, Sk);
      vt_r.load(vp, a.v_ss, (kt + 1) * kF32Tile, Sk);
    }
    const int kb = kt * kF32Tile;
    uint32_t mcur = 0;
    if (DROPOUT) {  // one 32-key block per tile, drawn in block order (DropStream)
      const uint32_t hb = dg.half_bits(hl);
      const uint32_t word = hb | xor32_u(hb);
      if (hl == 0 && mrow) mrow[kt] = word;
      mcur = hb >> (4 * hl);
    }
    if (CAUSAL && kb > qw + 31) continue;  // every key of the tile is after this wave's queries
    f32x16 st = mm_rows<D>(lds_k + r * LDR + hl * (D / 2), qf, f32x16{});
    if constexpr (BIAS) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        float bv[4];
        bias4<float>(brow, kb + 8 * g + 4 * hl, a.Sk, bv);
#pragma unroll
        for (int e = 0; e < 4; ++e) st[4 * g + e] += bv[e];
      }
    }
    if (kb + kF32Tile > Sk || (CAUSAL && kb + kF32Tile - 1 > qw)) {
      const int lim = CAUSAL ? min(Sk, qrow + 1) : Sk;
#pragma unroll
      for (int i = 0; i < 16; ++i)
        if (kb + kappa(i, hl) >= lim) st[i] = -INFINITY;
    }
    float tmax = -INFINITY;
#pragma unroll
    for (int i = 0; i < 16; ++i) tmax = fmaxf(tmax, st[i]);
    tmax = fmaxf(tmax, xor32_f(tmax));
    const float mnew = fmaxf(m, tmax);
    const float muse = mnew == -INFINITY ? 0.f : mnew;
    const float alpha = __builtin_amdgcn_exp2f((m - muse) * kLog2e);
    const float ms = -muse * kLog2e;
    m = mnew;
    float psum = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const float p = __builtin_amdgcn_exp2f(fmaf(st[i], kLog2e, ms));
      psum += p;
      st[i] = DROPOUT ? __builtin_bit_cast(float, __builtin_bit_cast(int, p) &
                                                      __builtin_amdgcn_sbfe((int)mcur, (i & 3) + 8 * (i >> 2), 1))
                      : p;
    }
    l = l * alpha + psum;
#pragma unroll
    for (int db = 0; db < D / 32; ++db)
#pragma unroll
      for (int i = 0; i < 16; ++i) o[db][i] *= alpha;
    mm_acc<D>(lds_vt, r, hl, st, o);  // O^T += V^T . P^T
  }
  const float ltot = l + xor32_f(l);
  if (qrow < a.Sq) {
    const float inv = ltot > 0.f ? (DROPOUT ? a.drop_scale : 1.f) / ltot : 0.f;
    store_rows<D>((float*)a.o + b * a.o_bs + h * a.o_hs + (int64_t)qrow * a.o_ss, hl, o, inv);
    if (hl == 0 && a.lse) a.lse[(int64_t)bh * a.Sq + qrow] = ltot > 0.f ? m + logf(ltot) : INFINITY;
  }
}

// ---------------------------------------------------------------------------------------------
// dK / dV: grid (B*H, key blocks of 128), key-stationary, query steps of 32
// ---------------------------------------------------------------------------------------------
template <int D, bool CAUSAL, bool DROPOUT, bool BIAS>
__global__ void __launch_bounds__(256) attn_f32_bwd_dkdv_kernel(AttnArgs a, const float* __restrict__ dout,
                                                                const float* __restrict__ delta, float* dk,
                                                                float* dv) {
  constexpr int LDR = D + 4;
  __shared__ __attribute__((aligned(16))) float lds_q[kF32Tile * LDR];
  __shared__ __attribute__((aligned(16))) float lds_qt[D * kF32LdT];
  __shared__ __attribute__((aligned(16))) float lds_do[kF32Tile * LDR];
  __shared__ __attribute__((aligned(16))) float lds_dot[D * kF32LdT];
  __shared__ __attribute__((aligned(16))) float lds_lse[kF32Tile], lds_delta[kF32Tile];
  __shared__ uint32_t lds_mw[kF32Tile * kF32Waves];  // dropout words [query][wave's 32-key block]
  const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int r = lane & 31, hl = lane >> 5;
  const int bh = blockIdx.x, b = bh / a.H, h = bh % a.H;
  const int k0 = blockIdx.y * kF32Rows;  // causal: block 0 (the most queries) first
  const int kw = k0 + 32 * wid;
  const int key = kw + r;
  const int Sk = a.k_lens ? min(a.k_lens[b], a.Sk) : a.Sk;
  const float* qp = (const float*)a.q + b * a.q_bs + h * a.q_hs;
  const float* dop = dout + b * a.do_bs + h * a.do_hs;
  const float* bcol = BIAS ? (const float*)a.bias + b * a.bias_bs + h * a.bias_hs + min(key, a.Sk - 1) : nullptr;

  float kf[D / 2], vf[D / 2];
  row_regs<D>((const float*)a.k + b * a.k_bs + h * a.k_hs + (int64_t)key * a.k_ss, key < Sk, hl, 1.f, kf);
  row_regs<D>((const float*)a.v + b * a.v_bs + h * a.v_hs + (int64_t)key * a.v_ss, key < Sk, hl, 1.f, vf);
  f32x16 dkt[D / 32], dvt[D / 32];
#pragma unroll
  for (int i = 0; i < D / 32; ++i) dkt[i] = dvt[i] = f32x16{};

  const int qbeg = CAUSAL ? min(k0, a.Sq) / kF32Tile * kF32Tile : 0;  // queries < k0 see no key of the block
  const int qend = k0 < Sk ? a.Sq : qbeg;
  const bool wave_keys = kw < Sk;
  const uint32_t* mw32 = (const uint32_t*)a.dmask;
  const int64_t wpr = a.mask_words >> 1;  // 32-bit words per row

  Tile32<D> q_r, do_r;
  if (qbeg < qend) {
    q_r.load(qp, a.q_ss, qbeg, a.Sq, a.scale);
    do_r.load(dop, a.do_ss, qbeg, a.Sq);
  }
  for (int qb = qbeg; qb < qend; qb += kF32Tile) {
    lds_barrier();
    q_r.rows(lds_q);
    q_r.cols(lds_qt);
    do_r.rows(lds_do);
    do_r.cols(lds_dot);
    if (threadIdx.x < kF32Tile) {
      const int q = qb + threadIdx.x;
      lds_lse[threadIdx.x] = q < a.Sq ? a.lse[(int64_t)bh * a.Sq + q] : INFINITY;
      lds_delta[threadIdx.x] = q < a.Sq ? delta[(int64_t)bh * a.Sq + q] : 0.f;
    }
    if (DROPOUT && threadIdx.x < kF32Tile * kF32Waves) {
      const int q = qb + (threadIdx.x >> 2), blk = (k0 >> 5) + (threadIdx.x & 3);
      lds_mw[threadIdx.x] = q < a.Sq && blk * 32 < Sk ? mw32[((int64_t)bh * a.Sq + q) * wpr + blk] : 0u;
    }
    lds_barrier();
    if (qb + kF32Tile < qend) {
      q_r.load(qp, a.q_ss, qb + kF32Tile, a.Sq, a.scale);
      do_r.load(dop, a.do_ss, qb + kF32Tile, a.Sq);
    }
    if (!wave_keys || (CAUSAL && qb + kF32Tile - 1 < kw)) continue;  // wave-uniform: nothing visible
    // S = (scale Q) . K^T, dP = dO . V^T: lane (key, half) holds queries qb + kappa(i, half)
    const f32x16 s = mm_rows<D>(lds_q + r * LDR + hl * (D / 2), kf, f32x16{});
    const f32x16 dp = mm_rows<D>(lds_do + r * LDR + hl * (D / 2), vf, f32x16{});
    f32x16 p, ds;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const float4 lse4 = *(const float4*)(lds_lse + 8 * g + 4 * hl);
      const float4 del4 = *(const float4*)(lds_delta + 8 * g + 4 * hl);
      const float lse[4] = {lse4.x, lse4.y, lse4.z, lse4.w};
      const float del[4] = {del4.x, del4.y, del4.z, del4.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int i = 4 * g + e;
        const int ql = 8 * g + 4 * hl + e;
        float sv = s[i];
        if (BIAS) sv += qb + ql < a.Sq ? bcol[(int64_t)(qb + ql) * a.bias_qs] : 0.f;
        float pv = __builtin_amdgcn_exp2f((sv - lse[e]) * kLog2e);
        if (key >= Sk || (CAUSAL && key > qb + ql)) pv = 0.f;
        float dpv = dp[i];
        float pk = pv;
        if (DROPOUT) {
          const bool keep = (lds_mw[ql * kF32Waves + wid] >> r) & 1u;
          pk = keep ? pv : 0.f;
          dpv = keep ? dpv * a.drop_scale : 0.f;
        }
        p[i] = pk;
        ds[i] = pv * (dpv - del[e]);
      }
    }
    if (BIAS && a.dbias) {  // trainable bias: its gradient is dS (see attention_impl.h)
      float* dcol = a.dbias + b * a.dbias_bs + h * a.dbias_hs + key;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int q = qb + kappa(i, hl);
        if (q < a.Sq && key < a.Sk) {
          float* dst = dcol + (int64_t)q * a.dbias_qs;
          if (a.dbias_atomic) atomicAdd(dst, ds[i]);
          else *dst = ds[i];
        }
      }
    }
    mm_acc<D>(lds_dot, r, hl, p, dvt);   // dV^T += dO^T . P (dropped: the 1/(1-p) in the epilogue)
    mm_acc<D>(lds_qt, r, hl, ds, dkt);   // dK^T += (scale Q)^T . dS
  }
  if (key < a.Sk) {
    store_rows<D>(dv + b * a.dv_bs + h * a.dv_hs + (int64_t)key * a.dv_ss, hl, dvt, DROPOUT ? a.drop_scale : 1.f);
    store_rows<D>(dk + b * a.dk_bs + h * a.dk_hs + (int64_t)key * a.dk_ss, hl, dkt, 1.f);
  }
}

// ---------------------------------------------------------------------------------------------
// dQ: grid (B*H, query blocks of 128), query-stationary, key tiles of 32
// ---------------------------------------------------------------------------------------------
template <int D, bool CAUSAL, bool DROPOUT, bool BIAS>
__global__ void __launch_bounds__(256) attn_f32_bwd_dq_kernel(AttnArgs a, const float* __restrict__ dout,
                                                              const float* __restrict__ delta) {
  constexpr int LDR = D + 4;
  __shared__ __attribute__((aligned(16))) float lds_k[kF32Tile * LDR];
  __shared__ __attribute__((aligned(16))) float lds_kt[D * kF32LdT];
  __shared__ __attribute__((aligned(16))) float lds_v[kF32Tile * LDR];
  const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int r = lane & 31, hl = lane >> 5;
  const int bh = blockIdx.x, b = bh / a.H, h = bh % a.H;
  const int q0 = (CAUSAL ? gridDim.y - 1 - blockIdx.y : blockIdx.y) * kF32Rows;
  const int qw = q0 + 32 * wid;
  const int qrow = qw + r;
  const bool qok = qrow < a.Sq;
  const int Sk = a.k_lens ? min(a.k_lens[b], a.Sk) : a.Sk;
  const float* kp = (const float*)a.k + b * a.k_bs + h * a.k_hs;
  const float* vp = (const float*)a.v + b * a.v_bs + h * a.v_hs;
  const float* brow = BIAS ? bias_row<float>(a, b, h, qrow) : nullptr;

  float qf[D / 2], dof[D / 2];
  row_regs<D>((const float*)a.q + b * a.q_bs + h * a.q_hs + (int64_t)qrow * a.q_ss, qok, hl, a.scale, qf);
  row_regs<D>(dout + b * a.do_bs + h * a.do_hs + (int64_t)qrow * a.do_ss, qok, hl, 1.f, dof);
  const float lse = qok ? a.lse[(int64_t)bh * a.Sq + qrow] : INFINITY;
  const float del = qok ? delta[(int64_t)bh * a.Sq + qrow] : 0.f;
  const uint32_t* mrow = DROPOUT && qok ? (const uint32_t*)(a.dmask + ((int64_t)bh * a.Sq + qrow) * a.mask_words) : nullptr;
  f32x16 dqt[D / 32];
#pragma unroll
  for (int i = 0; i < D / 32; ++i) dqt[i] = f32x16{};

  const int kend = CAUSAL ? min(Sk, q0 + kF32Rows) : Sk;
  const int ntiles = (kend + kF32Tile - 1) / kF32Tile;
  Tile32<D> k_r, v_r;
  if (ntiles > 0) {
    k_r.load(kp, a.k_ss, 0, Sk);
    v_r.load(vp, a.v_ss, 0, Sk);
  }
  for (int kt = 0; kt < ntiles; ++kt) {
    lds_barrier();
    k_r.rows(lds_k);
    k_r.cols(lds_kt);
    v_r.rows(lds_v);
    lds_barrier();
    if (kt + 1 < ntiles) {
      k_r.load(kp, a.k_ss, (kt + 1) * kF32Tile, Sk);
      v_r.load(vp, a.v_ss, (kt + 1) * kF32Tile, Sk);
    }
    const int kb = kt * kF32Tile;
    if (CAUSAL && kb > qw + 31) continue;
    // S^T = K . (scale Q)^T, dP^T = V . dO^T: lane (query, half) holds keys kb + kappa(i, half)
    f32x16 s = mm_rows<D>(lds_k + r * LDR + hl * (D / 2), qf, f32x16{});
    const f32x16 dp = mm_rows<D>(lds_v + r * LDR + hl * (D / 2), dof, f32x16{});
    const uint32_t mcur = DROPOUT && mrow ? mrow[kt] >> (4 * hl) : 0u;
    const int lim = CAUSAL ? min(Sk, qrow + 1) : Sk;
    f32x16 ds;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      float bv[4] = {0.f, 0.f, 0.f, 0.f};
      if (BIAS) bias4<float>(brow, kb + 8 * g + 4 * hl, a.Sk, bv);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int i = 4 * g + e;
        float pv = __builtin_amdgcn_exp2f((s[i] + bv[e] - lse) * kLog2e);
        if (kb + kappa(i, hl) >= lim) pv = 0.f;
        float dpv = dp[i];
        if (DROPOUT) dpv = (mcur >> ((i & 3) + 8 * (i >> 2))) & 1u ? dpv * a.drop_scale : 0.f;
        ds[i] = pv * (dpv - del);
      }
    }
    mm_acc<D>(lds_kt, r, hl, ds, dqt);  // dQ^T += K^T . dS^T
  }
  if (qok) store_rows<D>((float*)a.dq + b * a.dq_bs + h * a.dq_hs + (int64_t)qrow * a.dq_ss, hl, dqt, a.scale);
}

#define F32_DISPATCH_B(X, NAME, ...)                  \
  if (X) { constexpr bool NAME = true; __VA_ARGS__; } \
  else { constexpr bool NAME = false; __VA_ARGS__; }

template <int D>
int fwd_d(const AttnArgs& a, hipStream_t s) {
  const dim3 grid(a.B * a.H, (a.Sq + kF32Rows - 1) / kF32Rows);
  F32_DISPATCH_B(a.causal, C, F32_DISPATCH_B(a.drop_thresh > 0, DR, F32_DISPATCH_B(a.bias != nullptr, BI, {
    hipLaunchKernelGGL((attn_f32_fwd_kernel<D, C, DR, BI>), grid, dim3(256), 0, s, a);
  })));
  return (int)hipGetLastError();
}

template <int D>
int bwd_d(const AttnArgs& a, const float* dout, float* delta, float* dk, float* dv, hipStream_t s) {
  const dim3 dgrid((a.Sq * (D / 8) + 255) / 256, a.B * a.H);
  hipLaunchKernelGGL((attn_bwd_delta_kernel<float, D>), dgrid, dim3(256), 0, s, a, (const void*)dout, delta);
  const dim3 kgrid(a.B * a.H, (a.Sk + kF32Rows - 1) / kF32Rows);
  const dim3 qgrid(a.B * a.H, (a.Sq + kF32Rows - 1) / kF32Rows);
  F32_DISPATCH_B(a.causal, C, F32_DISPATCH_B(a.drop_thresh > 0, DR, F32_DISPATCH_B(a.bias != nullptr, BI, {
    hipLaunchKernelGGL((attn_f32_bwd_dkdv_kernel<D, C, DR, BI>), kgrid, dim3(256), 0, s, a, dout,
                       (const float*)delta, dk, dv);
    hipLaunchKernelGGL((attn_f32_bwd_dq_kernel<D, C, DR, BI>), qgrid, dim3(256), 0, s, a, dout,
                       (const float*)delta);
  })));
  return (int)hipGetLastError();
}

}  // namespace

int attn_fwd_f32(const AttnArgs& a, hipStream_t s) {
  switch (a.D) {
    case 32: return fwd_d<32>(a, s);
    case 64: return fwd_d<64>(a, s);
    case 128: return fwd_d<128>(a, s);
    default: return -1;
  }
}

int attn_bwd_f32(const AttnArgs& a, const void* dout, float* delta_ws, void* dk, void* dv, hipStream_t s) {
  if (!delta_ws) return -4;
  if (a.dsum) return -5;  // the packed-QKV bias-gradient fusion is a 16-bit-path feature
  const float* d = (const float*)dout;
  switch (a.D) {
    case 32: return bwd_d<32>(a, d, delta_ws, (float*)dk, (float*)dv, s);
    case 64: return bwd_d<64>(a, d, delta_ws, (float*)dk, (float*)dv, s);
    case 128: return bwd_d<128>(a, d, delta_ws, (float*)dk, (float*)dv, s);
    default: return -1;
  }
}

}  // namespace apex
