// Hand-written MFMA GEMM for gfx950 with fused epilogues (the transformer dense layers).
//
//   C[M,N] = epilogue( A[M,K] . B[N,K]^T )      A, B, C row-major, bf16 or fp16, fp32 accumulate
//
// Both operands are K-contiguous ("NT"): the forward projections (X . W^T) directly, and the
// input-gradient GEMMs (dY . W) through a transposed copy of W (transpose_2d below).
// Weight gradients (contraction over tokens): the transposed-read instantiation (gemm_tt, split-K
// fp32 slabs) for the shapes where it beats hipBLASLt, the library split-K otherwise (fused.py).
//
// Epilogues (fused into the tile write, so the activation never makes an extra HBM round
// trip — the separate bias/GELU/residual kernels they replace each read+wrote [M,N]):
//   EPI_NONE      C = acc
//   EPI_BIAS      C = acc + bias[n]
//   EPI_BIAS_GELU H = acc + bias[n] (pre-activation, kept for backward), C = gelu(H)
//   EPI_DGELU     C = acc * gelu'(H[m,n])   and per-(256-row tile, wave row) column partial sums
//                 of C written to `part` (the bias gradient, finished by partial_colsum)
//   EPI_RESID     C = acc + R[m,n]          (residual-gradient accumulation)
//   EPI_BIAS_GELU_TANH / EPI_DGELU_TANH: the same with the tanh-approximated GELU (GPT-2)
//   EPI_BIAS_GELU_D / _TANH_D  C = gelu(H) and gelu'(H) stored instead of H: the derivative shares
//                 the exp / erf (or sigmoid) of the GELU, so it is a few FMAs here, and the backward
//                 epilogue becomes
//   EPI_MUL       C = acc * G[m,n] with the bias-gradient partials of EPI_DGELU — a multiply
//                 instead of the erf/exp evaluation that made the dGELU epilogue VALU-bound
//                 (404 vs 201 us main loop at M=32768 N=4096 K=1024, profiles/r1_gemm_stagger.json)
//
// Tiling (CDNA4, cdna_hip_programming.md §5):
//  * 256x256 output tile, BK = 64, 512 threads = 8 waves as 2 (M) x 4 (N); each wave owns a
//    128 x 64 sub-tile = 8 x 4 fragments of v_mfma_f32_16x16x32 (128 fp32 accumulators/lane).
//  * The MFMA is issued "swapped" (A-operand = B rows, B-operand = A rows) so each lane ends
//    with 4 consecutive N-columns of one M-row: 8-byte vector epilogue loads/stores.
//  * Global -> LDS by global_load_lds_dwordx4 (16 B per lane, no VGPR round trip), double
//    buffered (2 x 64 KB), the next K-tile in flight across the barrier (counted vmcnt, raw
//    s_barrier — never __syncthreads(), whose fence would drain the prefetch).
//  * LDS image: 128-byte rows (64 bf16 of K), 16-byte chunk c of row r stored at chunk
//    c ^ ((r >> 1) & 7). glds writes lane-linear, so the XOR is applied to the per-lane SOURCE
//    address and again on the ds_read_b128: every 16-lane ds_read_b128 group then touches 16
//    distinct 16-B slots of the 256-B bank row (conflict-free).
//  * blockIdx -> tile: bijective XCD remap (each XCD gets a contiguous tile range) then
//    GROUP_M=8 panel ordering, so concurrently running tiles on one XCD share A/B panels in L2.
#include "common.h"
#include "kernels.h"
#include "fp8_pack.h"

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <type_traits>

namespace apex {
namespace {

// G_GROUP_M: M-tiles per panel of the tile order (consecutive workgroups walk GROUP_M M-tiles down
// one N column before moving right); APEX_G_GROUP_M overrides it at build time (lab sweeps)
#ifndef APEX_G_GROUP_M
#define APEX_G_GROUP_M 8
#endif
// APEX_GEMM_NT_GELU_D=1 / APEX_GEMM_NT_PLAIN=1 (A/B builds, off): the persistent bias+GELU_D epilogue
// stores both outputs / the plain and bias-only epilogues store C non-temporally. Isolated, bias+GELU_D
// ran 858 -> 821 us and a plain K = 1024 product 179 -> 164 us (profiles/r6_gemm_nt_stores.jsonl); in the
// BERT step the GELU_D form was neutral (4156 vs 4155 seq/s, 3 interleaved pairs,
// profiles/r6_gemm_nt_stores.jsonl): the next GEMM then reads its operand from HBM
#ifndef APEX_GEMM_NT_GELU_D
#define APEX_GEMM_NT_GELU_D 0
#endif
#ifndef APEX_GEMM_NT_PLAIN
#define APEX_GEMM_NT_PLAIN 0
#endif
constexpr int GB_M = 256, GB_N = 256, GB_K = 64, G_THREADS = 512, G_GROUP_M = APEX_G_GROUP_M;
constexpr int G_TILE_BYTES = GB_M * GB_K * 2;       // one operand tile: 32 KB
constexpr int G_BUF_BYTES = 2 * G_TILE_BYTES;       // A + B: 64 KB
constexpr int G_LDS_BYTES = 2 * G_BUF_BYTES;        // double buffered: 128 KB

typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <typename T> __device__ __forceinline__ f32x4 mfma16(const s16x8& a, const s16x8& b, const f32x4& c);
template <> __device__ __forceinline__ f32x4 mfma16<bf16>(const s16x8& a, const s16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
template <> __device__ __forceinline__ f32x4 mfma16<f16>(const s16x8& a, const s16x8& b, const f32x4& c) {
  typedef _Float16 h8 __attribute__((ext_vector_type(8)));
  return __builtin_amdgcn_mfma_f32_16x16x32_f16((h8)a, (h8)b, c, 0, 0, 0);
}

// FP8 (gfx950 f8f6f4 block-scaled MFMA, 16x16x128, 2x the bf16 rate): the 32 bytes of a lane's
// operand are the SAME two 16-byte LDS chunks the bf16 path reads for its two 16x16x32 K-steps
// (chunks lk and lk + 4 of the 128-byte K-tile row). The K order inside the instruction is thus a
// permutation of the tile's K, identical for both operands, so the dot products are unchanged and
// the LDS reads stay conflict-free. Block scales are all 2^0 (E8M0 127): the per-tensor scales
// are applied in the epilogue (alpha). Formats: 0 = e4m3 (OCP fn), 1 = e5m2.
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x8 __attribute__((ext_vector_type(8)));
template <int FMT_A, int FMT_B>
__device__ __forceinline__ f32x4 mfma_f8(const s16x8& a0, const s16x8& a1, const s16x8& b0, const s16x8& b1,
                                         const f32x4& c) {
  const i32x4 xa0 = __builtin_bit_cast(i32x4, a0), xa1 = __builtin_bit_cast(i32x4, a1);
  const i32x4 xb0 = __builtin_bit_cast(i32x4, b0), xb1 = __builtin_bit_cast(i32x4, b1);
  const i32x8 a = __builtin_shufflevector(xa0, xa1, 0, 1, 2, 3, 4, 5, 6, 7);
  const i32x8 b = __builtin_shufflevector(xb0, xb1, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, FMT_A, FMT_B, 0, 0x7F7F7F7F, 0, 0x7F7F7F7F);
}

// the lane id computed afresh (volatile: never CSE'd with an earlier copy or hoisted out of a loop), so
// no VGPR holding it — or an address derived from it — stays live across a K loop: the fp8 main loop
// runs at the 256-VGPR limit, and in the persistent kernel one more live register spills inside it
__device__ __forceinline__ int lane_id_fresh() {
  int l;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
  return l;
}

__device__ __forceinline__ void glds16(const void* g, void* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                   (__attribute__((address_space(3))) void*)lds_wave_base, 16, 0, 0);
}

// Branch-free erf (Abramowitz & Stegun 7.1.26, |error| <= 1.5e-7): one v_rcp, one v_exp and
// seven FMAs instead of ocml's erff (whose inlined branches made the epilogue 10x larger).
// Two values at a time: the polynomial runs on packed f32 (v_pk_fma_f32 / v_pk_mul_f32), the
// epilogue is VALU-bound on the GELU work (it runs after the MFMA main loop, not beside it).
typedef float f32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ f32x2 pk_fma(f32x2 a, f32x2 b, f32x2 c) { return __builtin_elementwise_fma(a, b, c); }
__device__ __forceinline__ f32x2 splat(float v) { return f32x2{v, v}; }

// Phi(x) = 0.5 (1 + erf(x / sqrt 2)) given e = exp(-x^2 / 2), the same A&S 7.1.26 polynomial with
// the 1/sqrt(2) folded into p and the 0.5 into the coefficients: Phi = 0.5 + sign(x) (0.5 - q),
// q = poly'(t) t e (two packed instructions fewer per pair than
// evaluating erf(x / sqrt 2) and then 0.5 (1 + erf))
__device__ __forceinline__ f32x2 cdf2(f32x2 x, f32x2 e) {
  const f32x2 ax = __builtin_elementwise_abs(x);
  const f32x2 d = pk_fma(splat(0.3275911f * 0.70710678118654752f), ax, splat(1.f));
  const f32x2 t = f32x2{__builtin_amdgcn_rcpf(d[0]), __builtin_amdgcn_rcpf(d[1])};
  f32x2 p = pk_fma(splat(0.5f * 1.061405429f), t, splat(0.5f * -1.453152027f));
  p = pk_fma(p, t, splat(0.5f * 1.421413741f));
  p = pk_fma(p, t, splat(0.5f * -0.284496736f));
  p = pk_fma(p, t, splat(0.5f * 0.254829592f));
  const f32x2 r = pk_fma(-p * t, e, splat(0.5f));  // 0.5 erf(|x| / sqrt 2)
  return splat(0.5f) + f32x2{copysignf(r[0], x[0]), copysignf(r[1], x[1])};
}
// exp(-x^2/2) via v_exp_f32 (2^y)
__device__ __forceinline__ f32x2 exp_neg_half_sq2(f32x2 x) {
  const f32x2 y = splat(-0.72134752044448170f) * x * x;
  return f32x2{__builtin_amdgcn_exp2f(y[0]), __builtin_amdgcn_exp2f(y[1])};
}
__device__ __forceinline__ f32x2 gelu2(f32x2 x) { return x * cdf2(x, exp_neg_half_sq2(x)); }
// tanh-approximated GELU (GPT-2): x * sigmoid(2u), u = sqrt(2/pi) (x + 0.044715 x^3)
__device__ __forceinline__ f32x2 sig2u(f32x2 x) {
  const f32x2 u = splat(-2.f * 0.7978845608028654f * 1.4426950408889634f) * pk_fma(splat(0.044715f) * x, x * x, x);
  const f32x2 d = splat(1.f) + f32x2{__builtin_amdgcn_exp2f(u[0]), __builtin_amdgcn_exp2f(u[1])};
  return f32x2{__builtin_amdgcn_rcpf(d[0]), __builtin_amdgcn_rcpf(d[1])};
}
__device__ __forceinline__ f32x2 gelu_tanh2(f32x2 x) { return x * sig2u(x); }
__device__ __forceinline__ f32x2 gelu_tanh_grad2(f32x2 x) {
  const f32x2 sg = sig2u(x);
  const f32x2 du = splat(2.f * 0.7978845608028654f) * pk_fma(splat(3.f * 0.044715f) * x, x, splat(1.f));
  return pk_fma(x * sg * (splat(1.f) - sg), du, sg);
}
// gelu(x) and gelu'(x) from one exp / erf (or one sigmoid for the tanh form)
__device__ __forceinline__ void gelu_and_grad2(f32x2 x, bool tanh_form, f32x2& y, f32x2& g) {
  if (tanh_form) {
    const f32x2 sg = sig2u(x);
    y = x * sg;
    const f32x2 du = splat(2.f * 0.7978845608028654f) * pk_fma(splat(3.f * 0.044715f) * x, x, splat(1.f));
    g = pk_fma(y * (splat(1.f) - sg), du, sg);
  } else {
    const f32x2 e = exp_neg_half_sq2(x);
    const f32x2 cdf = cdf2(x, e);
    y = x * cdf;
    g = pk_fma(x * splat(0.39894228040143268f), e, cdf);
  }
}
__device__ __forceinline__ f32x2 gelu_grad2(f32x2 x) {
  const f32x2 e = exp_neg_half_sq2(x);
  const f32x2 cdf = cdf2(x, e);
  return pk_fma(x * splat(0.39894228040143268f), e, cdf);
}

template <typename T>
__device__ __forceinline__ void load4(const T* p, float (&v)[4]) {
  Pack<T, 4> pk = *reinterpret_cast<const Pack<T, 4>*>(p);
#pragma unroll
  for (int i = 0; i < 4; ++i) v[i] = to_f(pk.v[i]);
}
template <typename T>
__device__ __forceinline__ void store4(T* p, const float (&v)[4]) {
  Pack<T, 4> pk;
#pragma unroll
  for (int i = 0; i < 4; ++i) pk.v[i] = from_f<T>(v[i]);
  *reinterpret_cast<Pack<T, 4>*>(p) = pk;
}

__device__ __forceinline__ s16x8 lds_frag(const char* tile, int r, int c) {
  return *reinterpret_cast<const s16x8*>(tile + r * 128 + ((c ^ ((r >> 1) & 7)) << 4));
}

__device__ __forceinline__ void bar() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

// One operand K-tile = 32 glds pieces of 1 KB; wave `wid` owns pieces wid*4 .. wid*4+3 and
// stage_pieces issues pieces [p0, p0+2) of them.
//  TR = false (operand [rows][K], K contiguous): piece = 8 rows x 128 B of K; image [256 rows][64 K],
//    chunk c of row r at c ^ ((r >> 1) & 7).
//  TR = true (operand stored [K][rows], rows contiguous — the weight-gradient GEMM, where the
//    contraction runs over tokens): piece = 2 K-rows x 512 B; image [64 K][256 rows], chunk c of
//    K-row r at c ^ ftr(r); fragments are gathered with ds_read_b64_tr_b16 (hardware transpose).
//    fp8 (the fp8 weight gradient): K-tile = 128 K-rows of 256 B, piece = 4 K-rows, chunk c of
//    K-row r at c ^ ftr8(r); fragments from ds_read_b64_tr_b8.
__device__ __forceinline__ int ftr(int r) { return 2 * (r & 3) + 8 * ((r >> 3) & 1); }
// A tr_b8 read's 32-lane half covers K-rows r0 + q and r0 + 16 + q (q = 0..7, r0 % 8 == 0), 8 bytes
// each of one 16-byte chunk: (r & 7) | bit 4 of r puts those 16 rows on 16 distinct slots (64 banks)
__device__ __forceinline__ int ftr8(int r) { return (r & 7) | (((r >> 4) & 1) << 3); }

template <typename T, bool TR>
__device__ __forceinline__ void stage_pieces(const T* __restrict__ g, int64_t ld, int row0, int rows, int k0,
                                             char* lds_tile, int wid, int lane, int p0) {
#pragma unroll
  for (int j = p0; j < p0 + 2; ++j) {
    const int piece = wid * 4 + j;
    if constexpr (TR) {
      constexpr int LPR = 16 * (int)sizeof(T);  // lanes (16-byte chunks) per K-row: 32 (16-bit), 16 (fp8)
      const int r = piece * (64 / LPR) + lane / LPR;
      const int chunk = (lane % LPR) ^ (sizeof(T) == 1 ? ftr8(r) : ftr(r));
      // partial tiles (rows % 256, e.g. GPT-2's 1600 / 4800): chunks past the last row read the
      // last full chunk instead (rows % 8 == 0) — they only feed output rows / columns the
      // bounds-checked epilogue does not store, and the last K-row never reads past the tensor
      int col = row0 + chunk * (16 / (int)sizeof(T));
      col = col < rows ? col : rows - 16 / (int)sizeof(T);
      glds16(g + (int64_t)(k0 + r) * ld + col, lds_tile + piece * 1024);
    } else {
      const int r = piece * 8 + (lane >> 3);
      const int chunk = (lane & 7) ^ ((r >> 1) & 7);
      int gr = row0 + r;
      gr = gr < rows ? gr : rows - 1;
      glds16(g + (int64_t)gr * ld + k0 + chunk * (16 / (int)sizeof(T)), lds_tile + piece * 1024);
    }
  }
}

typedef short s16x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ s16x4 lds_tr16(const char* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(p));
}
typedef int i32x2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ i32x2v lds_tr8(const char* p) {
  return __builtin_amdgcn_ds_read_tr8_b64_v2i32((__attribute__((address_space(3))) i32x2v*)(p));
}

// MFMA fragment for tile rows rb .. rb+15, K step s (32 wide): lane holds rows rb + lr,
// K = 32s + 8 lk .. +7. ES = operand element bytes (1: fp8, where the 16 bytes are K = 64s + 16lk ..
// +15, the chunk 4s + lk the NT image's lds_frag reads — see mfma_f8).
template <bool TR, int ES = 2>
__device__ __forceinline__ s16x8 frag(const char* tile, int rb, int s, int lr, int lk) {
  if constexpr (TR && ES == 1) {
    // two 8(K) x 16(rows) byte blocks (ds_read_b64_tr_b8): lane 2q+p of a 16-lane group addresses
    // K-row 64s + 16lk + 8h + q, rows rb + 8p .. +7; it receives row rb + lr, K-rows 8h .. 8h+7
    const int q = lr >> 1, pp = lr & 1;
    const int cl = rb >> 4;
    const int r0 = s * 64 + 16 * lk + q, r1 = r0 + 8;
    const i32x2v lo = lds_tr8(tile + r0 * 256 + ((cl ^ ftr8(r0)) << 4) + pp * 8);
    const i32x2v hi = lds_tr8(tile + r1 * 256 + ((cl ^ ftr8(r1)) << 4) + pp * 8);
    return __builtin_bit_cast(s16x8, i32x4{lo[0], lo[1], hi[0], hi[1]});
  } else if constexpr (TR) {
    // two 4(K) x 16(rows) transposed blocks: lane 4q+p of a 16-lane group addresses K-row
    // 32s + 8lk + 4h + q, rows rb + 4p .. +3; it receives row rb + lr, K 4h .. 4h+3
    const int q = lr >> 2, pp = lr & 3;
    const int cl = (rb >> 3) + (pp >> 1);
    const int r0 = s * 32 + 8 * lk + q, r1 = r0 + 4;
    const s16x4 lo = lds_tr16(tile + r0 * 512 + ((cl ^ ftr(r0)) << 4) + (pp & 1) * 8);
    const s16x4 hi = lds_tr16(tile + r1 * 512 + ((cl ^ ftr(r1)) << 4) + (pp & 1) * 8);
    return s16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  } else {
    return lds_frag(tile, rb + lr, s * 4 + lk);
  }
}

// Main loop schedule ("ping-pong", cdna_hip_programming.md §5 256² template, own phase plan):
// the 8 waves form two groups by M half (wr); group 1 runs one barrier behind group 0, so in
// every barrier interval one group issues its 16 MFMAs while the other issues its LDS reads
// and global->LDS copies on the same SIMDs. Per K-tile and wave, four phases, each
//   R: ds_read subtile, 2 glds pieces, [vmcnt], lgkmcnt(0)  | barrier
//   M: 16 x mfma_16x16x32 (one 64x32 quadrant, K = 64)      | barrier
//     p1  R: A rows mh=0 (8 frags) + B cols nh=0 (4)   stage A(t+1) pieces 0,1 -> other buffer
//     p2  R: B cols nh=1 (4)                           stage A(t+1) pieces 2,3
//     p3  R: A rows mh=1 (8)                           stage B(t+2) pieces 0,1 -> this buffer
//     p4  R: -                                         stage B(t+2) pieces 2,3; vmcnt(4)
//     quadrants (mh,nh): p1 (0,0)  p2 (0,1)  p3 (1,1)  p4 (1,0)
// WAR: B of this buffer is last read in p2 and A in p3; lgkmcnt(0) before each barrier retires
// the reads, so restaging one phase later (B(t+2) in p3) is safe; A(t+1) goes to the buffer whose
// A was last read in the previous tile's p3. RAW: vmcnt(4) in p4 retires everything but B(t+2)
// (i.e. A(t+1), B(t+1)) before the barrier that precedes the next tile's first read.
// Measured alternatives (profiles/r1_gemm_ksweep_variants.jsonl, same box, interleaved): LDS wait
// after the barrier with the glds moved to p2/p4 — within 1 %; BK = 32 with four buffers and one
// 32-MFMA phase per K-tile (half the barriers, loads 3 tiles ahead) — 12-15 % slower (the glds
// issue then sits inside the MFMA section); 256x128 tiles at two workgroups per CU (BK 32, three
// stages, no ping-pong; profiles/r1_gemm_*_2wg_variant.jsonl) — its epilogue does overlap the
// other workgroup's MFMAs (K = 64: 55 vs 65 us at N = 4096) but the main loop is ~60 % slower;
// two phases per K-tile with the whole tile read in the first R section (half the barriers, next
// loads 4 sections ahead, 256 VGPRs; profiles/r1_gemm_ksweep_2phase.jsonl) — within 1 %; the two
// glds pieces of each phase issued from inside the MFMA section (after 8 of its 16 MFMAs) instead
// of the R section, same buffers and waits (vmcnt(2) in R4) — 5-7 % slower on every BERT shape
// at M = 98304 (profiles/r2_gemm_glds_in_mma_ab.jsonl, same box).
// hipBLASLt's kernel on the same shape (rocprof): one wave per SIMD with 128x128 wave tiles (256
// AGPR accumulators), 74 % MFMA busy vs 64 % here. That geometry in HIP source (fragments
// software-pipelined under 64-MFMA halves) makes hipcc shuffle ~220 accumulator copies
// (v_accvgpr_read/write) per K-tile through the loop-carried phis, so it is not used. rocprof on the 32768x1024x4096 case: MFMA busy 65 %
// of SIMD cycles at 1.98 GHz, zero LDS bank conflicts.
template <typename T, bool TR, int FA, int FB, int DBG, bool FRESH = false>
__device__ __forceinline__ void mainloop_bk64_loop(const T* __restrict__ A, const T* __restrict__ B, int M, int N,
                                                   int K, int64_t lda, int64_t ldb, int m0, int n0, char* smem,
                                                   int wid, int wr, int wc, int lane, f32x4 (&acc)[4][8]);
template <typename T, bool TR, int FA = -1, int FB = -1, int DBG = 0>
__device__ __forceinline__ void mainloop_bk64(const T* __restrict__ A, const T* __restrict__ B, int M, int N, int K,
                                              int64_t lda, int64_t ldb, int m0, int n0, char* smem, int wid, int wr,
                                              int wc, int lane, f32x4 (&acc)[4][8]) {
  // one K-tile = 128 bytes of every row: 64 bf16/f16 elements or 128 fp8 ones
  constexpr bool F8 = FA >= 0;
  static_assert(!F8 || sizeof(T) == 1, "fp8: uint8 codes");
  constexpr int BKE = 128 / (int)sizeof(T);
  const int nt = K / BKE;
  // prologue: A(0), B(0) -> buf0, B(1) -> buf1; retire tile 0
  stage_pieces<T, TR>(A, lda, m0, M, 0, smem, wid, lane, 0);
  stage_pieces<T, TR>(A, lda, m0, M, 0, smem, wid, lane, 2);
  stage_pieces<T, TR>(B, ldb, n0, N, 0, smem + G_TILE_BYTES, wid, lane, 0);
  stage_pieces<T, TR>(B, ldb, n0, N, 0, smem + G_TILE_BYTES, wid, lane, 2);
  if (nt > 1) {
    stage_pieces<T, TR>(B, ldb, n0, N, BKE, smem + G_BUF_BYTES + G_TILE_BYTES, wid, lane, 0);
    stage_pieces<T, TR>(B, ldb, n0, N, BKE, smem + G_BUF_BYTES + G_TILE_BYTES, wid, lane, 2);
    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  bar();
  if (wr == 1) bar();  // stagger group 1 by one barrier
  mainloop_bk64_loop<T, TR, FA, FB, DBG>(A, B, M, N, K, lda, ldb, m0, n0, smem, wid, wr, wc, lane, acc);
}

// mainloop_bk64's K loop (tile 0 staged and retired, the wave groups staggered): also the fp8 body of
// the persistent kernel, which sets FRESH: the LDS-DMA source addresses are recomputed from a fresh
// lane id every K-tile instead of being kept in 16 VGPRs across the loop (there they spilled, and each
// reload waited, in vmcnt order, for every load and store in flight)
template <typename T, bool TR, int FA, int FB, int DBG, bool FRESH>
__device__ __forceinline__ void mainloop_bk64_loop(const T* __restrict__ A, const T* __restrict__ B, int M, int N,
                                                   int K, int64_t lda, int64_t ldb, int m0, int n0, char* smem,
                                                   int wid, int wr, int wc, int lane_in, f32x4 (&acc)[4][8]) {
  constexpr bool F8 = FA >= 0;
  constexpr int BKE = 128 / (int)sizeof(T);
  const int nt = K / BKE;
  const int lr = lane_in & 15, lk = lane_in >> 4;
  s16x8 fa[4][2], fb0[2][2], fb1[2][2];
  for (int t = 0; t < nt; ++t) {
    const int lane = FRESH ? lane_id_fresh() : lane_in;
    char* cur = smem + (t & 1) * G_BUF_BYTES;
    char* oth = smem + ((t + 1) & 1) * G_BUF_BYTES;
    const char* ta = cur;
    const char* tb = cur + G_TILE_BYTES;
    const bool ld_a = t + 1 < nt, ld_b = t + 2 < nt;
    // ---------------- p1: A mh=0, B nh=0; stage A(t+1) pieces 0,1 ----------------
#pragma unroll
    for (int j = 0; j < 2; ++j)
      if constexpr (!(DBG & 128)) for (int s = 0; s < 2; ++s) fb0[j][s] = frag<TR, sizeof(T)>(tb, wc * 64 + j * 16, s, lr, lk);
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if constexpr (!(DBG & 128)) for (int s = 0; s < 2; ++s) fa[i][s] = frag<TR, sizeof(T)>(ta, wr * 128 + i * 16, s, lr, lk);
    if (ld_a && !(DBG & 32)) stage_pieces<T, TR>(A, lda, m0, M, (t + 1) * BKE, oth, wid, lane, 0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if constexpr (!(DBG & 64)) bar();
    __builtin_amdgcn_s_setprio(1);
    if constexpr (F8) {
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[j][i] = mfma_f8<FB, FA>(fb0[j][0], fb0[j][1], fa[i][0], fa[i][1], acc[j][i]);
    } else {
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[j][i] = mfma16<T>(fb0[j][s], fa[i][s], acc[j][i]);
    }
    __builtin_amdgcn_s_setprio(0);
    if constexpr (!(DBG & 64)) bar();
    // ---------------- p2: B nh=1; stage A(t+1) pieces 2,3 ----------------
#pragma unroll
    for (int j = 0; j < 2; ++j)
      if constexpr (!(DBG & 128)) for (int s = 0; s < 2; ++s) fb1[j][s] = frag<TR, sizeof(T)>(tb, wc * 64 + 32 + j * 16, s, lr, lk);
    if (ld_a && !(DBG & 32)) stage_pieces<T, TR>(A, lda, m0, M, (t + 1) * BKE, oth, wid, lane, 2);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if constexpr (!(DBG & 64)) bar();
    __builtin_amdgcn_s_setprio(1);
    if constexpr (F8) {
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[2 + j][i] = mfma_f8<FB, FA>(fb1[j][0], fb1[j][1], fa[i][0], fa[i][1], acc[2 + j][i]);
    } else {
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[2 + j][i] = mfma16<T>(fb1[j][s], fa[i][s], acc[2 + j][i]);
    }
    __builtin_amdgcn_s_setprio(0);
    if constexpr (!(DBG & 64)) bar();
    // ---------------- p3: A mh=1; stage B(t+2) pieces 0,1 into this buffer ----------------
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if constexpr (!(DBG & 128)) for (int s = 0; s < 2; ++s) fa[i][s] = frag<TR, sizeof(T)>(ta, wr * 128 + 64 + i * 16, s, lr, lk);
    if (ld_b && !(DBG & 32)) stage_pieces<T, TR>(B, ldb, n0, N, (t + 2) * BKE, cur + G_TILE_BYTES, wid, lane, 0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if constexpr (!(DBG & 64)) bar();
    __builtin_amdgcn_s_setprio(1);
    if constexpr (F8) {
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[2 + j][4 + i] = mfma_f8<FB, FA>(fb1[j][0], fb1[j][1], fa[i][0], fa[i][1], acc[2 + j][4 + i]);
    } else {
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[2 + j][4 + i] = mfma16<T>(fb1[j][s], fa[i][s], acc[2 + j][4 + i]);
    }
    __builtin_amdgcn_s_setprio(0);
    if constexpr (!(DBG & 64)) bar();
    // ---------------- p4: stage B(t+2) pieces 2,3; retire A(t+1), B(t+1) ----------------
    if (ld_b) {
      if constexpr (!(DBG & 32)) stage_pieces<T, TR>(B, ldb, n0, N, (t + 2) * BKE, cur + G_TILE_BYTES, wid, lane, 2);
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    if constexpr (!(DBG & 64)) bar();
    __builtin_amdgcn_s_setprio(1);
    if constexpr (F8) {
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[j][4 + i] = mfma_f8<FB, FA>(fb0[j][0], fb0[j][1], fa[i][0], fa[i][1], acc[j][4 + i]);
    } else {
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[j][4 + i] = mfma16<T>(fb0[j][s], fa[i][s], acc[j][4 + i]);
    }
    __builtin_amdgcn_s_setprio(0);
    if constexpr (!(DBG & 64)) bar();
  }
}

// ---- "balanced" variant of the same schedule: the production main loop (DBG bit 1024 selects the
// one above, for lab A/B) ----------------------------------------------------------------------------
// The loop above reads 12 fragments in p1, 4 in p2, 8 in p3 and none in p4; p1's read section is the
// long pole of the ping-pong (the other group's 16-MFMA section has to cover it). Here the quadrant
// order alternates per K-tile — even tiles (0,0) (0,1) (1,1) (1,0), odd tiles (0,1) (0,0) (1,0) (1,1)
// — so the B half a tile starts with is the one its predecessor ended without, and p4 reads it from
// the other buffer for the next tile: 8 / 4 / 8 / 4 fragments per phase. That needs B(t+1) landed
// one phase earlier: p3 waits for it (vmcnt(6): only A(t+1) and B(t+2)'s first pieces stay in
// flight), and the barriers after p3 make it visible. WAR is unchanged: B(t+1) is last read in
// tile t+1's p2, before B(t+3) is staged over it in p3. Measured against the loop above
// (profiles/r4_gemm_balanced_loop.jsonl, same box, interleaved, outputs bit-identical): NT 8192^3
// 1.49 -> 1.53 PF/s, BERT M = 98304 shapes 1-5 % faster (FFN2 dgrad + residual 642 -> 618 us);
// transposed-read weight gradients 2-8 % (two ds_read_b64_tr_b16 per fragment: the read sections
// are longer there, so evening them out pays more).
template <bool TR, int ES = 2>
__device__ __forceinline__ void read_fa(s16x8 (&fa)[4][2], const char* ta, int rb, int lr, int lk) {
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int s = 0; s < 2; ++s) fa[i][s] = frag<TR, ES>(ta, rb + i * 16, s, lr, lk);
}
template <bool TR, int ES = 2>
__device__ __forceinline__ void read_fb(s16x8 (&fb)[2][2], const char* tb, int cb, int lr, int lk) {
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int s = 0; s < 2; ++s) fb[j][s] = frag<TR, ES>(tb, cb + j * 16, s, lr, lk);
}
template <typename T, int FA, int FB, int MH, int NH>
__device__ __forceinline__ void quad_mma(f32x4 (&acc)[4][8], const s16x8 (&fa)[4][2], const s16x8 (&fb)[2][2]) {
  __builtin_amdgcn_s_setprio(1);
  if constexpr (FA >= 0) {
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int i = 0; i < 4; ++i)
        acc[2 * NH + j][4 * MH + i] = mfma_f8<FB, FA>(fb[j][0], fb[j][1], fa[i][0], fa[i][1], acc[2 * NH + j][4 * MH + i]);
  } else {
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[2 * NH + j][4 * MH + i] = mfma16<T>(fb[j][s], fa[i][s], acc[2 * NH + j][4 * MH + i]);
  }
  __builtin_amdgcn_s_setprio(0);
}

template <typename T, bool TR, int FA, int FB, int DBG, int PAR>
__device__ __forceinline__ void bal_tile(int t, int nt, const T* __restrict__ A, const T* __restrict__ B, int M, int N,
                                         int64_t lda, int64_t ldb, int m0, int n0, char* smem, int wid, int wr, int wc,
                                         int lane, f32x4 (&acc)[4][8], s16x8 (&fa)[4][2], s16x8 (&fb)[2][2][2]) {
  constexpr int BKE = 128 / (int)sizeof(T);
  constexpr int OP = 1 - PAR;
  const int lr = lane & 15, lk = lane >> 4;
  // t & 1 == PAR, but kept opaque (an SGPR the compiler cannot fold): with a constant buffer base
  // per parity hipcc keeps separate fragment-address registers for both buffers and spills
  int pb = t & 1;
  asm("" : "+s"(pb));
  char* cur = smem + pb * G_BUF_BYTES;
  char* oth = smem + (pb ^ 1) * G_BUF_BYTES;
  const char* ta = cur;
  const char* tb = cur + G_TILE_BYTES;
  const bool ld_a = t + 1 < nt, ld_b = t + 2 < nt;
  constexpr bool RD = !(DBG & 128), GL = !(DBG & 32), BR = !(DBG & 64);
  // p1: A rows mh=0; stage A(t+1) pieces 0,1
  if constexpr (RD) read_fa<TR, sizeof(T)>(fa, ta, wr * 128, lr, lk);
  if (GL && ld_a) stage_pieces<T, TR>(A, lda, m0, M, (t + 1) * BKE, oth, wid, lane, 0);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  if constexpr (BR) bar();
  quad_mma<T, FA, FB, 0, PAR>(acc, fa, fb[PAR]);
  if constexpr (BR) bar();
  // p2: B half OP; stage A(t+1) pieces 2,3
  if constexpr (RD) read_fb<TR, sizeof(T)>(fb[OP], tb, wc * 64 + OP * 32, lr, lk);
  if (GL && ld_a) stage_pieces<T, TR>(A, lda, m0, M, (t + 1) * BKE, oth, wid, lane, 2);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  if constexpr (BR) bar();
  quad_mma<T, FA, FB, 0, OP>(acc, fa, fb[OP]);
  if constexpr (BR) bar();
  // p3: A rows mh=1; stage B(t+2) pieces 0,1 into this buffer; retire B(t+1) for p4
  if constexpr (RD) read_fa<TR, sizeof(T)>(fa, ta, wr * 128 + 64, lr, lk);
  if (ld_b) {
    if constexpr (GL) stage_pieces<T, TR>(B, ldb, n0, N, (t + 2) * BKE, cur + G_TILE_BYTES, wid, lane, 0);
    asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  } else if (ld_a) {
    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  if constexpr (BR) bar();
  quad_mma<T, FA, FB, 1, OP>(acc, fa, fb[OP]);
  if constexpr (BR) bar();
  // p4: next tile's first B half (OP) from the other buffer; stage B(t+2) pieces 2,3; retire A(t+1).
  // (Unconditional: after the last tile it reads stale LDS that nothing uses — a conditional load
  // would keep the old fragment live across the phase and cost registers.)
  if constexpr (RD) read_fb<TR, sizeof(T)>(fb[OP], oth + G_TILE_BYTES, wc * 64 + OP * 32, lr, lk);
  if (ld_b) {
    if constexpr (GL) stage_pieces<T, TR>(B, ldb, n0, N, (t + 2) * BKE, cur + G_TILE_BYTES, wid, lane, 2);
    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  if constexpr (BR) bar();
  quad_mma<T, FA, FB, 1, PAR>(acc, fa, fb[PAR]);
  if constexpr (BR) bar();
}

template <typename T, bool TR, int FA = -1, int FB = -1, int DBG = 0>
__device__ __forceinline__ void mainloop_bal(const T* __restrict__ A, const T* __restrict__ B, int M, int N, int K,
                                             int64_t lda, int64_t ldb, int m0, int n0, char* smem, int wid, int wr,
                                             int wc, int lane, f32x4 (&acc)[4][8]) {
  constexpr int BKE = 128 / (int)sizeof(T);
  const int nt = K / BKE;
  stage_pieces<T, TR>(A, lda, m0, M, 0, smem, wid, lane, 0);
  stage_pieces<T, TR>(A, lda, m0, M, 0, smem, wid, lane, 2);
  stage_pieces<T, TR>(B, ldb, n0, N, 0, smem + G_TILE_BYTES, wid, lane, 0);
  stage_pieces<T, TR>(B, ldb, n0, N, 0, smem + G_TILE_BYTES, wid, lane, 2);
  if (nt > 1) {
    stage_pieces<T, TR>(B, ldb, n0, N, BKE, smem + G_BUF_BYTES + G_TILE_BYTES, wid, lane, 0);
    stage_pieces<T, TR>(B, ldb, n0, N, BKE, smem + G_BUF_BYTES + G_TILE_BYTES, wid, lane, 2);
    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  bar();
  if (wr == 1) bar();  // stagger group 1 by one barrier
  s16x8 fa[4][2], fb[2][2][2];
  const int lr = lane & 15, lk = lane >> 4;
  if constexpr (!(DBG & 128)) read_fb<TR, sizeof(T)>(fb[0], smem + G_TILE_BYTES, wc * 64, lr, lk);  // tile 0's first B half
  int t = 0;
  for (; t + 1 < nt; t += 2) {
    bal_tile<T, TR, FA, FB, DBG, 0>(t, nt, A, B, M, N, lda, ldb, m0, n0, smem, wid, wr, wc, lane, acc, fa, fb);
    bal_tile<T, TR, FA, FB, DBG, 1>(t + 1, nt, A, B, M, N, lda, ldb, m0, n0, smem, wid, wr, wc, lane, acc, fa, fb);
  }
  if (t < nt) bal_tile<T, TR, FA, FB, DBG, 0>(t, nt, A, B, M, N, lda, ldb, m0, n0, smem, wid, wr, wc, lane, acc, fa, fb);
}

// Buffer resource for a wave-uniform base address (the epilogue's full-tile path): every lane
// addresses rows through ONE 32-bit voffset plus an SGPR soffset per row slot, instead of a 64-bit
// VGPR address pair per access (32 pairs per lane for a load+store epilogue, which the scheduler
// hoisted and spilled). Inputs go through readfirstlane so no waterfall loop is emitted
// (cdna_hip_programming.md T8 / T20).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t wave_rsrc(const void* p, uint32_t bytes) {
  const uint64_t a = (uint64_t)p;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), (short)0,
                                           (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}

// Epilogue shared by both kernels (wave tile 128 x 64 at rows m0 + wr*128, cols n0 + wc*64).
// Rounds the accumulators of a 128 x 64 wave tile (acc[J0 .. J0+3][*]) to T and writes them into the
// wave's 16 KB LDS region in the layout the epilogue reads back (see epilogue()).
// I0 / NI: the fragment rows staged (NI = 4: one 64-row half of the wave tile into an 8 KB region,
// local rows 0..63; the row's XOR pattern only depends on row & 15, so it is the same either way)
template <typename T, int J0, int NJ, int I0 = 0, int NI = 8>
__device__ __forceinline__ void stage_acc(const f32x4 (&acc)[NJ][8], char* reg, int lane, float alpha) {
  const int lr = lane & 15, lk = lane >> 4;
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int ii = 0; ii < NI; ++ii) {
      const int i = I0 + ii;
      const int row = ii * 16 + lr;
      const int chunk = (2 * j + (lk >> 1)) ^ (row & 7);
      const int half = (lk & 1) ^ ((row >> 3) & 1);
      Pack<T, 4> pk;
#pragma unroll
      for (int e = 0; e < 4; ++e) pk.v[e] = from_f<T>(acc[J0 + j][i][e] * alpha);
      *reinterpret_cast<Pack<T, 4>*>(reg + row * 128 + chunk * 16 + half * 8) = pk;
    }
}

// STAGED: the accumulators are already in `reg` (stage_acc), `acc` is not read
// Q8 (1 + fp8 format, 0 = off): the C output's fp8 codes are written too (q8.y, ldc bytes per row,
// scaled by q8.scale[0], max|C| into q8.amax) — the next GEMM's fp8 operand without a standalone
// quantise pass over C
// Loads the compiler does not see (the persistent kernel's epilogue): with LDS-DMA pieces of the next
// tile in flight, hipcc waits vmcnt(0) before the first use of any load it issued itself, i.e. the
// epilogue would stall on the next tile's prologue. These load through a descriptor held in SGPRs
// (built from wave-uniform values: s_nop 4 covers the SGPR-write -> buffer-read hazard) and are
// retired by explicit counted waits (asm_wait8 / asm_wait16) that name every destination register.
typedef unsigned u32x4g __attribute__((ext_vector_type(4)));
typedef int i32x4s __attribute__((ext_vector_type(4)));
__device__ __forceinline__ i32x4s sgpr_rsrc(const void* p, uint32_t bytes) {
  const uint64_t a = (uint64_t)p;
  return i32x4s{(int)__builtin_amdgcn_readfirstlane((uint32_t)a),
                (int)__builtin_amdgcn_readfirstlane((uint32_t)(a >> 32)) & 0xffff,
                (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000};
}
__device__ __forceinline__ u32x4g asm_load16(const i32x4s& rs, uint32_t voff, int soff) {
  u32x4g d;
  asm volatile("s_nop 4\n\tbuffer_load_dwordx4 %0, %1, %2, %3 offen" : "=v"(d) : "v"(voff), "s"(rs), "s"(soff) : "memory");
  return d;
}
template <int N>
__device__ __forceinline__ void asm_wait(u32x4g (&r)[8]) {
  asm volatile("s_waitcnt vmcnt(%8)"
               : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]), "+v"(r[6]), "+v"(r[7])
               : "n"(N)
               : "memory");
  __builtin_amdgcn_sched_barrier(0);
}
template <int N>
__device__ __forceinline__ void asm_wait1(u32x4g& r) {
  asm volatile("s_waitcnt vmcnt(%1)" : "+v"(r) : "n"(N) : "memory");
  __builtin_amdgcn_sched_barrier(0);
}
struct NoHook {
  __device__ __forceinline__ void operator()() const {}
};

// HALVES (the persistent kernel): `reg` is an 8 KB region; each 64-row half of the wave tile is staged
// into it right before its 8 row slots are read back (the other 64 KB of LDS hold the next tile's
// first K-tile meanwhile)
// With HALVES the epilogue's own loads (bias, [M, N] input) are asm loads issued BEFORE `pre()` (the
// caller's hook: the next tile's LDS-DMA pieces, exactly 8 per wave) and retired by counted waits that
// leave those pieces (and this epilogue's stores) in flight.
// XD (lab diagnostics, tools/gemmlab; production 0): bit 0 skips the epilogue math (the stored values
// are the rounded accumulators, same loads and stores), bit 1 skips every global store of the epilogue,
// bit 2 stores the second output (H / gelu') non-temporally, bit 3 stores C non-temporally.
// Bit 4 (production, fp8 codes-only outputs, Q8Out::only): C itself is not stored — its fp8 codes
// (and the GELU_D derivative / the MUL bias-grad partials) are: the fp8 step's consumers of the MLP
// hidden activation and its gradient read only the codes (apex.fp8 codes_only_ok)
template <typename T, int EPI, bool EDGE, int J0 = 0, int NJ = 4, bool STAGED = false, int Q8 = 0,
          bool HALVES = false, typename Hook = NoHook, int XD = 0>
__device__ __forceinline__ void epilogue(const f32x4 (&acc)[NJ][8], char* reg, T* __restrict__ C, int M, int N,
                                         int64_t ldc, const T* __restrict__ bias, const T* __restrict__ aux,
                                         int64_t ldaux, T* __restrict__ aux_out, float* __restrict__ part, int m0,
                                         int n0, int tm, int wr, int wc, int lane, float alpha = 1.f,
                                         const Q8Out& q8 = Q8Out{}, const Hook& pre = Hook{},
                                         float* q8_defer = nullptr) {
  // HALVES + Q8: the codes of the multiply / dGELU epilogues are stashed and emitted per half, and the
  // running max|C| goes to *q8_defer (the persistent kernel issues one amax atomic per workgroup at its
  // end: an atomic here would sit between the next tile's LDS-DMA pieces and their counted wait)
  static_assert(!HALVES || (!STAGED && !EDGE), "halved staging: full tiles, accumulators in registers");
  const int lr = lane & 15, lk = lane >> 4;
  // acc[j][i] holds rows wr*128 + i*16 + lr, cols wc*64 + j*16 + 4*lk .. +3 of the tile. The fp32
  // accumulators are rounded to T and transposed through the wave's own 16 KB LDS region
  // ([128 rows][64 cols], 16-B chunks XOR-swizzled by row, 8-B halves swapped on rows 8..15 of every
  // 16 so the ds_write_b64 groups are conflict-free); then every lane owns 8 consecutive columns of
  // 16 rows ("row slots" it = 0..15, rows lane/8 + 8 it of the wave tile), and the epilogue math
  // (bias, GELU, dGELU, residual) runs on 16-byte vectors with 16-byte loads/stores (8 lanes = one
  // 128-B row run). Rounding before the bias matches the unfused composition (GEMM output in T,
  // then the bias/activation kernel in fp32).
  //
  // Register budget (the kernel runs at 256 VGPRs): the slots are processed in two halves of 8, and
  // the [M, N] input operand of EPI_RESID / EPI_MUL / EPI_DGELU is loaded a half AHEAD — the first
  // half's 8 x 16 B per lane are issued before the accumulators go through LDS (the HBM latency
  // hides behind the transposition), the second half's while the first half computes and stores.
  // Global accesses go through buffer resources based at the wave tile's origin: full tiles use one
  // per-lane voffset plus an SGPR soffset per slot; edge tiles a per-slot voffset that points past
  // the resource for rows >= M or columns >= N (loads return 0, stores are dropped). With 64-bit
  // flat addresses per access and all 16 slots at once, these epilogues spilled 120-340 B per lane
  // to scratch (137 scratch instructions in EPI_MUL).
  // Measured alternative (profiles/r2_gemm_regroup_epilogue_ab.jsonl): the accumulators regrouped
  // in registers by v_permlane16_swap instead of the LDS transposition (no LDS, no barrier, every
  // lane 8 consecutive columns) — correct, but 2-10 % SLOWER (FFN2 dgrad x gelu' 796 -> 869 us):
  // each 16-byte-per-lane access then covers 16 rows x 64 B instead of 8 rows x 128 B.
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  constexpr bool GELU_D = EPI == EPI_BIAS_GELU_D || EPI == EPI_BIAS_GELU_TANH_D;
  constexpr bool GELU_FWD = EPI == EPI_BIAS_GELU || EPI == EPI_BIAS_GELU_TANH || GELU_D;
  constexpr bool DGELU = EPI == EPI_DGELU || EPI == EPI_DGELU_TANH;
  constexpr bool MUL = EPI == EPI_MUL;
  constexpr bool COLSUM = DGELU || MUL;
  constexpr bool TANH = EPI == EPI_BIAS_GELU_TANH || EPI == EPI_DGELU_TANH || EPI == EPI_BIAS_GELU_TANH_D;
  constexpr bool AUX_IN = DGELU || MUL || EPI == EPI_RESID;

  const int ncol = n0 + wc * 64 + (lane & 7) * 8;
  const int wrow0 = m0 + wr * 128, wcol0 = n0 + wc * 64;
  const int lrow = lane >> 3, lcol = (lane & 7) * 8;
  auto wave_res = [&](const T* base, int64_t ld) {
    return wave_rsrc(base + (int64_t)wrow0 * ld + wcol0, (uint32_t)(128 * ld * (int64_t)sizeof(T)));
  };
  // bounds-aware per-slot offset (any tile)
  auto voff_g = [&](int64_t ld, int slot) -> uint32_t {
    const int r = lrow + slot * 8;
    return (wrow0 + r < M && ncol < N) ? (uint32_t)((r * ld + lcol) * (int64_t)sizeof(T)) : 0x80000000u;
  };
  const __amdgpu_buffer_rsrc_t rs_c = wave_res(C, ldc);
  __amdgpu_buffer_rsrc_t rs_o = rs_c, rs_x = rs_c, rs_q = rs_c;
  float q8s = 0.f, q8mx = 0.f;
  if constexpr (Q8 != 0) {
    q8s = q8.scale[0];
    rs_q = wave_rsrc(q8.y + (int64_t)wrow0 * ldc + wcol0, (uint32_t)(128 * ldc));
  }
  if constexpr (GELU_FWD) rs_o = wave_res(aux_out, ldc);
  if constexpr (AUX_IN) rs_x = wave_res(aux, ldaux);
  auto unpack = [&](const u32x4& x, float (&v)[8]) {
    Pack<T, 8> pk = *reinterpret_cast<const Pack<T, 8>*>(&x);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = to_f(pk.v[e]);
  };
  auto pack = [&](const float (&v)[8]) {
    Pack<T, 8> pk;
#pragma unroll
    for (int e = 0; e < 8; ++e) pk.v[e] = from_f<T>(v[e]);
    return *reinterpret_cast<const u32x4*>(&pk);
  };

  // F (EDGE = false: the launch has only full tiles, M % 256 == 0 and N % 256 == 0) or the
  // bounds-checked form for every tile. One variant per kernel, no runtime branch: with both
  // variants in one kernel the compiler hoisted their common code (conversions, LDS reads,
  // unpacks) above the branch and spilled.
  {
    constexpr bool F = !EDGE;
    auto voff = [&](int64_t ld, int slot) -> uint32_t {
      if constexpr (F) return (uint32_t)((lrow * ld + lcol) * (int64_t)sizeof(T));
      return voff_g(ld, slot);
    };
    auto soff = [&](int64_t ld, int slot) -> int { return F ? (int)(slot * 8 * ld * (int64_t)sizeof(T)) : 0; };
    // stores take the slot offset in voffset with soffset = 0: with a register soffset hipcc
    // (ROCm 7.2) does not count the gfx950 store-data hazard — a VALU overwrote the data VGPRs of
    // a buffer_store_dwordx4 right after issue and corrupted a dword of the stored row (seen on
    // the GPU: sporadic dwords of EPI_BIAS_GELU's pre-activation output)
    // non-temporal stores (build options above; XD bits 2 / 3 force them in the lab): nt on the second
    // output (H / gelu') and / or on C
    constexpr int NTX = XD | (HALVES && GELU_D && APEX_GEMM_NT_GELU_D ? 12 : 0) |
                        (HALVES && (EPI == EPI_NONE || EPI == EPI_BIAS) && APEX_GEMM_NT_PLAIN ? 8 : 0);
    auto st = [&](const __amdgpu_buffer_rsrc_t& rs, int slot, const u32x4& x) {
      if constexpr (XD & 2) {  // no store: keep the value live
        asm volatile("" ::"v"(x));
      } else if constexpr (NTX & 12) {  // non-temporal: aux 2 = nt
        const bool o = &rs == &rs_o;
        if (o ? (NTX & 4) : (NTX & 8))
          __builtin_amdgcn_raw_buffer_store_b128(x, rs, voff(ldc, slot) + (uint32_t)soff(ldc, slot), 0, 2);
        else
          __builtin_amdgcn_raw_buffer_store_b128(x, rs, voff(ldc, slot) + (uint32_t)soff(ldc, slot), 0, 0);
      } else {
        __builtin_amdgcn_raw_buffer_store_b128(x, rs, voff(ldc, slot) + (uint32_t)soff(ldc, slot), 0, 0);
      }
    };
    // first half of the input operand in flight (sched_barriers pin the phase order: left alone,
    // the scheduler hoists both halves' loads above the transposition and spills around them)
    u32x4 ra[8];
    constexpr bool HAS_BIAS = EPI == EPI_BIAS || GELU_FWD;
    u32x4g braw = u32x4g{0u, 0u, 0u, 0u};
    i32x4s rsx_s = i32x4s{0, 0, 0, 0};
    if constexpr (HALVES) {
      if constexpr (AUX_IN) {
        rsx_s = sgpr_rsrc(aux + (int64_t)wrow0 * ldaux + wcol0, (uint32_t)(128 * ldaux * (int64_t)sizeof(T)));
#pragma unroll
        for (int it = 0; it < 8; ++it) ra[it] = asm_load16(rsx_s, voff(ldaux, it), soff(ldaux, it));
        pre();
        __builtin_amdgcn_sched_barrier(0);
        stage_acc<T, J0, NJ, 0, 4>(acc, reg, lane, alpha);
        __builtin_amdgcn_sched_barrier(0);
        asm_wait<8>(ra);  // the 8 pieces of pre() are younger
      } else {
        if constexpr (HAS_BIAS) braw = asm_load16(sgpr_rsrc(bias + n0 + wc * 64, 128), (uint32_t)((lane & 7) * 16), 0);
        pre();
        __builtin_amdgcn_sched_barrier(0);
        stage_acc<T, J0, NJ, 0, 4>(acc, reg, lane, alpha);
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (HAS_BIAS) asm_wait1<8>(braw);
      }
    } else if constexpr (AUX_IN) {
#pragma unroll
      for (int it = 0; it < 8; ++it) ra[it] = __builtin_amdgcn_raw_buffer_load_b128(rs_x, voff(ldaux, it), soff(ldaux, it), 0);
    }
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (!STAGED && !HALVES) stage_acc<T, J0, NJ>(acc, reg, lane, alpha);
    __builtin_amdgcn_sched_barrier(0);
    float bv[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if constexpr (HAS_BIAS) {
      if constexpr (HALVES) {
        unpack(*reinterpret_cast<const u32x4*>(&braw), bv);
      } else {
        const int nc = ncol < N ? ncol : N - 8;  // (N % 8 == 0: edge lanes read a valid chunk, unused)
        unpack(*reinterpret_cast<const u32x4*>(bias + nc), bv);
      }
    }
    float csum[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    u32x4 rb[8];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      u32x4 rc[8];
      if constexpr (HALVES) {
        if (h == 1) {  // (half 0 was staged before the first wait; LDS ops of one wave run in order)
          stage_acc<T, J0, NJ, 4, 4>(acc, reg, lane, alpha);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
#pragma unroll
      for (int it = 0; it < 8; ++it) {
        const int row = ((HALVES ? 0 : 8 * h) + it) * 8 + lrow, c = lane & 7;
        u32x4 x = *reinterpret_cast<const u32x4*>(reg + row * 128 + ((c ^ (row & 7)) << 4));
        if ((row >> 3) & 1) x = u32x4{x[2], x[3], x[0], x[1]};
        rc[it] = x;
      }
      if constexpr (AUX_IN) {
        if constexpr (HALVES) {
          // second half of the input: issued now, retired at h = 1 behind the 8 stores of h = 0
          if (h == 0) {
#pragma unroll
            for (int it = 0; it < 8; ++it) rb[it] = asm_load16(rsx_s, voff(ldaux, 8 + it), soff(ldaux, 8 + it));
          } else {
            asm_wait<Q8 != 0 ? 16 : 8>(rb);  // (half 0's stores, and with Q8 its codes, are younger)
          }
        } else if (h == 0) {
#pragma unroll
          for (int it = 0; it < 8; ++it)
            rb[it] = __builtin_amdgcn_raw_buffer_load_b128(rs_x, voff(ldaux, 8 + it), soff(ldaux, 8 + it), 0);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int it = 0; it < 8; ++it) {
        const int slot = 8 * h + it;
        u32x4 out = rc[it];
        if constexpr ((XD & 1) && EPI != EPI_NONE) {  // same bytes, no math
          if constexpr (GELU_D) st(rs_o, slot, out);
          if constexpr (AUX_IN) out = out ^ (h == 0 ? ra[it] : rb[it]);
        } else if constexpr (EPI != EPI_NONE) {
          float v[8];
          unpack(rc[it], v);
          if constexpr (EPI == EPI_BIAS) {
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] += bv[e];
          } else if constexpr (GELU_FWD) {
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] += bv[e];
            if constexpr (!GELU_D) {
              const u32x4 hraw = pack(v);
              st(rs_o, slot, hraw);
              unpack(hraw, v);  // GELU of the stored (rounded) pre-activation: what the backward's dGELU sees
            }
            // GELU_D stores no pre-activation: gelu and gelu' both come from the fp32 H here (no
            // round trip through 16 bits: 12 VALU instructions per 8 elements fewer)
            float gd[8];
#pragma unroll
            for (int e = 0; e < 8; e += 2) {
              if constexpr (GELU_D) {
                f32x2 gv, gg;
                gelu_and_grad2(f32x2{v[e], v[e + 1]}, TANH, gv, gg);
                v[e] = gv[0];
                v[e + 1] = gv[1];
                gd[e] = gg[0];
                gd[e + 1] = gg[1];
              } else {
                const f32x2 gv = TANH ? gelu_tanh2(f32x2{v[e], v[e + 1]}) : gelu2(f32x2{v[e], v[e + 1]});
                v[e] = gv[0];
                v[e + 1] = gv[1];
              }
            }
            if constexpr (GELU_D) st(rs_o, slot, pack(gd));
          } else {
            float x[8];
            unpack(h == 0 ? ra[it] : rb[it], x);
            const bool ok = F || (wrow0 + lrow + 8 * slot < M && ncol < N);
#pragma unroll
            for (int e = 0; e < 8; e += 2) {
              if constexpr (DGELU) {
                const f32x2 gg = TANH ? gelu_tanh_grad2(f32x2{x[e], x[e + 1]}) : gelu_grad2(f32x2{x[e], x[e + 1]});
                v[e] = ok ? v[e] * gg[0] : 0.f;
                v[e + 1] = ok ? v[e + 1] * gg[1] : 0.f;
              } else if constexpr (MUL) {
                v[e] = ok ? v[e] * x[e] : 0.f;
                v[e + 1] = ok ? v[e + 1] * x[e + 1] : 0.f;
              } else {
                v[e] += x[e];
                v[e + 1] += x[e + 1];
              }
            }
          }
          out = pack(v);
          if constexpr (COLSUM || Q8 != 0) {
            float r[8];
            unpack(out, r);  // the bias grad / the fp8 codes take the stored (rounded) values
            if constexpr (COLSUM) {
#pragma unroll
              for (int e = 0; e < 8; ++e) csum[e] += r[e];
              // fp8 codes later, from LDS: the slot's chunk (read above, this lane's alone) takes the
              // stored value back — inline, the codes' live ranges spilled ~100 VGPRs in these variants
              if constexpr (Q8 != 0) {
                const int row = (HALVES ? it : slot) * 8 + lrow;
                *reinterpret_cast<u32x4*>(reg + row * 128 + (((lane & 7) ^ (row & 7)) << 4)) = out;
              }
            }
            if constexpr (Q8 != 0 && !COLSUM) {
              typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
#pragma unroll
              for (int e = 0; e < 8; ++e) {
                q8mx = fmaxf(q8mx, fabsf(r[e]));
                r[e] *= q8s;
              }
              const u32x2 w = u32x2{f8_pack4<Q8 - 1>(r[0], r[1], r[2], r[3]), f8_pack4<Q8 - 1>(r[4], r[5], r[6], r[7])};
              const int qr = lrow + slot * 8;
              const uint32_t qo = (F || (wrow0 + qr < M && ncol < N)) ? (uint32_t)(qr * ldc + lcol) : 0x80000000u;
              __builtin_amdgcn_raw_buffer_store_b64(w, rs_q, qo, 0, 0);
            }
          }
        }
        if constexpr (!(XD & 16)) st(rs_c, slot, out);
        // one slot at a time: unpacking every slot's operands up front (16 bf16 -> 16 fp32 per
        // slot, hoisted by the scheduler) is what pushed these epilogues past 256 VGPRs
        __builtin_amdgcn_sched_barrier(0);
      }
      if constexpr (HALVES && Q8 != 0 && COLSUM) {  // this half's stashed outputs -> fp8 codes
        typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
#pragma unroll 4
        for (int it = 0; it < 8; ++it) {
          const int row = it * 8 + lrow;
          float r[8];
          unpack(*reinterpret_cast<const u32x4*>(reg + row * 128 + (((lane & 7) ^ (row & 7)) << 4)), r);
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            q8mx = fmaxf(q8mx, fabsf(r[e]));
            r[e] *= q8s;
          }
          const u32x2 w = u32x2{f8_pack4<Q8 - 1>(r[0], r[1], r[2], r[3]), f8_pack4<Q8 - 1>(r[4], r[5], r[6], r[7])};
          __builtin_amdgcn_raw_buffer_store_b64(w, rs_q, (uint32_t)(((8 * h + it) * 8 + lrow) * ldc + lcol), 0, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    if constexpr (COLSUM) {
      // lanes l, l^8, l^16, ... share the column chunk: reduce over the wave's 8 row slots
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float x = csum[e];
        x += __shfl_xor(x, 8, 64);
        x += __shfl_xor(x, 16, 64);
        x += __shfl_xor(x, 32, 64);
        csum[e] = x;
      }
      // waves wc = 0..3 of one wr cover disjoint columns: one partial row per (tile, wr)
      if (!(XD & 2) && lane < 8 && ncol < N) {
        float* pp = part + (int64_t)(tm * 2 + wr) * N + ncol;
        *reinterpret_cast<f32x4*>(pp) = f32x4{csum[0], csum[1], csum[2], csum[3]};
        *reinterpret_cast<f32x4*>(pp + 4) = f32x4{csum[4], csum[5], csum[6], csum[7]};
      }
    }
    if constexpr (Q8 != 0 && COLSUM && !HALVES) {  // the stashed outputs -> fp8 codes
      typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
#pragma unroll 4
      for (int slot = 0; slot < 16; ++slot) {
        const int row = slot * 8 + lrow;
        float r[8];
        unpack(*reinterpret_cast<const u32x4*>(reg + row * 128 + (((lane & 7) ^ (row & 7)) << 4)), r);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          q8mx = fmaxf(q8mx, fabsf(r[e]));
          r[e] *= q8s;
        }
        const u32x2 w = u32x2{f8_pack4<Q8 - 1>(r[0], r[1], r[2], r[3]), f8_pack4<Q8 - 1>(r[4], r[5], r[6], r[7])};
        const uint32_t qo = (F || (wrow0 + row < M && ncol < N)) ? (uint32_t)(row * ldc + lcol) : 0x80000000u;
        __builtin_amdgcn_raw_buffer_store_b64(w, rs_q, qo, 0, 0);
      }
    }
    if constexpr (Q8 != 0 && HALVES) {
      *q8_defer = fmaxf(*q8_defer, q8mx);
    } else if constexpr (Q8 != 0) {  // one amax atomic per wave, filtered by a plain read (amax only grows)
      const float m = f8_wave_max(q8mx);
      if (lane == 0 && m > 0.f && m > *(volatile float*)q8.amax) f8_atomic_max_pos(q8.amax, m);
    }
  }
}

// Launch control word (kernel argument `ctl`, no device-variable load in the kernel): bits 0..14
// first-round stagger units, bit 15 the split-major XCD remap (kCtlSplitXcd), bits 16.. diagnostics mode (2 = skip the epilogue: main-loop-only
// timing, tools/gemm_epi_cost.py). Both are host statics set by gemm_set_dbg().
// First-round stagger (experiment, off by default): half of the first round's workgroups (bid & 8)
// sleep `units` x s_sleep(127) before starting, offsetting every later tile on those CUs so their
// epilogues run beside the other half's main loops. Isolated GEMMs at M = 32768 (tools/gemm_stagger.py):
// bias+GELU 362 -> 312 us; the BERT step was 2.4 % SLOWER (profiles/r1_gemm_stagger.json); at
// M = 98304 no unit count helps any fused shape (profiles/r3_gemmlab_w8_stagger.jsonl).
int h_gemm_dbg = 0, h_gemm_stagger = 0;  // stagger: > 0 forced units, < 0 forced off, 0 launcher's
// ctl bit 15: split-major XCD remap of split-K (transposed-read) launches, APEX_GEMM_SPLIT_XCD=0 turns
// it off (A/B)
constexpr int kCtlSplitXcd = 0x8000;
inline bool host_split_xcd() {
  static int on = -1;
  if (on == -1) {
    const char* e = getenv("APEX_GEMM_SPLIT_XCD");
    on = (e && e[0] == '0') ? 0 : 1;
  }
  return on == 1;
}

// T: output / epilogue dtype; TI: operand dtype (T, or uint8_t fp8 with formats FA (A) / FB (B) and
// the dequantisation alpha = alpha_a[0] * alpha_b[0] read on the device)
template <typename T, int EPI, bool TR, bool EDGE, typename TI = T, int FA = -1, int FB = -1, int DBG = 0,
          int Q8 = 0, bool NOC = false>
__global__ void __launch_bounds__(G_THREADS) gemm_nt_kernel(const TI* __restrict__ A, const TI* __restrict__ B,
                                                            T* __restrict__ C, int M, int N, int K, int64_t lda,
                                                            int64_t ldb, int64_t ldc, const T* __restrict__ bias,
                                                            const T* __restrict__ aux, int64_t ldaux,
                                                            T* __restrict__ aux_out, float* __restrict__ part,
                                                            int ctl, const float* __restrict__ alpha_a = nullptr,
                                                            const float* __restrict__ alpha_b = nullptr,
                                                            Q8Out q8 = Q8Out{}) {
  __shared__ __attribute__((aligned(16))) char smem[G_LDS_BYTES];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid >> 2, wc = wid & 3;
  const int lr = lane & 15, lk = lane >> 4;

  // ---- tile mapping: bijective XCD remap, then GROUP_M panel order ----
  const int tiles_m = (M + GB_M - 1) / GB_M, tiles_n = (N + GB_N - 1) / GB_N;
  const int nwg = tiles_m * tiles_n;
  const int bid = blockIdx.x;
  int wg, split = TR ? (int)blockIdx.y : 0;
  if (TR && (ctl & kCtlSplitXcd) && gridDim.y > 1) {
    // split-K: the remap runs over (split, tile) jointly in dispatch order, split-major, so the
    // workgroups an XCD holds share one K-range and meet each other's A / B panels in its L2 (tile-
    // major, each dY panel of a weight gradient was streamed by every XCD holding one of its tiles)
    const int L = bid + nwg * (int)blockIdx.y, nall = nwg * (int)gridDim.y;
    const int xcd = L & 7, q = nall >> 3, rr = nall & 7;
    const int v = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (L >> 3);
    split = v / nwg;
    wg = v - split * nwg;
  } else {
    const int xcd = bid & 7, q = nwg >> 3, rr = nwg & 7;
    wg = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (bid >> 3);
  }
  const int group = G_GROUP_M * tiles_n;
  const int first_m = (wg / group) * G_GROUP_M;
  const int gm = min(tiles_m - first_m, G_GROUP_M);
  const int tm = first_m + (wg % group) % gm;
  const int tn = (wg % group) / gm;
  const int m0 = tm * GB_M, n0 = tn * GB_N;

  f32x4 acc[4][8];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
  // DBG bit 2048 (lab timeline trace, bf16 kernels only): per workgroup the 100 MHz real-time clock at
  // start, after the main loop and after the epilogue's stores completed, plus HW_ID / XCC_ID, into
  // the uint64 buffer passed as alpha_a (unused by the 16-bit kernels)
  uint64_t tr0 = 0, tr1 = 0;
  if constexpr (DBG & 2048) tr0 = __builtin_amdgcn_s_memrealtime();

  {
    const int st = ctl & 0x7fff;
    if (st > 0 && bid < 256 && (bid & 8)) {
      for (int i = 0; i < st; ++i) __builtin_amdgcn_s_sleep(127);
    }
  }
  if constexpr (TR) {
    // split-K slice of the transposed-read launches: K = ALL contraction rows, cut into gridDim.y slices
    // of whole K-tiles, [split * T / S, (split + 1) * T / S) for T K-tiles (the slices differ by at most
    // one K-tile: any slice count fills the CUs, e.g. BERT's QKV weight gradient, 48 tiles, at 5 slices
    // = 240 workgroups where 4 gave 192)
    constexpr int BKT = 128 / (int)sizeof(TI);  // rows per K-tile (64 16-bit, 128 fp8)
    const int nkt = K / BKT, ns = (int)gridDim.y;
    const int kb = (int)((int64_t)split * nkt / ns), ke = (int)((int64_t)(split + 1) * nkt / ns);
    A += (int64_t)kb * BKT * lda;
    B += (int64_t)kb * BKT * ldb;
    K = (ke - kb) * BKT;
  }
  // mainloop_bal for the 16-bit kernels; the fp8 instantiations and the edge-tile dGELU / multiply
  // epilogues keep the previous schedule (their epilogues hold more registers: the balanced loop's
  // extra live fragment spilled 50-240 VGPRs in fp8, 2 -> 52 in edge EPI_MUL). DBG bit 1024 forces
  // the previous one (lab A/B).
  constexpr bool EDGE_HEAVY = EDGE && (EPI == EPI_MUL || EPI == EPI_DGELU || EPI == EPI_DGELU_TANH);
  if constexpr ((DBG & 1024) || FA >= 0 || EDGE_HEAVY)
    mainloop_bk64<TI, TR, FA, FB, DBG>(A, B, M, N, K, lda, ldb, m0, n0, smem, wid, wr, wc, lane, acc);
  else
    mainloop_bal<TI, TR, FA, FB, DBG>(A, B, M, N, K, lda, ldb, m0, n0, smem, wid, wr, wc, lane, acc);
  if (wr == 0) bar();  // re-align the groups
  bar();               // every wave is past its last ds_read: LDS is free for the epilogue
  if constexpr (DBG & 2048) tr1 = __builtin_amdgcn_s_memrealtime();
  if constexpr (EPI == EPI_F32) {
    // fp32 slab (split-K partials): each lane stores its 4 consecutive columns per fragment
    // (fp8 operands: dequantised here, alpha = the two per-tensor inverse scales)
    float* out = part + (int64_t)split * M * ldc;
    float sc = 1.f;
    if constexpr (FA >= 0) sc = alpha_a[0] * alpha_b[0];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = n0 + wc * 64 + j * 16 + 4 * lk;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int m = m0 + wr * 128 + i * 16 + lr;
        if (m < M && n < N) *reinterpret_cast<f32x4*>(out + (int64_t)m * ldc + n) = acc[j][i] * sc;
      }
    }
    return;
  }
  if constexpr (EPI == EPI_F32_ACC) {
    // part[m, n] += acc in fp32 (one K slice: gemm_tt_acc's main_grad accumulation), in two halves
    // of 16 fragments whose 16-byte loads are all issued before the first add
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
      f32x4 prev[2][8];
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) {
        const int n = n0 + wc * 64 + (2 * hf + jj) * 16 + 4 * lk;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const int m = m0 + wr * 128 + i * 16 + lr;
          prev[jj][i] = m < M && n < N ? *reinterpret_cast<const f32x4*>(part + (int64_t)m * ldc + n) : f32x4{};
        }
      }
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) {
        const int n = n0 + wc * 64 + (2 * hf + jj) * 16 + 4 * lk;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const int m = m0 + wr * 128 + i * 16 + lr;
          if (m < M && n < N) *reinterpret_cast<f32x4*>(part + (int64_t)m * ldc + n) = prev[jj][i] + acc[2 * hf + jj][i];
        }
      }
    }
    return;
  }

  if (__builtin_expect((ctl >> 16) == 2, 0) || (DBG & 512)) {  // keep the accumulators live, store nothing
    float t = 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int i = 0; i < 8; ++i) t += acc[j][i][0] + acc[j][i][1] + acc[j][i][2] + acc[j][i][3];
    if (t == 1.2345e-30f) C[0] = from_f<T>(t);
    return;
  }
  float alpha = 1.f;
  if constexpr (FA >= 0) alpha = alpha_a[0] * alpha_b[0];
  epilogue<T, EPI, EDGE, 0, 4, false, Q8, false, NoHook, NOC ? 16 : 0>(acc, smem + wid * 16384, C, M, N, ldc, bias,
                                                                        aux, ldaux, aux_out, part, m0, n0, tm, wr, wc,
                                                                        lane, alpha, q8);
  if constexpr ((DBG & 2048) && FA < 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    bar();
    const uint64_t tr2 = __builtin_amdgcn_s_memrealtime();
    if (tid == 0) {
      uint32_t hw, xcc;
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
      uint64_t* tp = (uint64_t*)alpha_a + (int64_t)bid * 4;
      tp[0] = tr0;
      tp[1] = tr1;
      tp[2] = tr2;
      tp[3] = (uint64_t)hw | ((uint64_t)xcc << 32);
    }
  }
}


// ============================================================================================
// Persistent kernel: one workgroup per CU walks the tile list; the next tile's first K-tile is
// loaded while this tile's epilogue runs.
//
// The timeline trace of the one-tile-per-workgroup kernel (tools/gemmlab LAB_TRACE,
// profiles/r5_gemm_trace_m98304.jsonl) puts 3.2-11.4 us of epilogue and ~0.5 us of dispatch gap
// after each 25-28 us main loop at K = 1024, and the main loop itself includes the prologue: the
// first K-tile's 64 KB arriving while every CU's new workgroup asks for its own at once. Here the
// workgroup, after its last main-loop read of LDS:
//   1. issues the NEXT tile's A(0) and B(0) (buffer 0, 64 KB) — they load during the epilogue;
//   2. runs the epilogue with its accumulators staged through buffer 1 in two 64-row halves (8 KB per
//      wave instead of 16 KB);
//   3. barrier (buffer 1 free), issues B(1) into it, and waits for A(0) / B(0) with a COUNTED vmcnt
//      that leaves this epilogue's stores (and B(1)) in flight: loads, stores and LDS-DMA retire in
//      issue order, so vmcnt(stores + 4) retires exactly the 8 older pieces;
//   4. re-staggers the wave groups and enters the next tile's main loop (mainloop_bal's body).
// Tiles: workgroup b takes virtual block ids b, b + G, b + 2G, ... (G = grid, a multiple of 8) through
// the same bijective XCD remap + GROUP_M order as gemm_nt_kernel, so the tiles an XCD runs at once
// are the same adjacent ones. Full tiles only (M, N multiples of 256), 16-bit NT, no fp8 codes.
__device__ __forceinline__ void tile_coords(int v, int tiles_m, int tiles_n, int& m0, int& n0, int& tm) {
  const int nwg = tiles_m * tiles_n;
  const int xcd = v & 7, q = nwg >> 3, rr = nwg & 7;
  const int wg = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (v >> 3);
  const int group = G_GROUP_M * tiles_n;
  const int first_m = (wg / group) * G_GROUP_M;
  const int gm = min(tiles_m - first_m, G_GROUP_M);
  tm = first_m + (wg % group) % gm;
  const int tn = (wg % group) / gm;
  m0 = tm * GB_M;
  n0 = tn * GB_N;
}

// vector-memory instructions one wave's epilogue issues after the next tile's A(0) / B(0) pieces,
// counting only those that can still be in flight at the wait: the stores (its loads are consumed
// inside the epilogue, so they have retired). Must not exceed the true count (a larger vmcnt would
// let A(0) / B(0) through unretired): C 16, + pre-activation or gelu' 16, + the bias-grad partial row
// 2 (lanes 0..7).
template <int EPI, int Q8 = 0> constexpr int epi_stores() {
  constexpr bool GELU_FWD = EPI == EPI_BIAS_GELU || EPI == EPI_BIAS_GELU_TANH || EPI == EPI_BIAS_GELU_D ||
                            EPI == EPI_BIAS_GELU_TANH_D;
  constexpr bool COLSUM = EPI == EPI_DGELU || EPI == EPI_DGELU_TANH || EPI == EPI_MUL;
  return 16 + (GELU_FWD ? 16 : 0) + (COLSUM ? 2 : 0) + (Q8 != 0 ? 16 : 0);  // (+ the fp8 codes, 8 B per slot)
}

// fp8 (TI = uint8_t codes, formats FA / FB, dequantised by alpha_a[0] * alpha_b[0]; Q8: the output's
// own fp8 codes too): the same tile walk with mainloop_bk64's body (the fp8 instantiations keep it:
// the balanced loop's extra live fragment spills there) and 128-element K-tiles.
template <typename T, int EPI, typename TI = T, int FA = -1, int FB = -1, int Q8 = 0, int DBG = 0>
__global__ void __launch_bounds__(G_THREADS) gemm_persist_kernel(const TI* __restrict__ A, const TI* __restrict__ B,
                                                                 T* __restrict__ C, int M, int N, int K, int64_t lda,
                                                                 int64_t ldb, int64_t ldc, const T* __restrict__ bias,
                                                                 const T* __restrict__ aux, int64_t ldaux,
                                                                 T* __restrict__ aux_out, float* __restrict__ part,
                                                                 uint64_t* __restrict__ trace,
                                                                 const float* __restrict__ alpha_a = nullptr,
                                                                 const float* __restrict__ alpha_b = nullptr,
                                                                 Q8Out q8 = Q8Out{}) {
  __shared__ __attribute__((aligned(16))) char smem[G_LDS_BYTES];
  __shared__ float q8red[G_THREADS / 64];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid >> 2, wc = wid & 3;
  const int tiles_m = M / GB_M, tiles_n = N / GB_N, nwg = tiles_m * tiles_n;
  const int G = gridDim.x;
  constexpr bool F8 = FA >= 0;
  constexpr int BKE = 128 / (int)sizeof(TI);
  const int nt = K / BKE;
  int v = blockIdx.x;
  if (v >= nwg) return;  // (the host sizes the grid to at most the tile count)
  float alpha = 1.f;
  if constexpr (F8) alpha = alpha_a[0] * alpha_b[0];
  if constexpr (Q8 != 0) {  // per-wave running max|C| over the tiles, in LDS (no register across the K loop)
    if (lane == 0) q8red[wid] = 0.f;
  }
  int m0, n0, tm;
  tile_coords(v, tiles_m, tiles_n, m0, n0, tm);
  // first tile's prologue (mainloop_bal's): A(0), B(0) -> buffer 0, B(1) -> buffer 1
  stage_pieces<TI, false>(A, lda, m0, M, 0, smem, wid, lane, 0);
  stage_pieces<TI, false>(A, lda, m0, M, 0, smem, wid, lane, 2);
  stage_pieces<TI, false>(B, ldb, n0, N, 0, smem + G_TILE_BYTES, wid, lane, 0);
  stage_pieces<TI, false>(B, ldb, n0, N, 0, smem + G_TILE_BYTES, wid, lane, 2);
  if (nt > 1) {
    stage_pieces<TI, false>(B, ldb, n0, N, BKE, smem + G_BUF_BYTES + G_TILE_BYTES, wid, lane, 0);
    stage_pieces<TI, false>(B, ldb, n0, N, BKE, smem + G_BUF_BYTES + G_TILE_BYTES, wid, lane, 2);
    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  bar();
  for (;;) {
    uint64_t tr0 = 0, tr1 = 0;
    if constexpr (DBG & 2048) tr0 = __builtin_amdgcn_s_memrealtime();
    f32x4 acc[4][8];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (wr == 1) bar();  // stagger group 1 by one barrier
    // the K loop's per-lane addresses from an opaque lane copy: recomputed per tile rather than kept
    // live through the epilogue (where they spilled, and a scratch reload at the next tile's start
    // waits, in vmcnt order, for every epilogue store still in flight)
    const int lane_k = lane_id_fresh();
    if constexpr (F8) {
      mainloop_bk64_loop<TI, false, FA, FB, 0, true>(A, B, M, N, K, lda, ldb, m0, n0, smem, wid, wr, wc, lane_k, acc);
    } else {
      const int lrk = lane_k & 15, lkk = lane_k >> 4;
      s16x8 fa[4][2], fb[2][2][2];
      read_fb<false>(fb[0], smem + G_TILE_BYTES, wc * 64, lrk, lkk);  // tile 0's first B half
      int t = 0;
      for (; t + 1 < nt; t += 2) {
        bal_tile<TI, false, -1, -1, 0, 0>(t, nt, A, B, M, N, lda, ldb, m0, n0, smem, wid, wr, wc, lane_k, acc, fa, fb);
        bal_tile<TI, false, -1, -1, 0, 1>(t + 1, nt, A, B, M, N, lda, ldb, m0, n0, smem, wid, wr, wc, lane_k, acc, fa,
                                          fb);
      }
      if (t < nt)
        bal_tile<TI, false, -1, -1, 0, 0>(t, nt, A, B, M, N, lda, ldb, m0, n0, smem, wid, wr, wc, lane_k, acc, fa, fb);
    }
    if (wr == 0) bar();  // re-align the groups
    bar();               // every wave is past its last ds_read of this tile
    if constexpr (DBG & 2048) tr1 = __builtin_amdgcn_s_memrealtime();
    const int vn = v + G;
    const bool more = vn < nwg;
    int m1 = 0, n1 = 0, tm1 = 0;
    // an opaque copy of the lane id: everything the epilogue and the next tile's staging derive from
    // it is computed here, not hoisted above the K loop (where it stayed live and spilled ~55 VGPRs)
    const int lane_e = lane_id_fresh();
    if (more) {
      tile_coords(vn, tiles_m, tiles_n, m1, n1, tm1);
    } else {  // the last tile re-loads its own first K-tile (unused): the epilogue's counted waits
      m1 = m0;  // assume exactly 8 pieces behind its first loads
      n1 = n0;
    }
    // the next tile's A(0), B(0): issued by the epilogue after its own first loads (hook)
    auto next_k0 = [&]() {
      stage_pieces<TI, false>(A, lda, m1, M, 0, smem, wid, lane_e, 0);
      stage_pieces<TI, false>(A, lda, m1, M, 0, smem, wid, lane_e, 2);
      stage_pieces<TI, false>(B, ldb, n1, N, 0, smem + G_TILE_BYTES, wid, lane_e, 0);
      stage_pieces<TI, false>(B, ldb, n1, N, 0, smem + G_TILE_BYTES, wid, lane_e, 2);
    };
    __builtin_amdgcn_sched_barrier(0);
    float q8w = 0.f;
    epilogue<T, EPI, false, 0, 4, false, Q8, true, decltype(next_k0), (DBG >> 12) & 15>(acc, smem + G_BUF_BYTES + wid * 8192, C, M, N, ldc, bias, aux,
                                                    ldaux, aux_out, part, m0, n0, tm, wr, wc, lane_e, alpha, q8,
                                                    next_k0, &q8w);
    if constexpr (Q8 != 0) {
      const float m = f8_wave_max(q8w);
      if (lane_e == 0) q8red[wid] = fmaxf(q8red[wid], m);
    }
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (DBG & 2048) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      bar();
      const uint64_t tr2 = __builtin_amdgcn_s_memrealtime();
      if (tid == 0) {
        uint32_t hw, xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        uint64_t* tp = trace + (int64_t)v * 4;
        tp[0] = tr0;
        tp[1] = tr1;
        tp[2] = tr2;
        tp[3] = (uint64_t)hw | ((uint64_t)xcc << 32);
      }
    }
    if (!more) break;
    bar();  // every wave is done with its epilogue region: buffer 1 is free
    if (nt > 1) {
      stage_pieces<TI, false>(B, ldb, n1, N, BKE, smem + G_BUF_BYTES + G_TILE_BYTES, wid, lane_e, 0);
      stage_pieces<TI, false>(B, ldb, n1, N, BKE, smem + G_BUF_BYTES + G_TILE_BYTES, wid, lane_e, 2);
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(((DBG >> 12) & 2 ? 0 : epi_stores<EPI, Q8>()) + 4) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"((DBG >> 12) & 2 ? 0 : epi_stores<EPI, Q8>()) : "memory");
    }
    bar();  // A(0), B(0) of the next tile visible to every wave
    v = vn;
    m0 = m1;
    n0 = n1;
    tm = tm1;
  }
  if constexpr (Q8 != 0) {  // one amax atomic per workgroup, after its last tile
    bar();
    if (wid == 0 && lane_id_fresh() == 0) {
      float mm = 0.f;
#pragma unroll
      for (int w = 0; w < G_THREADS / 64; ++w) mm = fmaxf(mm, q8red[w]);
      if (mm > 0.f) f8_atomic_max_pos(q8.amax, mm);
    }
  }
}


// 2-D transpose out[C][R] = in[R][C] (16-bit elements). Each lane transposes an 8x8 block in
// registers: 8 x 16-B row loads, 8 x 16-B row stores. A wave is 8 (along C) x 8 (along R) blocks,
// so every load and every store instruction moves whole 128-B row runs. Edge blocks fall back to
// element-wise accesses.
template <typename T>
__global__ void __launch_bounds__(256) transpose_kernel(const T* __restrict__ in, T* __restrict__ out, int R, int Cc) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int bc = lane & 7, br = lane >> 3;
  // block tile = 64 (C) x 256 (R) per workgroup: 4 waves along R
  const int c0 = blockIdx.x * 64 + bc * 8;
  const int r0 = blockIdx.y * 256 + wid * 64 + br * 8;
  if (c0 + 8 <= Cc && r0 + 8 <= R && (Cc % 8) == 0 && (R % 8) == 0) {
    s16x8 v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = *reinterpret_cast<const s16x8*>(in + (int64_t)(r0 + k) * Cc + c0);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      s16x8 o;
#pragma unroll
      for (int k = 0; k < 8; ++k) o[k] = v[k][i];
      *reinterpret_cast<s16x8*>(out + (int64_t)(c0 + i) * R + r0) = o;
    }
  } else {
    for (int k = 0; k < 8; ++k)
      for (int i = 0; i < 8; ++i)
        if (r0 + k < R && c0 + i < Cc) out[(int64_t)(c0 + i) * R + r0 + k] = in[(int64_t)(r0 + k) * Cc + c0 + i];
  }
}

// per-epilogue first-round stagger units from APEX_GEMM_STAGGER="epi:units,..." (experiment; read once)
inline int host_stagger(int epi) {
  static int table[16] = {-1};
  if (table[0] == -1) {
    for (int& t : table) t = 0;
    if (const char* e = getenv("APEX_GEMM_STAGGER")) {
      int ep = 0, u = 0;
      const char* p = e;
      while (*p) {
        if (sscanf(p, "%d:%d", &ep, &u) == 2 && ep >= 0 && ep < 16) table[ep] = u;
        while (*p && *p != ',') ++p;
        if (*p == ',') ++p;
      }
    }
  }
  return table[epi];
}

// Persistent kernel (gemm_persist_kernel) for full-tile 16-bit NT launches: APEX_GEMM_PERSIST=0 turns it
// off (A/B). Measured against the one-tile-per-workgroup kernel at the BERT shapes, same process,
// interleaved, bit-identical outputs (profiles/r5_gemm_persist_m98304.jsonl): 0.7-3.6 % faster on
// every shape (plain / bias 3.6 %, residual 1-3 %, GELU_D 1.9 %, multiply 0.7 %).
// h_gemm_persist / h_gemm_persist_f8: -1 = the environment's choice (read once), 0 / 1 forced by
// gemm_set_persist() (the tests compare both kernels bitwise in one process)
int h_gemm_persist = -1, h_gemm_persist_f8 = -1;
inline bool host_persist() {
  static int on = -1;
  if (on == -1) {
    const char* e = getenv("APEX_GEMM_PERSIST");
    on = (e && e[0] == '0') ? 0 : 1;
  }
  return h_gemm_persist >= 0 ? h_gemm_persist == 1 : on == 1;
}
inline int host_cus() {
  static int cus = 0;
  if (cus == 0) {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
    cus = n;
  }
  return cus;
}

template <typename T, int EPI, bool TR = false>
void launch_gemm(const GemmArgs& g, hipStream_t s) {
  const int tiles = ((g.M + GB_M - 1) / GB_M) * ((g.N + GB_N - 1) / GB_N);
  if constexpr (!TR && EPI != EPI_F32 && EPI != EPI_F32_ACC) {
    if (g.M % GB_M == 0 && g.N % GB_N == 0 && tiles > host_cus() && host_persist() && h_gemm_dbg == 0 &&
        h_gemm_stagger <= 0) {
      // more tiles than CUs: one workgroup per CU walks them (the grid stays a multiple of 8)
      const int grid = (host_cus() / 8) * 8;
      hipLaunchKernelGGL((gemm_persist_kernel<T, EPI>), dim3(grid), dim3(G_THREADS), 0, s, (const T*)g.A, (const T*)g.B,
                         (T*)g.C, g.M, g.N, g.K, g.lda, g.ldb, g.ldc, (const T*)g.bias, (const T*)g.aux, g.ldaux,
                         (T*)g.aux_out, g.part, (uint64_t*)nullptr);
      return;
    }
  }
  const int units = h_gemm_stagger > 0 ? h_gemm_stagger : h_gemm_stagger < 0 ? 0 : host_stagger(EPI);
  const int stagger = (units & 0x7fff) | (TR && host_split_xcd() ? kCtlSplitXcd : 0) |
                      (h_gemm_dbg << 16);  // the kernel's ctl word
  const bool edge = g.M % GB_M != 0 || g.N % GB_N != 0;
  if (edge)  // (the transposed-read weight-gradient kernels too: partial tiles since round 5)
    hipLaunchKernelGGL((gemm_nt_kernel<T, EPI, TR, true>), dim3(tiles, TR ? g.splits : 1), dim3(G_THREADS), 0, s,
                       (const T*)g.A, (const T*)g.B, (T*)g.C, g.M, g.N, g.K, g.lda, g.ldb, g.ldc, (const T*)g.bias,
                       (const T*)g.aux, g.ldaux, (T*)g.aux_out, g.part, stagger);
  else
    hipLaunchKernelGGL((gemm_nt_kernel<T, EPI, TR, false>), dim3(tiles, TR ? g.splits : 1), dim3(G_THREADS), 0, s,
                       (const T*)g.A, (const T*)g.B, (T*)g.C, g.M, g.N, g.K, g.lda, g.ldb, g.ldc, (const T*)g.bias,
                       (const T*)g.aux, g.ldaux, (T*)g.aux_out, g.part, stagger);
}

// fp8 launches on the persistent kernel: OFF by default (APEX_GEMM_PERSIST_F8=1 turns it on). Measured
// at the BERT fp8 shapes, M = 98304 (tools/fp8_persist_bench.py, same box, bit-identical outputs):
// first SLOWER on every shape (profiles/r5_fp8_persist_ab.jsonl: FFN2 forward 487 vs 418 us, FFN1
// dgrad + residual 635 vs 438) — the fp8 main loop runs at the 256-VGPR limit, and in the persistent
// kernel a spilled staging address was reloaded inside the K loop behind the previous tile's epilogue
// stores (loads, stores and scratch retire in vmcnt order). With the staging addresses recomputed from
// a fresh lane id per K-tile (FRESH, 0 scratch): still 2-5 % slower except the out-projection forward,
// fp8 BERT step 156.2 vs 155.2 ms (profiles/r5_fp8_persist_ab_v2.jsonl).
inline bool host_persist_f8() {
  static int on = -1;
  if (on == -1) {
    const char* e = getenv("APEX_GEMM_PERSIST_F8");
    on = (e && e[0] == '1') ? 1 : 0;
  }
  return (h_gemm_persist_f8 >= 0 ? h_gemm_persist_f8 == 1 : on == 1) && host_persist();
}

template <typename T, int EPI, int FA, int FB>
void launch_gemm_f8(const GemmArgs& g, hipStream_t s) {
  const int tiles = ((g.M + GB_M - 1) / GB_M) * ((g.N + GB_N - 1) / GB_N);
  // fp8 codes of C for the next GEMM (the MLP's hidden activation forward, its gradient backward)
  constexpr bool Q8_OK = EPI == EPI_BIAS_GELU || EPI == EPI_BIAS_GELU_TANH || EPI == EPI_BIAS_GELU_D ||
                         EPI == EPI_BIAS_GELU_TANH_D || EPI == EPI_MUL || EPI == EPI_DGELU || EPI == EPI_DGELU_TANH;
  if (g.M % GB_M == 0 && g.N % GB_N == 0 && tiles > host_cus() && host_persist_f8()) {
    const int grid = (host_cus() / 8) * 8;
    auto go = [&](auto q_c) {
      hipLaunchKernelGGL((gemm_persist_kernel<T, EPI, uint8_t, FA, FB, decltype(q_c)::value>), dim3(grid),
                         dim3(G_THREADS), 0, s, (const uint8_t*)g.A, (const uint8_t*)g.B, (T*)g.C, g.M, g.N, g.K, g.lda,
                         g.ldb, g.ldc, (const T*)g.bias, (const T*)g.aux, g.ldaux, (T*)g.aux_out, g.part,
                         (uint64_t*)nullptr, g.alpha_a, g.alpha_b, g.q8);
    };
    if constexpr (Q8_OK) {
      if (g.q8.y) {
        if (g.q8.fmt == 0) go(std::integral_constant<int, 1>{});
        else go(std::integral_constant<int, 2>{});
        return;
      }
    }
    go(std::integral_constant<int, 0>{});
    return;
  }
  // codes-only C (Q8Out::only): the bias+GELU+derivative forward and the multiply backward on full
  // tiles; elsewhere the flag is ignored (C written as well: a superset, never wrong)
  constexpr bool NOC_OK = EPI == EPI_BIAS_GELU_D || EPI == EPI_BIAS_GELU_TANH_D || EPI == EPI_MUL;
  if constexpr (Q8_OK) {
    if (g.q8.y) {
      auto go = [&](auto edge_c, auto q_c, auto noc_c) {
        hipLaunchKernelGGL((gemm_nt_kernel<T, EPI, false, decltype(edge_c)::value, uint8_t, FA, FB, 0,
                                           decltype(q_c)::value, decltype(noc_c)::value>),
                           dim3(tiles), dim3(G_THREADS), 0, s, (const uint8_t*)g.A, (const uint8_t*)g.B, (T*)g.C, g.M,
                           g.N, g.K, g.lda, g.ldb, g.ldc, (const T*)g.bias, (const T*)g.aux, g.ldaux, (T*)g.aux_out,
                           g.part, 0, g.alpha_a, g.alpha_b, g.q8);
      };
      const bool edge = g.M % GB_M != 0 || g.N % GB_N != 0;
      if constexpr (NOC_OK) {
        if (g.q8.only && !edge) {
          if (g.q8.fmt == 0) go(std::false_type{}, std::integral_constant<int, 1>{}, std::true_type{});
          else go(std::false_type{}, std::integral_constant<int, 2>{}, std::true_type{});
          return;
        }
      }
      if (g.q8.fmt == 0) {
        if (edge) go(std::true_type{}, std::integral_constant<int, 1>{}, std::false_type{});
        else go(std::false_type{}, std::integral_constant<int, 1>{}, std::false_type{});
      } else {
        if (edge) go(std::true_type{}, std::integral_constant<int, 2>{}, std::false_type{});
        else go(std::false_type{}, std::integral_constant<int, 2>{}, std::false_type{});
      }
      return;
    }
  }
  if (g.M % GB_M != 0 || g.N % GB_N != 0)
    hipLaunchKernelGGL((gemm_nt_kernel<T, EPI, false, true, uint8_t, FA, FB>), dim3(tiles), dim3(G_THREADS), 0, s,
                       (const uint8_t*)g.A, (const uint8_t*)g.B, (T*)g.C, g.M, g.N, g.K, g.lda, g.ldb, g.ldc,
                       (const T*)g.bias, (const T*)g.aux, g.ldaux, (T*)g.aux_out, g.part, 0, g.alpha_a, g.alpha_b);
  else
    hipLaunchKernelGGL((gemm_nt_kernel<T, EPI, false, false, uint8_t, FA, FB>), dim3(tiles), dim3(G_THREADS), 0, s,
                       (const uint8_t*)g.A, (const uint8_t*)g.B, (T*)g.C, g.M, g.N, g.K, g.lda, g.ldb, g.ldc,
                       (const T*)g.bias, (const T*)g.aux, g.ldaux, (T*)g.aux_out, g.part, 0, g.alpha_a, g.alpha_b);
}

template <typename T, int FA, int FB>
int gemm_dispatch_f8(const GemmArgs& g, hipStream_t s) {
  switch (g.epi) {
    case EPI_NONE: launch_gemm_f8<T, EPI_NONE, FA, FB>(g, s); break;
    case EPI_BIAS: launch_gemm_f8<T, EPI_BIAS, FA, FB>(g, s); break;
    case EPI_RESID: launch_gemm_f8<T, EPI_RESID, FA, FB>(g, s); break;
    case EPI_BIAS_GELU: launch_gemm_f8<T, EPI_BIAS_GELU, FA, FB>(g, s); break;
    case EPI_BIAS_GELU_TANH: launch_gemm_f8<T, EPI_BIAS_GELU_TANH, FA, FB>(g, s); break;
    case EPI_DGELU: launch_gemm_f8<T, EPI_DGELU, FA, FB>(g, s); break;
    case EPI_DGELU_TANH: launch_gemm_f8<T, EPI_DGELU_TANH, FA, FB>(g, s); break;
    case EPI_BIAS_GELU_D: launch_gemm_f8<T, EPI_BIAS_GELU_D, FA, FB>(g, s); break;
    case EPI_BIAS_GELU_TANH_D: launch_gemm_f8<T, EPI_BIAS_GELU_TANH_D, FA, FB>(g, s); break;
    case EPI_MUL: launch_gemm_f8<T, EPI_MUL, FA, FB>(g, s); break;
    default: return -3;
  }
  return (int)hipGetLastError();
}

template <typename T>
int gemm_dispatch(const GemmArgs& g, hipStream_t s) {
  switch (g.epi) {
    case EPI_NONE: launch_gemm<T, EPI_NONE>(g, s); break;
    case EPI_BIAS: launch_gemm<T, EPI_BIAS>(g, s); break;
    case EPI_BIAS_GELU: launch_gemm<T, EPI_BIAS_GELU>(g, s); break;
    case EPI_DGELU: launch_gemm<T, EPI_DGELU>(g, s); break;
    case EPI_BIAS_GELU_TANH: launch_gemm<T, EPI_BIAS_GELU_TANH>(g, s); break;
    case EPI_DGELU_TANH: launch_gemm<T, EPI_DGELU_TANH>(g, s); break;
    case EPI_RESID: launch_gemm<T, EPI_RESID>(g, s); break;
    case EPI_BIAS_GELU_D: launch_gemm<T, EPI_BIAS_GELU_D>(g, s); break;
    case EPI_BIAS_GELU_TANH_D: launch_gemm<T, EPI_BIAS_GELU_TANH_D>(g, s); break;
    case EPI_MUL: launch_gemm<T, EPI_MUL>(g, s); break;
    default: return -3;
  }
  return (int)hipGetLastError();
}

}  // namespace

bool gemm_supported(int M, int N, int K, int64_t lda, int64_t ldb, int64_t ldc) {
  // ldc < 2^22: the epilogue addresses a 128-row wave tile through 32-bit buffer offsets
  return M > 0 && N > 0 && K > 0 && K % GB_K == 0 && N % 8 == 0 && lda % 8 == 0 && ldb % 8 == 0 && ldc % 8 == 0 &&
         ldc < (1 << 22) &&
         (int64_t)M * lda < (1ll << 40);
}

int64_t gemm_part_rows(int M) { return (int64_t)((M + GB_M - 1) / GB_M) * 2; }

int gemm_set_dbg(int v) {
  // v < 0: -v = stagger units (experiment); v >= 0: diagnostics mode
  if (v < 0) {  // -100: force no stagger; -200: launcher's choice; -k: k units
    h_gemm_stagger = v == -100 ? -1 : v == -200 ? 0 : -v;
    return 0;
  }
  h_gemm_dbg = v;
  return 0;
}

// which = 0: the 16-bit persistent kernel, 1: the fp8 one; v = 1 on, 0 off, -1 back to the environment's
// choice. Returns the previous forced value.
int gemm_set_persist(int which, int v) {
  int& h = which == 1 ? h_gemm_persist_f8 : h_gemm_persist;
  const int prev = h;
  h = v < 0 ? -1 : (v ? 1 : 0);
  return prev;
}

int gemm_nt(const GemmArgs& g, int dt, hipStream_t s) {
  if (!gemm_supported(g.M, g.N, g.K, g.lda, g.ldb, g.ldc)) return -2;
  if (g.aux && g.ldaux >= (1 << 22)) return -2;  // 32-bit buffer offsets in the epilogue
  if (dt == kBF16Code) return gemm_dispatch<bf16>(g, s);
  if (dt == kF16Code) return gemm_dispatch<f16>(g, s);
  return -1;
}

bool gemm_f8_supported(int M, int N, int K, int64_t lda, int64_t ldb, int64_t ldc) {
  return M > 0 && N > 0 && K > 0 && K % 128 == 0 && N % 8 == 0 && lda % 16 == 0 && ldb % 16 == 0 && ldc % 8 == 0 &&
         ldc < (1 << 22) &&
         (int64_t)M * lda < (1ll << 40);
}

int gemm_nt_f8(const GemmArgs& g, int fmt_a, int fmt_b, int out_dt, hipStream_t s) {
  // A (activations / gradients): e4m3 (0) or e5m2 (1); B (weights): e4m3
  if (!gemm_f8_supported(g.M, g.N, g.K, g.lda, g.ldb, g.ldc) || fmt_b != 0 || !g.alpha_a || !g.alpha_b) return -2;
  if (g.aux && g.ldaux >= (1 << 22)) return -2;
  if (out_dt == kBF16Code) {
    if (fmt_a == 0) return gemm_dispatch_f8<bf16, 0, 0>(g, s);
    if (fmt_a == 1) return gemm_dispatch_f8<bf16, 1, 0>(g, s);
  } else if (out_dt == kF16Code) {
    if (fmt_a == 0) return gemm_dispatch_f8<f16, 0, 0>(g, s);
    if (fmt_a == 1) return gemm_dispatch_f8<f16, 1, 0>(g, s);
  }
  return -1;
}

bool gemm_tt_supported(int P, int Q, int R, int splits, int64_t lda, int64_t ldb) {
  // P, Q: any multiple of 8 (partial 256-tiles: clamped staging + bounds-checked epilogues)
  return P > 0 && Q > 0 && splits > 0 && P % 8 == 0 && Q % 8 == 0 && R % GB_K == 0 && R / GB_K >= splits &&
         lda % 8 == 0 && ldb % 8 == 0;
}

int gemm_tt(const GemmArgs& g, int dt, hipStream_t s) {
  // C[P=M, Q=N] (+)= sum_r A[r, p] B[r, q]; g.K = ALL contraction rows (g.splits slices of whole K-tiles,
  // sizes within one K-tile of each other); g.part = fp32 slabs
  // [splits, M, N] when g.epi == EPI_F32, the fp32 [M, N] accumulator (+=) when EPI_F32_ACC, else g.C
  // in the operand dtype (splits must be 1 except for EPI_F32)
  if (!gemm_tt_supported(g.M, g.N, g.K, g.splits, g.lda, g.ldb)) return -2;
  if (g.epi != EPI_F32 && ((g.epi != EPI_NONE && g.epi != EPI_F32_ACC) || g.splits != 1)) return -3;
  if (dt == kBF16Code) {
    if (g.epi == EPI_F32) launch_gemm<bf16, EPI_F32, true>(g, s);
    else if (g.epi == EPI_F32_ACC) launch_gemm<bf16, EPI_F32_ACC, true>(g, s);
    else launch_gemm<bf16, EPI_NONE, true>(g, s);
  } else if (dt == kF16Code) {
    if (g.epi == EPI_F32) launch_gemm<f16, EPI_F32, true>(g, s);
    else if (g.epi == EPI_F32_ACC) launch_gemm<f16, EPI_F32_ACC, true>(g, s);
    else launch_gemm<f16, EPI_NONE, true>(g, s);
  } else {
    return -1;
  }
  return (int)hipGetLastError();
}

bool gemm_tt_f8_supported(int P, int Q, int R, int splits, int64_t lda, int64_t ldb) {
  // fp8 codes: 16-byte chunks of 16 columns (partial 256-tiles clamp to the last full chunk)
  return P > 0 && Q > 0 && splits > 0 && P % 16 == 0 && Q % 16 == 0 && R % 128 == 0 && R / 128 >= splits &&
         lda % 16 == 0 && ldb % 16 == 0;
}

// fp8 weight gradient: fp32 slabs [splits, P, Q] of alpha_a alpha_b sum_r A[r, p] B[r, q] over the
// uint8 codes A (format fmt_a: the output gradient, e5m2 in the hybrid recipe) and B (fmt_b: the
// layer input, e4m3); the transposed-read main loop with ds_read_b64_tr_b8 fragments
template <int FA, int FB>
void launch_gemm_tt_f8(const GemmArgs& g, hipStream_t s) {
  const int tiles = ((g.M + GB_M - 1) / GB_M) * ((g.N + GB_N - 1) / GB_N);
  if (g.M % GB_M != 0 || g.N % GB_N != 0)
    hipLaunchKernelGGL((gemm_nt_kernel<bf16, EPI_F32, true, true, uint8_t, FA, FB>), dim3(tiles, g.splits),
                       dim3(G_THREADS), 0, s, (const uint8_t*)g.A, (const uint8_t*)g.B, (bf16*)nullptr, g.M, g.N, g.K,
                       g.lda, g.ldb, g.ldc, (const bf16*)nullptr, (const bf16*)nullptr, (int64_t)0, (bf16*)nullptr,
                       g.part, host_split_xcd() ? kCtlSplitXcd : 0, g.alpha_a, g.alpha_b);
  else
    hipLaunchKernelGGL((gemm_nt_kernel<bf16, EPI_F32, true, false, uint8_t, FA, FB>), dim3(tiles, g.splits),
                       dim3(G_THREADS), 0, s, (const uint8_t*)g.A, (const uint8_t*)g.B, (bf16*)nullptr, g.M, g.N, g.K,
                       g.lda, g.ldb, g.ldc, (const bf16*)nullptr, (const bf16*)nullptr, (int64_t)0, (bf16*)nullptr,
                       g.part, host_split_xcd() ? kCtlSplitXcd : 0, g.alpha_a, g.alpha_b);
}

int gemm_tt_f8(const GemmArgs& g, int fmt_a, int fmt_b, hipStream_t s) {
  if (!gemm_tt_f8_supported(g.M, g.N, g.K, g.splits, g.lda, g.ldb) || !g.alpha_a || !g.alpha_b ||
      !g.part)
    return -2;
  if (fmt_a == 1 && fmt_b == 0) launch_gemm_tt_f8<1, 0>(g, s);
  else if (fmt_a == 0 && fmt_b == 0) launch_gemm_tt_f8<0, 0>(g, s);
  else return -1;
  return (int)hipGetLastError();
}

int gemm_bias_grad(const float* part, int parts, int N, void* out, int odt, hipStream_t s) {
  if (odt == kBF16Code) launch_partial_colsum<bf16>(part, parts, N, N, (bf16*)out, s);
  else if (odt == kF16Code) launch_partial_colsum<f16>(part, parts, N, N, (f16*)out, s);
  else if (odt == kF32Code) launch_partial_colsum<float>(part, parts, N, N, (float*)out, s);
  else return -1;
  return (int)hipGetLastError();
}

int transpose_2d(const void* in, void* out, int R, int C, int dt, hipStream_t s) {
  if (R == 0 || C == 0) return 0;
  dim3 grid((C + 63) / 64, (R + 255) / 256);
  if (dt == kBF16Code)
    hipLaunchKernelGGL((transpose_kernel<bf16>), grid, dim3(256), 0, s, (const bf16*)in, (bf16*)out, R, C);
  else if (dt == kF16Code)
    hipLaunchKernelGGL((transpose_kernel<f16>), grid, dim3(256), 0, s, (const f16*)in, (f16*)out, R, C);
  else
    return -1;
  return (int)hipGetLastError();
}

}  // namespace apex
