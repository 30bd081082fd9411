// Lab-only GEMM variants (measured negatives, kept for A/B in tools/gemmlab/lab.hip; never part of the
// production extension): the four-wave 128x128-wave-tile kernel (w4 / w4r), the two-workgroup
// 256x128 kernel (w2g), the 32x32x16-fragment kernel (m32) and the per-wave software-pipelined kernel
// (w8p). Results and reasons they lost are in profiles/README.md (rounds 3-4). Included by lab.hip
// right after csrc/gemm.hip, inside the same anonymous namespace.
#pragma once
namespace apex {
namespace {
// ============================================================================================
// Four-wave kernel ("w4"): the same 256 x 256 x 64 output tile and LDS image, but 256 threads =
// ONE wave per SIMD, each wave a 128 x 128 sub-tile (8 x 8 fragments of v_mfma_f32_16x16x32,
// 256 fp32 accumulators). Per K-tile and wave: 128 MFMAs (2048 matrix-pipe cycles) against 32
// ds_read_b128 and 16 LDS-DMA pieces — half the LDS read bytes per FLOP of the 8-wave 128 x 64
// layout (whose read sections outran its 16-MFMA compute sections: 64 % MFMA busy). The wave
// interleaves its own reads with its MFMAs (no ping-pong partner); one barrier per K-tile:
//   s = 0: 64 MFMAs on fragments (k 0..31), the k 32..63 fragments read meanwhile
//   s = 1: 32 MFMAs (rows 0..3) | vmcnt(0) + lgkmcnt(0) | barrier | read the NEXT tile's k 0..31
//          fragments and issue the tile-after-next's 16 LDS-DMA pieces into the buffer just
//          released | 32 MFMAs (rows 4..7)
// RAW: tile t+1 was issued right after the barrier of tile t-1 and is waited for (vmcnt(0)) before
// the barrier of tile t, ~1.5 K-tiles later; WAR: the barrier of tile t follows every wave's last
// read of tile t's buffer (lgkmcnt(0)), so tile t+2 may overwrite it right after.
// Operands are staged by buffer_load ... lds off a per-operand buffer resource (one 32-bit
// voffset per piece and lane, the K-tile in soffset): rows past M / N read zero (no clamping).
constexpr int W_THREADS = 256;

// MFMA with the accumulator pinned to the AGPR file ("+a"): all 256 accumulators of a 128 x 128
// wave tile fill the AGPR file exactly, and with the builtin hipcc parks some of them in VGPRs and
// shuffles ~400 v_accvgpr moves per K-tile through the loop phis. The asm statement is one MFMA
// whose only hazard partner is the next MFMA on the same accumulator (an accumulate chain, no wait
// states) and, after the loop, the epilogue's reads (mfma_drain).
template <typename T> __device__ __forceinline__ void mfma16_acc(f32x4& c, const s16x8& a, const s16x8& b);
// The statements are volatile: hipcc does not see them as MFMAs, so it would neither order its own
// v_accvgpr reads of the results behind the MFMA latency nor keep them in issue order; volatile asm
// keeps program order among these, the waits and the fences below.
template <> __device__ __forceinline__ void mfma16_acc<bf16>(f32x4& c, const s16x8& a, const s16x8& b) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(c) : "v"(a), "v"(b));
}
template <> __device__ __forceinline__ void mfma16_acc<f16>(f32x4& c, const s16x8& a, const s16x8& b) {
  asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, %0" : "+a"(c) : "v"(a), "v"(b));
}
// Hazard fences around an asm-MFMA region. Entry: the accumulators' initial v_accvgpr_writes are
// complete before the first MFMA reads them as SrcC. Exit: 16 wait states after the last MFMA (an
// 8-pass XDL result read by a VALU needs 12), then an empty "+a" statement per accumulator so no
// v_accvgpr_read of a result is scheduled above the wait (a volatile asm alone orders nothing but
// memory and other volatile statements: the reads were hoisted between the last MFMAs and returned
// pre-MFMA values — one k-step missing from the output).
template <int NJ, int NI>
__device__ __forceinline__ void acc_fence(f32x4 (&acc)[NJ][NI]) {
#pragma unroll
  for (int j = 0; j < NJ; ++j)
#pragma unroll
    for (int i = 0; i < NI; ++i) asm volatile("" : "+a"(acc[j][i]));
}
template <int NJ, int NI>
__device__ __forceinline__ void mfma_enter(f32x4 (&acc)[NJ][NI]) {
  acc_fence(acc);
  asm volatile("s_nop 4" ::: "memory");
}
template <int NJ, int NI>
__device__ __forceinline__ void mfma_drain(f32x4 (&acc)[NJ][NI]) {
  asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");
  acc_fence(acc);
}

__device__ __forceinline__ void bglds16(__amdgpu_buffer_rsrc_t rs, char* lds, uint32_t voff, uint32_t soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)lds, 16, voff, soff, 0, 0);
}

// per-lane byte offset of glds piece p (0..31) of an operand K-tile, relative to the tile origin
template <typename T, bool TR>
__device__ __forceinline__ uint32_t piece_voff(int p, int lane, int64_t ld) {
  if constexpr (TR) {
    const int r = p * 2 + (lane >> 5);
    const int chunk = (lane & 31) ^ ftr(r);
    return (uint32_t)(r * ld * (int64_t)sizeof(T) + chunk * 16);
  } else {
    const int r = p * 8 + (lane >> 3);
    const int chunk = (lane & 7) ^ ((r >> 1) & 7);
    return (uint32_t)(r * ld * (int64_t)sizeof(T) + chunk * 16);
  }
}

template <typename T, bool TR, int DBG = 0>
__device__ __forceinline__ void mainloop_w4(__amdgpu_buffer_rsrc_t rsa, __amdgpu_buffer_rsrc_t rsb,
                                            const uint32_t (&va)[8], const uint32_t (&vb)[8], uint32_t tsa,
                                            uint32_t tsb, int nt, char* smem, int wid, int wr, int wc, int lane,
                                            f32x4 (&acc)[8][8]) {
  const int lr = lane & 15, lk = lane >> 4;
  // glds piece q (0..15) of K-tile t into buffer buf: A pieces on even q, B pieces on odd q
  auto stage1 = [&](int t, int buf, int q) {
    char* base = smem + buf * G_BUF_BYTES + wid * 8 * 1024 + (q >> 1) * 1024;
    if (q & 1) bglds16(rsb, base + G_TILE_BYTES, vb[q >> 1], (uint32_t)t * tsb);
    else bglds16(rsa, base, va[q >> 1], (uint32_t)t * tsa);
  };
  // fragment read q (0..15) of k-step s: B columns 0..7 first (the first MFMA row needs all of
  // them), then A rows 0..7
  auto read1 = [&](const char* buf, int s, int q, s16x8(&fa)[8], s16x8(&fb)[8]) {
    if (q < 8) fb[q] = frag<TR>(buf + G_TILE_BYTES, wc * 128 + q * 16, s, lr, lk);
    else fa[q - 8] = frag<TR>(buf, wr * 128 + (q - 8) * 16, s, lr, lk);
  };
  auto mma1 = [&](const s16x8(&fa)[8], const s16x8(&fb)[8], int l) {  // l = i * 8 + j
    mfma16_acc<T>(acc[l & 7][l >> 3], fb[l & 7], fa[l >> 3]);
  };
#pragma unroll
  for (int q = 0; q < 16; ++q) stage1(0, 0, q);
  if (nt > 1) {
#pragma unroll
    for (int q = 0; q < 16; ++q) stage1(1, 1, q);
    asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  bar();
  s16x8 fa0[8], fb0[8], fa1[8], fb1[8];
#pragma unroll
  for (int q = 0; q < 16; ++q) read1(smem, 0, q, fa0, fb0);
  // One K-tile. NEXT: read the next tile's k 0..31 fragments; STAGE: issue tile t + 2.
  auto body = [&](int t, auto next_c, auto stage_c) {
    constexpr bool NEXT = decltype(next_c)::value, STAGE = decltype(stage_c)::value;
    const char* cur = smem + (t & 1) * G_BUF_BYTES;
    const char* nxt = smem + ((t + 1) & 1) * G_BUF_BYTES;
    // s = 0: 64 MFMAs, one fragment read of k-step 1 per 4
    if constexpr (DBG & 1) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if constexpr (DBG & 4) {
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      bar();
    }
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      if constexpr (!(DBG & 128)) read1(cur, 1, q, fa1, fb1);
      if constexpr (DBG & 8) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if constexpr (DBG & 2) asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");
        mma1(fa0, fb0, 4 * q + u);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    if constexpr (DBG & 1) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    // s = 1, rows 0..3
#pragma unroll
    for (int l = 0; l < 32; ++l) {
      if constexpr (DBG & 2) asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");
      mma1(fa1, fb1, l);
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    if constexpr (!(DBG & 64)) bar();
    // s = 1, rows 4..7: next tile's first fragments + the tile-after-next's LDS-DMA pieces
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      if constexpr (NEXT && !(DBG & 128)) read1(nxt, 0, q, fa0, fb0);
      if constexpr (STAGE && !(DBG & 32)) stage1(t + 2, t & 1, q);
      if constexpr (DBG & 8) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        if constexpr (DBG & 2) asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");
        mma1(fa1, fb1, 32 + 2 * q + u);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  for (int t = 0; t < nt - 2; ++t) body(t, std::true_type{}, std::true_type{});
  if (nt > 1) body(nt - 2, std::true_type{}, std::false_type{});
  body(nt - 1, std::false_type{}, std::false_type{});
}

// Register-staged variant of mainloop_w4: LDS-DMA pieces cost the lone wave of a SIMD 60-185 issue
// cycles each beside its MFMAs (no partner wave to cover them): 16 per K-tile took ~20 % of the
// kernel (tools/gemmlab, w4 with the glds removed: 858 -> 688 us at 8192^3). Here each wave loads
// its 16 pieces (16 B per lane, the same source-swizzled offsets) into 64 VGPRs one K-tile ahead
// and writes them to the lane-linear LDS image with ds_write_b128:
//   phase A (s = 0, 64 MFMAs): per 4 MFMAs one fragment read of k-step 1, one ds_write of tile
//     t+1 (loaded during tile t-1) into the buffer released at the previous barrier, and the
//     global load of the same piece of tile t+2 into the register just written out
//   B1 (s = 1 rows 0..3) | lgkmcnt(0) + barrier | B2 (rows 4..7) + the next tile's k 0..31 reads
// The barrier needs no vmcnt: the loads in flight target registers, not LDS.
template <typename T, bool TR, int DBG = 0>
__device__ __forceinline__ void mainloop_w4r(__amdgpu_buffer_rsrc_t rsa, __amdgpu_buffer_rsrc_t rsb,
                                             const uint32_t (&va)[8], const uint32_t (&vb)[8], uint32_t tsa,
                                             uint32_t tsb, int nt, char* smem, int wid, int wr, int wc, int lane,
                                             f32x4 (&acc)[8][8]) {
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  const int lr = lane & 15, lk = lane >> 4;
  u32x4 stg[16];
  auto gload = [&](int t, int q) {
    if (q & 1) stg[q] = __builtin_amdgcn_raw_buffer_load_b128(rsb, vb[q >> 1], (uint32_t)t * tsb, 0);
    else stg[q] = __builtin_amdgcn_raw_buffer_load_b128(rsa, va[q >> 1], (uint32_t)t * tsa, 0);
  };
  char* wbase = smem + wid * 8 * 1024 + lane * 16;
  auto swrite = [&](int buf, int q) {
    *reinterpret_cast<u32x4*>(wbase + buf * G_BUF_BYTES + (q & 1) * G_TILE_BYTES + (q >> 1) * 1024) = stg[q];
  };
  auto read1 = [&](const char* buf, int s, int q, s16x8(&fa)[8], s16x8(&fb)[8]) {
    if (q < 8) fb[q] = frag<TR>(buf + G_TILE_BYTES, wc * 128 + q * 16, s, lr, lk);
    else fa[q - 8] = frag<TR>(buf, wr * 128 + (q - 8) * 16, s, lr, lk);
  };
  auto mma1 = [&](const s16x8(&fa)[8], const s16x8(&fb)[8], int l) {
    mfma16_acc<T>(acc[l & 7][l >> 3], fb[l & 7], fa[l >> 3]);
  };
#pragma unroll
  for (int q = 0; q < 16; ++q) gload(0, q);
#pragma unroll
  for (int q = 0; q < 16; ++q) swrite(0, q);
  if (nt > 1) {
#pragma unroll
    for (int q = 0; q < 16; ++q) gload(1, q);
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  bar();
  s16x8 fa0[8], fb0[8], fa1[8], fb1[8];
#pragma unroll
  for (int q = 0; q < 16; ++q) read1(smem, 0, q, fa0, fb0);
  auto body = [&](int t, auto next_c, auto stage_c) {
    constexpr bool NEXT = decltype(next_c)::value, STAGE = decltype(stage_c)::value;
    const char* cur = smem + (t & 1) * G_BUF_BYTES;
    const char* nxt = smem + ((t + 1) & 1) * G_BUF_BYTES;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      read1(cur, 1, q, fa1, fb1);
      if constexpr (NEXT) swrite((t + 1) & 1, q);
      if constexpr (STAGE) gload(t + 2, q);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int u = 0; u < 4; ++u) mma1(fa0, fb0, 4 * q + u);
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int l = 0; l < 32; ++l) mma1(fa1, fb1, l);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    bar();
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      if constexpr (NEXT) read1(nxt, 0, q, fa0, fb0);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int u = 0; u < 2; ++u) mma1(fa1, fb1, 32 + 2 * q + u);
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  for (int t = 0; t < nt - 2; ++t) body(t, std::true_type{}, std::true_type{});
  if (nt > 1) body(nt - 2, std::true_type{}, std::false_type{});
  body(nt - 1, std::false_type{}, std::false_type{});
}

template <typename T, int EPI, bool TR, bool EDGE, int DBG = 0>
__global__ void __launch_bounds__(W_THREADS, 1) gemm_w4_kernel(const T* __restrict__ A, const T* __restrict__ B,
                                                               T* __restrict__ C, int M, int N, int K, int64_t lda,
                                                               int64_t ldb, int64_t ldc, const T* __restrict__ bias,
                                                               const T* __restrict__ aux, int64_t ldaux,
                                                               T* __restrict__ aux_out, float* __restrict__ part) {
  __shared__ __attribute__((aligned(16))) char smem[G_LDS_BYTES];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid >> 1, wc = wid & 1;
  const int lr = lane & 15, lk = lane >> 4;

  const int tiles_m = (M + GB_M - 1) / GB_M, tiles_n = (N + GB_N - 1) / GB_N;
  const int nwg = tiles_m * tiles_n;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, q = nwg >> 3, rr = nwg & 7;
  const int wg = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (bid >> 3);
  const int group = G_GROUP_M * tiles_n;
  const int first_m = (wg / group) * G_GROUP_M;
  const int gm = min(tiles_m - first_m, G_GROUP_M);
  const int tm = first_m + (wg % group) % gm;
  const int tn = (wg % group) / gm;
  const int m0 = tm * GB_M, n0 = tn * GB_N;

  uint32_t va[8], vb[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    va[j] = piece_voff<T, TR>(wid * 8 + j, lane, lda);
    vb[j] = piece_voff<T, TR>(wid * 8 + j, lane, ldb);
  }
  __amdgpu_buffer_rsrc_t rsa, rsb;
  uint32_t tsa, tsb;
  if constexpr (TR) {  // [K][rows]: split-K slice blockIdx.y = K-rows [y*K, (y+1)*K)
    const T* a0 = A + (int64_t)blockIdx.y * K * lda + m0;
    const T* b0 = B + (int64_t)blockIdx.y * K * ldb + n0;
    rsa = wave_rsrc(a0, 0xFFFFFFFFu);
    rsb = wave_rsrc(b0, 0xFFFFFFFFu);
    tsa = (uint32_t)(GB_K * lda * (int64_t)sizeof(T));
    tsb = (uint32_t)(GB_K * ldb * (int64_t)sizeof(T));
  } else {
    const int ra = min(M - m0, GB_M), rb = min(N - n0, GB_N);
    rsa = wave_rsrc(A + (int64_t)m0 * lda, (uint32_t)(ra * lda * (int64_t)sizeof(T)));
    rsb = wave_rsrc(B + (int64_t)n0 * ldb, (uint32_t)(rb * ldb * (int64_t)sizeof(T)));
    tsa = tsb = GB_K * sizeof(T);
  }

  f32x4 acc[8][8];
#pragma unroll
  for (int j = 0; j < 8; ++j)
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};

  mfma_enter(acc);
  if constexpr (DBG & 256)
    mainloop_w4r<T, TR, DBG>(rsa, rsb, va, vb, tsa, tsb, K / GB_K, smem, wid, wr, wc, lane, acc);
  else
    mainloop_w4<T, TR, DBG>(rsa, rsb, va, vb, tsa, tsb, K / GB_K, smem, wid, wr, wc, lane, acc);
  mfma_drain(acc);
  if constexpr (DBG & 16) {
#pragma unroll
    for (int i = 0; i < 16; ++i) asm volatile("s_nop 15" ::: "memory");
  }
  bar();  // every wave is past its last ds_read: LDS is free for the epilogue
  if constexpr (EPI == EPI_F32) {
    float* out = part + (int64_t)blockIdx.y * M * ldc;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int n = n0 + wc * 128 + j * 16 + 4 * lk;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int m = m0 + wr * 128 + i * 16 + lr;
        if (m < M && n < N) *reinterpret_cast<f32x4*>(out + (int64_t)m * ldc + n) = acc[j][i];
      }
    }
    return;
  }
  if constexpr (DBG & 512) {  // keep the accumulators live, store nothing
    float t = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
      for (int i = 0; i < 8; ++i) t += acc[j][i][0] + acc[j][i][1] + acc[j][i][2] + acc[j][i][3];
    if (t == 1.2345e-30f) C[0] = from_f<T>(t);
    return;
  }
  // all 256 accumulators to LDS first (as bf16 the wave's 128 x 128 tile fills its two 16 KB regions),
  // then the two 64-column halves: the accumulators are dead before the epilogue math starts
  char* reg0 = smem + (wid * 2) * 16384;
  char* reg1 = reg0 + 16384;
  stage_acc<T, 0, 8>(acc, reg0, lane, 1.f);
  stage_acc<T, 4, 8>(acc, reg1, lane, 1.f);
  __builtin_amdgcn_sched_barrier(0);
  epilogue<T, EPI, EDGE, 0, 8, true>(acc, reg0, C, M, N, ldc, bias, aux, ldaux, aux_out, part, m0, n0, tm, wr, wc * 2,
                                     lane);
  epilogue<T, EPI, EDGE, 4, 8, true>(acc, reg1, C, M, N, ldc, bias, aux, ldaux, aux_out, part, m0, n0, tm, wr,
                                     wc * 2 + 1, lane);
}

// ============================================================================================
// Two-workgroups-per-CU kernel ("w2g"): 256 x 128 output tiles, BK = 32, three LDS stages (72 KB),
// 256 threads = 4 waves as 2 (M) x 2 (N), each wave the same 128 x 64 sub-tile as the 8-wave
// kernel (acc[4][8], same epilogue). Two resident workgroups put two independent waves on every
// SIMD: while one workgroup runs its epilogue (HBM-bound bias / GELU / residual stores: 20-37 % of
// the 8-wave kernel at M = 98304, tools/gemmlab *_noepi) the other keeps the matrix pipe busy, and
// inside the main loops each wave's LDS reads and DMA issue are covered by its partner's MFMAs
// (no explicit ping-pong). Per K-tile and wave: 32 MFMAs, 12 ds_read_b128, 6 LDS-DMA pieces:
//   MFMA rows 0..3 | vmcnt(6) (tile t+1 landed, t+2 in flight) + barrier | read tile t+1's
//   fragments into the other register set, issue tile t+3 into the stage tile t used
//   (released by this barrier) | MFMA rows 4..7
// LDS image: 64-byte rows (32 K), 16-byte chunk c of row r at c ^ (2 * ((r >> 2) & 1)) — every
// 16-lane ds_read_b128 group hits 16 distinct bank quads (checked exhaustively); the XOR is
// applied to the DMA's per-lane source offset (the DMA writes lane-linear).
constexpr int W2_BN = 128, W2_BK = 32, W2_STAGES = 3;
constexpr int W2_A_BYTES = GB_M * W2_BK * 2, W2_B_BYTES = W2_BN * W2_BK * 2;  // 16 KB, 8 KB
constexpr int W2_STAGE_BYTES = W2_A_BYTES + W2_B_BYTES;                       // 24 KB
constexpr int W2_LDS_BYTES = W2_STAGES * W2_STAGE_BYTES;                      // 72 KB

__device__ __forceinline__ int w2_swz(int r) { return ((r >> 2) & 1) << 1; }

__device__ __forceinline__ s16x8 w2_frag(const char* tile, int r, int lk) {
  return *reinterpret_cast<const s16x8*>(tile + r * 64 + ((lk ^ w2_swz(r)) << 4));
}

template <typename T, int EPI, bool EDGE>
__global__ void __launch_bounds__(W_THREADS, 2) gemm_w2g_kernel(const T* __restrict__ A, const T* __restrict__ B,
                                                                T* __restrict__ C, int M, int N, int K, int64_t lda,
                                                                int64_t ldb, int64_t ldc, const T* __restrict__ bias,
                                                                const T* __restrict__ aux, int64_t ldaux,
                                                                T* __restrict__ aux_out, float* __restrict__ part) {
  __shared__ __attribute__((aligned(16))) char smem[W2_LDS_BYTES];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid >> 1, wc = wid & 1;
  const int lr = lane & 15, lk = lane >> 4;

  const int tiles_m = (M + GB_M - 1) / GB_M, tiles_n = (N + W2_BN - 1) / W2_BN;
  const int nwg = tiles_m * tiles_n;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, q = nwg >> 3, rr = nwg & 7;
  const int wg = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (bid >> 3);
  const int group = G_GROUP_M * tiles_n;
  const int first_m = (wg / group) * G_GROUP_M;
  const int gm = min(tiles_m - first_m, G_GROUP_M);
  const int tm = first_m + (wg % group) % gm;
  const int tn = (wg % group) / gm;
  const int m0 = tm * GB_M, n0 = tn * W2_BN;

  // this wave's 6 pieces per K-tile: A pieces 4w .. 4w+3 (16 rows each), B pieces 2w, 2w+1
  uint32_t va[4], vb[2];
  const int prow = lane >> 2, pc = lane & 3;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int r = (wid * 4 + j) * 16 + prow;
    va[j] = (uint32_t)(r * lda * (int64_t)sizeof(T) + ((pc ^ w2_swz(r)) << 4));
  }
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int r = (wid * 2 + j) * 16 + prow;
    vb[j] = (uint32_t)(r * ldb * (int64_t)sizeof(T) + ((pc ^ w2_swz(r)) << 4));
  }
  const int ra = min(M - m0, GB_M), rb = min(N - n0, W2_BN);
  const __amdgpu_buffer_rsrc_t rsa = wave_rsrc(A + (int64_t)m0 * lda, (uint32_t)(ra * lda * (int64_t)sizeof(T)));
  const __amdgpu_buffer_rsrc_t rsb = wave_rsrc(B + (int64_t)n0 * ldb, (uint32_t)(rb * ldb * (int64_t)sizeof(T)));
  constexpr uint32_t TS = W2_BK * sizeof(T);  // K-tile stride in bytes (soffset)
  auto stage = [&](int t, int st) {
    char* base = smem + st * W2_STAGE_BYTES;
#pragma unroll
    for (int j = 0; j < 4; ++j) bglds16(rsa, base + (wid * 4 + j) * 1024, va[j], (uint32_t)t * TS);
#pragma unroll
    for (int j = 0; j < 2; ++j) bglds16(rsb, base + W2_A_BYTES + (wid * 2 + j) * 1024, vb[j], (uint32_t)t * TS);
  };
  auto load = [&](int st, s16x8(&fa)[8], s16x8(&fb)[4]) {
    const char* base = smem + st * W2_STAGE_BYTES;
#pragma unroll
    for (int j = 0; j < 4; ++j) fb[j] = w2_frag(base + W2_A_BYTES, wc * 64 + j * 16 + lr, lk);
#pragma unroll
    for (int i = 0; i < 8; ++i) fa[i] = w2_frag(base, wr * 128 + i * 16 + lr, lk);
  };

  f32x4 acc[4][8];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto mma = [&](const s16x8(&fa)[8], const s16x8(&fb)[4], int i0) {
#pragma unroll
    for (int i = i0; i < i0 + 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[j][i] = mfma16<T>(fb[j], fa[i], acc[j][i]);
  };

  const int nt = K / W2_BK;
  stage(0, 0);
  if (nt > 1) stage(1, 1);
  if (nt > 2) stage(2, 2);
  if (nt > 2) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
  else if (nt > 1) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  bar();
  s16x8 fa0[8], fb0[4], fa1[8], fb1[4];
  load(0, fa0, fb0);
  // one K-tile on register set (fa, fb); the next tile's fragments go to (ga, gb)
  auto body = [&](int t, s16x8(&fa)[8], s16x8(&fb)[4], s16x8(&ga)[8], s16x8(&gb)[4]) {
    mma(fa, fb, 0);
    // tile t+1 landed: of this wave's pieces, only tile t+2's (issued at the previous barrier)
    // may still be in flight
    if (t + 2 < nt) asm volatile("s_waitcnt vmcnt(6) lgkmcnt(0)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    bar();
    if (t + 1 < nt) load((t + 1) % W2_STAGES, ga, gb);
    if (t + 3 < nt) stage(t + 3, t % W2_STAGES);
    mma(fa, fb, 4);
  };
  // steady state: six K-tiles per trip (register set t % 2, stage t % 3 compile-time constants;
  // every tile of the trip has its t+3 to issue), then the generic tail
  auto fast = [&](int t, auto u_c, s16x8(&fa)[8], s16x8(&fb)[4], s16x8(&ga)[8], s16x8(&gb)[4]) {
    constexpr int U = decltype(u_c)::value;
    mma(fa, fb, 0);
    asm volatile("s_waitcnt vmcnt(6) lgkmcnt(0)" ::: "memory");
    bar();
    load((U + 1) % W2_STAGES, ga, gb);
    stage(t + 3, U % W2_STAGES);
    mma(fa, fb, 4);
  };
  int t = 0;
  for (; t + 6 <= nt - 3; t += 6) {
    fast(t, std::integral_constant<int, 0>{}, fa0, fb0, fa1, fb1);
    fast(t + 1, std::integral_constant<int, 1>{}, fa1, fb1, fa0, fb0);
    fast(t + 2, std::integral_constant<int, 2>{}, fa0, fb0, fa1, fb1);
    fast(t + 3, std::integral_constant<int, 3>{}, fa1, fb1, fa0, fb0);
    fast(t + 4, std::integral_constant<int, 4>{}, fa0, fb0, fa1, fb1);
    fast(t + 5, std::integral_constant<int, 5>{}, fa1, fb1, fa0, fb0);
  }
  for (; t + 1 < nt; t += 2) {
    body(t, fa0, fb0, fa1, fb1);
    body(t + 1, fa1, fb1, fa0, fb0);
  }
  if (t < nt) body(t, fa0, fb0, fa1, fb1);
  bar();  // every wave is past its last ds_read: LDS is free for the epilogue
  if constexpr (false) {
    float x = 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int i = 0; i < 8; ++i) x += acc[j][i][0] + acc[j][i][1] + acc[j][i][2] + acc[j][i][3];
    if (x == 1.2345e-30f) C[0] = from_f<T>(x);
    return;
  }
  epilogue<T, EPI, EDGE>(acc, smem + wid * 16384, C, M, N, ldc, bias, aux, ldaux, aux_out, part, m0, n0, tm, wr, wc,
                         lane);
}

// ============================================================================================
// "m32" variant of the 8-wave ping-pong kernel: identical tiles, LDS image, staging, phases, waits
// and epilogue, but the fragments are v_mfma_f32_32x32x16 instead of 16x16x32. Per K-tile and
// wave the 128 x 64 sub-tile is 4 x 2 blocks of 32 x 32 over 4 K-steps of 16: 32 MFMAs of 32
// cycles (vs 64 of 16) against the same 24 ds_read_b128 (a 32 x 16 fragment is also 16 B per
// lane: row rb + (lane & 31), K chunk 2 s + (lane >> 5), conflict-free under the same XOR
// swizzle) — the LDS bytes per FLOP are fixed by the wave tile, not the fragment shape; what
// changes is that each MFMA holds the SIMD's issue for 8 of 32 cycles instead of 8 of 16, so the
// partner wave's ds_reads / glds issue gets 3x the free slots per MFMA
// (MI355X_MICROARCH.md, 'vector-instruction ISSUE cost'). Swapped operands as in the 16x16 kernel:
// the accumulator of block (n-block jb, m-block ib) holds, in lane l, M-row 32 ib + (l & 31) and
// N-columns 32 jb + 8 g + 4 (l >> 5) + e in register 4 g + e, which stage_acc32 writes into the
// epilogue's LDS image (the shared epilogue() then runs unchanged with STAGED = true).
typedef float f32x16g __attribute__((ext_vector_type(16)));
__device__ __forceinline__ f32x16g mfma32_bf16(const s16x8& a, const s16x8& b, const f32x16g& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

template <typename T>
__device__ __forceinline__ void mainloop_m32(const T* __restrict__ A, const T* __restrict__ B, int M, int N, int K,
                                             int64_t lda, int64_t ldb, int m0, int n0, char* smem, int wid, int wr,
                                             int wc, int lane, f32x16g (&acc)[2][4]) {
  constexpr int BKE = 64;
  const int nt = K / BKE;
  const int l32 = lane & 31, lh = lane >> 5;
  stage_pieces<T, false>(A, lda, m0, M, 0, smem, wid, lane, 0);
  stage_pieces<T, false>(A, lda, m0, M, 0, smem, wid, lane, 2);
  stage_pieces<T, false>(B, ldb, n0, N, 0, smem + G_TILE_BYTES, wid, lane, 0);
  stage_pieces<T, false>(B, ldb, n0, N, 0, smem + G_TILE_BYTES, wid, lane, 2);
  if (nt > 1) {
    stage_pieces<T, false>(B, ldb, n0, N, BKE, smem + G_BUF_BYTES + G_TILE_BYTES, wid, lane, 0);
    stage_pieces<T, false>(B, ldb, n0, N, BKE, smem + G_BUF_BYTES + G_TILE_BYTES, wid, lane, 2);
    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  bar();
  if (wr == 1) bar();

  s16x8 fa[2][4], fb0[4], fb1[4];
  for (int t = 0; t < nt; ++t) {
    char* cur = smem + (t & 1) * G_BUF_BYTES;
    char* oth = smem + ((t + 1) & 1) * G_BUF_BYTES;
    const char* ta = cur;
    const char* tb = cur + G_TILE_BYTES;
    const bool ld_a = t + 1 < nt, ld_b = t + 2 < nt;
    // p1: A rows 0..63 of the wave, B cols 0..31; stage A(t+1) pieces 0,1
#pragma unroll
    for (int s = 0; s < 4; ++s) fb0[s] = lds_frag(tb, wc * 64 + l32, 2 * s + lh);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int s = 0; s < 4; ++s) fa[i][s] = lds_frag(ta, wr * 128 + i * 32 + l32, 2 * s + lh);
    if (ld_a) stage_pieces<T, false>(A, lda, m0, M, (t + 1) * BKE, oth, wid, lane, 0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    bar();
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int i = 0; i < 2; ++i) acc[0][i] = mfma32_bf16(fb0[s], fa[i][s], acc[0][i]);
    __builtin_amdgcn_s_setprio(0);
    bar();
    // p2: B cols 32..63; stage A(t+1) pieces 2,3
#pragma unroll
    for (int s = 0; s < 4; ++s) fb1[s] = lds_frag(tb, wc * 64 + 32 + l32, 2 * s + lh);
    if (ld_a) stage_pieces<T, false>(A, lda, m0, M, (t + 1) * BKE, oth, wid, lane, 2);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    bar();
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int i = 0; i < 2; ++i) acc[1][i] = mfma32_bf16(fb1[s], fa[i][s], acc[1][i]);
    __builtin_amdgcn_s_setprio(0);
    bar();
    // p3: A rows 64..127; stage B(t+2) pieces 0,1 into this buffer
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int s = 0; s < 4; ++s) fa[i][s] = lds_frag(ta, wr * 128 + 64 + i * 32 + l32, 2 * s + lh);
    if (ld_b) stage_pieces<T, false>(B, ldb, n0, N, (t + 2) * BKE, cur + G_TILE_BYTES, wid, lane, 0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    bar();
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int i = 0; i < 2; ++i) acc[1][2 + i] = mfma32_bf16(fb1[s], fa[i][s], acc[1][2 + i]);
    __builtin_amdgcn_s_setprio(0);
    bar();
    // p4: stage B(t+2) pieces 2,3; retire A(t+1), B(t+1)
    if (ld_b) {
      stage_pieces<T, false>(B, ldb, n0, N, (t + 2) * BKE, cur + G_TILE_BYTES, wid, lane, 2);
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    bar();
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int i = 0; i < 2; ++i) acc[0][2 + i] = mfma32_bf16(fb0[s], fa[i][s], acc[0][2 + i]);
    __builtin_amdgcn_s_setprio(0);
    bar();
  }
}

// the m32 accumulators into the epilogue's LDS image (see stage_acc: element (row, col) of the
// wave tile, col = 4 q + e, lives at row * 128 + ((q >> 1) ^ (row & 7)) * 16 + ((q & 1) ^ ((row >> 3) & 1)) * 8)
template <typename T>
__device__ __forceinline__ void stage_acc32(const f32x16g (&acc)[2][4], char* reg, int lane) {
  const int l32 = lane & 31, lh = lane >> 5;
#pragma unroll
  for (int jb = 0; jb < 2; ++jb)
#pragma unroll
    for (int ib = 0; ib < 4; ++ib) {
      const int row = ib * 32 + l32;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int chunk = (4 * jb + g) ^ (row & 7);
        const int half = lh ^ ((row >> 3) & 1);
        Pack<T, 4> pk;
#pragma unroll
        for (int e = 0; e < 4; ++e) pk.v[e] = from_f<T>(acc[jb][ib][4 * g + e]);
        *reinterpret_cast<Pack<T, 4>*>(reg + row * 128 + chunk * 16 + half * 8) = pk;
      }
    }
}

template <typename T, int EPI, bool EDGE, int DBG = 0>
__global__ void __launch_bounds__(G_THREADS) gemm_m32_kernel(const T* __restrict__ A, const T* __restrict__ B,
                                                             T* __restrict__ C, int M, int N, int K, int64_t lda,
                                                             int64_t ldb, int64_t ldc, const T* __restrict__ bias,
                                                             const T* __restrict__ aux, int64_t ldaux,
                                                             T* __restrict__ aux_out, float* __restrict__ part) {
  __shared__ __attribute__((aligned(16))) char smem[G_LDS_BYTES];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid >> 2, wc = wid & 3;
  const int tiles_m = (M + GB_M - 1) / GB_M, tiles_n = (N + GB_N - 1) / GB_N;
  const int nwg = tiles_m * tiles_n;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, q = nwg >> 3, rr = nwg & 7;
  const int wg = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (bid >> 3);
  const int group = G_GROUP_M * tiles_n;
  const int first_m = (wg / group) * G_GROUP_M;
  const int gm = min(tiles_m - first_m, G_GROUP_M);
  const int tm = first_m + (wg % group) % gm;
  const int tn = (wg % group) / gm;
  const int m0 = tm * GB_M, n0 = tn * GB_N;
  f32x16g acc[2][4];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[j][i] = f32x16g{};
  mainloop_m32<T>(A, B, M, N, K, lda, ldb, m0, n0, smem, wid, wr, wc, lane, acc);
  if (wr == 0) bar();
  bar();
  if constexpr (DBG & 512) {  // keep the accumulators live, store nothing
    float t = 0.f;
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int e = 0; e < 16; ++e) t += acc[j][i][e];
    if (t == 1.2345e-30f) C[0] = from_f<T>(t);
    return;
  }
  char* reg = smem + wid * 16384;
  stage_acc32<T>(acc, reg, lane);
  const f32x4 dummy[4][8] = {};
  epilogue<T, EPI, EDGE, 0, 4, true>(dummy, reg, C, M, N, ldc, bias, aux, ldaux, aux_out, part, m0, n0, tm, wr, wc,
                                     lane);
}

// ============================================================================================
// "w8p": the 8-wave kernel without the ping-pong. Same 256 x 256 x 64 tiles, LDS image, glds
// staging, wave tiles (128 x 64, 8 x 4 fragments of 16x16x32) and epilogue, but every wave
// software-pipelines its own fragment reads one K-step (32 of K) ahead of its MFMAs, and the
// workgroup meets at ONE barrier per K-tile instead of eight:
//   k-step 0 of tile t: 32 MFMAs on F0(t) | the 12 ds_read_b128 of F1(t) interleaved
//   vmcnt(0) (tile t+1 landed) + lgkmcnt(0) (F1(t) in registers) | barrier
//   issue tile t+2's glds into tile t's buffer (free: every wave is past its reads of it)
//   k-step 1 of tile t: 32 MFMAs on F1(t) | the 12 reads of F0(t+1) from the other buffer
// The ping-pong's read sections end in lgkmcnt(0) + a barrier each, so their LDS latency (and the
// 12-read section's queueing) is exposed whenever it outlasts the partner group's 16-MFMA section
// (profiles/r3_gemmlab_w8_ablation.txt: no ds_read -29 %, i.e. the reads are not hidden). Here a
// read has a whole K-step (32 MFMAs of its own wave, 64 on the SIMD) to land. Costs: 96 VGPRs of
// double-buffered fragments next to the 128 accumulators, and tile t+1's copies get one K-tile
// (~1 us) of flight time instead of the ping-pong's two for B.
// Registers: fragments are double-buffered per HALF K-step (A: 4 row fragments of one 64-row half,
// B: the 4 column fragments of one K-step), 64 VGPRs next to the 128 accumulators — a whole
// K-step of both (96 VGPRs) did not fit the 256 of a two-waves-per-SIMD kernel (334 spilled).
// Four stages per K-tile (K-step s, row half h), 16 MFMAs each, the next stage's fragments read
// during the current one:
//   (0,0) reads A(s0,h1)          (0,1) reads A(s1,h0) + B(s1)
//   (1,0) reads A(s1,h1) | vmcnt(0) + lgkmcnt(0), barrier, glds of tile t+2 into this buffer
//   (1,1) reads A(s0,h0) + B(s0) of tile t+1 from the other buffer
template <int NI>
__device__ __forceinline__ void w8p_fa(const char* buf, int wr, int h, int s, int lr, int lk, s16x8 (&fa)[NI]) {
#pragma unroll
  for (int i = 0; i < NI; ++i) fa[i] = frag<false>(buf, wr * 128 + h * 64 + i * 16, s, lr, lk);
}
__device__ __forceinline__ void w8p_fb(const char* buf, int wc, int s, int lr, int lk, s16x8 (&fb)[4]) {
#pragma unroll
  for (int j = 0; j < 4; ++j) fb[j] = frag<false>(buf + G_TILE_BYTES, wc * 64 + j * 16, s, lr, lk);
}

// 16 MFMAs of one stage (rows of half h) with NR fragment reads interleaved
template <typename T, int NR>
__device__ __forceinline__ void w8p_stage(const s16x8 (&fa)[4], const s16x8 (&fb)[4], f32x4 (&acc)[4][8], int h) {
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[j][4 * h + i] = mfma16<T>(fb[j], fa[i], acc[j][4 * h + i]);
  constexpr int PER = NR > 0 ? 16 / NR : 16;
#ifndef W8P_NOSCHED
#pragma unroll
  for (int g = 0; g < NR; ++g) {
    __builtin_amdgcn_sched_group_barrier(0x008, PER, 0);  // MFMA
    __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);        // DS read
  }
#endif
}

template <typename T>
__device__ __forceinline__ void mainloop_w8p(const T* __restrict__ A, const T* __restrict__ B, int M, int N, int K,
                                             int64_t lda, int64_t ldb, int m0, int n0, char* smem, int wid, int wr,
                                             int wc, int lane, f32x4 (&acc)[4][8]) {
  constexpr int BKE = 64;
  const int nt = K / BKE;
  const int lr = lane & 15, lk = lane >> 4;
  // glds through buffer resources (wave-uniform bases in SGPRs, one 32-bit voffset per piece and
  // lane, the K-tile in soffset; rows past M / N read zero): 64-bit flat addresses per piece were
  // spilled to scratch here, and every reload's vmcnt(0) then also waited for the copies in flight
  const __amdgpu_buffer_rsrc_t rsa =
      wave_rsrc(A + (int64_t)m0 * lda, (uint32_t)(min(M - m0, GB_M) * lda * (int64_t)sizeof(T)));
  const __amdgpu_buffer_rsrc_t rsb =
      wave_rsrc(B + (int64_t)n0 * ldb, (uint32_t)(min(N - n0, GB_N) * ldb * (int64_t)sizeof(T)));
  uint32_t va[4], vb[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    va[j] = piece_voff<T, false>(wid * 4 + j, lane, lda);
    vb[j] = piece_voff<T, false>(wid * 4 + j, lane, ldb);
  }
  auto stage_tile = [&](int t, char* buf) {
    const uint32_t so = (uint32_t)(t * BKE * (int)sizeof(T));
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      bglds16(rsa, buf + (wid * 4 + j) * 1024, va[j], so);
      bglds16(rsb, buf + G_TILE_BYTES + (wid * 4 + j) * 1024, vb[j], so);
    }
  };
  stage_tile(0, smem);
  if (nt > 1) {
    stage_tile(1, smem + G_BUF_BYTES);
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");  // tile 0's 8 pieces (tile 1's stay in flight)
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  bar();
  s16x8 fa0[4], fa1[4], fb0[4], fb1[4];
  w8p_fa<4>(smem, wr, 0, 0, lr, lk, fa0);
  w8p_fb(smem, wc, 0, lr, lk, fb0);
  // unrolled by two so each half's buffers are compile-time (no per-iteration buffer select; the
  // fragment registers keep their places across the back edge)
  auto iter = [&](const int t, char* cur, char* nxt) {
    w8p_fa<4>(cur, wr, 1, 0, lr, lk, fa1);  // (0,0): reads A(s0,h1)
    w8p_stage<T, 4>(fa0, fb0, acc, 0);
    w8p_fa<4>(cur, wr, 0, 1, lr, lk, fa0);  // (0,1): reads A(s1,h0) + B(s1)
    w8p_fb(cur, wc, 1, lr, lk, fb1);
    w8p_stage<T, 8>(fa1, fb0, acc, 1);
    w8p_fa<4>(cur, wr, 1, 1, lr, lk, fa1);  // (1,0): reads A(s1,h1)
    w8p_stage<T, 4>(fa0, fb1, acc, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // tile t+1 landed (this wave's pieces)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's reads of tile t retired
    bar();
    if (t + 2 < nt) stage_tile(t + 2, cur);
    if (t + 1 < nt) {  // (1,1): reads A(s0,h0) + B(s0) of tile t+1
      w8p_fa<4>(nxt, wr, 0, 0, lr, lk, fa0);
      w8p_fb(nxt, wc, 0, lr, lk, fb0);
      w8p_stage<T, 8>(fa1, fb1, acc, 1);
    } else {
      w8p_stage<T, 0>(fa1, fb1, acc, 1);
    }
  };
  for (int t = 0; t < nt; t += 2) {
    iter(t, smem, smem + G_BUF_BYTES);
    if (t + 1 < nt) iter(t + 1, smem + G_BUF_BYTES, smem);
  }
}

template <typename T, int EPI, bool EDGE, int DBG = 0>
__global__ void __launch_bounds__(G_THREADS) gemm_w8p_kernel(const T* __restrict__ A, const T* __restrict__ B,
                                                             T* __restrict__ C, int M, int N, int K, int64_t lda,
                                                             int64_t ldb, int64_t ldc, const T* __restrict__ bias,
                                                             const T* __restrict__ aux, int64_t ldaux,
                                                             T* __restrict__ aux_out, float* __restrict__ part) {
  __shared__ __attribute__((aligned(16))) char smem[G_LDS_BYTES];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid >> 2, wc = wid & 3;
  const int tiles_m = (M + GB_M - 1) / GB_M, tiles_n = (N + GB_N - 1) / GB_N;
  const int nwg = tiles_m * tiles_n;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, q = nwg >> 3, rr = nwg & 7;
  const int wg = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (bid >> 3);
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
  mainloop_w8p<T>(A, B, M, N, K, lda, ldb, m0, n0, smem, wid, wr, wc, lane, acc);
  bar();  // every wave is past its last ds_read: LDS is free for the epilogue
  if constexpr (DBG & 512) {
    float t = 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int i = 0; i < 8; ++i) t += acc[j][i][0] + acc[j][i][1] + acc[j][i][2] + acc[j][i][3];
    if (t == 1.2345e-30f) C[0] = from_f<T>(t);
    return;
  }
  epilogue<T, EPI, EDGE, 0, 4, false>(acc, smem + wid * 16384, C, M, N, ldc, bias, aux, ldaux, aux_out, part, m0, n0,
                                      tm, wr, wc, lane);
}

}  // namespace
}  // namespace apex
