// Weight-gradient GEMM lab (no torch): the transposed-read (TR) path of csrc/gemm.hip
// (C[P, Q] = sum_r A[r, p] B[r, q], split-K over r into fp32 slabs) at the BERT-Large weight
// shapes, with ablations, against the NT kernel on a problem of the same tile count and per-tile
// contraction length. Build + run (GPU box):
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -Icsrc tools/gemmlab/tr_lab.hip -o labbin/trlab
//   labbin/trlab P Q R splits [rounds=5] [reps=10]
// Variants:
//   tr_f32       production (EPI_F32 slabs)
//   tr_noepi     main loop only (accumulators kept live, nothing stored)
//   tr_nodsread  ... and no fragment ds_reads
//   tr_noglds    ... and no global->LDS copies (main loop: barriers + ds_reads + MFMAs)
//   *_old        the same with the previous main loop (mainloop_bk64, DBG bit 1024; production is
//                mainloop_bal); its fp32 slabs are compared with production's (max |diff|, "maxdiff")
//   nt_f32 / nt_noepi   the NT kernel on [P*splits, R/splits] x [Q, R/splits] (same tiles, same
//                per-tile K, operands K-contiguous)
// One JSON line per variant: us per call (min / median over rounds), PF/s.
#include "../../csrc/gemm.hip"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

using namespace apex;

#define CK(x)                                                                                     \
  do {                                                                                            \
    hipError_t e_ = (x);                                                                          \
    if (e_ != hipSuccess) {                                                                       \
      fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__);      \
      exit(2);                                                                                    \
    }                                                                                             \
  } while (0)

__global__ void fill_kernel(bf16* p, int64_t n, uint32_t seed) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    h ^= h >> 16; h *= 0x85ebca6bu; h ^= h >> 13;
    p[i] = (bf16)((h & 0xFFFF) / 32768.f - 1.f);
  }
}

__global__ void maxdiff_kernel(const float* a, const float* b, int64_t n, float* out) {
  float m = 0.f;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const float d = fabsf(a[i] - b[i]);
    if (!(d <= m)) m = d;
  }
  for (int o = 32; o; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  if ((threadIdx.x & 63) == 0) atomicMax((int*)out, __float_as_int(m));
}

struct Prob {
  bf16 *A, *B, *C;
  float* part;
  int P, Q, R, S;
};

template <int EPI, int DBG>
void tr(const Prob& p, hipStream_t s) {
  const int tiles = (p.P / GB_M) * (p.Q / GB_N);
  hipLaunchKernelGGL((gemm_nt_kernel<bf16, EPI, true, false, bf16, -1, -1, DBG>), dim3(tiles, p.S), dim3(G_THREADS), 0,
                     s, p.A, p.B, p.C, p.P, p.Q, p.R, (int64_t)p.P, (int64_t)p.Q, (int64_t)p.Q, nullptr, nullptr,
                     (int64_t)0, nullptr, p.part, 0);
}

// the four-wave kernel (one wave per SIMD, 128 x 128 wave tiles: half the fragment reads per FLOP
// of the 8-wave 128 x 64 tile, which matters most for the transposed reads' doubled LDS instruction
// count); DBG 256 = its register-staged loop
template <int EPI, int DBG>
void tr_w4(const Prob& p, hipStream_t s) {
  const int tiles = (p.P / GB_M) * (p.Q / GB_N);
  hipLaunchKernelGGL((gemm_w4_kernel<bf16, EPI, true, false, DBG>), dim3(tiles, p.S), dim3(W_THREADS), 0, s, p.A, p.B,
                     p.C, p.P, p.Q, p.R / p.S, (int64_t)p.P, (int64_t)p.Q, (int64_t)p.Q, nullptr, nullptr, (int64_t)0,
                     nullptr, p.part);
}

template <int EPI, int DBG>
void nt(const Prob& p, hipStream_t s) {
  const int Kc = p.R / p.S, M = p.P * p.S;
  const int tiles = (M / GB_M) * (p.Q / GB_N);
  hipLaunchKernelGGL((gemm_nt_kernel<bf16, EPI, false, false, bf16, -1, -1, DBG>), dim3(tiles), dim3(G_THREADS), 0, s,
                     p.A, p.B, p.C, M, p.Q, Kc, (int64_t)Kc, (int64_t)Kc, (int64_t)p.Q, nullptr, nullptr, (int64_t)0,
                     nullptr, p.part, 0);
}

int main(int argc, char** argv) {
  if (argc < 5) {
    fprintf(stderr, "usage: %s P Q R splits [rounds] [reps]\n", argv[0]);
    return 1;
  }
  Prob p;
  p.P = atoi(argv[1]);
  p.Q = atoi(argv[2]);
  p.R = atoi(argv[3]);
  p.S = atoi(argv[4]);
  const int rounds = argc > 5 ? atoi(argv[5]) : 5;
  const int reps = argc > 6 ? atoi(argv[6]) : 10;
  if (p.P % 256 || p.Q % 256 || p.R % (p.S * 64)) {
    fprintf(stderr, "P, Q must be multiples of 256 and R of 64 * splits\n");
    return 1;
  }
  const int64_t nA = (int64_t)p.R * p.P, nB = (int64_t)p.R * p.Q;
  CK(hipMalloc(&p.A, nA * 2));
  CK(hipMalloc(&p.B, nB * 2));
  CK(hipMalloc(&p.C, (int64_t)p.P * p.S * p.Q * 2));
  CK(hipMalloc(&p.part, (int64_t)p.S * p.P * p.Q * 4));
  hipStream_t s;
  CK(hipStreamCreate(&s));
  hipLaunchKernelGGL(fill_kernel, dim3(2048), dim3(256), 0, s, p.A, nA, 1u);
  hipLaunchKernelGGL(fill_kernel, dim3(2048), dim3(256), 0, s, p.B, nB, 2u);
  CK(hipStreamSynchronize(s));
  struct V {
    const char* name;
    void (*fn)(const Prob&, hipStream_t);
  };
  std::vector<V> vs = {{"tr_f32", tr<EPI_F32, 0>},
                       {"tr_w4_f32", tr_w4<EPI_F32, 0>},
                       {"tr_w4r_f32", tr_w4<EPI_F32, 256>},
                       {"tr_f32_old", tr<EPI_F32, 1024>},
                       {"tr_noepi", tr<EPI_NONE, 512>},
                       {"tr_noepi_old", tr<EPI_NONE, 512 + 1024>},
                       {"tr_nodsread", tr<EPI_NONE, 512 + 128>},
                       {"tr_noglds", tr<EPI_NONE, 512 + 32>},
                       {"nt_f32", nt<EPI_F32, 0>},
                       {"nt_f32_old", nt<EPI_F32, 1024>},
                       {"nt_noepi", nt<EPI_NONE, 512>},
                       {"nt_nodsread", nt<EPI_NONE, 512 + 128>}};
  // correctness: each *_f32_old slab set against the production loop's
  const int64_t nP = (int64_t)p.S * p.P * p.Q;
  float *ref, *dmax;
  CK(hipMalloc(&ref, nP * 4));
  CK(hipMalloc(&dmax, 4));
  std::vector<float> diff(vs.size(), -1.f);
  for (size_t v = 0; v < vs.size(); ++v) {
    const std::string nm = vs[v].name;
    if (nm == "tr_f32" || nm == "nt_f32") {
      vs[v].fn(p, s);
      CK(hipMemcpyAsync(ref, p.part, nP * 4, hipMemcpyDeviceToDevice, s));
    } else if (nm == "tr_f32_old" || nm == "nt_f32_old" || nm == "tr_w4_f32" || nm == "tr_w4r_f32") {
      CK(hipMemsetAsync(p.part, 0, nP * 4, s));
      vs[v].fn(p, s);
      CK(hipMemsetAsync(dmax, 0, 4, s));
      hipLaunchKernelGGL(maxdiff_kernel, dim3(1024), dim3(256), 0, s, p.part, ref, nP, dmax);
      CK(hipMemcpyAsync(&diff[v], dmax, 4, hipMemcpyDeviceToHost, s));
    }
    CK(hipStreamSynchronize(s));
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<std::vector<float>> t(vs.size());
  for (int r = 0; r < rounds; ++r)
    for (size_t v = 0; v < vs.size(); ++v) {
      vs[v].fn(p, s);
      CK(hipGetLastError());
      CK(hipEventRecord(e0, s));
      for (int i = 0; i < reps; ++i) vs[v].fn(p, s);
      CK(hipEventRecord(e1, s));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      t[v].push_back(ms * 1000.f / reps);
    }
  const double flop = 2.0 * p.P * p.Q * (double)p.R;
  for (size_t v = 0; v < vs.size(); ++v) {
    std::vector<float> x = t[v];
    std::sort(x.begin(), x.end());
    printf("{\"P\": %d, \"Q\": %d, \"R\": %d, \"splits\": %d, \"variant\": \"%s\", \"us_min\": %.1f, \"us_med\": %.1f, "
           "\"pflops\": %.3f, \"maxdiff\": %g}\n",
           p.P, p.Q, p.R, p.S, vs[v].name, x[0], x[x.size() / 2], flop / (x[0] * 1e-6) / 1e15, diff[v]);
  }
  fflush(stdout);
  return 0;
}
