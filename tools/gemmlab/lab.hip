// Standalone GEMM lab (no torch): times kernel variants of csrc/gemm.hip against each other on
// random bf16 operands, interleaved in one process, and checks every variant's output against the
// 8-wave reference kernel. Build + run (GPU box):
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -Icsrc tools/gemmlab/lab.hip -o build/gemmlab
//   build/gemmlab M N K [epi=0] [rounds=5] [reps=10]
// Prints one JSON line per variant: us per call (min / median over rounds), PF/s, max |diff|.
#include "../../csrc/gemm.hip"
#include "lab_variants.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <vector>

using namespace apex;

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      exit(2);                                                                       \
    }                                                                                \
  } while (0)

__global__ void fill_kernel(bf16* p, int64_t n, uint32_t seed, float scale) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    h ^= h >> 16; h *= 0x85ebca6bu; h ^= h >> 13; h *= 0xc2b2ae35u; h ^= h >> 16;
    p[i] = (bf16)(((h & 0xFFFFFF) / 8388608.f - 1.f) * scale);
  }
}

__global__ void maxdiff_kernel(const bf16* a, const bf16* b, int64_t n, float* out) {
  float m = 0.f;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    float d = fabsf((float)a[i] - (float)b[i]);
    if (!(d <= m)) m = d;  // NaN propagates
  }
  for (int o = 32; o; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  if ((threadIdx.x & 63) == 0) atomicMax((int*)out, __float_as_int(m));
}

// error census: count of |a - b| > thr per 16 x 16 fragment position inside the 256 x 256 tile
__global__ void errmap_kernel(const bf16* a, const bf16* b, int M, int N, float thr, unsigned* hist) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < (int64_t)M * N; i += (int64_t)gridDim.x * blockDim.x) {
    const float d = fabsf((float)a[i] - (float)b[i]);
    if (!(d <= thr)) {
      const int r = (int)(i / N) & 255, c = (int)(i % N) & 255;
      atomicAdd(&hist[(r >> 4) * 16 + (c >> 4)], 1u);
    }
  }
}

struct Bufs {
  bf16 *A, *B, *bias, *aux, *C, *Cref, *aux_out, *aux_ref;
  float* part;
  int M, N, K;
};

typedef void (*Launch)(const Bufs&, int epi, hipStream_t);

template <int EPI, int DBG = 0, int STAGGER = 0>
void launch_old(const Bufs& b, hipStream_t s) {
  const int tiles = ((b.M + 255) / 256) * ((b.N + 255) / 256);
  if (b.M % 256 || b.N % 256)  // partial tiles: the bounds-checked instantiation (as launch_gemm)
    hipLaunchKernelGGL((gemm_nt_kernel<bf16, EPI, false, true, bf16, -1, -1, DBG>), dim3(tiles), dim3(512), 0, s, b.A, b.B, b.C,
                       b.M, b.N, b.K, (int64_t)b.K, (int64_t)b.K, (int64_t)b.N, b.bias, b.aux, (int64_t)b.N, b.aux_out, b.part,
                       STAGGER, nullptr, nullptr);
  else
    hipLaunchKernelGGL((gemm_nt_kernel<bf16, EPI, false, false, bf16, -1, -1, DBG>), dim3(tiles), dim3(512), 0, s, b.A, b.B, b.C,
                       b.M, b.N, b.K, (int64_t)b.K, (int64_t)b.K, (int64_t)b.N, b.bias, b.aux, (int64_t)b.N, b.aux_out, b.part,
                       STAGGER, nullptr, nullptr);
}
// timeline trace (LAB_TRACE): the production kernel with DBG bit 2048, 4 x uint64 per workgroup
uint64_t* g_trace = nullptr;
template <int EPI>
void launch_trace(const Bufs& b, hipStream_t s) {
  const int tiles = ((b.M + 255) / 256) * ((b.N + 255) / 256);
  hipLaunchKernelGGL((gemm_nt_kernel<bf16, EPI, false, false, bf16, -1, -1, 2048>), dim3(tiles), dim3(512), 0, s, b.A, b.B,
                     b.C, b.M, b.N, b.K, (int64_t)b.K, (int64_t)b.K, (int64_t)b.N, b.bias, b.aux, (int64_t)b.N, b.aux_out,
                     b.part, 0, (const float*)g_trace, nullptr);
}

int g_cus = 0;
template <int EPI, int DBG = 0>
void launch_persist(const Bufs& b, hipStream_t s) {
  const int tiles = (b.M / 256) * (b.N / 256);
  const int grid = std::min(tiles, g_cus);
  hipLaunchKernelGGL((gemm_persist_kernel<bf16, EPI, bf16, -1, -1, 0, DBG>), dim3(grid), dim3(512), 0, s, b.A, b.B, b.C, b.M, b.N, b.K,
                     (int64_t)b.K, (int64_t)b.K, (int64_t)b.N, b.bias, b.aux, (int64_t)b.N, b.aux_out, b.part, g_trace);
}

// Summary of one traced launch: per-phase durations, the gap between a workgroup's end and the next
// start on the same CU, and how many workgroups sit in their epilogue at the same time (lockstep).
void trace_summary(const Bufs& b, int epi, hipStream_t s, void (*fn)(const Bufs&, hipStream_t)) {
  const int tiles = ((b.M + 255) / 256) * ((b.N + 255) / 256);
  static int call = 0;
  const char* tname = (call++ % 2) ? "persist" : "w8";
  CK(hipMalloc(&g_trace, (size_t)tiles * 32));
  fn(b, s);
  CK(hipMemsetAsync(g_trace, 0, (size_t)tiles * 32, s));
  fn(b, s);
  std::vector<uint64_t> h((size_t)tiles * 4);
  CK(hipMemcpyAsync(h.data(), g_trace, (size_t)tiles * 32, hipMemcpyDeviceToHost, s));
  CK(hipStreamSynchronize(s));
  CK(hipFree(g_trace));
  g_trace = nullptr;
  uint64_t t0 = ~0ull, tend = 0;
  for (int i = 0; i < tiles; ++i) {
    t0 = std::min(t0, h[i * 4]);
    tend = std::max(tend, h[i * 4 + 2]);
  }
  std::vector<double> ml, ep, gaps;
  std::vector<std::pair<uint64_t, int>> ev;  // (time, +1 epilogue start / -1 end)
  std::map<uint64_t, std::vector<std::pair<uint64_t, uint64_t>>> percu;
  for (int i = 0; i < tiles; ++i) {
    const uint64_t a = h[i * 4], m = h[i * 4 + 1], e = h[i * 4 + 2], id = h[i * 4 + 3];
    ml.push_back((m - a) * 0.01);
    ep.push_back((e - m) * 0.01);
    const uint64_t hw = id & 0xffffffffull, xcc = id >> 32;
    const uint64_t cu = ((xcc & 0xf) << 16) | (((hw >> 13) & 7) << 8) | (((hw >> 12) & 1) << 4) | ((hw >> 8) & 0xf);
    percu[cu].push_back({a, e});
    ev.push_back({m, +1});
    ev.push_back({e, -1});
  }
  for (auto& kv : percu) {
    auto v = kv.second;
    std::sort(v.begin(), v.end());
    for (size_t j = 1; j < v.size(); ++j) gaps.push_back(((double)v[j].first - (double)v[j - 1].second) * 0.01);
  }
  std::sort(ev.begin(), ev.end());
  // time-weighted histogram of the number of workgroups in their epilogue
  int cur = 0, peak = 0;
  double w[5] = {0, 0, 0, 0, 0};  // 0, 1-63, 64-127, 128-191, 192+
  for (size_t j = 0; j + 1 < ev.size(); ++j) {
    cur += ev[j].second;
    peak = std::max(peak, cur);
    const double dt = (double)(ev[j + 1].first - ev[j].first) * 0.01;
    w[cur == 0 ? 0 : 1 + std::min(3, cur / 64)] += dt;
  }
  auto med = [](std::vector<double> v) {
    if (v.empty()) return 0.0;
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
  };
  auto mean = [](const std::vector<double>& v) {
    double t = 0;
    for (double x : v) t += x;
    return v.empty() ? 0.0 : t / v.size();
  };
  const double span = (tend - t0) * 0.01;
  printf("{\"trace\": \"%s\", \"M\": %d, \"N\": %d, \"K\": %d, \"epi\": %d, \"span_us\": %.1f, \"cus\": %zu, "
         "\"mainloop_us_med\": %.2f, \"mainloop_us_mean\": %.2f, \"epi_us_med\": %.2f, \"epi_us_mean\": %.2f, "
         "\"gap_us_med\": %.2f, \"gap_us_mean\": %.2f, \"epi_concurrency_peak\": %d, "
         "\"time_frac_epi_wgs\": {\"0\": %.3f, \"1-63\": %.3f, \"64-127\": %.3f, \"128-191\": %.3f, \"192+\": %.3f}}\n",
         tname, b.M, b.N, b.K, epi, span, percu.size(), med(ml), mean(ml), med(ep), mean(ep), med(gaps), mean(gaps), peak,
         w[0] / span, w[1] / span, w[2] / span, w[3] / span, w[4] / span);
  fflush(stdout);
}

template <int EPI, int DBG = 0>
void launch_w4(const Bufs& b, hipStream_t s) {
  const int tiles = ((b.M + 255) / 256) * ((b.N + 255) / 256);
  hipLaunchKernelGGL((gemm_w4_kernel<bf16, EPI, false, false, DBG>), dim3(tiles), dim3(256), 0, s, b.A, b.B, b.C, b.M, b.N,
                     b.K, (int64_t)b.K, (int64_t)b.K, (int64_t)b.N, b.bias, b.aux, (int64_t)b.N, b.aux_out, b.part);
}

template <int EPI>
void launch_w2g(const Bufs& b, hipStream_t s) {
  const int tiles = ((b.M + 255) / 256) * ((b.N + 127) / 128);
  hipLaunchKernelGGL((gemm_w2g_kernel<bf16, EPI, false>), dim3(tiles), dim3(256), 0, s, b.A, b.B, b.C, b.M, b.N, b.K,
                     (int64_t)b.K, (int64_t)b.K, (int64_t)b.N, b.bias, b.aux, (int64_t)b.N, b.aux_out, b.part);
}

template <int EPI, int DBG = 0>
void launch_m32(const Bufs& b, hipStream_t s) {
  const int tiles = ((b.M + 255) / 256) * ((b.N + 255) / 256);
  hipLaunchKernelGGL((gemm_m32_kernel<bf16, EPI, false, DBG>), dim3(tiles), dim3(512), 0, s, b.A, b.B, b.C, b.M, b.N,
                     b.K, (int64_t)b.K, (int64_t)b.K, (int64_t)b.N, b.bias, b.aux, (int64_t)b.N, b.aux_out, b.part);
}

template <int EPI, int DBG = 0>
void launch_w8p(const Bufs& b, hipStream_t s) {
  const int tiles = ((b.M + 255) / 256) * ((b.N + 255) / 256);
  hipLaunchKernelGGL((gemm_w8p_kernel<bf16, EPI, false, DBG>), dim3(tiles), dim3(512), 0, s, b.A, b.B, b.C, b.M, b.N,
                     b.K, (int64_t)b.K, (int64_t)b.K, (int64_t)b.N, b.bias, b.aux, (int64_t)b.N, b.aux_out, b.part);
}

template <int EPI>
void run_epi(Bufs& b, int rounds, int reps, hipStream_t s) {
  struct V {
    const char* name;
    void (*fn)(const Bufs&, hipStream_t);
  };
  std::vector<V> vs = {{"w8", launch_old<EPI>}, {"w8old", launch_old<EPI, 1024>}};
  // the other variants have no bounds-checked form: full tiles only
  const bool full = b.M % 256 == 0 && b.N % 256 == 0;
  if (full && getenv("LAB_W8P")) vs.push_back({"w8p", launch_w8p<EPI>});
  if (full && getenv("LAB_M32")) vs.push_back({"w8m32", launch_m32<EPI>});
  if (full && getenv("LAB_W2G")) vs.push_back({"w2g", launch_w2g<EPI>});
  if (full && getenv("LAB_NOEPI")) {
    vs.push_back({"w8_noepi", launch_old<EPI, 512>});
    vs.push_back({"w8p_noepi", launch_w8p<EPI, 512>});
  }
  if (full && getenv("LAB_W4")) {
    vs.push_back({"w4", launch_w4<EPI>});
    vs.push_back({"w4r", launch_w4<EPI, 256>});
  }
  if (full && getenv("LAB_DBG")) {
    vs.push_back({"w8_noglds", launch_old<EPI, 32>});
    vs.push_back({"w8_nobar", launch_old<EPI, 64>});
    vs.push_back({"w8_nodsread", launch_old<EPI, 128>});
    vs.push_back({"w8_nomem", launch_old<EPI, 32 + 64 + 128>});
    vs.push_back({"w8_noepi", launch_old<EPI, 512>});
  }
  if (full && getenv("LAB_STAGGER")) {
    vs.push_back({"w8_st1", launch_old<EPI, 0, 1>});
    vs.push_back({"w8_st2", launch_old<EPI, 0, 2>});
    vs.push_back({"w8_st3", launch_old<EPI, 0, 3>});
    vs.push_back({"w8_st5", launch_old<EPI, 0, 5>});
  }
  if (full && getenv("LAB_TRACE")) {
    trace_summary(b, EPI, s, launch_trace<EPI>);
    trace_summary(b, EPI, s, launch_persist<EPI, 2048>);
  }
  if (full && !getenv("LAB_NOPERSIST")) vs.push_back({"w8pers", launch_persist<EPI>});
  if (full && getenv("LAB_PXD")) {  // persistent-kernel epilogue diagnostics (epilogue XD bits)
    vs.push_back({"pers_nomath", launch_persist<EPI, 4096>});
    vs.push_back({"pers_nostore", launch_persist<EPI, 8192>});
    vs.push_back({"pers_nomath_nostore", launch_persist<EPI, 12288>});
  }
  if (full && getenv("LAB_NT")) {  // non-temporal epilogue stores (XD bits 2, 3)
    vs.push_back({"pers_nt_aux", launch_persist<EPI, 16384>});
    vs.push_back({"pers_nt_c", launch_persist<EPI, 32768>});
    vs.push_back({"pers_nt_both", launch_persist<EPI, 49152>});
  }
  const int64_t MN = (int64_t)b.M * b.N;
  float* dmax;
  CK(hipMalloc(&dmax, 4));
  // reference output from the 8-wave kernel
  bf16* C0 = b.C;
  bf16* AO0 = b.aux_out;
  b.C = b.Cref;
  b.aux_out = b.aux_ref;
  vs[0].fn(b, s);
  b.C = C0;
  b.aux_out = AO0;
  CK(hipStreamSynchronize(s));
  std::vector<std::vector<float>> t(vs.size());
  std::vector<float> diff(vs.size(), 0.f);
  for (size_t v = 0; v < vs.size(); ++v) {
    CK(hipMemsetAsync(b.C, 0, MN * 2, s));
    vs[v].fn(b, s);
    CK(hipMemsetAsync(dmax, 0, 4, s));
    hipLaunchKernelGGL(maxdiff_kernel, dim3(1024), dim3(256), 0, s, b.C, b.Cref, MN, dmax);
    CK(hipMemcpyAsync(&diff[v], dmax, 4, hipMemcpyDeviceToHost, s));
    CK(hipStreamSynchronize(s));
    if (getenv("LAB_ERRMAP") && diff[v] > 0.02f) {
      unsigned* dh;
      CK(hipMalloc(&dh, 256 * 4));
      CK(hipMemsetAsync(dh, 0, 256 * 4, s));
      hipLaunchKernelGGL(errmap_kernel, dim3(1024), dim3(256), 0, s, b.C, b.Cref, b.M, b.N, 0.02f, dh);
      unsigned h[256];
      CK(hipMemcpyAsync(h, dh, 256 * 4, hipMemcpyDeviceToHost, s));
      CK(hipStreamSynchronize(s));
      printf("errmap %s (rows: fragment row 0..15 of the tile; cols: fragment col 0..15)\n", vs[v].name);
      for (int r = 0; r < 16; ++r) {
        for (int c = 0; c < 16; ++c) printf("%7u", h[r * 16 + c]);
        printf("\n");
      }
      CK(hipFree(dh));
    }
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int r = 0; r < rounds; ++r)
    for (size_t v = 0; v < vs.size(); ++v) {
      vs[v].fn(b, s);  // warm
      CK(hipEventRecord(e0, s));
      for (int i = 0; i < reps; ++i) vs[v].fn(b, s);
      CK(hipEventRecord(e1, s));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      t[v].push_back(ms * 1000.f / reps);
    }
  const double flop = 2.0 * b.M * b.N * b.K;
  for (size_t v = 0; v < vs.size(); ++v) {
    std::vector<float> x = t[v];
    std::sort(x.begin(), x.end());
    printf("{\"M\": %d, \"N\": %d, \"K\": %d, \"epi\": %d, \"variant\": \"%s\", \"us_min\": %.1f, \"us_med\": %.1f, "
           "\"pflops\": %.3f, \"maxdiff\": %g}\n",
           b.M, b.N, b.K, EPI, vs[v].name, x[0], x[x.size() / 2], flop / (x[0] * 1e-6) / 1e15, diff[v]);
  }
  fflush(stdout);
  CK(hipFree(dmax));
}

int main(int argc, char** argv) {
  if (argc < 4) {
    fprintf(stderr, "usage: %s M N K [epi] [rounds] [reps]\n", argv[0]);
    return 1;
  }
  Bufs b;
  b.M = atoi(argv[1]);
  b.N = atoi(argv[2]);
  b.K = atoi(argv[3]);
  if (b.K % 64 || b.N % 8 || b.M <= 0) {  // what gemm_supported() requires of every launch
    fprintf(stderr, "K must be a multiple of 64 and N of 8\n");
    return 1;
  }
  const int epi = argc > 4 ? atoi(argv[4]) : 0;
  const int rounds = argc > 5 ? atoi(argv[5]) : 5;
  const int reps = argc > 6 ? atoi(argv[6]) : 10;
  const int64_t MK = (int64_t)b.M * b.K, NK = (int64_t)b.N * b.K, MN = (int64_t)b.M * b.N;
  CK(hipMalloc(&b.A, MK * 2));
  CK(hipMalloc(&b.B, NK * 2));
  CK(hipMalloc(&b.bias, b.N * 2));
  CK(hipMalloc(&b.aux, MN * 2));
  CK(hipMalloc(&b.C, MN * 2));
  CK(hipMalloc(&b.Cref, MN * 2));
  CK(hipMalloc(&b.aux_out, MN * 2));
  CK(hipMalloc(&b.aux_ref, MN * 2));
  CK(hipMalloc(&b.part, (int64_t)((b.M + 255) / 256) * 2 * b.N * 4));
  hipStream_t s;
  CK(hipStreamCreate(&s));
  CK(hipDeviceGetAttribute(&g_cus, hipDeviceAttributeMultiprocessorCount, 0));
  hipLaunchKernelGGL(fill_kernel, dim3(2048), dim3(256), 0, s, b.A, MK, 1u, 1.f);
  hipLaunchKernelGGL(fill_kernel, dim3(2048), dim3(256), 0, s, b.B, NK, 2u, 1.f / sqrtf((float)b.K));
  hipLaunchKernelGGL(fill_kernel, dim3(64), dim3(256), 0, s, b.bias, (int64_t)b.N, 3u, 0.1f);
  hipLaunchKernelGGL(fill_kernel, dim3(2048), dim3(256), 0, s, b.aux, MN, 4u, 1.f);
  CK(hipStreamSynchronize(s));
  switch (epi) {
    case 0: run_epi<EPI_NONE>(b, rounds, reps, s); break;
    case 1: run_epi<EPI_BIAS>(b, rounds, reps, s); break;
    case 4: run_epi<EPI_RESID>(b, rounds, reps, s); break;
    case 8: run_epi<EPI_BIAS_GELU_D>(b, rounds, reps, s); break;
    case 10: run_epi<EPI_MUL>(b, rounds, reps, s); break;
    default: fprintf(stderr, "epi %d not in the lab\n", epi); return 1;
  }
  return 0;
}
