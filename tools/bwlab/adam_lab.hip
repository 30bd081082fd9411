// Standalone bandwidth lab for the fused Adam step (no torch): fp32 grad, fp32 master param,
// fp32 m / v, bf16 param copy = 30 B per parameter. Variants differ only in how the lanes walk
// the chunk (lane-contiguous 16-B vectors per wave instruction vs 8 contiguous elements per lane),
// how many vector groups a lane keeps in flight, non-temporal loads / stores, and the grid.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/bwlab/adam_lab.hip -o build/adam_lab
//   build/adam_lab [n_params=536870912] [reps=10]
// One JSON line per variant: us per step, TB/s (algorithmic, 30 B / param), max |diff| vs V0.
#include <hip/hip_bf16.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                              \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      exit(2);                                                                             \
    }                                                                                      \
  } while (0)

typedef __hip_bfloat16 bf16;
typedef float f4 __attribute__((ext_vector_type(4)));

struct Args {
  const float* g;
  float* p;
  float* m;
  float* v;
  bf16* c;
  int64_t n;
  int chunk;
  float lr, b1, b2, eps, wd, rbc1, rbc2;
};

__device__ __forceinline__ float adam1(float g, float& p, float& m, float& v, const Args& a) {
  m = a.b1 * m + (1.f - a.b1) * g;
  v = a.b2 * v + (1.f - a.b2) * g * g;
  const float den = sqrtf(v * a.rbc2) + a.eps;
  const float u = (m * a.rbc1) / den + a.wd * p;
  p -= a.lr * u;
  return p;
}

template <bool NT>
__device__ __forceinline__ f4 ld4(const float* q) {
  if constexpr (NT) return __builtin_nontemporal_load(reinterpret_cast<const f4*>(q));
  return *reinterpret_cast<const f4*>(q);
}
template <bool NT>
__device__ __forceinline__ void st4(float* q, f4 x) {
  if constexpr (NT)
    __builtin_nontemporal_store(x, reinterpret_cast<f4*>(q));
  else
    *reinterpret_cast<f4*>(q) = x;
}
template <bool NT>
__device__ __forceinline__ void st_bf4(bf16* q, f4 x) {
  typedef unsigned u2 __attribute__((ext_vector_type(2)));
  union {
    bf16 h[4];
    u2 u;
  } pk;
  pk.h[0] = (bf16)x[0];
  pk.h[1] = (bf16)x[1];
  pk.h[2] = (bf16)x[2];
  pk.h[3] = (bf16)x[3];
  if constexpr (NT)
    __builtin_nontemporal_store(pk.u, reinterpret_cast<u2*>(q));
  else
    *reinterpret_cast<u2*>(q) = pk.u;
}

// V0: the production layout — 8 contiguous elements per lane per iteration (two 16-B loads per
// stream per lane, each wave instruction covering every other 16 B of a 2 KB span).
__global__ void __launch_bounds__(256) adam_v0(Args a) {
  const int64_t nchunks = (a.n + a.chunk - 1) / a.chunk;
  for (int64_t c = blockIdx.x; c < nchunks; c += gridDim.x) {
    const int64_t s = c * a.chunk;
    const int64_t len = std::min<int64_t>(a.chunk, a.n - s);
    for (int64_t i = threadIdx.x * 8; i < len; i += 256 * 8) {
      const int64_t j = s + i;
      f4 g[2], p[2], m[2], v[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        g[h] = ld4<false>(a.g + j + 4 * h);
        p[h] = ld4<false>(a.p + j + 4 * h);
        m[h] = ld4<false>(a.m + j + 4 * h);
        v[h] = ld4<false>(a.v + j + 4 * h);
      }
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          float pp = p[h][k], mm = m[h][k], vv = v[h][k];
          adam1(g[h][k], pp, mm, vv, a);
          p[h][k] = pp;
          m[h][k] = mm;
          v[h][k] = vv;
        }
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        st4<false>(a.p + j + 4 * h, p[h]);
        st4<false>(a.m + j + 4 * h, m[h]);
        st4<false>(a.v + j + 4 * h, v[h]);
        st_bf4<false>(a.c + j + 4 * h, p[h]);
      }
    }
  }
}

// V1: lane-contiguous — group u of a lane sits at i + u * 1024 (a wave instruction covers 1 KB
// contiguous); U groups (4 fp32 each) loaded before any compute / store.
template <int U, bool NTL, bool NTS>
__global__ void __launch_bounds__(256) adam_v1(Args a) {
  const int64_t nchunks = (a.n + a.chunk - 1) / a.chunk;
  constexpr int STEP = 256 * 4 * U;
  for (int64_t c = blockIdx.x; c < nchunks; c += gridDim.x) {
    const int64_t s = c * a.chunk;
    const int64_t len = std::min<int64_t>(a.chunk, a.n - s);  // lab: multiple of STEP
    for (int64_t i = threadIdx.x * 4; i < len; i += STEP) {
      f4 g[U], p[U], m[U], v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t j = s + i + u * 1024;
        g[u] = ld4<NTL>(a.g + j);
        p[u] = ld4<NTL>(a.p + j);
        m[u] = ld4<NTL>(a.m + j);
        v[u] = ld4<NTL>(a.v + j);
      }
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          float pp = p[u][k], mm = m[u][k], vv = v[u][k];
          adam1(g[u][k], pp, mm, vv, a);
          p[u][k] = pp;
          m[u][k] = mm;
          v[u][k] = vv;
        }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t j = s + i + u * 1024;
        st4<NTS>(a.p + j, p[u]);
        st4<NTS>(a.m + j, m[u]);
        st4<NTS>(a.v + j, v[u]);
        st_bf4<NTS>(a.c + j, p[u]);
      }
    }
  }
}

// ceilings: 16-B copy (read 1 stream, write 1) and read-only sum over the same 4 fp32 streams
template <bool NT>
__global__ void __launch_bounds__(256) copy_k(Args a) {
  const int64_t n4 = a.n / 4;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256)
    st4<NT>(a.m + 4 * i, ld4<NT>(a.p + 4 * i));
}
__global__ void __launch_bounds__(256) read_k(Args a) {
  const int64_t n4 = a.n / 4;
  f4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256)
    acc += ld4<true>(a.g + 4 * i) + ld4<true>(a.p + 4 * i) + ld4<true>(a.m + 4 * i) + ld4<true>(a.v + 4 * i);
  if (acc[0] + acc[1] + acc[2] + acc[3] == 1234.5f) a.c[0] = (bf16)1.f;
}

__global__ void fill(float* x, int64_t n, uint32_t seed, float lo, float hi) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    h ^= h >> 16;
    h *= 0x85ebca6bu;
    h ^= h >> 13;
    x[i] = lo + (hi - lo) * ((h & 0xFFFFFF) / 16777216.f);
  }
}

__global__ void maxdiff(const float* a, const float* b, int64_t n, float* out) {
  float m = 0.f;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    m = fmaxf(m, fabsf(a[i] - b[i]));
  for (int o = 32; o; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  if ((threadIdx.x & 63) == 0) atomicMax((int*)out, __float_as_int(m));
}

int main(int argc, char** argv) {
  const int64_t n = argc > 1 ? atoll(argv[1]) : (1LL << 29);
  const int reps = argc > 2 ? atoi(argv[2]) : 10;
  Args a{};
  float *g, *p, *m, *v, *p0, *m0, *v0, *pref;
  bf16* c;
  CK(hipMalloc(&g, n * 4));
  CK(hipMalloc(&p, n * 4));
  CK(hipMalloc(&m, n * 4));
  CK(hipMalloc(&v, n * 4));
  CK(hipMalloc(&p0, n * 4));
  CK(hipMalloc(&m0, n * 4));
  CK(hipMalloc(&v0, n * 4));
  CK(hipMalloc(&pref, n * 4));
  CK(hipMalloc(&c, n * 2));
  hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, g, n, 1u, -1.f, 1.f);
  hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, p0, n, 2u, -1.f, 1.f);
  hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, m0, n, 3u, -0.1f, 0.1f);
  hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, v0, n, 4u, 0.f, 0.01f);
  a.g = g;
  a.p = p;
  a.m = m;
  a.v = v;
  a.c = c;
  a.n = n;
  a.lr = 1e-3f;
  a.b1 = 0.9f;
  a.b2 = 0.999f;
  a.eps = 1e-8f;
  a.wd = 0.01f;
  a.rbc1 = 1.f / (1.f - 0.9f);
  a.rbc2 = 1.f / (1.f - 0.999f);
  struct V {
    const char* name;
    void (*k)(Args);
    int grid;
    int chunk;
  };
  std::vector<V> vs = {
      {"v0_prod_grid2048", adam_v0, 2048, 32768},
      {"v1_u1_grid2048", adam_v1<1, false, false>, 2048, 32768},
      {"v1_u2_grid2048", adam_v1<2, false, false>, 2048, 32768},
      {"v1_u4_grid2048", adam_v1<4, false, false>, 2048, 32768},
      {"v1_u2_nts", adam_v1<2, false, true>, 2048, 32768},
      {"v1_u2_ntl_nts", adam_v1<2, true, true>, 2048, 32768},
      {"v1_u4_nts", adam_v1<4, false, true>, 2048, 32768},
      {"v1_u4_ntl_nts", adam_v1<4, true, true>, 2048, 32768},
      {"v1_u2_nts_grid1024", adam_v1<2, false, true>, 1024, 32768},
      {"v1_u2_nts_grid4096", adam_v1<2, false, true>, 4096, 32768},
      {"v1_u2_nts_chunk65536", adam_v1<2, false, true>, 2048, 65536},
      {"v1_u4_nts_chunk131072", adam_v1<4, false, true>, 2048, 131072},
      {"v1_u2_nts_fullgrid", adam_v1<2, false, true>, 0, 32768},
      {"v1_u8_ntl_nts", adam_v1<8, true, true>, 2048, 32768},
      {"v1_u4_ntl", adam_v1<4, true, false>, 2048, 32768},
      {"v1_u4_ntl_nts_grid1024", adam_v1<4, true, true>, 1024, 32768},
      {"v1_u4_ntl_nts_grid4096", adam_v1<4, true, true>, 4096, 32768},
      {"v1_u4_ntl_nts_fullgrid", adam_v1<4, true, true>, 0, 32768},
      {"ceiling_copy_16B", copy_k<false>, 8192, 32768},
      {"ceiling_copy_16B_nt", copy_k<true>, 8192, 32768},
      {"ceiling_read4_nt", read_k, 8192, 32768},
  };
  float* dmax;
  CK(hipMalloc(&dmax, 4));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (size_t k = 0; k < vs.size(); ++k) {
    a.chunk = vs[k].chunk;
    const int64_t nchunks = (n + a.chunk - 1) / a.chunk;
    const int grid = vs[k].grid ? vs[k].grid : (int)nchunks;
    // correctness: one step from the same start state
    CK(hipMemcpy(p, p0, n * 4, hipMemcpyDeviceToDevice));
    CK(hipMemcpy(m, m0, n * 4, hipMemcpyDeviceToDevice));
    CK(hipMemcpy(v, v0, n * 4, hipMemcpyDeviceToDevice));
    hipLaunchKernelGGL(vs[k].k, dim3(grid), dim3(256), 0, 0, a);
    float diff = 0.f;
    if (k == 0) {
      CK(hipMemcpy(pref, p, n * 4, hipMemcpyDeviceToDevice));
    } else {
      CK(hipMemset(dmax, 0, 4));
      hipLaunchKernelGGL(maxdiff, dim3(2048), dim3(256), 0, 0, p, pref, n, dmax);
      CK(hipMemcpy(&diff, dmax, 4, hipMemcpyDeviceToHost));
    }
    std::vector<float> t;
    for (int r = 0; r < 3; ++r) {
      hipLaunchKernelGGL(vs[k].k, dim3(grid), dim3(256), 0, 0, a);
      CK(hipEventRecord(e0, 0));
      for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(vs[k].k, dim3(grid), dim3(256), 0, 0, a);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      t.push_back(ms * 1000.f / reps);
    }
    std::sort(t.begin(), t.end());
    const double bytes = strstr(vs[k].name, "copy") ? 8.0 * n : strstr(vs[k].name, "read4") ? 16.0 * n : 30.0 * n;
    printf("{\"variant\": \"%s\", \"n\": %lld, \"grid\": %d, \"chunk\": %d, \"us\": %.1f, \"tbs\": %.3f, \"maxdiff\": %g}\n",
           vs[k].name, (long long)n, grid, a.chunk, t[0], bytes / (t[0] * 1e-6) / 1e12, diff);
    fflush(stdout);
  }
  return 0;
}
