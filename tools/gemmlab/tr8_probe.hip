#include <hip/hip_runtime.h>
#include <cstdio>
typedef int i32x2 __attribute__((ext_vector_type(2)));
__global__ void k(const int* addr, unsigned char* out) {
  __shared__ unsigned char s[4096];
  for (int i = threadIdx.x; i < 4096; i += 64) s[i] = (unsigned char)(i & 255);
  __syncthreads();
  i32x2 v = __builtin_amdgcn_ds_read_tr8_b64_v2i32((__attribute__((address_space(3))) i32x2*)(s + addr[threadIdx.x]));
  *(i32x2*)(out + threadIdx.x * 8) = v;
}
int main() {
  int ha[64]; unsigned char ho[512];
  // lane 2q+p (within 16-lane group g) -> row q (row stride 16 B + group offset 128*g... use distinct), cols 8p
  for (int l = 0; l < 64; ++l) { int g = l >> 4, i = l & 15, q = i >> 1, p = i & 1; ha[l] = g * 1024 + q * 128 + 8 * p; }
  int* da; unsigned char* dout;
  hipMalloc(&da, sizeof ha); hipMalloc(&dout, 512);
  hipMemcpy(da, ha, sizeof ha, hipMemcpyHostToDevice);
  k<<<1, 64>>>(da, dout);
  hipMemcpy(ho, dout, 512, hipMemcpyDeviceToHost);
  int ok = 1;
  for (int l = 0; l < 64; ++l) {
    int g = l >> 4, i = l & 15;
    printf("lane %2d:", l);
    for (int b = 0; b < 8; ++b) {
      int off = ho[l * 8 + b];  // byte value = addr & 255; decode row q, col c
      printf(" %3d", off);
      // expected under hypothesis: row b, col i -> addr g*1024 + b*128 + i
      int exp = (g * 1024 + b * 128 + i) & 255;
      if (off != exp) ok = 0;
    }
    printf("\n");
  }
  printf("HYPOTHESIS %s\n", ok ? "OK" : "FAIL");
  return 0;
}
