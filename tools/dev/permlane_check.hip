// Prints the lane mapping of __builtin_amdgcn_permlane{32,16}_swap on the GPU (development check).
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(unsigned* o) {
  const unsigned l = threadIdx.x;
  unsigned a = 1000 + l, b = 2000 + l;
  auto x = __builtin_amdgcn_permlane32_swap(a, b, false, false);
  o[l] = x[0];
  o[64 + l] = x[1];
  auto y = __builtin_amdgcn_permlane16_swap(a, b, false, false);
  o[128 + l] = y[0];
  o[192 + l] = y[1];
}
int main() {
  unsigned* d;
  unsigned h[256];
  hipMalloc(&d, 1024);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  hipMemcpy(h, d, 1024, hipMemcpyDeviceToHost);
  const char* nm[4] = {"p32 a'", "p32 b'", "p16 a'", "p16 b'"};
  for (int t = 0; t < 4; ++t) {
    printf("%s:", nm[t]);
    for (int l = 0; l < 64; l += 8) printf(" [%d]=%u", l, h[t * 64 + l]);
    printf(" [17]=%u [33]=%u [49]=%u\n", h[t * 64 + 17], h[t * 64 + 33], h[t * 64 + 49]);
  }
  return 0;
}
