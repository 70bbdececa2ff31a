// Which SIMD each wave of a workgroup runs on (HW_REG_HW_ID bits [5:4]; CU bits [11:8]):
// 1024-, 512- and 256-thread blocks, a few blocks each.
//   hipcc -O3 --offload-arch=gfx950 tools/simd_map.hip -o tools/simd_map
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void map_kernel(int* out) {
  const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4);   // HW_ID, 32 bits
  if ((threadIdx.x & 63) == 0) out[blockIdx.x * 16 + (threadIdx.x >> 6)] = (int)hw;
}

int main() {
  int* d;
  hipMalloc(&d, 64 * 16 * sizeof(int));
  int h[64 * 16];
  for (int threads : {1024, 512, 256}) {
    hipMemset(d, 0xff, sizeof(h));
    hipLaunchKernelGGL(map_kernel, dim3(4), dim3(threads), 0, 0, d);
    hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    printf("%d threads per block: wave -> simd (cu)\n", threads);
    for (int b = 0; b < 4; ++b) {
      printf("  block %d:", b);
      for (int w = 0; w < threads / 64; ++w) {
        const unsigned v = (unsigned)h[b * 16 + w];
        printf(" %u(%u)", (v >> 4) & 3, (v >> 8) & 15);
      }
      printf("\n");
    }
  }
  return 0;
}
