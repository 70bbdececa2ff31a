// Per-launch cost of back-to-back kernels on one stream (HIP events over N launches):
// empty kernels of 1 and 60 workgroups, the same after a kernel that dirties ~32 MB of L2
// lines, and the same N empty kernels replayed from a hipGraph.
//   hipcc -O3 --offload-arch=gfx950 tools/launch_floor.hip -o tools/launch_floor
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__global__ void empty_kernel(int* p) {
  if (p && threadIdx.x == 1023) p[0] = 1;   // never true: keeps the kernel non-trivial
}

// busy-waits `ns` nanoseconds (wall clock, 100 MHz) and writes one value per thread
__global__ void spin_kernel(double* x, long long ns) {
  const long long t0 = wall_clock64();
  while ((wall_clock64() - t0) * 10 < ns) __builtin_amdgcn_s_sleep(1);
  x[blockIdx.x * (long)blockDim.x + threadIdx.x] = 1.0;
}

__global__ void dirty_kernel(double* x, long n) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    x[i] = (double)i;
}

int main() {
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const int N = 2000;
  const long nd = 4L << 20;   // 32 MB of doubles
  double* x;
  CK(hipMalloc(&x, nd * sizeof(double)));
  float ms;
  for (int grid : {1, 60, 480}) {
    for (int rep = 0; rep < 2; ++rep) {
      CK(hipEventRecord(a, s));
      for (int i = 0; i < N; ++i) hipLaunchKernelGGL(empty_kernel, dim3(grid), dim3(256), 0, s, nullptr);
      CK(hipEventRecord(b, s));
      CK(hipEventSynchronize(b));
      CK(hipEventElapsedTime(&ms, a, b));
    }
    printf("empty kernel, %4d workgroups: %.2f us per launch\n", grid, 1e3 * ms / N);
  }
  // dirty + empty pairs: cost of the empty kernel after a kernel that wrote 32 MB
  {
    const int M = 200;
    for (int rep = 0; rep < 2; ++rep) {
      CK(hipEventRecord(a, s));
      for (int i = 0; i < M; ++i) hipLaunchKernelGGL(dirty_kernel, dim3(1024), dim3(256), 0, s, x, nd);
      CK(hipEventRecord(b, s));
      CK(hipEventSynchronize(b));
      CK(hipEventElapsedTime(&ms, a, b));
    }
    const float only = ms / M;
    for (int rep = 0; rep < 2; ++rep) {
      CK(hipEventRecord(a, s));
      for (int i = 0; i < M; ++i) {
        hipLaunchKernelGGL(dirty_kernel, dim3(1024), dim3(256), 0, s, x, nd);
        hipLaunchKernelGGL(empty_kernel, dim3(60), dim3(256), 0, s, nullptr);
      }
      CK(hipEventRecord(b, s));
      CK(hipEventSynchronize(b));
      CK(hipEventElapsedTime(&ms, a, b));
    }
    printf("32 MB write kernel: %.2f us; + empty 60-workgroup kernel after it: +%.2f us\n",
           1e3 * only, 1e3 * (ms / M - only));
  }
  // a ~40 us kernel of 489 workgroups (the 62.5k-slice sweep's shape) alone, then followed
  // by an empty 60-workgroup kernel: what the second launch adds to the pair
  {
    const int M = 200;
    float solo = 0, pair = 0;
    for (int rep = 0; rep < 2; ++rep) {
      CK(hipEventRecord(a, s));
      for (int i = 0; i < M; ++i) hipLaunchKernelGGL(spin_kernel, dim3(489), dim3(256), 0, s, x, 40000LL);
      CK(hipEventRecord(b, s));
      CK(hipEventSynchronize(b));
      CK(hipEventElapsedTime(&solo, a, b));
      CK(hipEventRecord(a, s));
      for (int i = 0; i < M; ++i) {
        hipLaunchKernelGGL(spin_kernel, dim3(489), dim3(256), 0, s, x, 40000LL);
        hipLaunchKernelGGL(empty_kernel, dim3(60), dim3(256), 0, s, nullptr);
      }
      CK(hipEventRecord(b, s));
      CK(hipEventSynchronize(b));
      CK(hipEventElapsedTime(&pair, a, b));
    }
    printf("spin kernel (489 x 256, ~40 us): %.2f us; + empty 60-workgroup kernel: +%.2f us\n",
           1e3 * solo / M, 1e3 * (pair - solo) / M);
  }
  if (getenv("NO_GRAPH")) { CK(hipFree(x)); return 0; }
  // graph replay of N empty kernels
  {
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    for (int i = 0; i < 200; ++i) hipLaunchKernelGGL(empty_kernel, dim3(60), dim3(256), 0, s, nullptr);
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    for (int rep = 0; rep < 3; ++rep) {
      CK(hipEventRecord(a, s));
      for (int i = 0; i < 10; ++i) CK(hipGraphLaunch(ge, s));
      CK(hipEventRecord(b, s));
      CK(hipEventSynchronize(b));
      CK(hipEventElapsedTime(&ms, a, b));
    }
    printf("graph of 200 empty 60-workgroup kernels: %.2f us per kernel\n", 1e3 * ms / 2000);
  }
  CK(hipFree(x));
  return 0;
}
