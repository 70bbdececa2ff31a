// Identical-VA probe: can two processes on ONE GPU whose
// device allocations sit at identical virtual addresses read each other's cached data?
// No engine code, no IPC, no mailboxes: each process allocates the same sequence of buffers
// (same sizes, same order -> the same VAs, printed), then for `iters` rounds rewrites its
// buffers with a (rank, round)-specific pattern and re-reads them many times from small grids
// (the working set is L1 / L2 resident), counting every value that is not this process's own
// pattern.  `offset` MB of padding allocated first moves this process's VAs (the control).
//   hipcc -O3 --offload-arch=gfx950 tools/va_probe.hip -o tools/va_probe
//   ./tools/va_probe RANK ITERS OFFSET_MB
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

__device__ __forceinline__ double pattern(long j, int rank, int round) {
  return (double)(j % 100003) + 1e6 * rank + 1e9 * (round & 1023);
}

__global__ void fill(double* x, long n, int rank, int round) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    x[i] = pattern(i, rank, round);
}

// every thread re-reads 64 values of the buffer (strided), checks them against its own pattern
__global__ void check(const double* x, long n, int rank, int round, unsigned long long* bad,
                      double* foreign) {
  const long i = blockIdx.x * (long)blockDim.x + threadIdx.x;
  unsigned long long nb = 0;
  double seen = 0.0;
  for (int k = 0; k < 64; ++k) {
    const long j = (i + (long)k * 97) % n;
    const double v = x[j];
    if (v != pattern(j, rank, round)) {
      ++nb;
      seen = v;
    }
  }
  if (nb) {
    atomicAdd(bad, nb);
    *foreign = seen;
  }
}

int main(int argc, char** argv) {
  const int rank = argc > 1 ? atoi(argv[1]) : 0;
  const int iters = argc > 2 ? atoi(argv[2]) : 2000;
  const long offset_mb = argc > 3 ? atol(argv[3]) : 0;
  CK(hipSetDevice(0));
  void* pad = nullptr;
  if (offset_mb > 0) CK(hipMalloc(&pad, (size_t)offset_mb << 20));
  const long n_small = 4096, n_big = 1 << 22;   // 32 KB (L1-sized) and 32 MB (L2 / L3)
  double *small, *big, *foreign;
  unsigned long long* bad;
  CK(hipMalloc(&small, n_small * 8));
  CK(hipMalloc(&big, n_big * 8));
  CK(hipMalloc(&bad, 8));
  CK(hipMalloc(&foreign, 8));
  CK(hipMemset(bad, 0, 8));
  CK(hipMemset(foreign, 0, 8));
  printf("rank %d offset %ld MB: small %p big %p\n", rank, offset_mb, (void*)small, (void*)big);
  fflush(stdout);
  for (int r = 0; r < iters; ++r) {
    hipLaunchKernelGGL(fill, 64, 256, 0, 0, small, n_small, rank, r);
    hipLaunchKernelGGL(fill, 1024, 256, 0, 0, big, n_big, rank, r);
    for (int q = 0; q < 4; ++q) {
      hipLaunchKernelGGL(check, 16, 256, 0, 0, small, n_small, rank, r, bad, foreign);
      hipLaunchKernelGGL(check, 512, 256, 0, 0, big, n_big, rank, r, bad, foreign);
    }
  }
  CK(hipDeviceSynchronize());
  unsigned long long nb = 0;
  double f = 0;
  CK(hipMemcpy(&nb, bad, 8, hipMemcpyDeviceToHost));
  CK(hipMemcpy(&f, foreign, 8, hipMemcpyDeviceToHost));
  const double reads = (double)iters * 4 * (16 + 512) * 256 * 64;
  printf("rank %d: %llu wrong values of %.3g reads%s%.17g\n", rank, nb, reads,
         nb ? " (last wrong value " : "", nb ? f : 0.0);
  if (nb) printf(")\n");
  return nb ? 2 : 0;
}
