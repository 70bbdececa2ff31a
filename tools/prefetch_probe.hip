// Memory-pattern probe of the contracted sweep with an explicit prefetch distance: per step,
// every wavelength reads the two T-bracket rows of one table and one stale flux row, and writes
// one flux row (32 B per update, 59 steps); the loads of step k + PF are issued at step k into a
// register ring (unrolled by PF, so every ring index is static).  A dependent recurrence keeps
// every value live.  Sizes: 62.5k (the 8-GPU slice) and 500k wavelengths.
//   hipcc -O3 --offload-arch=gfx950 tools/prefetch_probe.hip -o tools/prefetch_probe
#include <hip/hip_runtime.h>
#include <cstdio>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

constexpr int NS = 59;

__device__ __forceinline__ long row_of(int k) { return (long)k * 16 + (k * 7) % 15; }

template <int PF>
__global__ __launch_bounds__(256) void sweep_pf(const double* __restrict__ tab,
                                               const double* __restrict__ st,
                                               double* __restrict__ out, long n, long pitch) {
  const long j0 = blockIdx.x * 256L + threadIdx.x;
  const long j = j0 < n ? j0 : n - 1;
  double lo[PF], hi[PF], sv[PF];
  auto load = [&](int k, double& a, double& b, double& s) {
    k = k < NS ? k : NS - 1;
    const double* r = tab + row_of(k) * pitch + j;
    a = __builtin_nontemporal_load(r);
    b = __builtin_nontemporal_load(r + pitch);
    s = st[(long)k * n + j];
  };
#pragma unroll
  for (int b = 0; b < PF; ++b) load(b, lo[b], hi[b], sv[b]);
  double acc = 0.0;
  for (int k0 = 0; k0 < NS; k0 += PF) {
#pragma unroll
    for (int b = 0; b < PF; ++b) {
      const int k = k0 + b;
      if (k >= NS) break;
      const double v = sv[b] + lo[b] * 0.5 + hi[b] * 0.25;
      load(k + PF, lo[b], hi[b], sv[b]);
      acc = acc * 0.999 + v;
      if (j0 < n) out[(long)k * n + j] = acc;
    }
  }
}

template <int PF>
int run(long n, long pitch, const double* tab, const double* st, double* out) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int nb = (int)((n + 255) / 256);
  for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(sweep_pf<PF>, nb, 256, 0, 0, tab, st, out, n, pitch);
  CK(hipDeviceSynchronize());
  const int reps = 20;
  CK(hipEventRecord(e0));
  for (int r = 0; r < reps; ++r)
    hipLaunchKernelGGL(sweep_pf<PF>, nb, 256, 0, 0, tab, st, out, n, pitch);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  const double t = ms / reps * 1e-3;
  printf("n %7ld  PF %2d  %.4f ms  %.2f TB/s\n", n, PF, t * 1e3, 32.0 * NS * n / t / 1e12);
  return 0;
}

int main() {
  for (long n : {62500L, 500000L}) {
    const long pitch = (n + 63) / 64 * 64;
    const size_t rows = 60 * 16;
    double *tab, *st, *out;
    CK(hipMalloc(&tab, rows * pitch * 8));
    CK(hipMalloc(&st, (size_t)NS * n * 8));
    CK(hipMalloc(&out, (size_t)NS * n * 8));
    CK(hipMemset(tab, 0, rows * pitch * 8));
    CK(hipMemset(st, 0, (size_t)NS * n * 8));
    for (int rep = 0; rep < 2; ++rep) {
      if (run<1>(n, pitch, tab, st, out) || run<2>(n, pitch, tab, st, out) ||
          run<4>(n, pitch, tab, st, out) || run<8>(n, pitch, tab, st, out) ||
          run<16>(n, pitch, tab, st, out))
        return 1;
    }
    CK(hipFree(tab));
    CK(hipFree(st));
    CK(hipFree(out));
  }
  return 0;
}
