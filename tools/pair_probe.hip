// HBM access-pattern probe for the contracted sweep (32 B per update): per step, every
// wavelength reads the two T-bracket rows of one table, one stale flux, and writes one flux.
//   sep1:  [row][lambda] table, rows lo / hi (two streams), one wavelength per lane (the engine)
//   pair1: [row][lambda][2] table (lo, hi adjacent), one 16 B load per lane
//   sep2:  [row][lambda] table, two adjacent wavelengths per lane (16 B loads / stores)
//   pair2: [row][lambda][2] table, two wavelengths per lane (2 x 16 B loads)
// Same bytes, a dependent recurrence so nothing is dead.  Sizes: 500k and 62.5k lambda.
//   hipcc -O3 --offload-arch=gfx950 tools/pair_probe.hip -o tools/pair_probe
#include <hip/hip_runtime.h>
#include <cstdio>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

constexpr int NS = 59;

__device__ __forceinline__ long row_of(int k) { return (long)k * 16 + (k * 7) % 15; }

__global__ __launch_bounds__(256) void sep1(const double* tab, const double* st, double* out,
                                           long n, long pitch) {
  const long j = blockIdx.x * 256L + threadIdx.x;
  if (j >= n) return;
  double acc = 0.0;
  for (int k = 0; k < NS; ++k) {
    const double* r = tab + row_of(k) * pitch + j;
    const double v = st[(long)k * n + j] + r[0] * 0.5 + r[pitch] * 0.25;
    acc = acc * 0.999 + v;
    out[(long)k * n + j] = acc;
  }
}

__global__ __launch_bounds__(256) void pair1(const double* tab, const double* st, double* out,
                                            long n, long pitch) {
  const long j = blockIdx.x * 256L + threadIdx.x;
  if (j >= n) return;
  double acc = 0.0;
  for (int k = 0; k < NS; ++k) {
    const double2 t = *reinterpret_cast<const double2*>(tab + (row_of(k) * pitch + j) * 2);
    const double v = st[(long)k * n + j] + t.x * 0.5 + t.y * 0.25;
    acc = acc * 0.999 + v;
    out[(long)k * n + j] = acc;
  }
}

__global__ __launch_bounds__(256) void sep2(const double* tab, const double* st, double* out,
                                           long n, long pitch) {
  const long j = (blockIdx.x * 256L + threadIdx.x) * 2;
  if (j >= n) return;
  double a0 = 0.0, a1 = 0.0;
  for (int k = 0; k < NS; ++k) {
    const double* r = tab + row_of(k) * pitch + j;
    const double2 lo = *reinterpret_cast<const double2*>(r);
    const double2 hi = *reinterpret_cast<const double2*>(r + pitch);
    const double2 s = *reinterpret_cast<const double2*>(st + (long)k * n + j);
    a0 = a0 * 0.999 + (s.x + lo.x * 0.5 + hi.x * 0.25);
    a1 = a1 * 0.999 + (s.y + lo.y * 0.5 + hi.y * 0.25);
    *reinterpret_cast<double2*>(out + (long)k * n + j) = make_double2(a0, a1);
  }
}

__global__ __launch_bounds__(256) void pair2(const double* tab, const double* st, double* out,
                                            long n, long pitch) {
  const long j = (blockIdx.x * 256L + threadIdx.x) * 2;
  if (j >= n) return;
  double a0 = 0.0, a1 = 0.0;
  for (int k = 0; k < NS; ++k) {
    const double2* r = reinterpret_cast<const double2*>(tab + (row_of(k) * pitch + j) * 2);
    const double2 t0 = r[0], t1 = r[1];
    const double2 s = *reinterpret_cast<const double2*>(st + (long)k * n + j);
    a0 = a0 * 0.999 + (s.x + t0.x * 0.5 + t0.y * 0.25);
    a1 = a1 * 0.999 + (s.y + t1.x * 0.5 + t1.y * 0.25);
    *reinterpret_cast<double2*>(out + (long)k * n + j) = make_double2(a0, a1);
  }
}

int main() {
  for (long n : {500000L, 62500L}) {
    const long pitch = (n + 63) / 64 * 64;
    const size_t rows = 60 * 16;
    double *tab, *tabp, *st, *out;
    CK(hipMalloc(&tab, rows * pitch * sizeof(double)));
    CK(hipMalloc(&tabp, rows * pitch * 2 * sizeof(double)));
    CK(hipMalloc(&st, (size_t)NS * n * sizeof(double)));
    CK(hipMalloc(&out, (size_t)NS * n * sizeof(double)));
    CK(hipMemset(tab, 0, rows * pitch * sizeof(double)));
    CK(hipMemset(tabp, 0, rows * pitch * 2 * sizeof(double)));
    CK(hipMemset(st, 0, (size_t)NS * n * sizeof(double)));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const int b1 = (int)((n + 255) / 256), b2 = (int)((n / 2 + 255) / 256);
    const double bytes = (double)NS * n * 32.0;
    for (int rep = 0; rep < 3; ++rep) {
      float ms[4];
      for (int v = 0; v < 4; ++v) {
        CK(hipEventRecord(a));
        for (int i = 0; i < 20; ++i) {
          if (v == 0) hipLaunchKernelGGL(sep1, dim3(b1), dim3(256), 0, 0, tab, st, out, n, pitch);
          if (v == 1) hipLaunchKernelGGL(pair1, dim3(b1), dim3(256), 0, 0, tabp, st, out, n, pitch);
          if (v == 2) hipLaunchKernelGGL(sep2, dim3(b2), dim3(256), 0, 0, tab, st, out, n, pitch);
          if (v == 3) hipLaunchKernelGGL(pair2, dim3(b2), dim3(256), 0, 0, tabp, st, out, n, pitch);
        }
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        CK(hipEventElapsedTime(&ms[v], a, b));
        ms[v] /= 20;
      }
      printf("n %ld  sep1 %.4f ms %.2f TB/s  pair1 %.4f ms %.2f  sep2 %.4f ms %.2f  pair2 %.4f ms %.2f\n",
             n, ms[0], bytes / (ms[0] * 1e-3) / 1e12, ms[1], bytes / (ms[1] * 1e-3) / 1e12,
             ms[2], bytes / (ms[2] * 1e-3) / 1e12, ms[3], bytes / (ms[3] * 1e-3) / 1e12);
    }
    CK(hipFree(tab)); CK(hipFree(tabp)); CK(hipFree(st)); CK(hipFree(out));
  }
  return 0;
}
