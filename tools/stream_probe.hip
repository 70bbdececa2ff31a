// HBM access-pattern probe for the per-species sweep (144 B per update at S = 8): per step,
// every lane reads two T-bracket rows of S species tables plus one stale flux and writes one
// flux.  "separate": one table per species, [row][lambda] (the engine's layout: 16 row streams
// per step); "interleaved": one table [row][lambda][S] (2 streams of S contiguous doubles per
// lane).  Same bytes, same arithmetic (a dependent sum so nothing is dead).
//   hipcc -O3 --offload-arch=gfx950 tools/stream_probe.hip -o tools/stream_probe
#include <hip/hip_runtime.h>
#include <cstdio>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

constexpr int S = 8;
constexpr int NS = 59;          // steps per sweep
constexpr int NROW = 60 * 16;   // (p, T) rows per species

__global__ __launch_bounds__(256) void separate(const double* const* tab, const double* stale,
                                               double* out, long n, long pitch) {
  const long j = blockIdx.x * 256L + threadIdx.x;
  if (j >= n) return;
  double acc = 0.0;
  for (int k = 0; k < NS; ++k) {
    const long row = (long)k * 16 + (k * 7) % 15;          // layer's p row, a T bracket
    double v = stale[(long)k * n + j];
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const double* r = tab[s] + row * pitch + j;
      v += r[0] * 0.5 + r[pitch] * 0.25;
    }
    acc = acc * 0.999 + v;
    out[(long)k * n + j] = acc;
  }
}

__global__ __launch_bounds__(256) void interleaved(const double* tab, const double* stale,
                                                  double* out, long n, long pitch) {
  const long j = blockIdx.x * 256L + threadIdx.x;
  if (j >= n) return;
  double acc = 0.0;
  for (int k = 0; k < NS; ++k) {
    const long row = (long)k * 16 + (k * 7) % 15;
    double v = stale[(long)k * n + j];
    const double2* lo = reinterpret_cast<const double2*>(tab + (row * pitch + j) * S);
    const double2* hi = reinterpret_cast<const double2*>(tab + ((row + 1) * pitch + j) * S);
#pragma unroll
    for (int s = 0; s < S / 2; ++s) {
      const double2 a = lo[s], b = hi[s];
      v += a.x * 0.5 + b.x * 0.25;
      v += a.y * 0.5 + b.y * 0.25;
    }
    acc = acc * 0.999 + v;
    out[(long)k * n + j] = acc;
  }
}

int main() {
  const long n = 500000, pitch = 500032;
  const size_t tab_elems = (size_t)NROW * pitch;
  double* tabs[S];
  for (int s = 0; s < S; ++s) {
    CK(hipMalloc(&tabs[s], tab_elems * sizeof(double)));
    CK(hipMemset(tabs[s], 0, tab_elems * sizeof(double)));
  }
  double* il;
  CK(hipMalloc(&il, tab_elems * S * sizeof(double)));
  CK(hipMemset(il, 0, tab_elems * S * sizeof(double)));
  double **dtabs, *stale, *out;
  CK(hipMalloc(&dtabs, sizeof(tabs)));
  CK(hipMemcpy(dtabs, tabs, sizeof(tabs), hipMemcpyHostToDevice));
  CK(hipMalloc(&stale, (size_t)NS * n * sizeof(double)));
  CK(hipMalloc(&out, (size_t)NS * n * sizeof(double)));
  CK(hipMemset(stale, 0, (size_t)NS * n * sizeof(double)));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const int blocks = (int)((n + 255) / 256);
  const double bytes = (double)NS * n * (16.0 * S + 16.0);
  for (int rep = 0; rep < 3; ++rep) {
    float ms_s, ms_i;
    CK(hipEventRecord(a));
    for (int i = 0; i < 10; ++i)
      hipLaunchKernelGGL(separate, dim3(blocks), dim3(256), 0, 0, dtabs, stale, out, n, pitch);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    CK(hipEventElapsedTime(&ms_s, a, b));
    CK(hipEventRecord(a));
    for (int i = 0; i < 10; ++i)
      hipLaunchKernelGGL(interleaved, dim3(blocks), dim3(256), 0, 0, il, stale, out, n, pitch);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    CK(hipEventElapsedTime(&ms_i, a, b));
    printf("separate %.3f ms (%.2f TB/s)   interleaved %.3f ms (%.2f TB/s)\n", ms_s / 10,
           bytes / (ms_s / 10 * 1e-3) / 1e12, ms_i / 10, bytes / (ms_i / 10 * 1e-3) / 1e12);
  }
  return 0;
}
