// Write-heavy roofline probe for K7 (the batched contraction): the C5 shape — 60 layers x
// 16 T rows x 100,032 columns per table row block, 8 tables read once, 32 per-atmosphere
// tables written — with trivial arithmetic, in three forms:
//   write   : the 24.6 GB of stores only (16 B per lane, 1 KiB contiguous per wave-instruction)
//   rw      : + the 6.15 GB of table reads (lane per column pair, 16 B per lane)
//   rw_nt   : the same with nontemporal stores
//   copy    : plain streaming copy of 6.15 GB (read+write reference)
//   hipcc -O3 --offload-arch=gfx950 tools/store_probe.hip -o tools/store_probe
#include <hip/hip_runtime.h>
#include <cstdio>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

typedef double dbl2 __attribute__((ext_vector_type(2)));
constexpr int S = 8, NATM = 32, NL = 60, NT = 16;
constexpr long PITCH = 100032;
constexpr long NCOL = NT * PITCH;              // columns per layer row block
constexpr long PER = NL * NCOL + 64;          // doubles per atmosphere table

template <int MODE>
__global__ __launch_bounds__(256) void k7_shape(const double* __restrict__ tab,
                                               double* __restrict__ eff) {
  const int l = blockIdx.y;
  const long c = ((long)blockIdx.x * 256 + threadIdx.x) * 2;
  if (c >= NCOL) return;
  const long row = (long)l * NCOL;
  dbl2 acc = {1.0, 2.0};
  if (MODE >= 1) {
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const dbl2 v = *reinterpret_cast<const dbl2*>(tab + (long)s * NL * NCOL + row + c);
      acc += v;
    }
  }
  for (int m = 0; m < NATM; ++m) {
    dbl2* p = reinterpret_cast<dbl2*>(eff + (long)m * PER + row + c);
    const dbl2 v = acc * (double)(m + 1);
    if (MODE == 2) __builtin_nontemporal_store(v, p);
    else *p = v;
  }
}

__global__ __launch_bounds__(256) void copy(const dbl2* __restrict__ a, dbl2* __restrict__ b,
                                           long n) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256)
    b[i] = a[i];
}

template <int MODE>
int run(const char* name, const double* tab, double* eff) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  dim3 grid((unsigned)((NCOL / 2 + 255) / 256), NL);
  hipLaunchKernelGGL(k7_shape<MODE>, grid, 256, 0, 0, tab, eff);
  CK(hipDeviceSynchronize());
  const int reps = 3;
  CK(hipEventRecord(e0));
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k7_shape<MODE>, grid, 256, 0, 0, tab, eff);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  const double t = ms / reps * 1e-3;
  const double wb = 8.0 * NATM * NL * NCOL, rb = MODE >= 1 ? 8.0 * S * NL * NCOL : 0.0;
  printf("%-6s %.3f ms  %.2f TB/s (%.1f GB written, %.1f GB read)\n", name, t * 1e3,
         (wb + rb) / t / 1e12, wb / 1e9, rb / 1e9);
  return 0;
}

int main() {
  double *tab, *eff;
  CK(hipMalloc(&tab, (size_t)S * NL * NCOL * 8));
  CK(hipMalloc(&eff, (size_t)NATM * PER * 8));
  CK(hipMemset(tab, 0, (size_t)S * NL * NCOL * 8));
  for (int rep = 0; rep < 2; ++rep) {
    if (run<0>("write", tab, eff) || run<1>("rw", tab, eff) || run<2>("rw_nt", tab, eff))
      return 1;
    const long n = (long)S * NL * NCOL / 2;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    hipLaunchKernelGGL(copy, 4096, 256, 0, 0, (const dbl2*)tab, (dbl2*)eff, n);
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL(copy, 4096, 256, 0, 0, (const dbl2*)tab, (dbl2*)eff, n);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("copy   %.3f ms  %.2f TB/s (6.1 GB read + written)\n", ms,
           2.0 * n * 16 / (ms * 1e-3) / 1e12);
  }
  return 0;
}
