// bw_probe.hip — HBM ceilings on MI355X for the sweep kernel's access mix (diagnostic tool).
//   hipcc -O3 --offload-arch=gfx950 tools/bw_probe.hip -o build/bw_probe && build/bw_probe
// Prints GB/s for: streaming read (8 B / 16 B per lane), copy, and a "sweep-like" pattern
// (per step 16 table rows + 1 flux row read, 2 flux rows written, rows 4 MB apart).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e = (x);                                                            \
    if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } \
  } while (0)

__global__ void read8(const double* __restrict__ a, int64_t n, double* out) {
  double s = 0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    s += a[i];
  if (s == 12345.678) out[0] = s;
}

__global__ void read16(const double2* __restrict__ a, int64_t n, double* out) {
  double s = 0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    double2 v = a[i];
    s += v.x + v.y;
  }
  if (s == 12345.678) out[0] = s;
}

__global__ void copy16(const double2* __restrict__ a, double2* __restrict__ b, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    b[i] = a[i];
}

// One lane per wavelength, loop over steps; rows of length nl.
template <int R>
__global__ __launch_bounds__(256) void pattern(const double* __restrict__ tab,
                                               const double* __restrict__ fin,
                                               double* __restrict__ fo1, double* __restrict__ fo2,
                                               int64_t nl, int steps) {
  const int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (j >= nl) return;
  double carry = 0;
  for (int k = 0; k < steps; ++k) {
    double s = 0;
#pragma unroll
    for (int r = 0; r < R; ++r) s += tab[((int64_t)k * R + r) * nl + j];
    s += fin[(int64_t)k * nl + j];
    carry = carry * 0.5 + s;
    fo1[(int64_t)k * nl + j] = carry;
    fo2[(int64_t)k * nl + j] = s;
  }
}

int main() {
  const int64_t N = (int64_t)1 << 29;  // 4 GiB of doubles
  double *a, *b, *out;
  CK(hipMalloc(&a, N * 8));
  CK(hipMalloc(&b, N * 8));
  CK(hipMalloc(&out, 64));
  CK(hipMemset(a, 0, N * 8));
  CK(hipMemset(b, 0, N * 8));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto timeit = [&](auto launch, double bytes, const char* name) {
    launch();
    CK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int r = 0; r < 5; ++r) {
      CK(hipEventRecord(e0));
      launch();
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      best = ms < best ? ms : best;
    }
    printf("%-40s %8.3f ms  %7.0f GB/s\n", name, best, bytes / (best * 1e-3) / 1e9);
    return 0;
  };
  const int grid = 256 * 8, blk = 256;
  timeit([&] { read8<<<grid, blk>>>(a, N, out); }, N * 8.0, "read 8B/lane (grid-stride)");
  timeit([&] { read16<<<grid, blk>>>((const double2*)a, N / 2, out); }, N * 8.0,
         "read 16B/lane (grid-stride)");
  timeit([&] { copy16<<<grid, blk>>>((const double2*)a, (double2*)b, N / 4); }, N / 4 * 32.0,
         "copy 16B/lane");
  // sweep-like: 500k wavelengths, 59 steps, 16 table rows + 1 read + 2 written per step
  const int64_t nl = 500000;
  const int steps = 59;
  double* tab = a;                         // 59*16*nl*8 = 3.8 GB
  double* fin = b;                         // 59*nl
  double* fo1 = b + (int64_t)steps * nl;
  double* fo2 = b + 2 * (int64_t)steps * nl;
  const double pbytes = (double)steps * nl * (16 + 1 + 2) * 8.0;
  timeit([&] { pattern<16><<<(nl + 255) / 256, 256>>>(tab, fin, fo1, fo2, nl, steps); }, pbytes,
         "sweep pattern 16r+1r+2w, 1 lane/lambda");
  const double pbytes8 = (double)steps * nl * (8 + 1 + 2) * 8.0;
  timeit([&] { pattern<8><<<(nl + 255) / 256, 256>>>(tab, fin, fo1, fo2, nl, steps); }, pbytes8,
         "sweep pattern 8r+1r+2w, 1 lane/lambda");
  return 0;
}
