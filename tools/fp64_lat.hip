// fp64 VALU latency / issue microbenchmark (one wave per SIMD): cycles per v_fma_f64 for K
// independent dependency chains, and for division / exp-like sequences.
//   hipcc -O3 --offload-arch=gfx950 tools/fp64_lat.hip -o tools/fp64_lat && ./tools/fp64_lat
#include <hip/hip_runtime.h>
#include <cstdio>

template <int K>
__global__ void chains(double* out, int n, long long* cyc) {
  double a[K];
  for (int k = 0; k < K; ++k) a[k] = threadIdx.x * 1e-3 + k;
  const double b = 0.999999, c = 1e-7;
  __syncthreads();
  const long long t0 = clock64();
#pragma unroll 32
  for (int i = 0; i < n; ++i) {
#pragma unroll
    for (int k = 0; k < K; ++k) a[k] = __builtin_fma(a[k], b, c);
  }
  const long long t1 = clock64();
  double s = 0;
  for (int k = 0; k < K; ++k) s += a[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int K>
void run(int waves_per_simd) {
  const int n = 4096;
  const int blocks = 256;               // one block per CU
  const int threads = 64 * 4 * waves_per_simd;
  double* out; long long* cyc;
  hipMalloc(&out, sizeof(double) * blocks * threads);
  hipMalloc(&cyc, sizeof(long long) * blocks);
  hipLaunchKernelGGL(chains<K>, dim3(blocks), dim3(threads), 0, 0, out, n, cyc);
  hipDeviceSynchronize();
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL(chains<K>, dim3(blocks), dim3(threads), 0, 0, out, n, cyc);
  hipEventRecord(e1); hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  long long c[256]; hipMemcpy(c, cyc, sizeof(c), hipMemcpyDeviceToHost);
  const double instr = (double)n * K;   // per wave
  printf("chains=%d waves/SIMD=%d: %.2f clock64 ticks per fma per wave; SIMD issue %.2f "
         "ns per wave-fma; kernel %.3f ms\n", K, waves_per_simd, c[0] / instr,
         ms * 1e6 / (instr * waves_per_simd), ms);
  hipFree(out); hipFree(cyc);
}

// dependent chains of one op kind (one wave per SIMD): ticks per op
template <int OP>
__global__ void opchain(double* out, int n, long long* cyc) {
  double x = 1.0 + threadIdx.x * 1e-6;
  __syncthreads();
  const long long t0 = clock64();
#pragma unroll 16
  for (int i = 0; i < n; ++i) {
    if (OP == 0) x = __builtin_amdgcn_rcp(x);                 // v_rcp_f64
    if (OP == 1) x = __builtin_amdgcn_rsq(x);                 // v_rsq_f64
    if (OP == 2) x = x * 1.0000001;                           // v_mul_f64
    if (OP == 3) { const double r = __builtin_amdgcn_rcp(x);  // division core a / x
                   double e = __builtin_fma(-x, r, 1.0); double r2 = __builtin_fma(r, e, r);
                   e = __builtin_fma(-x, r2, 1.0); r2 = __builtin_fma(r2, e, r2);
                   const double q = 1.5 * r2; const double rem = __builtin_fma(-x, q, 1.5);
                   x = __builtin_fma(rem, r2, q); }
    if (OP == 4) x = __builtin_amdgcn_ldexp(x, 1) * 0.5;     // v_ldexp_f64 + mul
  }
  const long long t1 = clock64();
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int OP>
void runop(const char* name, int per) {
  const int n = 4096, blocks = 256, threads = 256;   // one wave per SIMD
  double* out; long long* cyc;
  hipMalloc(&out, sizeof(double) * blocks * threads);
  hipMalloc(&cyc, sizeof(long long) * blocks);
  hipLaunchKernelGGL(opchain<OP>, dim3(blocks), dim3(threads), 0, 0, out, n, cyc);
  hipDeviceSynchronize();
  hipLaunchKernelGGL(opchain<OP>, dim3(blocks), dim3(threads), 0, 0, out, n, cyc);
  hipDeviceSynchronize();
  long long c[256]; hipMemcpy(c, cyc, sizeof(c), hipMemcpyDeviceToHost);
  printf("%-28s %.2f ticks per chain step (%d dependent VALU ops)\n", name, (double)c[0] / n, per);
  hipFree(out); hipFree(cyc);
}

int main() {
  runop<0>("v_rcp_f64 chain", 1);
  runop<1>("v_rsq_f64 chain", 1);
  runop<2>("v_mul_f64 chain", 1);
  runop<3>("division core chain", 8);
  runop<4>("ldexp + mul chain", 2);
  run<1>(1); run<2>(1); run<4>(1); run<8>(1);
  run<1>(2); run<2>(2); run<4>(2);
  run<1>(4); run<2>(4);
  return 0;
}
