// Device-wide barrier cost on MI355X: 245 co-resident blocks (one per CU) spin on a counter in
// uncached device memory.  "bar": barriers only; "xchg": the persistent small-slice exchange
// per half-iteration — every block stores 236 partial sums (uncached), barrier, blocks 0..235
// each sum one output over all blocks' partials and store it, barrier, every block reads the 236
// sums.  Reports microseconds per barrier / per exchange.
//   hipcc -O3 --offload-arch=gfx950 tools/gbar_probe.hip -o tools/gbar_probe
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <cstdio>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

constexpr int NV = 236;

__device__ __forceinline__ void gbar(unsigned long long* ctr, unsigned long long target,
                                     int* err) {
  __syncthreads();
  if (threadIdx.x == 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_fetch_add(ctr, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const long long t0 = wall_clock64();
    while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      if (wall_clock64() - t0 > 100000000LL) { *err = 1; break; }   // 1 s: give up, no hang
      __builtin_amdgcn_s_sleep(1);
    }
  }
  __syncthreads();
}

__global__ __launch_bounds__(1024) void bar(unsigned long long* ctr, int n, int* err) {
  const unsigned long long nb = gridDim.x;
  for (int i = 1; i <= n; ++i) gbar(ctr, nb * i, err);
}

// Two-level barrier: blocks b = g (mod 8) — one XCD each under the round-robin dispatch — count
// on their group's counter (own 256 B line); the last of a group bumps the top counter.
__device__ __forceinline__ void gbar2(unsigned long long* ctr, int i, int* err) {
  __syncthreads();
  if (threadIdx.x == 0) {
    const int nb = gridDim.x, g = blockIdx.x & 7;
    const unsigned long long gsz = (unsigned long long)((nb - g + 7) / 8);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned long long old = __hip_atomic_fetch_add(ctr + 32 * (g + 1), 1ull,
                                                          __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (old + 1 == gsz * i)
      __hip_atomic_fetch_add(ctr, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned long long target = 8ull * i;
    const long long t0 = wall_clock64();
    while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      if (wall_clock64() - t0 > 100000000LL) { *err = 1; break; }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  __syncthreads();
}

__global__ __launch_bounds__(1024) void bar2(unsigned long long* ctr, int n, int* err) {
  for (int i = 1; i <= n; ++i) gbar2(ctr, i, err);
}

__global__ __launch_bounds__(1024) void xchg(unsigned long long* ctr, double* part, double* sums,
                                             int n, int* err, double* sink) {
  const unsigned long long nb = gridDim.x;
  __shared__ double s[NV];
  double acc = 0.0;
  for (int i = 0; i < n; ++i) {
    if (threadIdx.x < NV)
      __hip_atomic_store(reinterpret_cast<unsigned long long*>(part + (size_t)threadIdx.x * nb + blockIdx.x),
                         __builtin_bit_cast(unsigned long long, (double)(i + blockIdx.x)),
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    gbar(ctr, nb * (2 * i + 1), err);
    if (blockIdx.x < NV) {   // one output per block: sum over the blocks' partials
      double v = 0.0;
      for (int b = threadIdx.x; b < (int)nb; b += blockDim.x)
        v += __builtin_bit_cast(double, __hip_atomic_load(
                 reinterpret_cast<unsigned long long*>(part + (size_t)blockIdx.x * nb + b),
                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
      for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
      if ((threadIdx.x & 63) == 0) s[threadIdx.x >> 6] = v;
      __syncthreads();
      if (threadIdx.x == 0) {
        double t = 0.0;
        for (int w = 0; w < (int)(blockDim.x / 64); ++w) t += s[w];
        __hip_atomic_store(reinterpret_cast<unsigned long long*>(sums + blockIdx.x),
                           __builtin_bit_cast(unsigned long long, t), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
    gbar(ctr, nb * (2 * i + 2), err);
    if (threadIdx.x < NV)
      s[threadIdx.x] = __builtin_bit_cast(double, __hip_atomic_load(
          reinterpret_cast<unsigned long long*>(sums + threadIdx.x), __ATOMIC_RELAXED,
          __HIP_MEMORY_SCOPE_SYSTEM));
    __syncthreads();
    acc += s[(i + threadIdx.x) % NV];
  }
  if (acc == -1.0) *sink = acc;
}

int main() {
  int dev = 0, ncu = 0;
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  const int nb = ncu < 245 ? ncu : 245;
  unsigned long long* ctr;
  double *part, *sums, *sink;
  int* err;
  CK(hipExtMallocWithFlags((void**)&ctr, 4096, hipDeviceMallocUncached));  // 9 counters, 256 B apart
  CK(hipExtMallocWithFlags((void**)&part, (size_t)NV * nb * 8, hipDeviceMallocUncached));
  CK(hipExtMallocWithFlags((void**)&sums, 4096, hipDeviceMallocUncached));
  CK(hipMalloc(&err, 4));
  CK(hipMalloc(&sink, 8));
  CK(hipMemset(err, 0, 4));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int rep = 0; rep < 3; ++rep) {
    const int n = 2000;
    float ms;
    CK(hipMemset(ctr, 0, 8));
    CK(hipEventRecord(a));
    hipLaunchKernelGGL(bar, dim3(nb), dim3(1024), 0, 0, ctr, n, err);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    CK(hipEventElapsedTime(&ms, a, b));
    float ms3;
    CK(hipMemset(ctr, 0, 4096));
    CK(hipEventRecord(a));
    hipLaunchKernelGGL(bar2, dim3(nb), dim3(1024), 0, 0, ctr, n, err);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    CK(hipEventElapsedTime(&ms3, a, b));
    float ms2;
    CK(hipMemset(ctr, 0, 8));
    CK(hipEventRecord(a));
    hipLaunchKernelGGL(xchg, dim3(nb), dim3(1024), 0, 0, ctr, part, sums, n, err, sink);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    CK(hipEventElapsedTime(&ms2, a, b));
    int e = 0;
    CK(hipMemcpy(&e, err, 4, hipMemcpyDeviceToHost));
    printf("%d blocks x 1024: barrier %.3f us, two-level barrier %.3f us, exchange (2 barriers + "
           "reduce) %.3f us, err %d\n", nb, ms * 1e3 / n, ms3 * 1e3 / n, ms2 * 1e3 / n, e);
  }
  return 0;
}
