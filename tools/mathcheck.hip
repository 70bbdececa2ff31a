// Bitwise check of frei_math.h (fm::exp / expm1 / div / sqrt, exp_neg, expm1_mid) against the
// ocml / IEEE forms on the GPU, and rcp_nr within one ulp: random inputs over the ranges the
// sweep uses (and well beyond), plus edge cases.
//   hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -std=c++17 -Ifrei_amd/csrc \
//         tools/mathcheck.hip -o tools/mathcheck && ./tools/mathcheck
// Prints mismatch counts per function and range; exit status 1 on any mismatch inside the
// ranges the sweep relies on (div operands within 2^+-450, sqrt arguments >= 2^-767).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdint>

#include "frei_math.h"

using namespace frei;

__device__ inline uint64_t mix(uint64_t x) {
  x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull;
  return x ^ (x >> 33);
}
__device__ inline double unif(uint64_t i, uint64_t salt) {
  return (double)(mix(i * 0x9e3779b97f4a7c15ull + salt) >> 11) * 0x1p-53;
}
__device__ inline bool same(double a, double b) {
  return __double_as_longlong(a) == __double_as_longlong(b) || (isnan(a) && isnan(b));
}

// kind: 0 exp on [lo, hi], 1 expm1 on [lo, hi], 2 div with log-uniform |a|,|b| in 2^[lo,hi]
// and random signs, 3 sqrt log-uniform in 2^[lo, hi]
__global__ void check(int kind, double lo, double hi, uint64_t n, unsigned long long* bad,
                      double* example) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * blockDim.x) {
    double x = lo + (hi - lo) * unif(i, 1 + kind), got, ref;
    if (kind == 0) { got = fm::exp(x); ref = ::exp(x); }
    else if (kind == 1) { got = fm::expm1(x); ref = ::expm1(x); }
    else if (kind == 2) {
      const double a = ldexp(1.0 + unif(i, 7), (int)floor(x)) * (unif(i, 8) < 0.5 ? -1 : 1);
      const double y = lo + (hi - lo) * unif(i, 9);
      const double b = ldexp(1.0 + unif(i, 10), (int)floor(y)) * (unif(i, 11) < 0.5 ? -1 : 1);
      got = fm::div(a, b); ref = a / b; x = a;
    } else if (kind == 3) {
      x = ldexp(1.0 + unif(i, 12), (int)floor(x));
      got = fm::sqrt(x); ref = ::sqrt(x);
    } else if (kind == 4) {
      got = fm::exp_neg(x); ref = ::exp(x);
    } else if (kind == 5) {
      got = fm::expm1_mid(x, fm::expm1_regs()); ref = ::expm1(x);
    } else {   // rcp_nr: within 1 ulp (two Newton steps) / 16 ulp (one) of the rounded 1 / b
      const double b = ldexp(1.0 + unif(i, 13), (int)floor(x)) * (unif(i, 14) < 0.5 ? -1 : 1);
      got = fm::rcp_nr(b); ref = 1.0 / b; x = b;
      const long long d = __double_as_longlong(got) - __double_as_longlong(ref);
      const long long tol = FREI_RCP_STEPS == 1 ? 16 : 1;
      if (d >= -tol && d <= tol) got = ref;
    }
    if (!same(got, ref)) {
      if (atomicAdd(bad, 1ull) == 0) { example[0] = x; example[1] = got; example[2] = ref; }
    }
  }
}

__global__ void edges(unsigned long long* bad) {
  const double inf = __builtin_inf(), nan = __builtin_nan("");
  const double xs[] = {0.0, -0.0, 1.0, -1.0, 1e-300, -1e-300, 709.78, 709.79, 1023.9, 1024.0,
                       1024.5, -745.1, -745.2, -1074.9, -1075.0, -1075.1, -36.9, -37.0,
                       -37.1, 1e-20, inf, -inf, nan, 0x1p-1022, 0x1p-1074};
  int b = 0;
  for (double x : xs) {
    b += !same(fm::exp(x), ::exp(x));
    b += !same(fm::expm1(x), ::expm1(x));
    if (x >= 0x1p-767 || x == 0.0 || x == inf || isnan(x)) b += !same(fm::sqrt(x), ::sqrt(x));
  }
  const double xn[] = {0.0, -0.0, -1e-300, -1.0, -745.1, -1074.9, -1075.0, -1075.1, -1100.0,
                       -1100.5, -1e6, -inf, nan};
  for (double x : xn) b += !same(fm::exp_neg(x), ::exp(x));
  b += !same(fm::div_big(3.0, inf), 0.0);
  b += !same(fm::div_big(3.0, 0x1p1000), 3.0 / 0x1p1000);
  *bad = b;
}

int main() {
  unsigned long long* d_bad;
  double* d_ex;
  hipMalloc(&d_bad, sizeof(unsigned long long));
  hipMalloc(&d_ex, 3 * sizeof(double));
  struct Case { const char* name; int kind; double lo, hi; bool must; };
  const Case cases[] = {
      {"exp   [-800, 0]   (sweep: exp(-2 sq dtau))", 0, -800.0, 0.0, true},
      {"exp   [-1100, 1100]", 0, -1100.0, 1100.0, true},
      {"expm1 [0, 750]    (Planck exponent)", 1, 0.0, 750.0, true},
      {"expm1 [-40, 2]", 1, -40.0, 2.0, true},
      {"div   |a|, |b| in 2^[-450, 450]", 2, -450.0, 450.0, true},
      {"div   2^[-1070, 1020] (guards dropped: may differ)", 2, -1070.0, 1020.0, false},
      {"sqrt  2^[-767, 1023]", 3, -767.0, 1023.0, true},
      {"sqrt  2^[-1074, -767] (scaling dropped: may differ)", 3, -1074.0, -767.0, false},
      {"exp_neg [-1200, 0] vs exp (sweep transmission)", 4, -1200.0, 0.0, true},
      {"expm1_mid [0, 600] vs expm1 (Planck, ordinary layers)", 5, 0.0, 600.0, true},
      {FREI_RCP_STEPS == 1 ? "rcp_nr within 16 ulp, |b| in 2^[-450, 450]"
                           : "rcp_nr within 1 ulp, |b| in 2^[-450, 450]", 6, -450.0, 450.0, true},
  };
  const uint64_t n = 1ull << 28;
  int fail = 0;
  for (const Case& c : cases) {
    hipMemset(d_bad, 0, sizeof(unsigned long long));
    hipLaunchKernelGGL(check, dim3(4096), dim3(256), 0, 0, c.kind, c.lo, c.hi, n, d_bad, d_ex);
    unsigned long long bad = 0;
    double ex[3] = {0, 0, 0};
    hipMemcpy(&bad, d_bad, sizeof(bad), hipMemcpyDeviceToHost);
    hipMemcpy(ex, d_ex, sizeof(ex), hipMemcpyDeviceToHost);
    printf("%-52s %llu / %llu differ", c.name, bad, (unsigned long long)n);
    if (bad) printf("  (e.g. x=%.17g got %.17g ref %.17g)", ex[0], ex[1], ex[2]);
    printf("\n");
    if (bad && c.must) fail = 1;
  }
  hipMemset(d_bad, 0, sizeof(unsigned long long));
  hipLaunchKernelGGL(edges, dim3(1), dim3(1), 0, 0, d_bad);
  unsigned long long bad = 0;
  hipMemcpy(&bad, d_bad, sizeof(bad), hipMemcpyDeviceToHost);
  printf("%-52s %llu differ\n", "edge cases (0, +-inf, NaN, range ends)", bad);
  if (bad) fail = 1;
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  return fail;
}
