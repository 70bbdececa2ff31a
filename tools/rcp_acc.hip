// Accuracy of gfx950's fp64 v_rcp_f64 / v_rsq_f64 and of one Newton-Raphson step on them,
// over random operands spanning [2^-40, 2^40] (max relative error vs the IEEE result, in ulp
// of the result).  Decides how many refinement steps the sweep's divisions need.
//   hipcc -O3 --offload-arch=gfx950 tools/rcp_acc.hip -o tools/rcp_acc
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <vector>

__global__ void probe(const double* b, double* out, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double x = b[i];
  const double r0 = __builtin_amdgcn_rcp(x);
  const double e = __builtin_fma(-x, r0, 1.0);
  const double r1 = __builtin_fma(r0, e, r0);
  const double y0 = __builtin_amdgcn_rsq(x);
  const double g = x * y0, h = y0 * 0.5;
  const double e2 = __builtin_fma(-h, g, 0.5);
  const double g1 = __builtin_fma(g, e2, g);   // sqrt after one coupled step
  const double q1 = 3.0 * r1;                 // quotient 3/x from one-step reciprocal
  const double rem = __builtin_fma(-x, q1, 3.0);
  const double q2 = __builtin_fma(rem, r1, q1);  // + residual correction
  out[7 * i + 0] = r0;
  out[7 * i + 1] = r1;
  out[7 * i + 2] = y0;
  out[7 * i + 3] = g1;
  out[7 * i + 4] = q1;
  out[7 * i + 5] = q2;
  out[7 * i + 6] = 3.0 / x;
}

static double ulp_err(double got, double ref) {
  if (got == ref) return 0.0;
  const double u = std::nextafter(std::fabs(ref), INFINITY) - std::fabs(ref);
  return std::fabs(got - ref) / u;
}

int main() {
  const int n = 1 << 22;
  std::vector<double> b(n), o(7 * (size_t)n);
  unsigned long long s = 88172645463325252ull;
  for (int i = 0; i < n; ++i) {
    s ^= s << 13; s ^= s >> 7; s ^= s << 17;
    const double u = (double)(s >> 11) * 0x1p-53;
    b[i] = std::ldexp(1.0 + u, (int)(s % 81) - 40);
  }
  double *db, *dout;
  hipMalloc(&db, n * sizeof(double));
  hipMalloc(&dout, 7 * (size_t)n * sizeof(double));
  hipMemcpy(db, b.data(), n * sizeof(double), hipMemcpyHostToDevice);
  hipLaunchKernelGGL(probe, dim3(n / 256), dim3(256), 0, 0, db, dout, n);
  hipMemcpy(o.data(), dout, 7 * (size_t)n * sizeof(double), hipMemcpyDeviceToHost);
  double m[7] = {0};
  long exact[7] = {0};
  for (int i = 0; i < n; ++i) {
    const double x = b[i];
    const double ref[7] = {1.0 / x, 1.0 / x, 1.0 / std::sqrt(x), std::sqrt(x), 3.0 / x, 3.0 / x,
                           3.0 / x};
    for (int k = 0; k < 7; ++k) {
      const double e = ulp_err(o[7 * (size_t)i + k], ref[k]);
      m[k] = e > m[k] ? e : m[k];
      exact[k] += (e == 0.0);
    }
  }
  const char* name[7] = {"rcp", "rcp+1NR", "rsq", "sqrt(rsq+1 step)", "3*(rcp+1NR)",
                         "3*(rcp+1NR)+residual", "3/x (IEEE)"};
  for (int k = 0; k < 7; ++k)
    printf("%-22s max %.4g ulp, exact %.4f\n", name[k], m[k], (double)exact[k] / n);
  return 0;
}
