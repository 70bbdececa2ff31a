// Unit check of frei::group_sum4<Q> (DPP / permlane-swap wave sums) against exact sums.
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 -Iinclude -Ifrei_amd/csrc tools/groupsum_check.hip
#include "../frei_amd/csrc/frei_kernels.hip"
#include <cstdio>
template <int Q>
__global__ void t(double* o) {
  int l = threadIdx.x;
  double q0 = l + 1, q1 = 1000 * (l + 1), q2 = 1e6 * (l + 1), q3 = 1e9 * (l + 1);
  o[l] = frei::group_sum4<Q>(q0, q1, q2, q3, l);
}
int main() {
  double* d; hipMalloc(&d, 3 * 64 * 8);
  hipLaunchKernelGGL(t<1>, dim3(1), dim3(64), 0, 0, d);
  hipLaunchKernelGGL(t<2>, dim3(1), dim3(64), 0, 0, d + 64);
  hipLaunchKernelGGL(t<4>, dim3(1), dim3(64), 0, 0, d + 128);
  double h[192]; hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  int Qs[3] = {1, 2, 4};
  for (int r = 0; r < 3; ++r) {
    int Q = Qs[r], bad = 0;
    for (int l = 0; l < 4 * Q; ++l) {
      int q = l % Q, b = (l / Q) & 1, c = (l / (2 * Q)) & 1, idx = 2 * b + c;
      double scale = idx == 0 ? 1 : idx == 1 ? 1000 : idx == 2 ? 1e6 : 1e9, want = 0;
      for (int m = q; m < 64; m += Q) want += scale * (m + 1);
      if (h[r * 64 + l] != want) { ++bad; printf("Q%d lane %d got %.17g want %.17g\n", Q, l, h[r * 64 + l], want); }
    }
    printf("Q%d: %d bad\n", Q, bad);
  }
  return 0;
}
