// frei_math.h — fp64 exp / expm1 / sqrt / division for the sweep kernels, bit-identical to
// the ocml / LLVM lowering they replace but cheaper on gfx950's VALU.
//
// Why: the sweep is fp64-VALU-bound, and three lowering choices cost ~25% of
// its instructions per flux update:
//   * ocml's exp Horner chain is emitted as `v_fmac_f64 acc(=c_k) += r * p`, so every
//     polynomial coefficient is first copied into a VGPR pair (two v_mov_b32 per term, ~18
//     VALU moves per call).  Here each term of the sweep's exp (exp_neg*) is one
//     `v_fma_f64 p, r, p, s[c_k]` with the coefficient in an SGPR pair (materialised by SALU
//     moves, off the VALU port).
//   * IEEE fp64 division is lowered with v_div_scale x2 / v_div_fmas / v_div_fixup around the
//     Newton-Raphson core.  Those only act when an operand is within ~2^768 of the exponent
//     range ends or denormal; every quotient the sweep forms (optical depths, Planck terms,
//     albedos, 1/chi) is far from them, so the bare core below returns the same bits.
//   * sqrt's denormal-range scaling (x < 2^-767) is likewise dropped: the sweep takes square
//     roots of 1 - w0 style quantities in (2^-53, 2].
//   * division and sqrt refine the hardware estimate with one Newton-Raphson step fewer than
//     the LLVM / ocml sequences: gfx950's v_rcp_f64 and
//     v_rsq_f64 are good to ~2^-24 and one step brings the reciprocal to <= 11 ulp
//     (tools/rcp_acc.hip), after which the quotient's residual correction (sqrt: the final
//     Newton correction) still rounds correctly — 0 differences from the IEEE result in 2^28
//     random operands per range (tools/mathcheck.hip).  Not a proof: a result within ~2^-45
//     ulp of a rounding midpoint could come out one ulp off (probability ~2^-44 per call).
//     -1.2 % sweep time at 500k, -3.9 % at 62.5k (profiles/r02_ab_short_div.txt).
// Otherwise every function keeps the exact operation sequence of the lowering it replaces
// (same constants, same fma order), so results are identical wherever the dropped guards
// would not fire; tools/mathcheck.hip checks that on the GPU over random and edge-case inputs.
#pragma once
#include <hip/hip_runtime.h>

namespace frei {
namespace fm {

// d = a * b + c with c held in an SGPR pair (wave-uniform constant).
__device__ __forceinline__ double fma_sc(double a, double b, double c) {
  double d;
  asm("v_fma_f64 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "s"(c));
  return d;
}

__device__ __forceinline__ double c64(unsigned long long bits) {
  return __builtin_bit_cast(double, bits);
}

// exp(x): ocml's own (the standalone two_stream form; the sweeps use exp_neg* below).  The
// SGPR-coefficient form of the whole-range exp pushed the one-lane sweep past the SGPR file (18
// spills), 2 % slower (profiles/r01_ab_fastmath.txt).
__device__ __forceinline__ double exp(double x) { return ::exp(x); }

// exp(x) for x <= 0 or NaN (a layer transmission exp(-2 sqrt(..) dtau)): ocml's sequence
// (round-to-nearest reduction by ln2 split in two, degree-11 Horner polynomial, two final fma
// with 1.0, ldexp) with the argument clamped at -1100 instead of its two range selects — below
// -1075 the final ldexp underflows to the same 0 ocml returns, so bit-identical for every
// x <= 0; NaN passes through.
// exp_neg's Horner terms as VOP3 fma with SGPR coefficients: otherwise the compiler keeps the
// coefficients in VGPRs and copies each into the accumulator of a two-address v_fmac (one
// extra move per term) — 174 vs 183 VALU instructions per flux update and -6 % sweep time
// at 500k despite a few SGPR spills (profiles/r02_ab_exp_sc.txt)
__device__ __forceinline__ double hfma(double r, double p, unsigned long long c) {
  return fma_sc(r, p, c64(c));
}
__device__ __forceinline__ double exp_neg(double x) {
  x = (x < -1100.0) ? -1100.0 : x;
  const double n = __builtin_rint(x * c64(0x3ff71547652b82feull));
  double r = __builtin_fma(c64(0xbfe62e42fefa39efull), n, x);
  r = __builtin_fma(c64(0xbc7abc9e3b39803full), n, r);
  double p = __builtin_fma(c64(0x3e5ade156a5dcb37ull), r, c64(0x3e928af3fca7ab0cull));
  p = hfma(r, p, 0x3ec71dee623fde64ull);
  p = hfma(r, p, 0x3efa01997c89e6b0ull);
  p = hfma(r, p, 0x3f2a01a014761f6eull);
  p = hfma(r, p, 0x3f56c16c1852b7b0ull);
  p = hfma(r, p, 0x3f81111111122322ull);
  p = hfma(r, p, 0x3fa55555555502a1ull);
  p = hfma(r, p, 0x3fc5555555555511ull);
  p = hfma(r, p, 0x3fe000000000000bull);
  p = __builtin_fma(r, p, 1.0);
  p = __builtin_fma(r, p, 1.0);
  return __builtin_ldexp(p, (int)n);
}

// exp_neg for an argument that cannot be NaN (the contracted-table sweeps: K3 is only built
// for NaN-free tables): the clamp is one v_max_f64 instead of a compare and two selects (maxNum
// would turn a NaN into -1100; here there is none).  Bit-identical to exp_neg otherwise.
__device__ __forceinline__ double exp_neg_nf(double x) {
  x = __builtin_fmax(x, -1100.0);
  const double n = __builtin_rint(x * c64(0x3ff71547652b82feull));
  double r = __builtin_fma(c64(0xbfe62e42fefa39efull), n, x);
  r = __builtin_fma(c64(0xbc7abc9e3b39803full), n, r);
  double p = __builtin_fma(c64(0x3e5ade156a5dcb37ull), r, c64(0x3e928af3fca7ab0cull));
  p = hfma(r, p, 0x3ec71dee623fde64ull);
  p = hfma(r, p, 0x3efa01997c89e6b0ull);
  p = hfma(r, p, 0x3f2a01a014761f6eull);
  p = hfma(r, p, 0x3f56c16c1852b7b0ull);
  p = hfma(r, p, 0x3f81111111122322ull);
  p = hfma(r, p, 0x3fa55555555502a1ull);
  p = hfma(r, p, 0x3fc5555555555511ull);
  p = hfma(r, p, 0x3fe000000000000bull);
  p = __builtin_fma(r, p, 1.0);
  p = __builtin_fma(r, p, 1.0);
  return __builtin_ldexp(p, (int)n);
}

// exp(x) for x <= 0 without the clamp (Planck factors, frei_kernels.hip planck_e): exp_neg's
// sequence, so bit-identical to it for x in [-1100, 0]; below, n stays an int32 and the final
// ldexp still underflows to 0.  NaN propagates; x = -inf gives NaN (a zero temperature).
__device__ __forceinline__ double exp_neg_unclamped(double x) {
  const double n = __builtin_rint(x * c64(0x3ff71547652b82feull));
  double r = __builtin_fma(c64(0xbfe62e42fefa39efull), n, x);
  r = __builtin_fma(c64(0xbc7abc9e3b39803full), n, r);
  double p = __builtin_fma(c64(0x3e5ade156a5dcb37ull), r, c64(0x3e928af3fca7ab0cull));
  p = hfma(r, p, 0x3ec71dee623fde64ull);
  p = hfma(r, p, 0x3efa01997c89e6b0ull);
  p = hfma(r, p, 0x3f2a01a014761f6eull);
  p = hfma(r, p, 0x3f56c16c1852b7b0ull);
  p = hfma(r, p, 0x3f81111111122322ull);
  p = hfma(r, p, 0x3fa55555555502a1ull);
  p = hfma(r, p, 0x3fc5555555555511ull);
  p = hfma(r, p, 0x3fe000000000000bull);
  p = __builtin_fma(r, p, 1.0);
  p = __builtin_fma(r, p, 1.0);
  return __builtin_ldexp(p, (int)n);
}

// 1 / b within one ulp: the reciprocal part of the division core below (rcp and two
// Newton-Raphson steps) without the quotient's final residual correction.  Used where the
// result only scales a sum (1 / chi of the flux update), so an ulp is not amplified.
// (One Newton step: within 11 ulp, two VALU fewer per update, 0..1.5 % sweep time —
// noise-level, profiles/r03/ab_rcp_steps.txt — but batched-vs-single temperatures then differ by
// 2e-11 after 3 iterations: not adopted.)
__device__ __forceinline__ double rcp_nr(double b) {
  double r = __builtin_amdgcn_rcp(b);
  double e = __builtin_fma(-b, r, 1.0);
  r = __builtin_fma(r, e, r);
  e = __builtin_fma(-b, r, 1.0);
  return __builtin_fma(r, e, r);
}

// a / b: LLVM's fp64 division core (rcp, one Newton-Raphson step where LLVM takes two,
// quotient, one residual correction) without the div_scale / div_fmas / div_fixup guards.
__device__ __forceinline__ double div(double a, double b) {
  double r = __builtin_amdgcn_rcp(b);
  const double e = __builtin_fma(-b, r, 1.0);
  r = __builtin_fma(r, e, r);
  const double q = a * r;
  const double rem = __builtin_fma(-b, q, a);
  return __builtin_fma(rem, r, q);
}

// sqrt(x): ocml's rsq + Newton-Raphson sequence (its last correction dropped) without the
// x < 2^-767 rescaling; +-0 and +inf pass through as in ocml.
__device__ __forceinline__ double sqrt(double x) {
  const double y = __builtin_amdgcn_rsq(x);
  double g = x * y;
  double h = y * 0.5;
  const double e = __builtin_fma(-h, g, 0.5);
  g = __builtin_fma(g, e, g);
  h = __builtin_fma(h, e, h);
  double d = __builtin_fma(-g, g, x);
  g = __builtin_fma(d, h, g);
  return __builtin_amdgcn_class(x, 0x260) ? x : g;   // +-0, +inf
}

// sqrt(x) for the sweep's square roots — E (E - w0), (E - w0) / E and 1 - w0 with
// w0 = sigma / (2 sigma + sum of table terms) <= 1/2 and E in [1, 1.21], i.e. x in (1/2, 1.21]
// for non-negative opacities: sqrt's sequence without the +-0 / +inf pass-through (three
// instructions), which only differs at exactly those inputs; NaN propagates as before.
__device__ __forceinline__ double sqrt_pos(double x) {
  const double y = __builtin_amdgcn_rsq(x);
  double g = x * y;
  double h = y * 0.5;
  const double e = __builtin_fma(-h, g, 0.5);
  g = __builtin_fma(g, e, g);
  h = __builtin_fma(h, e, h);
  double d = __builtin_fma(-g, g, x);
  g = __builtin_fma(d, h, g);
  return g;
}

}  // namespace fm
}  // namespace frei
