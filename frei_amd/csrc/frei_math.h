// frei_math.h — fp64 exp / expm1 / sqrt / division for the sweep kernels, bit-identical to
// the ocml / LLVM lowering they replace but cheaper on gfx950's VALU.
//
// Why: the sweep is fp64-VALU-bound, and three lowering choices cost ~25% of
// its instructions per flux update:
//   * ocml's exp/expm1 Horner chains are emitted as `v_fmac_f64 acc(=c_k) += r * p`, so every
//     polynomial coefficient is first copied into a VGPR pair (two v_mov_b32 per term, ~18
//     VALU moves per call).  Here each term is one `v_fma_f64 p, r, p, s[c_k]` with the
//     coefficient in an SGPR pair (materialised by SALU moves, off the VALU port).
//   * IEEE fp64 division is lowered with v_div_scale x2 / v_div_fmas / v_div_fixup around the
//     Newton-Raphson core.  Those only act when an operand is within ~2^768 of the exponent
//     range ends or denormal; every quotient the sweep forms (optical depths, Planck terms,
//     albedos, 1/chi) is far from them, so the bare core below returns the same bits.
//   * sqrt's denormal-range scaling (x < 2^-767) is likewise dropped: the sweep takes square
//     roots of 1 - w0 style quantities in (2^-53, 2].
//   * division and sqrt refine the hardware estimate with one Newton-Raphson step fewer than
//     the LLVM / ocml sequences (FREI_FM_DIV / FREI_FM_SQRT = 2): gfx950's v_rcp_f64 and
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

// A/B switches (tools/build_variant.sh -DFREI_FM_...=0|1|2): 0 selects the plain ocml / IEEE
// form, 1 the full-length sequences without range guards, 2 (div, sqrt) one step fewer.  FREI_FM_EXP is off: in the sweep the SGPR-held coefficients push the kernel past
// the SGPR file (18 spills through v_writelane/v_readlane), which measured 2% slower than the
// VGPR moves it removes (profiles/r01_ab_fastmath.txt).  Division and sqrt are on (-6%).
#ifndef FREI_FM_EXP
#define FREI_FM_EXP 0
#endif
#ifndef FREI_FM_EXPM1
#define FREI_FM_EXPM1 FREI_FM_EXP
#endif
#ifndef FREI_FM_DIV
#define FREI_FM_DIV 2
#endif
#ifndef FREI_FM_SQRT
#define FREI_FM_SQRT 2
#endif

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

// exp(x): ocml __ocml_exp_f64 (round-to-nearest reduction by ln2 split in two, degree-11
// Horner polynomial, two final fma with 1.0, ldexp; x > 1024 -> inf, x < -1075 -> 0).
__device__ __forceinline__ double exp(double x) {
#if !FREI_FM_EXP
  return ::exp(x);
#endif
  const double n = __builtin_rint(x * c64(0x3ff71547652b82feull));
  double r = __builtin_fma(c64(0xbfe62e42fefa39efull), n, x);
  r = __builtin_fma(c64(0xbc7abc9e3b39803full), n, r);
  double p = __builtin_fma(c64(0x3e5ade156a5dcb37ull), r, c64(0x3e928af3fca7ab0cull));
  p = fma_sc(r, p, c64(0x3ec71dee623fde64ull));
  p = fma_sc(r, p, c64(0x3efa01997c89e6b0ull));
  p = fma_sc(r, p, c64(0x3f2a01a014761f6eull));
  p = fma_sc(r, p, c64(0x3f56c16c1852b7b0ull));
  p = fma_sc(r, p, c64(0x3f81111111122322ull));
  p = fma_sc(r, p, c64(0x3fa55555555502a1ull));
  p = fma_sc(r, p, c64(0x3fc5555555555511ull));
  p = fma_sc(r, p, c64(0x3fe000000000000bull));
  p = __builtin_fma(r, p, 1.0);
  p = __builtin_fma(r, p, 1.0);
  double e = __builtin_ldexp(p, (int)n);
  e = (x > 1024.0) ? __builtin_inf() : e;   // NaN passes through, as in ocml
  return (x < -1075.0) ? 0.0 : e;
}

// expm1(x): ocml __ocml_expm1_f64 (same reduction, degree-12 polynomial for e^r - 1 - r,
// scale 2^n with the n = 1024 split, x > 709.78 -> inf, x < -37 -> -1).
__device__ __forceinline__ double expm1(double x) {
#if !FREI_FM_EXPM1
  return ::expm1(x);
#endif
  const double n = __builtin_rint(x * c64(0x3ff71547652b82feull));
  double r = __builtin_fma(c64(0xbfe62e42fefa39efull), n, x);
  r = __builtin_fma(c64(0xbc7abc9e3b39803full), n, r);
  double p = __builtin_fma(c64(0x3e21f32ea9d67f34ull), r, c64(0x3e5af4eb2a1b768bull));
  p = fma_sc(r, p, c64(0x3e927e500e0ac05bull));
  p = fma_sc(r, p, c64(0x3ec71de01b889c29ull));
  p = fma_sc(r, p, c64(0x3efa01a0197bcfd8ull));
  p = fma_sc(r, p, c64(0x3f2a01a01ac1a723ull));
  p = fma_sc(r, p, c64(0x3f56c16c16c18931ull));
  p = fma_sc(r, p, c64(0x3f81111111110056ull));
  p = fma_sc(r, p, c64(0x3fa5555555555552ull));
  p = fma_sc(r, p, c64(0x3fc5555555555557ull));
  p = r * __builtin_fma(r, p, 0.5);
  const bool top = (n == 1024.0);
  const double s = top ? c64(0x7fe0000000000000ull) : __builtin_ldexp(1.0, (int)n);
  const double t = s - 1.0;
  const double u = __builtin_fma(r, p, r);
  double y = __builtin_fma(s, u, t);
  y = top ? y + y : y;
  y = (x > c64(0x40862e42fefa39efull)) ? __builtin_inf() : y;
  return (x < -37.0) ? -1.0 : y;
}

// expm1 with its polynomial coefficients held in VGPRs for a whole kernel: the same
// operation sequence as fm::expm1 / ocml (bit-identical), but the coefficients are loaded
// once through an index the compiler cannot prove uniform (mbcnt of an empty mask = 0), so
// they cannot be rematerialised as literal moves inside the loop (two v_mov_b32 per term per
// call otherwise; 10 VGPR pairs instead).
__device__ const double kExpm1Coef[10] = {
    __builtin_bit_cast(double, 0x3e21f32ea9d67f34ull), __builtin_bit_cast(double, 0x3e5af4eb2a1b768bull),
    __builtin_bit_cast(double, 0x3e927e500e0ac05bull), __builtin_bit_cast(double, 0x3ec71de01b889c29ull),
    __builtin_bit_cast(double, 0x3efa01a0197bcfd8ull), __builtin_bit_cast(double, 0x3f2a01a01ac1a723ull),
    __builtin_bit_cast(double, 0x3f56c16c16c18931ull), __builtin_bit_cast(double, 0x3f81111111110056ull),
    __builtin_bit_cast(double, 0x3fa5555555555552ull), __builtin_bit_cast(double, 0x3fc5555555555557ull)};

struct Expm1Reg {
  double c[10];
};

__device__ __forceinline__ Expm1Reg expm1_regs() {
  const int z = (int)__builtin_amdgcn_mbcnt_lo(0u, 0u);
  Expm1Reg k;
#pragma unroll
  for (int i = 0; i < 10; ++i) k.c[i] = kExpm1Coef[i + z];
  return k;
}

__device__ __forceinline__ double expm1(double x, const Expm1Reg& k) {
  const double n = __builtin_rint(x * c64(0x3ff71547652b82feull));
  double r = __builtin_fma(c64(0xbfe62e42fefa39efull), n, x);
  r = __builtin_fma(c64(0xbc7abc9e3b39803full), n, r);
  double p = __builtin_fma(k.c[0], r, k.c[1]);
#pragma unroll
  for (int i = 2; i < 10; ++i) p = __builtin_fma(r, p, k.c[i]);
  p = r * __builtin_fma(r, p, 0.5);
  const bool top = (n == 1024.0);
  const double s = top ? c64(0x7fe0000000000000ull) : __builtin_ldexp(1.0, (int)n);
  const double t = s - 1.0;
  const double u = __builtin_fma(r, p, r);
  double y = __builtin_fma(s, u, t);
  y = top ? y + y : y;
  y = (x > c64(0x40862e42fefa39efull)) ? __builtin_inf() : y;
  return (x < -37.0) ? -1.0 : y;
}

// expm1(x) for a Planck exponent x in [0, 600] (every ordinary layer): the sequence of
// expm1(x, k) above without its range selects (n < 1024, no overflow, x > -37 all hold
// there), so bit-identical to ocml on that range.  The sweeps route x > 600 (very cold layers
// at short wavelengths, expm1 >= 2^865) to the full IEEE form.
__device__ __forceinline__ double expm1_mid(double x, const Expm1Reg& k) {
  const double n = __builtin_rint(x * c64(0x3ff71547652b82feull));
  double r = __builtin_fma(c64(0xbfe62e42fefa39efull), n, x);
  r = __builtin_fma(c64(0xbc7abc9e3b39803full), n, r);
  double p = __builtin_fma(k.c[0], r, k.c[1]);
#pragma unroll
  for (int i = 2; i < 10; ++i) p = __builtin_fma(r, p, k.c[i]);
  p = r * __builtin_fma(r, p, 0.5);
  const double s = __builtin_ldexp(1.0, (int)n);
  const double t = s - 1.0;
  const double u = __builtin_fma(r, p, r);
  return __builtin_fma(s, u, t);
}

// exp(x) for x <= 0 or NaN (a layer transmission exp(-2 sqrt(..) dtau)): ocml's sequence
// (fm::exp above) with the argument clamped at -1100 instead of its two range selects — below
// -1075 the final ldexp underflows to the same 0 ocml returns, so bit-identical for every
// x <= 0; NaN passes through.
// exp_neg's Horner terms as VOP3 fma with SGPR coefficients: otherwise the compiler keeps the
// coefficients in VGPRs and copies each into the accumulator of a two-address v_fmac (one
// extra move per term) — 174 vs 183 VALU instructions per flux update and -6 % sweep time
// at 500k despite a few SGPR spills (profiles/r02_ab_exp_sc.txt)
#ifndef FREI_EXP_SC
#define FREI_EXP_SC 1
#endif
__device__ __forceinline__ double hfma(double r, double p, unsigned long long c) {
#if FREI_EXP_SC
  return fma_sc(r, p, c64(c));
#else
  return __builtin_fma(r, p, c64(c));
#endif
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
// FREI_RCP_STEPS: Newton steps after v_rcp_f64 — 2 (default): within 1 ulp; 1: within 11 ulp,
// two VALU fewer per update, 0..1.5 % sweep time (noise-level, profiles/r03/ab_rcp_steps.txt) but
// batched-vs-single temperatures then differ by 2e-11 after 3 iterations: not adopted.
#ifndef FREI_RCP_STEPS
#define FREI_RCP_STEPS 2
#endif
__device__ __forceinline__ double rcp_nr(double b) {
  double r = __builtin_amdgcn_rcp(b);
  double e = __builtin_fma(-b, r, 1.0);
#if FREI_RCP_STEPS == 1
  return __builtin_fma(r, e, r);
#else
  r = __builtin_fma(r, e, r);
  e = __builtin_fma(-b, r, 1.0);
  return __builtin_fma(r, e, r);
#endif
}

// a / b: LLVM's fp64 division core (rcp, two Newton-Raphson steps — one with FREI_FM_DIV 2 —,
// quotient, one residual correction) without the div_scale / div_fmas / div_fixup guards.
__device__ __forceinline__ double div(double a, double b) {
#if !FREI_FM_DIV
  return a / b;
#endif
  double r = __builtin_amdgcn_rcp(b);
  double e = __builtin_fma(-b, r, 1.0);
  r = __builtin_fma(r, e, r);
#if FREI_FM_DIV != 2
  e = __builtin_fma(-b, r, 1.0);
  r = __builtin_fma(r, e, r);
#endif
  const double q = a * r;
  const double rem = __builtin_fma(-b, q, a);
  return __builtin_fma(rem, r, q);
}

// c / x for x from expm1 of a Planck exponent: x can exceed 2^900 (x -> inf for very cold
// layers at short wavelengths), where the unguarded core would lose the denormal quotient;
// those lanes take the IEEE division (a rarely taken, execz-skipped branch).
__device__ __forceinline__ double div_big(double a, double b) {
  double q = div(a, b);
  if (__builtin_expect(!(b < 0x1p900), 0)) q = a / b;
  return q;
}

// sqrt(x): ocml's rsq + Newton-Raphson sequence (its last correction dropped with
// FREI_FM_SQRT 2) without the x < 2^-767 rescaling; +-0 and +inf pass through as in ocml.
__device__ __forceinline__ double sqrt(double x) {
#if !FREI_FM_SQRT
  return ::sqrt(x);
#endif
  const double y = __builtin_amdgcn_rsq(x);
  double g = x * y;
  double h = y * 0.5;
  const double e = __builtin_fma(-h, g, 0.5);
  g = __builtin_fma(g, e, g);
  h = __builtin_fma(h, e, h);
  double d = __builtin_fma(-g, g, x);
  g = __builtin_fma(d, h, g);
#if FREI_FM_SQRT != 2
  d = __builtin_fma(-g, g, x);
  g = __builtin_fma(d, h, g);
#endif
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
#if FREI_FM_SQRT != 2
  d = __builtin_fma(-g, g, x);
  g = __builtin_fma(d, h, g);
#endif
  return g;
}

}  // namespace fm
}  // namespace frei
