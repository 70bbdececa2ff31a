// frei_kernels.hip — gfx950 (CDNA4) kernels of the two-stream radiative-transfer engine.
//
// Hot path of bmorris3/frei:
//   K1 sweep_kernel   one lane per wavelength bin, loop over layers inside the lane
//                     (emit: twostream.py:351-407, absorb: 486-536) with the species-summed
//                     opacity assembly fused in (K2, opacity.py:203-269), Planck reuse
//                     between adjacent layers, in-place flux update and the per-layer
//                     bolometric trapezoid partials (twostream.py:16-20, 396-398) reduced
//                     wave -> block in a fixed order.
//   reduce_kernel     deterministic sum of the per-block partials -> [steps][4].
//   update_kernel     K4/K5: per-layer scalar physics (twostream.py:23-43, 180-287) -> dT,
//                     T <- T - dT (Q11), absorb temperature history and the reference's
//                     convergence test (core.py:301-318), then the next sweep's
//                     per-layer interpolation terms (setup) — the T-P loop never leaves
//                     the device.
//
// Numerics: fp64 throughout, compiled with -ffp-contract=off and the reference's
// expression order, so results differ from NumPy only by the last-ulp differences of
// exp/expm1/sqrt (ocml vs libm).  See DESIGN.md "Parity".
#include <unordered_map>

#include "frei_device.h"
#include "frei_math.h"

namespace frei {

// ---------------------------------------------------------------- diagnostic trace
// FREI_TRACE builds only (tools/trace_probe.py): thread 0 of every block of the sweeps and
// the fused update appends (kernel kind, block, 4 wall-clock marks at 100 MHz) to a device
// ring — entry, end of the prologue, end of the main loop, exit — so one T-P half-iteration's
// launch latency, prologue, steps and drain can be read off without a profiler.  Beside the
// wall clock, entry and exit also stamp the shader-cycle counter (s_memtime): Δcycles ÷
// Δwall × 100 MHz is the clock the block ran at (MI355X_MICROARCH.md, DVFS item 6).
#ifdef FREI_TRACE
struct TraceRec {
  long long kind, block, t[4], cyc[2];
};
constexpr unsigned kTraceCap = 1u << 17;
__device__ TraceRec g_trace[kTraceCap];
__device__ unsigned int g_trace_n;
#define TRACE_DECL                                                           \
  long long tr_[4] = {wall_clock64(), 0, 0, 0};                              \
  const long long trc_ = (long long)__builtin_amdgcn_s_memtime()
#define TRACE_MARK(i) (tr_[i] = wall_clock64())
#define TRACE_PUT(kind)                                                      \
  do {                                                                       \
    tr_[3] = wall_clock64();                                                 \
    const long long trc1_ = (long long)__builtin_amdgcn_s_memtime();         \
    if (threadIdx.x == 0) {                                                  \
      const unsigned i_ = atomicAdd(&g_trace_n, 1u);                         \
      if (i_ < kTraceCap)                                                    \
        g_trace[i_] = TraceRec{(kind), (long long)blockIdx.x,                \
                               {tr_[0], tr_[1], tr_[2], tr_[3]},             \
                               {trc_, trc1_}};                               \
    }                                                                        \
  } while (0)
// Per-phase stamps of the producer/consumer sweep (tools/pipe_trace.py): lane 0 of every wave
// of sampled blocks (bx % 32 == 5) stamps the shader-cycle counter at the loop start and, per
// phase, on reaching the block barrier and on leaving it; the last launch per direction wins.
constexpr int kPtPh = 24;
__device__ long long g_ptrace[2 * 8 * 16 * (kPtPh + 1) * 2];
#define PT_STAMP(dir, bx, wv, ph, k)                                                       \
  do {                                                                                     \
    if (blockIdx.y == 0 && (bx) % 32 == 5 && (bx) / 32 < 8 && (threadIdx.x & 63) == 0 &&   \
        (ph) + 1 <= kPtPh)                                                                 \
      g_ptrace[(((((dir) * 8 + (bx) / 32) * 16 + (wv)) * (kPtPh + 1)) + (ph) + 1) * 2 + (k)] = \
          (long long)__builtin_amdgcn_s_memtime();                                         \
  } while (0)
#else
#define TRACE_DECL
#define TRACE_MARK(i)
#define TRACE_PUT(kind)
#define PT_STAMP(dir, bx, wv, ph, k)
#endif

// ---------------------------------------------------------------- device math
// twostream.py:64-67: 2hc^2/lam^5 / expm1(hc / (lam k T)).  The exponent is formed as
// (hc / (lam k)) * (1 / T) — a per-wavelength constant (host) times a per-layer one (the step
// record) — instead of one division per update: within 1.5 ulp of the reference's
// hc / ((lam k) T), which moves spectra and T by < 1e-13.
//
// The value is formed as c1 e / (1 - e) with e = exp(-x), from the transmission's exp (its
// coefficients are wave-uniform SGPR constants the sweep already holds) instead of an expm1
// whose ten coefficients occupied 20 VGPRs per lane: four VALU and 20 VGPRs fewer per update,
// no range guard (e in [0, 1]: the quotient never overflows, and e underflows to the
// reference's 0 at x > 745).  Error: a few ulp, growing as ~1 ulp / x for x < 1 (the
// cancellation in 1 - e) — 1e-15 relative at x = 0.1, far inside the 1e-10 parity bar.  A NaN
// temperature propagates.  Between x = 709.8 (where numpy's expm1 overflows, B = 0) and 745 it
// returns the subnormal c1 e instead of 0.
__device__ __forceinline__ double planck(double c1, double hcl, double iT) {
  const double e = fm::exp_neg_unclamped(-(hcl * iT));
  return fm::div(c1 * e, 1.0 - e);
}

// twostream.py:97-177 with g_0 = 0 (call sites 389, 518), E() of :70-94.
__device__ __forceinline__ void two_stream(double w0, double dtau, double B1, double B2,
                                           double F1u, double F2d, double& F2u,
                                           double& F1d) {
  // E = 1 where w0 <= 0.1 (twostream.py:90-94): then E * Emw, Emw / E and Bprime / (2 E)
  // are exact without the multiply/divide, and sqrt(E * Emw) == sqrt(Emw / E), so that
  // branch skips two divisions and a square root with bit-identical results.
  double E, Emw, sq, r, q;
  const double Bp = fm::div(B1 - B2, dtau);
  if (w0 > 0.1) {
    E = (1.225 - 0.1777 * w0) - 0.05582 * (w0 * w0);
    Emw = E - w0;
    sq = fm::sqrt(E * Emw);
    r = fm::sqrt(fm::div(Emw, E));
    q = fm::div(Bp, 2.0 * E);
  } else {
    E = 1.0;
    Emw = 1.0 - w0;
    sq = fm::sqrt(Emw);
    r = sq;
    q = Bp * 0.5;
  }
  const double Tr = fm::exp((-2.0 * sq) * dtau);
  const double zp = 0.5 * (1.0 + r);
  const double zm = 0.5 * (1.0 - r);
  const double Tr2 = Tr * Tr;
  const double zm2 = zm * zm;
  const double zp2 = zp * zp;
  const double chi = zm2 * Tr2 - zp2;
  const double xi = (zp * zm) * (1.0 - Tr2);
  const double psi = (zm2 - zp2) * Tr;
  const double pi_w = fm::div(kPi * (1.0 - w0), Emw);
  const double ic = fm::div(1.0, chi);
  F2u = ic * ((psi * F1u - xi * F2d) +
              pi_w * ((B2 * (chi + xi) - psi * B1) + q * ((chi - psi) - xi)));
  F1d = ic * ((psi * F2d - xi * F1u) +
              pi_w * ((B1 * (chi + xi) - psi * B2) + q * ((xi + psi) - chi)));
}

// propagate_fluxes with an asymmetry factor g0 (twostream.py:139-176, E of :89-94), the
// reference's numpy expression order term by term; IEEE operations throughout (standalone
// API only: E - w0 may be <= 0 for strongly back-scattering g0, giving NaN as numpy does).
__device__ __forceinline__ void two_stream_g(double w0, double g0, double dtau, double B1,
                                             double B2, double F1u, double F2d, double& F2u,
                                             double& F1d) {
  const double E = (w0 > 0.1) ? (((((1.225 - 0.1582 * g0) - 0.1777 * w0) - 0.07465 * (g0 * g0)) +
                                  (0.2351 * w0) * g0) - 0.05582 * (w0 * w0))
                              : 1.0;
  const double Emw = E - w0;
  const double wg = 1.0 - w0 * g0;
  const double Tr = ::exp((-2.0 * ::sqrt((E * Emw) * wg)) * dtau);
  const double r = ::sqrt((Emw / E) / wg);
  const double zp = 0.5 * (1.0 + r);
  const double zm = 0.5 * (1.0 - r);
  const double Tr2 = Tr * Tr;
  const double zm2 = zm * zm;
  const double zp2 = zp * zp;
  const double chi = zm2 * Tr2 - zp2;
  const double xi = (zp * zm) * (1.0 - Tr2);
  const double psi = (zm2 - zp2) * Tr;
  const double pi_w = (kPi * (1.0 - w0)) / Emw;
  const double q = ((B1 - B2) / dtau) / ((2.0 * E) * wg);
  const double ic = 1.0 / chi;
  F2u = ic * ((psi * F1u - xi * F2d) +
              pi_w * ((B2 * (chi + xi) - psi * B1) + q * ((chi - psi) - xi)));
  F1d = ic * ((psi * F2d - xi * F1u) +
              pi_w * ((B1 * (chi + xi) - psi * B2) + q * ((xi + psi) - chi)));
}

// Species-summed opacity at one wavelength (opacity.py:250-269).  FAST: every term is
// exactly two T-bracket rows of the layer's own pressure slab (pressure on a node).
template <int S, bool FAST>
__device__ __forceinline__ double kappa_at(const TermP* __restrict__ t, int nS, int64_t j,
                                           double sig) {
  double tot = 0.0;
  if constexpr (FAST) {
    double v[2 * S];
#pragma unroll
    for (int s = 0; s < S; ++s) {  // issue every table load before the first use
      v[2 * s] = __builtin_nontemporal_load(t[s].row[0] + j);
      v[2 * s + 1] = __builtin_nontemporal_load(t[s].row[1] + j);
    }
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const double acc = (0.0 + v[2 * s] * t[s].w[0]) + v[2 * s + 1] * t[s].w[1];
      double ops = t[s].mmr * acc;
      if (S > 1) ops = isnan(ops) ? 0.0 : ops;  // xarray nansum for S > 1 (Q8)
      tot = (s == 0) ? ops : tot + ops;
    }
  } else {
    for (int s = 0; s < nS; ++s) {
      double acc;
      if (t[s].nrow < 0) {  // single-T table: scipy interp1d over pressure
        const double lo = t[s].row[0][j], hi = t[s].row[1][j];
        acc = ((hi - lo) / t[s].dx) * t[s].x1 + lo;
      } else {
        acc = 0.0;
        for (int r = 0; r < t[s].nrow; ++r) acc = acc + t[s].row[r][j] * t[s].w[r];
      }
      double ops = t[s].mmr * acc;
      if (nS > 1) ops = isnan(ops) ? 0.0 : ops;
      tot = (s == 0) ? ops : tot + ops;
    }
  }
  return tot + sig;  // k includes sigma (Q1)
}

// ---------------------------------------------------------------- cross-lane sums
// DPP move of a double (two 32-bit halves): row_mask / bank_mask all, bound_ctrl off.
template <int CTRL>
__device__ __forceinline__ double dpp_bcast(double x) {
  const int2 v = __builtin_bit_cast(int2, x);
  int2 r;
  r.x = __builtin_amdgcn_mov_dpp(v.x, CTRL, 0xF, 0xF, false);
  r.y = __builtin_amdgcn_mov_dpp(v.y, CTRL, 0xF, 0xF, false);
  return __builtin_bit_cast(double, r);
}

// Value of lane ^ M for M <= 8, all on the VALU (no LDS round trip): quad_perm for 1 and 2,
// row_shl / row_shr selected by the lane's bit for 4, row_ror:8 (= xor 8) for 8.
template <int M>
__device__ __forceinline__ double lane_xor(double x, int lane) {
  static_assert(M == 1 || M == 2 || M == 4 || M == 8, "in-row exchange");
  if constexpr (M == 1) return dpp_bcast<0xB1>(x);            // quad_perm [1,0,3,2]
  if constexpr (M == 2) return dpp_bcast<0x4E>(x);            // quad_perm [2,3,0,1]
  if constexpr (M == 4) {
    // both moves on the full wave, then the select: a DPP inside a divergent branch would
    // read its partner lane while that lane is masked off
    const double down = dpp_bcast<0x114>(x);   // row_shr:4 (lane - 4)
    const double up = dpp_bcast<0x104>(x);     // row_shl:4 (lane + 4)
    return (lane & 4) ? down : up;
  }
  return dpp_bcast<0x128>(x);                                 // row_ror:8
}

// x(row r) + x(row r ^ 1) and x(half h) + x(half h ^ 1) through gfx950's
// v_permlane16_swap / v_permlane32_swap: both operands hold x, the swap leaves the even
// rows (halves) in one result and the odd ones in the other, so every lane adds the same
// two values in the same order.
__device__ __forceinline__ double rows_sum16(double x) {
  const int2 v = __builtin_bit_cast(int2, x);
  const auto lo = __builtin_amdgcn_permlane16_swap(v.x, v.x, false, false);
  const auto hi = __builtin_amdgcn_permlane16_swap(v.y, v.y, false, false);
  return __builtin_bit_cast(double, make_int2((int)lo[0], (int)hi[0])) +
         __builtin_bit_cast(double, make_int2((int)lo[1], (int)hi[1]));
}
__device__ __forceinline__ double rows_sum32(double x) {
  const int2 v = __builtin_bit_cast(int2, x);
  const auto lo = __builtin_amdgcn_permlane32_swap(v.x, v.x, false, false);
  const auto hi = __builtin_amdgcn_permlane32_swap(v.y, v.y, false, false);
  return __builtin_bit_cast(double, make_int2((int)lo[0], (int)hi[0])) +
         __builtin_bit_cast(double, make_int2((int)lo[1], (int)hi[1]));
}

// Sums of q0..q3 over the 64/Q lanes with the same lane mod Q (Q = 1: the whole wave).
// The first two butterfly levels exchange one of two values each, so afterwards every lane
// carries one partial sum: lane q + Q(b + 2c) ends with the sum of q[2b + c] over the lanes
// of its residue q.  Every level is a DPP or permlane-swap VALU operation (the shfl form
// costs one LDS round trip per level, which a one- or two-wave-per-SIMD slice cannot hide).
// Fixed tree: deterministic.
template <int Q, bool FULL = true>
__device__ __forceinline__ double group_sum4(double q0, double q1, double q2, double q3,
                                             int lane) {
  const bool b = lane & Q;
  const double r0 = lane_xor<Q>(b ? q0 : q2, lane);
  const double r1 = lane_xor<Q>(b ? q1 : q3, lane);
  const double x0 = (b ? q2 : q0) + r0;
  const double x1 = (b ? q3 : q1) + r1;
  const bool c = lane & (2 * Q);
  double y = (c ? x1 : x0) + lane_xor<2 * Q>(c ? x0 : x1, lane);
  if constexpr (Q == 1) {
    y += dpp_bcast<0x124>(y);   // row_ror:4 then row_ror:8: the 4 lanes of a residue mod 4
    y += dpp_bcast<0x128>(y);
  } else if constexpr (Q == 2) {
    y += dpp_bcast<0x128>(y);   // row_ror:8 (lane ^ 8)
  }
  if constexpr (!FULL) return y;   // per-row sums: the caller adds the 4 rows later
  return rows_sum32(rows_sum16(y));
}

// One-lane form: lane 0 ends with sum(q0), lane 2 with sum(q1), lane 1 with sum(q2), lane 3
// with sum(q3).
__device__ __forceinline__ double wave_sum4(double q0, double q1, double q2, double q3,
                                            int lane) {
  return group_sum4<1>(q0, q1, q2, q3, lane);
}

// The xor-32, 16, ..., 1 butterfly (acc += shfl_xor(acc, o)) on the VALU: permlane32 / 16 swaps
// for the half and row levels, DPP for the in-row ones.  Every level pairs the same lanes and
// adds the same two values (addition commutes), so the result is bit-identical to the shfl form
// without its LDS round trip per level.  Whole wave active.
__device__ __forceinline__ double butterfly_sum(double v, int lane) {
  v = rows_sum32(v);
  v = rows_sum16(v);
  v += lane_xor<8>(v, lane);
  v += lane_xor<4>(v, lane);
  v += lane_xor<2>(v, lane);
  v += lane_xor<1>(v, lane);
  return v;
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// ---------------------------------------------------------------- K1: sweep
template <int DIR, int S, bool FAST>
__global__ __launch_bounds__(kBlock) void sweep_kernel(SweepArgs a) {
  if (!a.force && *a.conv) return;
  extern __shared__ double red[];  // [wave][step][4]
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wv = tid >> 6;
  const int64_t nl = a.n_lam;
  const int64_t j0 = (int64_t)blockIdx.x * kBlock + tid;
  const bool act = j0 < nl;
  const int64_t j = act ? j0 : nl - 1;
  const double c1 = a.c1[j], hcl = a.hcl[j], sig = a.sig[j];
  const double wt = act ? a.wtr[j] : 0.0;
  double* __restrict__ Fu = a.F_up;
  double* __restrict__ Fd = a.F_down;
  const int nS = a.n_species;
  const int ns = a.n_steps;

  double carry, Bc;
  {
    const StepP s0 = a.steps[0];
    if (DIR == kEmit) {  // fresh F_up carried upward (twostream.py:383)
      carry = Fu[(int64_t)s0.layer * nl + j];
      Bc = planck(c1, hcl, s0.iT1);
    } else {             // fresh F_down carried downward (twostream.py:511)
      carry = Fd[(int64_t)(s0.layer + 1) * nl + j];
      Bc = planck(c1, hcl, s0.iT2);
    }
  }
  for (int k = 0; k < ns; ++k) {
    const StepP sp = a.steps[k];
    const int i = sp.layer;
    const double kap = kappa_at<S, FAST>(a.terms + (int64_t)k * nS, nS, j, sig);
    const double dtau = sp.dm * kap;             // twostream.py:227-231
    const double w0 = fm::div(sig, sig + kap);   // twostream.py:376-378
    double B1, B2, F1u, F2d;
    if (DIR == kEmit) {
      B1 = Bc;
      B2 = sp.top ? Bc : planck(c1, hcl, sp.iT2);
      F1u = carry;
      F2d = sp.top ? a.ftoa[j] : Fd[(int64_t)(i + 1) * nl + j];  // stale (Q2, Q3)
    } else {
      B2 = Bc;
      B1 = planck(c1, hcl, sp.iT1);
      F2d = carry;
      F1u = Fu[(int64_t)i * nl + j];                               // stale (Q2)
    }
    double F2u, F1d;
    two_stream(w0, dtau, B1, B2, F1u, F2d, F2u, F1d);
    if (act) {
      const bool st_up = (DIR == kEmit) ? !sp.top : (!a.live_only || i == 0);
      const bool st_dn = (DIR == kAbsorb) || !a.live_only || sp.top;
      if (st_up) Fu[(int64_t)(i + 1) * nl + j] = F2u;
      if (st_dn) Fd[(int64_t)i * nl + j] = F1d;
      if (a.dtaus) a.dtaus[(int64_t)(k + 1) * nl + j] = dtau;
    }
    const double y = wave_sum4(wt * F2u, wt * F2d, wt * F1u, wt * F1d, lane);
    if (lane < 4) red[((int64_t)wv * ns + k) * 4 + (lane & 1) * 2 + ((lane >> 1) & 1)] = y;
    if (DIR == kEmit) { carry = F2u; Bc = B2; } else { carry = F1d; Bc = B1; }
  }
  __syncthreads();
  const int nw = kBlock / 64;
  for (int idx = tid; idx < ns * 4; idx += kBlock) {
    double v = red[idx];
    for (int w = 1; w < nw; ++w) v += red[(int64_t)w * ns * 4 + idx];
    a.part[part_at(idx, blockIdx.x, gridDim.x, ns * 4)] = v;
  }
}

// ---------------------------------------------------------------- K1 fast path
// Software-pipelined: the next step's 2S table rows and its stale opposite-stream flux
// are loaded into registers while the current step computes, so HBM latency overlaps the
// fp64 two-stream arithmetic instead of serialising with it.
// (Measured and not adopted, profiles/design_notes_r01_r03.md and profiles/r04/: non-temporal
// row loads, write-through flux stores.)

// Issue priority by progress: a wave in quarter q of its layer loop runs at priority 3 - q, so
// waves that started late (second-round blocks) catch up instead of trailing alone at the end
// of the launch (the hardware otherwise favours the oldest wave).  DESIGN.md §3.
__device__ __forceinline__ void progress_priority(int k0, int ns) {
  switch ((4 * k0) / ns) {
    case 0: __builtin_amdgcn_s_setprio(3); break;
    case 1: __builtin_amdgcn_s_setprio(2); break;
    case 2: __builtin_amdgcn_s_setprio(1); break;
    default: __builtin_amdgcn_s_setprio(0); break;
  }
}

// Scheduling fence of the sweep's load ring.
__device__ __forceinline__ void ring_fence() { __builtin_amdgcn_sched_barrier(0); }
__device__ __forceinline__ void store_flux(double* p, double v) { *p = v; }
// A register-level dependence of a refill's address on the value that consumed the slot (no
// instruction): sched_barrier only orders the machine scheduler, while instruction selection had
// already placed the refill loads ahead of the opacity that reads the slot, so the old and new
// values overlapped and the loop latch copied the four row registers after waiting for their
// loads (s_waitcnt vmcnt(5..2) + five v_mov_b64 per two steps).
// (On the element index, not the pointer: a pointer out of an asm is generic, and its loads
// would become flat loads that also wait on the LDS counter.)
template <class I>
__device__ __forceinline__ I after_use(I idx, double used) {
  asm volatile("" : "+v"(idx) : "v"(used));
  return idx;
}
template <class I>
__device__ __forceinline__ I after_use(I idx, double used, double used2) {
  asm volatile("" : "+v"(idx) : "v"(used), "v"(used2));
  return idx;
}
// A value read on every path (no instruction): a load left pending on a rarely taken path makes
// the loop's merge blocks wait for everything issued after it (vmcnt is in order).
__device__ __forceinline__ void consume(double v) { asm volatile("" ::"v"(v)); }

// Carry-independent part of one step (everything in twostream.py:135-176 except the
// terms that multiply the carried flux).  Split out so two layers' coefficients form one
// straight-line block the scheduler interleaves (2x instruction-level parallelism per
// wave, which is what a 1-wave-per-SIMD slice — 500k lambda over 8 GPUs — needs).
// Wave-uniform value read from LDS, moved to SGPRs (keeps it out of the VGPR budget).
__device__ __forceinline__ double uni(double x) {
  const long long b = __double_as_longlong(x);
  const int lo = __builtin_amdgcn_readfirstlane((int)(b & 0xffffffffLL));
  const int hi = __builtin_amdgcn_readfirstlane((int)(b >> 32));
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
__device__ __forceinline__ int uni(int x) { return __builtin_amdgcn_readfirstlane(x); }
__device__ __forceinline__ int64_t uni(int64_t x) {
  return (int64_t)__double_as_longlong(uni(__longlong_as_double((long long)x)));
}

// (Step parameters that only feed arithmetic — T1, T2, dm, weights, mmr — are read from the
// LDS step table straight into VGPRs, a broadcast LDS read, not readfirstlane'd into SGPRs.)

// The step's coefficients are premultiplied by 1/chi (and pi_w), so a flux update is two fma on
// the carried input, F2u = (ic psi) F1u - (ic xi) F2d + (ic pi_w) Xu, instead of
// ic ((psi F1u - xi F2d) + pi_w Xu): a different association of the same products (an ulp or
// so, tools/lean_err.py), fewer instructions on the carried chain and four ring values per step
// in the producer/consumer sweep.  Every sweep form uses the same coefficients, so they stay
// bitwise identical to each other.
struct StepCoef {
  // psi, xi, Xu, Xd hold ic*psi, ic*xi, ic*Xu, ic*Xd:
  //   F2u = psi F1u - xi F2d + Xu, F1d = psi F2d - xi F1u + Xd (step_up / step_dn)
  double psi, xi, Xu, Xd;
  double dtau, Bnext;          // Bnext: Planck value the next layer reuses
  double F_st;                 // stale opposite-stream flux
  int layer, top;
};

// The flux update of one step from its coefficients (twostream.py:161-176).
__device__ __forceinline__ double step_up(double psi, double xi, double Xu, double F1u,
                                          double F2d) {
  return __builtin_fma(psi, F1u, __builtin_fma(-xi, F2d, Xu));
}
__device__ __forceinline__ double step_dn(double psi, double xi, double Xd, double F1u,
                                          double F2d) {
  return __builtin_fma(psi, F2d, __builtin_fma(-xi, F1u, Xd));
}

// Terms after E (twostream.py:143-176), same expression order as two_stream().  pi_w =
// pi (1 - w0) / (E - w0) comes from the caller (pi itself where E = 1); 1 / chi is formed
// within an ulp (it scales the whole update, nothing cancels after it); the transmission's exp
// argument is <= 0.  NF: the step's inputs cannot be NaN (contracted-table sweeps), so exp's
// clamp is a max.  The coefficients come out premultiplied by 1/chi (and pi_w): StepCoef.
template <bool NF = false>
__device__ __forceinline__ void coef_tail(double w0, double dtau, double B1, double B2,
                                          double sq, double r, double q, double pi_w,
                                          StepCoef& c) {
  (void)w0;
  const double Tr = NF ? fm::exp_neg_nf((-2.0 * sq) * dtau) : fm::exp_neg((-2.0 * sq) * dtau);
  // 0.5 (1 +- r) as one fma: fl((1 +- r) / 2) = fl(1 +- r) / 2 (scaling by 2 is exact), so the
  // same bits as the reference's add-then-halve in one instruction instead of two
  const double zp = __builtin_fma(0.5, r, 0.5);
  const double zm = __builtin_fma(-0.5, r, 0.5);
  const double Tr2 = Tr * Tr;
  const double zm2 = zm * zm;
  const double zp2 = zp * zp;
  // chi, xi, psi and the source brackets exactly as the reference forms them: their rounding
  // errors are correlated ((chi - psi) - xi cancels to O(dtau^2) in thin layers), so rewriting
  // any of them by an algebraic identity (psi = -r Tr, an fma for chi, (xi + psi) - chi as
  // -((chi - psi) - xi)) moved thin-layer fluxes by up to 1e-8 (tools/lean_err.py)
  const double chi = zm2 * Tr2 - zp2;
  const double xi = (zp * zm) * (1.0 - Tr2);
  const double psi = (zm2 - zp2) * Tr;
  const double ic = fm::rcp_nr(chi);
  const double u = chi + xi;
  const double icw = ic * pi_w;
  c.psi = ic * psi;
  c.xi = ic * xi;
  c.Xu = icw * ((B2 * u - psi * B1) + q * ((chi - psi) - xi));
  c.Xd = icw * ((B1 * u - psi * B2) + q * ((xi + psi) - chi));
  c.dtau = dtau;
}

// The E-dependent head of a step's coefficients (twostream.py:139-176; E of Deitrick 2020
// Eqn 19 where w0 > 0.1, else 1): sq = sqrt(E (E - w0)), r = sqrt((E - w0) / E), q = B' / 2E and
// pi_w, ahead of the shared coef_tail.  Every lane first takes the E = 1 values — there E Emw,
// Emw / E and B' / 2E are exact without the multiply / divide and sqrt(E Emw) == sqrt(Emw / E)
// (bit-identical, two divisions and a square root fewer), and pi (1 - w0) / (1 - w0) is pi
// within an ulp (the reference's own rounding of it).  Only when some lane of the wave has
// w0 > 0.1 does a wave-uniform branch patch those lanes with the general E (coef_head_general).
// One tail in the loop instead of one per branch: the duplicated tail had set the sweep's
// register budget (4 VGPRs).
struct CoefHead {
  double sq, r, q, pi_w;
};
__device__ __forceinline__ CoefHead coef_head_e1(double w0, double dtau, double B1, double B2) {
  CoefHead h;
  const double Emw = 1.0 - w0;
  h.sq = fm::sqrt_pos(Emw);
  h.r = h.sq;
  h.q = fm::div(B1 - B2, dtau) * 0.5;   // = div(div(B1 - B2, dtau), 2 E) at E = 1
  h.pi_w = kPi;   // pi (1 - w0) / (1 - w0): pi within an ulp
  return h;
}
__device__ __forceinline__ void coef_head_general(double w0, double dtau, double B1, double B2,
                                                  CoefHead& h) {
  if (w0 > 0.1) {
    const double E = (1.225 - 0.1777 * w0) - 0.05582 * (w0 * w0);
    const double Emw = E - w0;
    h.q = fm::div(fm::div(B1 - B2, dtau), 2.0 * E);
    h.pi_w = fm::div(kPi * (1.0 - w0), Emw);
    h.sq = fm::sqrt_pos(E * Emw);
    h.r = fm::sqrt_pos(fm::div(Emw, E));
  }
}

struct PreCoef {
  double w0, dtau, B1, B2;
};

// Per-step partial sums in LDS (a.red_rows):
//   0  one row per wave: a full DPP/permlane wave sum per step;
//   1  one row per (wave, 16-lane row): the wave sum stops after the in-row DPP levels and
//      the block epilogue adds 4x more partials;
//   2  (one-lane sweep, two steps in flight) staged: each lane parks its 4 weighted values
//      of both steps in a per-wave LDS tile; then every lane sums 8 consecutive lanes of one
//      of the 8 (step, quantity) outputs and three DPP levels finish the 64-lane sums —
//      about a third of the VALU work of a per-step butterfly, no block barrier.
__host__ __device__ inline int red_rows_per_block(int red_rows, int nw = kBlock / 64) {
  return nw * (red_rows == 1 ? 4 : 1);
}
// mode 2 tile: [wave][2 steps][4 quantities][64 lanes + 8 pad]; the pad staggers the rows
// over the LDS banks so the strided reads of the reduction are conflict-free
constexpr int kStageRow = 72;
__host__ __device__ inline int64_t red_lds_doubles(int red_rows, int ns, int nw = kBlock / 64) {
  return (int64_t)red_rows_per_block(red_rows, nw) * ns * 4 +
         (red_rows == 2 ? (int64_t)nw * 2 * 4 * kStageRow : 0);
}

// The sweep's step records formed in its own prologue (FastArgs.rec_on: contracted table,
// shared brackets, fixed mmr) from the temperatures the previous update kernel left: T, p and
// the sorted T nodes are staged in `scratch` (LDS), then thread k forms record k into `dst`
// (LDS) with setup_sweep's expressions — the records the update kernel would have written, bit
// for bit, without that kernel's record step on the critical path.  Ends with a block barrier.
__device__ __forceinline__ void step_s_core(const SetupArgs& u, const double* T, const double* P,
                                            const double* tnodes, const SpecMeta& sm,
                                            const PMeta& pm, int dir, int k, FastStepS& f);
__device__ inline void atm_view(SetupArgs& u, int m);
__host__ __device__ inline int64_t rec_scratch_doubles(const FastArgs& a) {
  return a.rec_on ? 2 * (int64_t)a.rec.n_layers + a.rec.n_tnodes : 0;
}
// Chained launch: a temperature the leading update workgroups publish by one write-through
// (sc1) store; polled by sc1 loads (global, never flat: they bypass this CU's L1) until it is
// no longer kPoisonT — the value is its own ready flag (an 8-byte granule, MI355X_MICROARCH.md
// "Valid forms" R2).  A bounded wait: after ch_timeout it flags ch_err and returns what it read.
using gu64 = __attribute__((address_space(1))) unsigned long long;
__device__ __forceinline__ unsigned long long chain_poll(const FastArgs& a, const void* p,
                                                         unsigned long long until_not,
                                                         unsigned long long want, bool eq) {
  const gu64* g = (const gu64*)p;
  unsigned long long v = __hip_atomic_load(g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const long long t0 = wall_clock64();
  while (eq ? (v >> 2) != want : v == until_not) {
    __builtin_amdgcn_s_sleep(1);
    v = __hip_atomic_load(g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // after one timeout every later wait gives up at once (the run has already failed): a
    // block's per-layer waits then end within one timeout, not one each
    const int e = __hip_atomic_load(a.ch_err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (e || wall_clock64() - t0 > a.ch_timeout) {
      if (!e) __hip_atomic_store(a.ch_err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      break;
    }
  }
  return v;
}

// Returns 1 (every thread, after a barrier) when a chained launch's update found the run
// converged: the caller's sweep block then returns, as an unchained sweep would at entry.
__device__ __forceinline__ int stage_records(const FastArgs& a, int dir, FastStepS* dst,
                                          double* scratch) {
  SetupArgs u = a.rec;
  if (a.n_atm > 1) atm_view(u, blockIdx.y);
  const int nL = u.n_layers, ns = nL - 1, ntn = u.n_tnodes;
  const int tid = threadIdx.x, nthr = blockDim.x;
  double* sT = scratch;
  double* sP = sT + nL;
  double* sN = sP + nL;
  int skip = 0, allc = 1;   // chained: run already converged / every layer converged
  if (a.ch_epoch) {
    // ONE lane polls (the update workgroups publish within about a microsecond of each other;
    // every lane polling would put hundreds of thousands of loads in flight on the same few
    // lines and slow the update itself), then every lane reads its layers once — polling on
    // only for a value not yet there
    if (tid == 0) (void)chain_poll(a, a.ch_epoch + (nL - 1), 0, a.ch_val, true);
    __syncthreads();
    for (int q = tid; q < nL; q += nthr) {
      sT[q] = __builtin_bit_cast(double, chain_poll(a, u.T + q, kPoisonT, 0, false));
      const unsigned long long g = chain_poll(a, a.ch_epoch + q, 0, a.ch_val, true);
      skip |= (int)((g >> 1) & 1);
      allc &= (int)(g & 1);
      sP[q] = u.p[q];
    }
  } else {
    for (int q = tid; q < nL; q += nthr) {
      sT[q] = u.T[q];
      sP[q] = u.p[q];
    }
  }
  for (int q = tid; q < ntn; q += nthr) sN[q] = u.tnodes[q];
  // this thread's first record's metadata, loaded with T / p (one global round trip in all)
  const SpecMeta sm = u.spec[0];
  const PMeta pm0 = u.pmeta[step_layer(dir, tid < ns ? tid : 0, nL)];
  if (a.ch_epoch) {
    // the update's convergence decision, formed from its per-layer granules: the sweep does
    // not run once the run has converged (as an unchained sweep returns at entry)
    // (logical block reductions: __syncthreads_or / _and return 0 or 1, not bit patterns)
    skip = __syncthreads_or(skip);
    allc = __syncthreads_and(allc);
    if ((skip || (a.ch_can_conv && allc)) && !a.force) return 1;
  } else {
    __syncthreads();
  }
  for (int k = tid; k < ns; k += nthr) {
    FastStepS f;
    step_s_core(u, sT, sP, sN, sm, k == tid ? pm0 : u.pmeta[step_layer(dir, k, nL)], dir, k,
                f);
    f.mmr[0] = 1.0;   // the contracted table's unit mixing ratio (MM1: never read)
    for (int s = 1; s < kMaxFastS; ++s) f.mmr[s] = 0.0;
    dst[k] = f;
  }
  __syncthreads();
  return 0;
}

// PD steps form one coefficient block; PF (a multiple of PD) is the prefetch distance: the
// loads of step k + PF are issued while step k computes, into a register ring of PF entries
// (the step loop is unrolled by PF, so every ring index is static).  PF > PD pays on small
// slices, where about one wave per SIMD cannot hide HBM latency with PD steps of loads alone.
template <int DIR, int S, int PD, bool NANCHK, bool SH, bool MM1, int PF, bool CH>
__device__ __forceinline__ void sweep_fast_body(
    FastArgs& a, const FastStep* __restrict__ st, const FastStepS* __restrict__ ss,
    double* __restrict__ Fu, double* __restrict__ Fd, double* __restrict__ part,
    double* __restrict__ dtaus, double* red, const int bx, const int nbx) {
  static_assert(!CH || SH, "chained: the step records are formed in the block (LDS)");
  static_assert(PD == 1 || PD == 2 || PD == 4, "prefetch depth 1, 2 or 4");
  static_assert(PF % PD == 0, "prefetch distance: a multiple of the coefficient block");
  static_assert(!MM1 || S == 1, "mmr = 1 only for the contracted single table");
  // staged partial sums (red_rows 2) reduce a pair of steps: the pair is one coefficient block
  // (PD = 2), or the two one-step blocks of a trip (PD = 1, PF = 2: fewer registers per wave)
  constexpr bool kPairs = PD == 2 || (PD == 1 && PF == 2);
  // no NaN reaches the coefficients: the contracted table is built from NaN-free tables, and
  // with S > 1 the tables were scanned (NaN-free, or NANCHK's nansum zeroes NaN terms); only a
  // single per-species table keeps the reference's NaN propagation (Q8)
  constexpr bool kNaNFree = MM1 || S > 1;
  {  // atmosphere of a batched launch (identity for one atmosphere)
    const int m = blockIdx.y;
    Fu += m * a.bs.flux;
    Fd += m * a.bs.flux;
    part += m * a.bs.part;
    if (dtaus) dtaus += m * a.bs.flux;
    st += m * a.bs.steps;
    ss += m * a.bs.steps;
    a.tab[0] += m * a.bs.tab;
    a.ftoa += m * a.bs.ftoa;
    a.conv += m;
  }
  if (!CH && !a.force && *a.conv) return;
  TRACE_DECL;
  // red: [wave][step][4], then (shared brackets) the step table
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wv = tid >> 6;
  const int64_t nl = a.n_lam;
  if (a.poison && bx == 0)   // the deferred update's output temperatures: "not published"
    for (int i = tid; i <= a.n_steps; i += kBlock)
      reinterpret_cast<unsigned long long*>(a.poison)[i] = kPoisonT;
  const int64_t j0 = (int64_t)bx * kBlock + tid;
  const bool act = j0 < nl;
  const int64_t j = act ? j0 : nl - 1;
  const double c1 = a.c1[j], hcl = a.hcl[j], sig = a.sig[j];
  const double wt = act ? a.wtr[j] : 0.0;
  const int ns = a.n_steps;
  // Shared brackets: stage the whole step table (ns x 120 B) in LDS once, so every step
  // reads its uniform parameters at LDS latency instead of scalar loads that miss the
  // K$ and L2 of a freshly scheduled CU (the step table was written by the update kernel).
  const FastStepS* sp = ss;
  if constexpr (SH) {
    double* lss = red + red_lds_doubles(a.red_rows, ns);
    constexpr int kW = sizeof(FastStepS) / sizeof(double);
    if (a.rec_on) {   // form the records here from the current T (the update wrote none)
      if (stage_records(a, DIR, reinterpret_cast<FastStepS*>(lss), lss + ns * kW)) return;
    } else {
      const double* g = reinterpret_cast<const double*>(ss);
      for (int idx = tid; idx < ns * kW; idx += kBlock) lss[idx] = g[idx];
      __syncthreads();
    }
    sp = reinterpret_cast<const FastStepS*>(lss);
  }
  TRACE_MARK(1);
  // Load the 2S table rows and the stale opposite-stream flux of step k into one buffer
  // (and, with shared brackets, the step's uniform parameters).
  // a step's layer and top flag follow from its index (step_layer; emit's top step is the
  // last one), so they need no step-table read
  auto layer_of = [&](int k) { return step_layer(DIR, k, ns + 1); };
  auto top_of = [&](int k) { return DIR == kEmit && k == ns - 1; };
  // Loads of a step: the 2S table rows (with shared brackets the row offset comes from the
  // step table) and the stale opposite-stream flux.  Unconditional, at clamped indices, so the
  // vmcnt bookkeeping stays static.
  auto load_rows = [&](int k, double (&v)[2 * S], double dep = 0.0) {
    k = k < ns ? k : ns - 1;
    if constexpr (SH) {
      const int64_t off = uni(sp[k].off);
#pragma unroll
      for (int s = 0; s < S; ++s) {
        const double* r = a.tab[s] + after_use(off + j, dep);
        v[2 * s] = *(r);
        v[2 * s + 1] = *(r + a.pitch);
      }
      return;
    }
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const double* r = a.tab[s] + after_use(st[k].off[s] + j, dep);
      v[2 * s] = *(r);
      v[2 * s + 1] = *(r + a.pitch);
    }
  };
  auto load_stale = [&](int k, double& stale) {
    k = k < ns ? k : ns - 1;
    const int i = layer_of(k);
    const double* src = (DIR == kEmit) ? (top_of(k) ? a.ftoa : Fd + (int64_t)(i + 1) * nl)
                                       : Fu + (int64_t)i * nl;
    stale = src[j];
  };
  // Species-summed opacity of step k from its row slot (opacity.py:250-269).
  auto opacity = [&](int k, const double (&v)[2 * S]) {
    const int kk = k < ns ? k : ns - 1;  // the last pair of a PD = 2 loop may be a dummy
    double tot = 0.0;
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const double vlo = v[2 * s], vhi = v[2 * s + 1];
      double ops;
      if constexpr (SH) {
        // (0 + a) + b == a + b for the non-negative table terms; the contracted table (MM1)
        // carries mmr = 1, whose product is the identity
        const double acc = vlo * (sp[kk].wlo) + vhi * (sp[kk].whi);
        ops = MM1 ? acc : (sp[kk].mmr[s]) * acc;
      } else {
        const double acc = vlo * st[kk].wlo[s] + vhi * st[kk].whi[s];
        ops = MM1 ? acc : st[kk].mmr[s] * acc;
      }
      // xarray nansum for S > 1 (Q8); compiled out when the tables hold no NaN (scan at load)
      if (NANCHK && S > 1) ops = isnan(ops) ? 0.0 : ops;
      tot = (s == 0) ? ops : tot + ops;
    }
    return tot;
  };
  // Phase A of step k from its opacity: dtau, single-scattering albedo and the Planck terms,
  // everything before E.
  // Bprev: emit -> B(T1) of this step, absorb -> B(T2) of this step (reuse, Q: B2 = next B1).
  // The step's new Planck value (emit: B(T2), absorb: B(T1)); formed ahead of the opacity so the
  // loop consumes (and refills) its row slots after both steps' Planck chains.
  auto planck_new = [&](int k) {
    const int kk = k < ns ? k : ns - 1;
    if constexpr (SH) return planck(c1, hcl, DIR == kEmit ? (sp[kk].iT2) : (sp[kk].iT1));
    else return planck(c1, hcl, DIR == kEmit ? st[kk].iT2 : st[kk].iT1);
  };
  auto coef = [&](int k, double tot, double Bprev, double X, StepCoef& c, PreCoef& pc) {
    const int kk = k < ns ? k : ns - 1;
    double dm;
    c.layer = layer_of(kk);
    c.top = top_of(kk);
    if constexpr (SH) dm = (sp[kk].dm);
    else dm = st[kk].dm;
    const double kap = tot + sig;
    const double dtau = dm * kap;
    const double w0 = fm::div(sig, sig + kap);
    double B1, B2;
    if (DIR == kEmit) {
      B1 = Bprev;
      B2 = c.top ? Bprev : X;
      c.Bnext = B2;
    } else {
      B2 = Bprev;
      B1 = X;
      c.Bnext = B1;
    }
    pc.w0 = w0;
    pc.dtau = dtau;
    pc.B1 = B1;
    pc.B2 = B2;
  };
  // Phase B for a group of steps: the E = 1 form when every lane of every step has
  // w0 <= 0.1 (a wave-uniform branch, so the group stays one straight-line block), else the
  // general form (bit-identical on the E = 1 lanes).
  auto coefB = [&](PreCoef (&pc)[PD], StepCoef (&c)[PD]) {
    bool e1 = true;
    CoefHead h[PD];
#pragma unroll
    for (int b = 0; b < PD; ++b) {
      e1 = e1 && !(pc[b].w0 > 0.1);
      h[b] = coef_head_e1(pc[b].w0, pc[b].dtau, pc[b].B1, pc[b].B2);
    }
    if (!__all(e1)) {   // rare: one step at a time (registers, not ILP)
#pragma unroll
      for (int b = 0; b < PD; ++b) {
        ring_fence();
        coef_head_general(pc[b].w0, pc[b].dtau, pc[b].B1, pc[b].B2, h[b]);
      }
      ring_fence();
    }
#pragma unroll
    for (int b = 0; b < PD; ++b)
      coef_tail<kNaNFree>(pc[b].w0, pc[b].dtau, pc[b].B1, pc[b].B2, h[b].sq, h[b].r, h[b].q,
                          h[b].pi_w, c[b]);
  };

  // Carry-dependent finish of step k: fluxes, stores, bolometric partials.
  double carry;
  auto finish = [&](int k, const StepCoef& c, double F_st) {
    // read the stale flux on every path, the dummy step past the end included: left pending
    // there, its load made the loop's merge block wait for the next rows before the refill
    consume(F_st);
    double F1u, F2d;
    if (DIR == kEmit) { F1u = carry; F2d = F_st; } else { F2d = carry; F1u = F_st; }
    const double F2u = step_up(c.psi, c.xi, c.Xu, F1u, F2d);
    const double F1d = step_dn(c.psi, c.xi, c.Xd, F1u, F2d);
    if (k >= ns) return;
    const int i = c.layer;
    if (act) {
      // live_only: inside the T-P loop skip the dead stores (emit's interior F_down rows
      // are rewritten by absorb before any read, absorb's F_up rows >= 2 by the next emit).
      const bool st_up = (DIR == kEmit) ? !c.top : (!a.live_only || i == 0);
      const bool st_dn = (DIR == kAbsorb) || !a.live_only || c.top;
      if (st_up) store_flux(Fu + (int64_t)(i + 1) * nl + j, F2u);
      if (st_dn) store_flux(Fd + (int64_t)i * nl + j, F1d);
      if (dtaus) dtaus[(int64_t)(k + 1) * nl + j] = c.dtau;
    }
    if (kPairs && a.red_rows == 2) {   // staged: reduced per pair of steps (stage_reduce)
      double* t = red + (int64_t)(kBlock / 64) * ns * 4 + ((wv * 2 + (k & 1)) * 4) * kStageRow +
                  lane;
      t[0] = wt * F2u;
      t[kStageRow] = wt * F2d;
      t[2 * kStageRow] = wt * F1u;
      t[3 * kStageRow] = wt * F1d;
      carry = (DIR == kEmit) ? F2u : F1d;
      return;
    }
    // row sums (DPP only); lanes 0..3 of each 16-lane row write them, the block epilogue
    // adds the 16 (wave, row) partials
    const int qi = (lane & 1) * 2 + ((lane >> 1) & 1);
    if (a.red_rows) {
      const double y = group_sum4<1, false>(wt * F2u, wt * F2d, wt * F1u, wt * F1d, lane);
      if ((lane & 15) < 4) red[((int64_t)(wv * 4 + (lane >> 4)) * ns + k) * 4 + qi] = y;
    } else {
      const double y = group_sum4<1>(wt * F2u, wt * F2d, wt * F1u, wt * F1d, lane);
      if (lane < 4) red[((int64_t)wv * ns + k) * 4 + qi] = y;
    }
    carry = (DIR == kEmit) ? F2u : F1d;
  };

  double Bc;
  {
    const int l0 = SH ? sp[0].layer : st[0].layer;
    const double iT10 = SH ? sp[0].iT1 : st[0].iT1, iT20 = SH ? sp[0].iT2 : st[0].iT2;
    if (DIR == kEmit) {
      carry = Fu[(int64_t)l0 * nl + j];
      Bc = planck(c1, hcl, iT10);
    } else {
      carry = Fd[(int64_t)(l0 + 1) * nl + j];
      Bc = planck(c1, hcl, iT20);
    }
  }
  // PD steps in flight: their loads are issued PD steps ahead, their coefficients form one
  // block (PD-way instruction-level parallelism), then the short carried recurrence.
  // Ring of PF steps' loads: slot (k mod PF) is refilled with step k + PF as soon as step k
  // has consumed it — the rows after the opacity sums, the stale flux after the flux update —
  // and a scheduling fence keeps every refill behind the last read of the slot's old value, so
  // the old and new values never live at once: each slot stays one register pair across the
  // loop's back edge, with no copy there (a copy of a register whose load is in flight would
  // make the compiler drain every outstanding load at the latch, vmcnt(0)).
  double vb[PF][2 * S], sb[PF];
  // rows first, then the stale fluxes: the order the loop refills them in, so the first trip's
  // waits on its rows are the loop's own (vmcnt is in order: a stale load issued between two
  // row loads would have to land before the opacity could read the later row)
#pragma unroll
  for (int b = 0; b < PF; ++b) load_rows(b, vb[b]);
  ring_fence();
#pragma unroll
  for (int b = 0; b < PF; ++b) load_stale(b, sb[b]);
  ring_fence();
  for (int k0 = 0; k0 < ns; k0 += PF) {
    progress_priority(k0, ns);
#pragma unroll
  for (int g = 0; g < PF / PD; ++g) {
    const int k = k0 + g * PD;
    // wave-uniform: no dummy coefficient blocks at the end (a pair's dummy second step runs,
    // unstored, so the pair's reduction below sees both steps)
    if (PF > PD && !(PD == 1 && kPairs) && k >= ns) break;
    if constexpr (PD == 1 && kPairs) ring_fence();   // one step at a time: registers, not ILP
    StepCoef c[PD];
    PreCoef pc[PD];
    double tot[PD], X[PD];
#pragma unroll
    for (int b = 0; b < PD; ++b) X[b] = planck_new(k + b);
#pragma unroll
    for (int b = 0; b < PD; ++b) tot[b] = opacity(k + b, vb[g * PD + b]);
    ring_fence();
#pragma unroll
    for (int b = 0; b < PD; ++b) load_rows(k + b + PF, vb[g * PD + b], tot[b]);
    double Bp = Bc;
#pragma unroll
    for (int b = 0; b < PD; ++b) {
      coef(k + b, tot[b], Bp, X[b], c[b], pc[b]);
      Bp = c[b].Bnext;
    }
    Bc = Bp;
    coefB(pc, c);
#pragma unroll
    for (int b = 0; b < PD; ++b) finish(k + b, c[b], sb[g * PD + b]);
    ring_fence();
#pragma unroll
    for (int b = 0; b < PD; ++b) load_stale(k + b + PF, sb[g * PD + b]);
    if constexpr (kPairs) {
      // the pair's 8 (step, quantity) sums over the wave's 64 lanes, once both are staged
      if (a.red_rows == 2 && (PD == 2 || (g & 1))) {
        const int kp = PD == 2 ? k : k - 1;   // the pair's first step
        __builtin_amdgcn_wave_barrier();
        const int o = lane >> 3;
        // lane r = lane & 7 of output o sums lanes r, r + 8, ..., r + 56 of that output's row
        const double* t = red + (int64_t)(kBlock / 64) * ns * 4 +
                          ((wv * 2 + (o >> 2)) * 4 + (o & 3)) * kStageRow + (lane & 7);
        double y = t[0];
#pragma unroll
        for (int i = 1; i < 8; ++i) y += t[8 * i];
        y += dpp_bcast<0xB1>(y);    // quad_perm [1,0,3,2]
        y += dpp_bcast<0x4E>(y);    // quad_perm [2,3,0,1]
        y += dpp_bcast<0x141>(y);   // row_half_mirror: the other quad of the 8-lane group
        const int ks = kp + (o >> 2);
        if ((lane & 7) == 0 && ks < ns) red[((int64_t)wv * ns + ks) * 4 + (o & 3)] = y;
        __builtin_amdgcn_wave_barrier();
      }
    }
  }
  }
  TRACE_MARK(2);
  __syncthreads();
  for (int idx = tid; idx < ns * 4; idx += kBlock) {
    double s = red[idx];
    for (int w = 1; w < red_rows_per_block(a.red_rows); ++w)
      s += red[(int64_t)w * ns * 4 + idx];
    part[part_at(idx, bx, nbx, ns * 4)] = s;
  }
  TRACE_PUT(CH ? 41 : 1);
}

template <int DIR, int S, int PD, bool NANCHK, bool SH, bool MM1, int PF>
__global__ __launch_bounds__(kBlock, 1) void sweep_fast_kernel(
    FastArgs a, const FastStep* __restrict__ st, const FastStepS* __restrict__ ss,
    double* __restrict__ Fu, double* __restrict__ Fd, double* __restrict__ part,
    double* __restrict__ dtaus) {
  extern __shared__ double red[];
  sweep_fast_body<DIR, S, PD, NANCHK, SH, MM1, PF, false>(a, st, ss, Fu, Fd, part, dtaus, red,
                                                         blockIdx.x, gridDim.x);
}

// ---------------------------------------------------------------- K1, grouped-lane form
// Small slices (e.g. 62.5k lambda per GPU over 8 GPUs) leave about one wave per SIMD, and a
// lone wave issues a vector instruction only every other slot.  This form spends Q = 2 or 4
// lanes per wavelength so the same slice runs Q times the waves: the Q lanes (q = lane mod Q)
// of a wavelength own its steps Qg + q, so within each group of Q sweep steps every lane
// computes one step's coefficients (one instruction stream for all Q).  Each lane forms its
// step's new Planck value and the group resolves (B1, B2) of all Q steps in order; the
// carried recurrence runs through the group's lanes in step order (carry broadcast by DPP
// quad_perm); each lane stores its own step; the bolometric terms of the Q steps reduce
// together over the 64/Q lanes of each q.  Fluxes are formed by the same expressions in the
// same order as the one-lane form (bit-identical); the bolometric partial sums use this
// form's own fixed summation tree.  One contracted table (K3), step table staged in LDS.
// quad_perm control reading sub-lane R of a lane's Q-group (Q = 2: two groups per quad)
template <int Q, int R>
constexpr int qp_from() {
  return Q == 4 ? R * 0x55 : (R | (R << 2) | ((R + 2) << 4) | ((R + 2) << 6));
}
template <int Q, int R>
__device__ __forceinline__ double from_lane(double x) {
  return dpp_bcast<qp_from<Q, R>()>(x);
}


// Block bx of nbx sweep blocks (a chained launch's sweep blocks follow its update workgroups);
// red: the dynamic LDS.  CH: chained — the temperatures and the convergence decision come from
// the leading update workgroups (stage_records polls them).
template <int DIR, int Q, int NW, bool CH>
__device__ __forceinline__ void sweep_group_body(
    FastArgs& a, const FastStepS* __restrict__ ss, double* __restrict__ Fu,
    double* __restrict__ Fd, double* __restrict__ part, double* __restrict__ dtaus,
    double* red, const int bx, const int nbx) {
  static_assert(Q == 2 || Q == 4, "2 or 4 lanes per wavelength");
  static_assert(NW == 4 || NW == 8, "4 or 8 waves per block");
  constexpr int kB = 64 * NW;   // threads per block
  {  // atmosphere of a batched launch (identity for one atmosphere)
    const int m = blockIdx.y;
    Fu += m * a.bs.flux;
    Fd += m * a.bs.flux;
    part += m * a.bs.part;
    if (dtaus) dtaus += m * a.bs.flux;
    ss += m * a.bs.steps;
    a.tab[0] += m * a.bs.tab;
    a.ftoa += m * a.bs.ftoa;
    a.conv += m;
  }
  if (!CH && !a.force && *a.conv) return;
  TRACE_DECL;
  // red: [wave][step][4], then the step table
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wv = tid >> 6;
  const int q = lane & (Q - 1);    // step residue this lane computes
  const int64_t nl = a.n_lam;
  // the deferred update's output temperatures start as "not published" (its own launch reads
  // them only after this one has ended)
  if (a.poison && bx == 0)
    for (int i = tid; i <= a.n_steps; i += kB)
      reinterpret_cast<unsigned long long*>(a.poison)[i] = kPoisonT;
  const int64_t j0 = (int64_t)bx * (kB / Q) + wv * (64 / Q) + lane / Q;
  const bool act = j0 < nl;
  const int64_t j = act ? j0 : nl - 1;
  const double c1 = a.c1[j], hcl = a.hcl[j], sig = a.sig[j];
  const double wt = act ? a.wtr[j] : 0.0;
  const int ns = a.n_steps;
  const double* __restrict__ tab = a.tab[0];
  double* lss = red + red_lds_doubles(a.red_rows, ns, NW);
  {
    constexpr int kW = sizeof(FastStepS) / sizeof(double);
    if (a.rec_on) {   // form the records here from the current T (the update wrote none)
      if (stage_records(a, DIR, reinterpret_cast<FastStepS*>(lss), lss + ns * kW)) return;
    } else {
      const double* g = reinterpret_cast<const double*>(ss);
      for (int idx = tid; idx < ns * kW; idx += kB) lss[idx] = g[idx];
      __syncthreads();
    }
  }
  const FastStepS* sp = reinterpret_cast<const FastStepS*>(lss);
  TRACE_MARK(1);
  auto clampk = [&](int k) { return k < ns ? k : ns - 1; };
  const int nL = ns + 1;
  // A step's layer and top flag follow from its index (step_layer; emit's top step is the
  // last), so only the bracket offset, weights, T and dm come from the LDS step table.
  auto is_top = [&](int k) { return DIR == kEmit && k >= ns - 1; };
  // Everything group g's phase A reads, issued together one group ahead: the LDS step
  // parameters with the table rows and the stale flux (their latency overlaps).
  struct Pre {
    double vlo, vhi, stale, wl, wh, dm, iT;
  };
  // per-lane running addresses, advanced by Q steps per load: this lane's stale row (emit:
  // F_down row k + 2; absorb: F_up row nL - 2 - k) and its table column
  const double* tabj = tab + j;
  const double* ftoaj = a.ftoa + j;
  const int64_t sstep = (DIR == kEmit ? (int64_t)Q : -(int64_t)Q) * nl;
  const double* pst = (DIR == kEmit) ? Fd + (int64_t)(q + 2) * nl + j
                                     : Fu + (int64_t)(nL - 2 - q) * nl + j;
  // Two loads per group buffer, each issued once the buffer's previous value is consumed (the
  // one-lane sweep's load ring, ring_fence): the table rows and step parameters right after
  // the opacity, the stale flux after the group's flux update — so no buffer value is live
  // across its refill and the loop's back edge needs no register copies (a copy of an
  // in-flight load drains every outstanding load there).
  int kr = q, kst = q;               // this lane's step of the next row / stale load
  // d1, d2: values formed from the buffer's previous contents (after_use: the refill is issued
  // after them, so old and new contents never live at once)
  auto load_rows = [&](Pre& P, double d1 = 0.0, double d2 = 0.0) {
    const FastStepS& st = sp[after_use(clampk(kr), d1, d2)];
    const double* r = tabj + st.off;
    P.wl = st.wlo;
    P.wh = st.whi;
    P.dm = st.dm;
    P.iT = DIR == kEmit ? st.iT2 : st.iT1;
    P.vlo = *(r);
    P.vhi = *(r + a.pitch);
    kr += Q;
  };
  auto load_stale = [&](Pre& P) {
    // emit's top step reads F_TOA; past the last step (dummy groups) any valid row serves
    const double* src = (DIR == kEmit) ? (kst >= ns - 1 ? ftoaj : pst)
                                       : (kst >= ns ? Fu + j : pst);
    P.stale = *src;
    pst += sstep;
    kst += Q;
  };
  double carry, carryB;
  {
    const int l0 = sp[0].layer;
    if (DIR == kEmit) {
      carry = Fu[(int64_t)l0 * nl + j];
      carryB = planck(c1, hcl, sp[0].iT1);
    } else {
      carry = Fd[(int64_t)(l0 + 1) * nl + j];
      carryB = planck(c1, hcl, sp[0].iT2);
    }
  }
  struct GroupA {
    double w0, dtau, B1, B2;
    int k;
  };
  // Phase A of this lane's step in group g (opacity, dtau, albedo, Planck chain of the
  // group); refills the group's row buffer with group g + 2.
  auto phaseA = [&](int g, Pre& P, GroupA& A) {
    const int k = Q * g + q;
    A.k = k;
    // each lane forms its step's new Planck value; the group gathers them and resolves
    // (B1, B2) of its steps in order (emit: B2 is new and becomes the next B1; absorb: B1 is
    // new and becomes the next B2; emit's top step keeps B2 = B1)
    const double X = planck(c1, hcl, P.iT);
    // contracted table: mmr = 1, and (0 + a) + b == a + b for its non-negative terms
    const double kap = (P.vlo * P.wl + P.vhi * P.wh) + sig;
    A.dtau = P.dm * kap;
    ring_fence();
    load_rows(P, A.dtau, X);
    A.w0 = fm::div(sig, sig + kap);
    // the step before this lane's holds the lane before it in the group (quad_perm
    // [0,0,2,2] for Q = 2, [0,0,1,2] for Q = 4), the group's first step the carried value;
    // emit's top step keeps B2 = B1 (it is the last step, so no later step reads it)
    const double Xp = dpp_bcast<Q == 2 ? 0xA0 : 0x90>(X);
    const double before = (q == 0) ? carryB : Xp;
    const double mine = (DIR == kEmit && is_top(k)) ? before : X;
    if (DIR == kEmit) {
      A.B1 = before;
      A.B2 = mine;
    } else {
      A.B2 = before;
      A.B1 = mine;
    }
    carryB = from_lane<Q, Q - 1>(mine);
  };
  // This lane's flux / dtau row pointers for its step of the current group: Q rows on per
  // group (up for emit, down for absorb), so the stores need no per-step row arithmetic.
  const int64_t rstep = (DIR == kEmit ? (int64_t)Q : -(int64_t)Q) * nl;
  double* pu = Fu + (int64_t)(step_layer(DIR, q, nL) + 1) * nl + j;
  double* pd = Fd + (int64_t)step_layer(DIR, q, nL) * nl + j;
  double* pt = (dtaus ? dtaus : Fu) + (int64_t)(q + 1) * nl + j;
  // Carried recurrence through the group (steps in order), stores of this lane's step and
  // the reduction of the group's bolometric terms.
  auto finish = [&](const GroupA& A, const StepCoef& c, const double F_st) {
    // the two fluxes of a step from its carried input (same expressions as the one-lane form)
    auto flux_up = [&](double in) {   // F_2_up
      const double F1u = (DIR == kEmit) ? in : F_st, F2d = (DIR == kEmit) ? F_st : in;
      return step_up(c.psi, c.xi, c.Xu, F1u, F2d);
    };
    auto flux_dn = [&](double in) {   // F_1_down
      const double F1u = (DIR == kEmit) ? in : F_st, F2d = (DIR == kEmit) ? F_st : in;
      return step_dn(c.psi, c.xi, c.Xd, F1u, F2d);
    };
    // the carried chain runs through the group's steps in order, each step in its own lane
    // (q == r); only the carried flux is formed in the chain, the other one once afterwards
    double cin = carry, own = 0.0, in_r = carry;
#pragma unroll
    for (int r = 0; r < Q; ++r) {
      const double out = (DIR == kEmit) ? flux_up(in_r) : flux_dn(in_r);  // lane q == r
      if (r == 0) {
        own = out;
      } else if (q == r) {
        cin = in_r;
        own = out;
      }
      if (r == 0) in_r = from_lane<Q, 0>(out);
      else if (r == 1) in_r = from_lane<Q, 1>(out);
      else if (r == 2) in_r = from_lane<Q, (Q == 4 ? 2 : 0)>(out);
      else in_r = from_lane<Q, (Q == 4 ? 3 : 0)>(out);
    }
    carry = in_r;
    const double F2u = (DIR == kEmit) ? own : flux_up(cin);
    const double F1d = (DIR == kEmit) ? flux_dn(cin) : own;
    const double F1u = (DIR == kEmit) ? cin : F_st;
    const double F2d = (DIR == kEmit) ? F_st : cin;
    const int k = A.k;
    if (act && k < ns) {
      // emit's top step and absorb's bottom step are both the last step (k = ns - 1)
      const bool last = k == ns - 1;
      const bool st_up = (DIR == kEmit) ? !last : (!a.live_only || last);
      const bool st_dn = (DIR == kAbsorb) || !a.live_only || last;
      if (st_up) store_flux(pu, F2u);
      if (st_dn) store_flux(pd, F1d);
      if (dtaus) *pt = c.dtau;
    }
    pu += rstep;
    pd += rstep;
    pt += (int64_t)Q * nl;
    if (a.red_rows == 2) {   // staged: reduced per pair of groups (below, main loop)
      double* t = red + (int64_t)NW * ns * 4 +
                  ((wv * 2 + ((k / Q) & 1)) * 4) * kStageRow + lane;
      t[0] = wt * F2u;
      t[kStageRow] = wt * F2d;
      t[2 * kStageRow] = wt * F1u;
      t[3 * kStageRow] = wt * F1d;
      return;
    }
    const int kq = (k - q) + (lane & (Q - 1));
    if (a.red_rows) {   // per-row sums; the block epilogue adds the 16 (wave, row) partials
      const double y = group_sum4<Q, false>(wt * F2u, wt * F2d, wt * F1u, wt * F1d, lane);
      const int r = lane & 15;
      if (r < 4 * Q && kq < ns)
        red[((int64_t)(wv * 4 + (lane >> 4)) * ns + kq) * 4 + ((r / Q) & 1) * 2 +
            ((r / (2 * Q)) & 1)] = y;
    } else {
      const double y = group_sum4<Q>(wt * F2u, wt * F2d, wt * F1u, wt * F1d, lane);
      if (lane < 4 * Q && kq < ns)
        red[((int64_t)wv * ns + kq) * 4 + ((lane / Q) & 1) * 2 + ((lane / (2 * Q)) & 1)] = y;
    }
  };
  const int ng = (ns + Q - 1) / Q;
  Pre pa, pb;                      // two groups in flight (4: measured no faster)
  load_rows(pa);   // rows, then stale fluxes: the loop's own refill order (vmcnt is in order)
  load_rows(pb);
  ring_fence();
  load_stale(pa);
  load_stale(pb);
  ring_fence();
  for (int g = 0; g < ng; g += 2) {
    // 8 waves: two per SIMD from ONE block, held level by a barrier every two group pairs —
    // left alone, the older wave takes the issue slots first and the younger one finishes
    // its last groups alone at single-wave speed (two 4-wave blocks per CU: the second-placed
    // blocks ended ~10 us after the first at 62.5k, profiles/r03/trace_blocks_62500.txt)
    if constexpr (NW == 8) {
      if ((g & 3) == 0) __syncthreads();
    }
    GroupA A0, A1;
    phaseA(g, pa, A0);
    phaseA(g + 1, pb, A1);   // a dummy group past the end is computed, not stored
    StepCoef c0, c1;
    CoefHead h0 = coef_head_e1(A0.w0, A0.dtau, A0.B1, A0.B2);
    CoefHead h1 = coef_head_e1(A1.w0, A1.dtau, A1.B1, A1.B2);
    if (!__all(!(A0.w0 > 0.1) && !(A1.w0 > 0.1))) {
      coef_head_general(A0.w0, A0.dtau, A0.B1, A0.B2, h0);
      coef_head_general(A1.w0, A1.dtau, A1.B1, A1.B2, h1);
    }
    // contracted table: NaN-free
    coef_tail<true>(A0.w0, A0.dtau, A0.B1, A0.B2, h0.sq, h0.r, h0.q, h0.pi_w, c0);
    coef_tail<true>(A1.w0, A1.dtau, A1.B1, A1.B2, h1.sq, h1.r, h1.q, h1.pi_w, c1);
    finish(A0, c0, pa.stale);
    consume(pb.stale);
    if (g + 1 < ng) finish(A1, c1, pb.stale);
    ring_fence();
    load_stale(pa);
    load_stale(pb);
    if (a.red_rows == 2) {
      // the 8Q (group, quantity, step residue) sums of the two groups over the wave's 64/Q
      // wavelengths: 8/Q lanes per output, each adds 8 staged values (residue qq, lanes
      // qq + Q r + 8 i), then DPP finishes over the 8/Q lanes
      __builtin_amdgcn_wave_barrier();
      constexpr int L = 8 / Q;                       // lanes per output
      const int o = lane / L, r = lane % L;
      const int p = o / (4 * Q), qi = (o / Q) & 3, qq = o % Q;
      const double* t = red + (int64_t)NW * ns * 4 +
                        ((wv * 2 + p) * 4 + qi) * kStageRow + qq + Q * r;
      double y = t[0];
#pragma unroll
      for (int i = 1; i < 8; ++i) y += t[8 * i];
      y += dpp_bcast<0xB1>(y);                       // quad_perm [1,0,3,2]
      if constexpr (L == 4) y += dpp_bcast<0x4E>(y);  // quad_perm [2,3,0,1]
      const int ks = Q * (g + p) + qq;
      if (r == 0 && ks < ns && (p == 0 || g + 1 < ng))
        red[((int64_t)wv * ns + ks) * 4 + qi] = y;
      __builtin_amdgcn_wave_barrier();
    }
  }
  TRACE_MARK(2);
  __syncthreads();
  for (int idx = tid; idx < ns * 4; idx += kB) {
    double s = red[idx];
    for (int w = 1; w < red_rows_per_block(a.red_rows, NW); ++w)
      s += red[(int64_t)w * ns * 4 + idx];
    part[part_at(idx, bx, nbx, ns * 4)] = s;
  }
  TRACE_PUT(CH ? 40 + Q : 10 + Q);
}

template <int DIR, int Q, int NW>
__global__ __launch_bounds__(64 * NW) void sweep_group_kernel(
    FastArgs a, const FastStepS* __restrict__ ss, double* __restrict__ Fu,
    double* __restrict__ Fd, double* __restrict__ part, double* __restrict__ dtaus) {
  extern __shared__ double red[];
  sweep_group_body<DIR, Q, NW, false>(a, ss, Fu, Fd, part, dtaus, red, blockIdx.x, gridDim.x);
}


// ---------------------------------------------------------------- K1, two wavelengths per lane
// The contracted one-table sweep (K3) with each lane carrying two adjacent wavelengths: half the
// waves of the one-lane form, so a 500k-lambda launch (3908 waves) is ONE round of the 4096
// wave slots at four waves per SIMD instead of 1.5 rounds of the one-lane form's five: no
// second-round blocks that start late and finish alone (measured: the one-lane sweep takes
// 0.40 ns per lambda at whole rounds, 0.41-0.43 ns at 1.25-1.5 rounds, profiles/r04/c8/rounds.txt).
// Every wavelength's flux recurrence is the one-lane form's, expression for expression (fluxes
// bit-identical); the two wavelengths' weighted bolometric terms are added in the lane first
// (fma(wt_b, F_b, wt_a F_a)) and then go through the one-lane form's staged reduction, so the
// partial sums follow this form's own fixed tree and each block writes half as many partials.
// 16-byte loads and stores (the pair is adjacent in every row; the host requires an even n_lam
// and the tables' pitch is even).  Loads two steps ahead (the one-lane ring), one step per
// coefficient block per wavelength (the two wavelengths are the block's two chains).
template <int DIR>
__global__ __launch_bounds__(kBlock, 1) void sweep_pair_kernel(
    FastArgs a, const FastStep* __restrict__ st, double* __restrict__ Fu,
    double* __restrict__ Fd, double* __restrict__ part, double* __restrict__ dtaus) {
  extern __shared__ double red[];
  using d2 = double2;
  {  // atmosphere of a batched launch (identity for one atmosphere)
    const int m = blockIdx.y;
    Fu += m * a.bs.flux;
    Fd += m * a.bs.flux;
    part += m * a.bs.part;
    if (dtaus) dtaus += m * a.bs.flux;
    st += m * a.bs.steps;
    a.tab[0] += m * a.bs.tab;
    a.ftoa += m * a.bs.ftoa;
    a.conv += m;
  }
  // the convergence flag: loaded now, tested once the first steps' loads are in flight (below)
  const bool conv0 = *a.conv && !a.force;   // (unconditional load: issued at once)
  TRACE_DECL;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wv = tid >> 6;
  const int bx = blockIdx.x, nbx = gridDim.x;
  const int64_t nl = a.n_lam;
  const int ns = a.n_steps;
  const int64_t j0 = 2 * ((int64_t)bx * kBlock + tid);   // the lane's first wavelength
  const bool act = j0 < nl;
  const int64_t j = act ? j0 : nl - 2;
  auto ld2 = [](const double* p) { return *reinterpret_cast<const d2*>(p); };
  auto st2 = [](double* p, d2 v) { *reinterpret_cast<d2*>(p) = v; };
  const d2 c1 = ld2(a.c1 + j), hcl = ld2(a.hcl + j), sig = ld2(a.sig + j);
  const d2 wt = act ? ld2(a.wtr + j) : d2{0.0, 0.0};
  TRACE_MARK(1);
  auto layer_of = [&](int k) { return step_layer(DIR, k, ns + 1); };
  auto top_of = [&](int k) { return DIR == kEmit && k == ns - 1; };
  auto clampk = [&](int k) { return k < ns ? k : ns - 1; };
  // lazy K3: the rows a record masks (off[1], wave-uniform) are contracted for this lane's two
  // wavelengths before the step loop — contract_kernel's sum, species in order — and read back
  // by the same lane (no other lane or block reads them in this launch).  In the prologue, not
  // at each refill: the check inside the loop cost 1.5-2 % per T-P iteration with the whole
  // table contracted (code in the hot loop), profiles/r06/lazy_k3/.
  auto contract_rows = [&](const FastStep& sk) {
    const int64_t mask = sk.off[1];
    const int l = sk.layer;
    for (int b = 0; b < 2; ++b) {
      if (!(mask & (1 << b))) continue;
      const int64_t o = sk.off[0] + b * a.pitch + j;
      d2 acc = ld2(a.ktab[0] + o);
      acc = d2{a.kmmr[l] * acc.x, a.kmmr[l] * acc.y};
#pragma unroll
      for (int s = 1; s < kMaxFastS; ++s) {   // (static indices: the arguments stay in SGPRs)
        if (s < a.kS) {
          const d2 v = ld2(a.ktab[s] + o);
          const double m = a.kmmr[(int64_t)s * a.kNL + l];
          acc = d2{acc.x + m * v.x, acc.y + m * v.y};
        }
      }
      st2(const_cast<double*>(a.tab[0]) + o, acc);
    }
  };
  auto load_rows = [&](int k, d2 (&v)[2], double dep1 = 0.0, double dep2 = 0.0) {
    const double* r = a.tab[0] + after_use(st[clampk(k)].off[0] + j, dep1, dep2);
    v[0] = ld2(r);
    v[1] = ld2(r + a.pitch);
  };
  auto load_stale = [&](int k, d2& stale) {
    k = clampk(k);
    const int i = layer_of(k);
    const double* src = (DIR == kEmit) ? (top_of(k) ? a.ftoa : Fd + (int64_t)(i + 1) * nl)
                                       : Fu + (int64_t)i * nl;
    stale = ld2(src + j);
  };
  if (a.kmmr)   // (only while the lazy table is incomplete)
    for (int k = 0; k < ns; ++k)
      if (st[k].off[1]) contract_rows(st[k]);
  d2 carry, Bc;
  {
    const int l0 = st[0].layer;
    const double iT = DIR == kEmit ? st[0].iT1 : st[0].iT2;
    carry = ld2((DIR == kEmit ? Fu + (int64_t)l0 * nl : Fd + (int64_t)(l0 + 1) * nl) + j);
    Bc = d2{planck(c1.x, hcl.x, iT), planck(c1.y, hcl.y, iT)};
  }
  d2 vb[2][2], sb[2];
  load_rows(0, vb[0]);   // rows first, then the stale fluxes (the loop's refill order)
  load_rows(1, vb[1]);
  ring_fence();
  load_stale(0, sb[0]);
  load_stale(1, sb[1]);
  ring_fence();
  if (conv0) return;   // converged: nothing stored yet
  double* tile = red + (int64_t)(kBlock / 64) * ns * 4;
  for (int k0 = 0; k0 < ns; k0 += 2) {
    progress_priority(k0, ns);
#pragma unroll
    for (int g = 0; g < 2; ++g) {
      const int k = k0 + g;
      // odd step counts: no work past the last step (the pair's reduction below then reads a
      // stale tile slot for it and writes nothing for it)
      if (k >= ns) break;
      const int kk = clampk(k);
      ring_fence();
      const FastStep& sk = st[kk];
      const double iTn = DIR == kEmit ? sk.iT2 : sk.iT1;
      const d2 X = {planck(c1.x, hcl.x, iTn), planck(c1.y, hcl.y, iTn)};
      // contracted table: mmr = 1, and (0 + a) + b == a + b for its non-negative terms
      const double wl = sk.wlo[0], wh = sk.whi[0], dm = sk.dm;
      const d2 tot = {vb[g][0].x * wl + vb[g][1].x * wh, vb[g][0].y * wl + vb[g][1].y * wh};
      ring_fence();
      load_rows(k + 2, vb[g], tot.x, tot.y);
      const bool top = top_of(kk);
      PreCoef pa, pb;
      {
        const double ka = tot.x + sig.x, kb = tot.y + sig.y;
        pa.dtau = dm * ka;
        pb.dtau = dm * kb;
        pa.w0 = fm::div(sig.x, sig.x + ka);
        pb.w0 = fm::div(sig.y, sig.y + kb);
      }
      if (DIR == kEmit) {
        pa.B1 = Bc.x; pa.B2 = top ? Bc.x : X.x;
        pb.B1 = Bc.y; pb.B2 = top ? Bc.y : X.y;
        Bc = d2{pa.B2, pb.B2};
      } else {
        pa.B2 = Bc.x; pa.B1 = X.x;
        pb.B2 = Bc.y; pb.B1 = X.y;
        Bc = X;
      }
      CoefHead ha = coef_head_e1(pa.w0, pa.dtau, pa.B1, pa.B2);
      CoefHead hb = coef_head_e1(pb.w0, pb.dtau, pb.B1, pb.B2);
      const bool e1 = !(pa.w0 > 0.1) && !(pb.w0 > 0.1);
      if (!__all(e1)) {   // rare: one wavelength at a time (registers, not ILP)
        ring_fence();
        coef_head_general(pa.w0, pa.dtau, pa.B1, pa.B2, ha);
        ring_fence();
        coef_head_general(pb.w0, pb.dtau, pb.B1, pb.B2, hb);
        ring_fence();
      }
      StepCoef ca, cb;
      coef_tail<true>(pa.w0, pa.dtau, pa.B1, pa.B2, ha.sq, ha.r, ha.q, ha.pi_w, ca);
      coef_tail<true>(pb.w0, pb.dtau, pb.B1, pb.B2, hb.sq, hb.r, hb.q, hb.pi_w, cb);
      // finish: the carried recurrence of both wavelengths, stores, staged weighted terms
      const d2 Fst = sb[g];
      consume(Fst.x);
      consume(Fst.y);
      const d2 F1u = (DIR == kEmit) ? carry : Fst, F2d = (DIR == kEmit) ? Fst : carry;
      const d2 F2u = {step_up(ca.psi, ca.xi, ca.Xu, F1u.x, F2d.x),
                      step_up(cb.psi, cb.xi, cb.Xu, F1u.y, F2d.y)};
      const d2 F1d = {step_dn(ca.psi, ca.xi, ca.Xd, F1u.x, F2d.x),
                      step_dn(cb.psi, cb.xi, cb.Xd, F1u.y, F2d.y)};
      if (k < ns) {
        const int i = layer_of(k);
        if (act) {
          const bool st_up = (DIR == kEmit) ? !top : (!a.live_only || i == 0);
          const bool st_dn = (DIR == kAbsorb) || !a.live_only || top;
          if (st_up) st2(Fu + (int64_t)(i + 1) * nl + j, F2u);
          if (st_dn) st2(Fd + (int64_t)i * nl + j, F1d);
          if (dtaus) st2(dtaus + (int64_t)(k + 1) * nl + j, d2{ca.dtau, cb.dtau});
        }
        double* t = tile + ((wv * 2 + (k & 1)) * 4) * kStageRow + lane;
        t[0] = __builtin_fma(wt.y, F2u.y, wt.x * F2u.x);
        t[kStageRow] = __builtin_fma(wt.y, F2d.y, wt.x * F2d.x);
        t[2 * kStageRow] = __builtin_fma(wt.y, F1u.y, wt.x * F1u.x);
        t[3 * kStageRow] = __builtin_fma(wt.y, F1d.y, wt.x * F1d.x);
        carry = (DIR == kEmit) ? F2u : F1d;
      }
      ring_fence();
      load_stale(k + 2, sb[g]);
    }
    // the pair's 8 (step, quantity) sums over the wave's 64 lanes (the one-lane form's stage)
    __builtin_amdgcn_wave_barrier();
    const int o = lane >> 3;
    const double* t = tile + ((wv * 2 + (o >> 2)) * 4 + (o & 3)) * kStageRow + (lane & 7);
    double y = t[0];
#pragma unroll
    for (int i = 1; i < 8; ++i) y += t[8 * i];
    y += dpp_bcast<0xB1>(y);    // quad_perm [1,0,3,2]
    y += dpp_bcast<0x4E>(y);    // quad_perm [2,3,0,1]
    y += dpp_bcast<0x141>(y);   // row_half_mirror: the other quad of the 8-lane group
    const int ks = k0 + (o >> 2);
    if ((lane & 7) == 0 && ks < ns) red[((int64_t)wv * ns + ks) * 4 + (o & 3)] = y;
    __builtin_amdgcn_wave_barrier();
  }
  TRACE_MARK(2);
  __syncthreads();
  for (int idx = tid; idx < ns * 4; idx += kBlock) {
    double sum = red[idx];
    for (int w = 1; w < kBlock / 64; ++w) sum += red[(int64_t)w * ns * 4 + idx];
    part[part_at(idx, bx, nbx, ns * 4)] = sum;
  }
  TRACE_PUT(2);
}

static size_t sweep_shm(const void* kernel, const FastArgs& a, size_t shm);
// Two wavelengths per lane (sweep_pair_kernel): nblocks = ceil(n_lam / 512).
void launch_sweep_pair(int dir, const FastArgs& a, int nblocks, hipStream_t st) {
  const size_t shm = (size_t)red_lds_doubles(2, a.n_steps) * sizeof(double);
  const dim3 grid(nblocks, a.n_atm > 1 ? a.n_atm : 1);
  if (dir == kEmit) {
    const auto k = sweep_pair_kernel<kEmit>;
    hipLaunchKernelGGL(k, grid, dim3(kBlock), sweep_shm(reinterpret_cast<const void*>(k), a, shm),
                       st, a, a.steps, a.F_up, a.F_down, a.part, a.dtaus);
  } else {
    const auto k = sweep_pair_kernel<kAbsorb>;
    hipLaunchKernelGGL(k, grid, dim3(kBlock), sweep_shm(reinterpret_cast<const void*>(k), a, shm),
                       st, a, a.steps, a.F_up, a.F_down, a.part, a.dtaus);
  }
}

// Dynamic LDS of a one-lane / grouped-lane sweep launch: at least a.min_lds bytes
// (FREI_SWEEP_LDS_KB), which caps the blocks resident per CU at 160 KiB / min_lds, so the
// dispatcher cannot stack three or four blocks on one CU while others hold one (small slices:
// the launch ends with its most loaded CU).  Above 64 KiB the kernel opts in first.
static size_t sweep_shm(const void* kernel, const FastArgs& a, size_t shm) {
  const size_t s = shm > (size_t)a.min_lds ? shm : (size_t)a.min_lds;
  if (s > 65536) {
    static std::unordered_map<const void*, size_t> optin;
    size_t& have = optin[kernel];
    if (s > have) {
      (void)hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)s);
      have = s;
    }
  }
  return s;
}

// Q lanes per wavelength, NW waves: 64 NW / Q wavelengths per block.
void launch_sweep_group(int dir, int Q, int NW, const FastArgs& a, int nblocks,
                        hipStream_t st) {
  const size_t shm = (size_t)red_lds_doubles(a.red_rows, a.n_steps, NW) * sizeof(double) +
                     (size_t)a.n_steps * sizeof(FastStepS) +
                     (size_t)rec_scratch_doubles(a) * sizeof(double);
  const dim3 grid(nblocks, a.n_atm > 1 ? a.n_atm : 1);
  auto go = [&](auto kernel, int nw) {
    const size_t s = sweep_shm(reinterpret_cast<const void*>(kernel), a, shm);
    hipLaunchKernelGGL(kernel, grid, dim3(64 * nw), s, st, a, a.ssteps, a.F_up, a.F_down,
                       a.part, a.dtaus);
  };
  if (NW == 8) {
    if (Q == 4) {
      if (dir == kEmit) go(sweep_group_kernel<kEmit, 4, 8>, 8);
      else go(sweep_group_kernel<kAbsorb, 4, 8>, 8);
    } else {
      if (dir == kEmit) go(sweep_group_kernel<kEmit, 2, 8>, 8);
      else go(sweep_group_kernel<kAbsorb, 2, 8>, 8);
    }
  } else if (Q == 4) {
    if (dir == kEmit) go(sweep_group_kernel<kEmit, 4, 4>, 4);
    else go(sweep_group_kernel<kAbsorb, 4, 4>, 4);
  } else {
    if (dir == kEmit) go(sweep_group_kernel<kEmit, 2, 4>, 4);
    else go(sweep_group_kernel<kAbsorb, 2, 4>, 4);
  }
}


// ---------------------------------------------------------------- K1, producer/consumer form
// Small slices again (the 8-GPU case), without the grouped form's replicated chain.  Only the
// carried recurrence F = ic ((psi F_in - xi F_st) + X) is sequential over a wavelength's steps;
// everything before it (opacity, dtau, albedo, Planck, E, the transmission, psi, xi, 1/chi and
// the source terms — ~85 % of a step's instructions) is independent per (step, wavelength).
// So per 64 wavelengths a block runs kPipeP = 3 producer waves and one consumer wave:
//   phase ph: producer p computes the coefficients of the M consecutive steps
//             ph G + p M ... (+ M - 1), G = 3 M, with the one-lane form's arithmetic (Planck
//             reused inside its M steps, formed afresh at the first) into an LDS ring slot
//             [ph & 1][G steps][psi, xi, Xu, Xd (, ic)][64 lanes] and writes dtau;
//             the consumer runs the carried chain over phase ph - 1's G steps from the other
//             slot (stale fluxes prefetched a phase ahead), stores the fluxes and stages the
//             bolometric terms exactly as the one-lane sweep does;
//   then one block barrier.
// Four times the waves of the one-lane form per wavelength, each with a short dependent chain,
// at ~1.1x its instructions per update (the extra Planck per M steps and the LDS hand-off).
// Fluxes and dtaus are bit-identical to the one-lane form (same expressions, same order); with
// NC = 4 consumers (256 wavelengths per block) the per-block bolometric partials are too (the
// same lanes, staged tile and wave order), so T and every output match the one-lane sweep bit
// for bit.  One contracted table (K3, mmr = 1); the step records come from the global step table
// through scalar loads.
constexpr int kPipeP = 3;    // producer waves per consumer wave
constexpr int kPipeNV = 4;   // psi, xi, Xu, Xd
constexpr int kStepDoubles = (int)(sizeof(FastStepS) / sizeof(double));
__host__ __device__ inline int64_t pipe_lds_doubles(int NC, int M, int ns) {
  return (int64_t)NC * 2 * (kPipeP * M) * kPipeNV * 64 + (int64_t)NC * 2 * 4 * kStageRow +
         (int64_t)NC * ns * 4 + (int64_t)ns * kStepDoubles;
}

template <int DIR, int NC, int M, int PF, bool CH, bool TL = false>
__device__ __forceinline__ void sweep_pipe_body(FastArgs& a, const FastStepS* __restrict__ ss,
                                                double* __restrict__ Fu, double* __restrict__ Fd,
                                                double* __restrict__ part,
                                                double* __restrict__ dtaus, double* lds,
                                                const int bx, const int nbx) {
  constexpr int G = kPipeP * M;   // steps per phase
  static_assert(PF == 1 || PF == 2, "table rows loaded one or two phases ahead");
  static_assert(G % 2 == 0, "phases hold whole step pairs (staged partial sums)");
  {  // atmosphere of a batched launch (identity for one atmosphere)
    const int m = blockIdx.y;
    Fu += m * a.bs.flux;
    Fd += m * a.bs.flux;
    part += m * a.bs.part;
    if (dtaus) dtaus += m * a.bs.flux;
    ss += m * a.bs.steps;
    a.tab[0] += m * a.bs.tab;
    a.ftoa += m * a.bs.ftoa;
    a.conv += m;
  }
  // the convergence flag: loaded now, tested once the step records' loads are in flight (below),
  // not a round trip of its own ahead of them
  const bool conv0 = !CH && *a.conv && !a.force;
  TRACE_DECL;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  if (a.poison && bx == 0)   // the deferred update's output temperatures: "not published"
    for (int i = tid; i <= a.n_steps; i += 256 * NC)
      reinterpret_cast<unsigned long long*>(a.poison)[i] = kPoisonT;
  const int sub = wv >> 2;    // 64-wavelength chunk of the block
  // 0 .. 2: producer, 3: consumer.  Waves w and w + 4 share a SIMD (profiles/r03/simd_map.txt),
  // so role = w & 3 would put all four consumers on one SIMD and the producers' work on the
  // other three.  The roles rotate per chunk (every SIMD holds three producers and one
  // consumer) and the consumer issues first (priority 2: its chain paces the phase): together
  // −4 µs per sweep at 62.5k λ (loop 33.2 → 29.6 µs, profiles/r03/pipe_layout/); either alone
  // is no faster.
  const int role = (wv + sub) & 3;
  if (role == kPipeP) __builtin_amdgcn_s_setprio(2);
  const int64_t nl = a.n_lam;
  const int64_t j0 = (int64_t)bx * (64 * NC) + sub * 64 + lane;
  const bool act = j0 < nl;
  const int64_t j = act ? j0 : nl - 1;
  const int ns = a.n_steps;
  const int nL = ns + 1;
  const int nph = (ns + G - 1) / G;
  double* ring = lds + (int64_t)sub * 2 * G * kPipeNV * 64;
  double* tile = lds + (int64_t)NC * 2 * G * kPipeNV * 64;   // [sub][2][4][kStageRow]
  double* red = tile + (int64_t)NC * 2 * 4 * kStageRow;      // [sub][ns][4]
  // the step records in LDS: formed here from the current T (a.rec_on, scratch in the ring,
  // which is not in use yet) or copied from the global step table
  FastStepS* lrec = reinterpret_cast<FastStepS*>(red + (int64_t)NC * ns * 4);
  if (a.rec_on) {
    if (conv0) return;
    if (stage_records(a, DIR, lrec, lds)) return;
  } else {
    const double* g = reinterpret_cast<const double*>(ss);
    double* l = reinterpret_cast<double*>(lrec);
    for (int idx = tid; idx < ns * kStepDoubles; idx += 256 * NC) l[idx] = g[idx];
    if (conv0) return;   // block-uniform, ahead of the barrier
    __syncthreads();
  }
  if constexpr (!TL) TRACE_MARK(1);
  auto rslot = [&](int ph, int s, int v) {
    return ring + ((((ph & 1) * G + s) * kPipeNV + v) << 6) + lane;
  };
  // TL (trailing update): right after the barrier that ends phase q + 1, wave 0 (a producer) sums
  // phase q's staged partials over the NC consumers — the order of the end-of-sweep epilogue
  // below, so the values are bitwise its — and publishes them by write-through stores into slots
  // that hold kPoisonT until then: the trailing update workgroups start on a layer as soon as
  // every block has published its steps, while the sweep runs on.  Step-major, [steps x 4][nbx]:
  // an update slot's 256 threads read one value of 64 consecutive blocks per load instruction
  // (block-major, each lane's load was a line of its own: 8k line requests per CU and poll pass,
  // ~4-7 us under the sweep's traffic, profiles/r06/tail/).
  auto publish = [&](int q) {
    if constexpr (TL) {
      const int idx = q * G * 4 + lane;
      if (wv == 0 && q >= 0 && lane < G * 4 && idx < ns * 4) {
        double v = red[idx];
        for (int w = 1; w < NC; ++w) v += red[(int64_t)w * ns * 4 + idx];
        __hip_atomic_store((gu64*)(a.tail_part + (int64_t)idx * nbx + bx),
                           __builtin_bit_cast(unsigned long long, v), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
      }
      if (q == 0) TRACE_MARK(1);   // (trace builds: phase 0 published)
    }
  };
  if (role < kPipeP) {
    // ---------------- producer
    const int p = role;
    const double c1 = a.c1[j], hcl = a.hcl[j], sig = a.sig[j];
    const double* __restrict__ tabj = a.tab[0] + j;
    // a phase's table rows and step parameters, loaded PF phases ahead (two buffers when
    // PF = 2: phases alternate between them, the loop below is unrolled by two)
    struct Buf {
      double vlo[M], vhi[M], wl[M], wh[M], dm[M], iTn[M], iT0;
    };
    auto load = [&](int ph, Buf& b) {
      const int kb = min(ph * G + p * M, ns - 1);
      b.iT0 = (DIR == kEmit) ? lrec[kb].iT1 : lrec[kb].iT2;
#pragma unroll
      for (int i = 0; i < M; ++i) {
        const int k = min(ph * G + p * M + i, ns - 1);
        const FastStepS& st = lrec[k];
        const double* r = tabj + st.off;
        b.vlo[i] = *(r);
        b.vhi[i] = *(r + a.pitch);
        b.wl[i] = st.wlo;
        b.wh[i] = st.whi;
        b.dm[i] = st.dm;
        b.iTn[i] = (DIR == kEmit) ? st.iT2 : st.iT1;
      }
    };
    auto produce = [&](int ph, Buf& b) {
      if (ph >= nph) return;
      const int kb = ph * G + p * M;
      PreCoef pc[M];
      StepCoef c[M];
      // the Planck value the first step reuses in the one-lane form: emit B(T1), absorb
      // B(T2) of step kb (the same inverse temperature as the previous step's new one)
      double Bp = planck(c1, hcl, b.iT0);
#pragma unroll
      for (int i = 0; i < M; ++i) {
        const double kap = (b.vlo[i] * b.wl[i] + b.vhi[i] * b.wh[i]) + sig;
        const double dtau = b.dm[i] * kap;
        pc[i].w0 = fm::div(sig, sig + kap);
        pc[i].dtau = dtau;
        if (DIR == kEmit) {
          const bool top = kb + i >= ns - 1;
          pc[i].B1 = Bp;
          pc[i].B2 = top ? Bp : planck(c1, hcl, b.iTn[i]);
          Bp = pc[i].B2;
        } else {
          pc[i].B2 = Bp;
          pc[i].B1 = planck(c1, hcl, b.iTn[i]);
          Bp = pc[i].B1;
        }
      }
      ring_fence();   // every read of b above precedes its refill
      load(ph + PF, b);
      bool e1 = true;
#pragma unroll
      for (int i = 0; i < M; ++i) e1 = e1 && !(pc[i].w0 > 0.1);
      {
        CoefHead h[M];
#pragma unroll
        for (int i = 0; i < M; ++i) h[i] = coef_head_e1(pc[i].w0, pc[i].dtau, pc[i].B1, pc[i].B2);
        if (!__all(e1)) {
#pragma unroll
          for (int i = 0; i < M; ++i)
            coef_head_general(pc[i].w0, pc[i].dtau, pc[i].B1, pc[i].B2, h[i]);
        }
#pragma unroll
        for (int i = 0; i < M; ++i)   // contracted table: NaN-free
          coef_tail<true>(pc[i].w0, pc[i].dtau, pc[i].B1, pc[i].B2, h[i].sq, h[i].r, h[i].q,
                          h[i].pi_w, c[i]);
      }
#pragma unroll
      for (int i = 0; i < M; ++i) {
        const int s = p * M + i;
        *rslot(ph, s, 0) = c[i].psi;
        *rslot(ph, s, 1) = c[i].xi;
        *rslot(ph, s, 2) = c[i].Xu;
        *rslot(ph, s, 3) = c[i].Xd;
        if (dtaus && act && kb + i < ns) dtaus[(int64_t)(kb + i + 1) * nl + j] = c[i].dtau;
      }
    };
    Buf b0, b1;
    load(0, b0);
    PT_STAMP(DIR, bx, wv, -1, 0);
    if constexpr (PF == 2) {
      load(1, b1);
      for (int ph = 0; ph <= nph; ph += 2) {   // nph + 1 barriers, like the consumer's
        produce(ph, b0);
        PT_STAMP(DIR, bx, wv, ph, 0);
        __syncthreads();
        PT_STAMP(DIR, bx, wv, ph, 1);
        publish(ph - 1);
        if (ph + 1 <= nph) {
          produce(ph + 1, b1);
          PT_STAMP(DIR, bx, wv, ph + 1, 0);
          __syncthreads();
          PT_STAMP(DIR, bx, wv, ph + 1, 1);
          publish(ph);
        }
      }
    } else {
      for (int ph = 0; ph <= nph; ++ph) {
        produce(ph, b0);
        PT_STAMP(DIR, bx, wv, ph, 0);
        __syncthreads();
        PT_STAMP(DIR, bx, wv, ph, 1);
        publish(ph - 1);
      }
    }
  } else {
    // ---------------- consumer
    const double wt = act ? a.wtr[j] : 0.0;
    double carry = (DIR == kEmit) ? Fu[(int64_t)step_layer(DIR, 0, nL) * nl + j]
                                  : Fd[(int64_t)(step_layer(DIR, 0, nL) + 1) * nl + j];
    // the stale opposite-stream flux of step ph G + i (clamped past the last step)
    auto stale = [&](int ph, int i) {
      const int k = min(ph * G + i, ns - 1);
      const int layer = step_layer(DIR, k, nL);
      const double* src = (DIR == kEmit)
                              ? (k == ns - 1 ? a.ftoa : Fd + (int64_t)(layer + 1) * nl)
                              : Fu + (int64_t)layer * nl;
      return src[j];
    };
    double* t0 = tile + (int64_t)sub * 2 * 4 * kStageRow;
    // step i of phase q: the carried chain, flux stores and staged bolometric terms (a pair's
    // 8 sums after its second step)
    // (rv: the step's psi, xi, Xu, Xd, read from the ring with the rest of its phase's)
    auto step = [&](int q, int i, double stv, const double (&rv)[kPipeNV]) {
      const int k = q * G + i;
      if (k < ns) {
        const double psi = rv[0], xi = rv[1], Xu = rv[2], Xd = rv[3];
        double F1u, F2d;
        if (DIR == kEmit) { F1u = carry; F2d = stv; } else { F2d = carry; F1u = stv; }
        const double F2u = step_up(psi, xi, Xu, F1u, F2d);
        const double F1d = step_dn(psi, xi, Xd, F1u, F2d);
        const int layer = step_layer(DIR, k, nL);
        const bool top = DIR == kEmit && k == ns - 1;
        if (act) {
          const bool st_up = (DIR == kEmit) ? !top : (!a.live_only || layer == 0);
          const bool st_dn = (DIR == kAbsorb) || !a.live_only || top;
          if constexpr (TL) {
            // write-through: the XCDs' L2s then hold no dirty flux lines while the trailing
            // update's P2P push makes its system-scope release (a writeback of this XCD's L2)
            if (st_up)
              __hip_atomic_store((gu64*)(Fu + (int64_t)(layer + 1) * nl + j),
                                 __builtin_bit_cast(unsigned long long, F2u), __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_AGENT);
            if (st_dn)
              __hip_atomic_store((gu64*)(Fd + (int64_t)layer * nl + j),
                                 __builtin_bit_cast(unsigned long long, F1d), __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_AGENT);
          } else {
            if (st_up) store_flux(Fu + (int64_t)(layer + 1) * nl + j, F2u);
            if (st_dn) store_flux(Fd + (int64_t)layer * nl + j, F1d);
          }
        }
        double* t = t0 + ((k & 1) * 4) * kStageRow + lane;
        t[0] = wt * F2u;
        t[kStageRow] = wt * F2d;
        t[2 * kStageRow] = wt * F1u;
        t[3 * kStageRow] = wt * F1d;
        carry = (DIR == kEmit) ? F2u : F1d;
      }
      if (i & 1) {   // the pair's 8 (step, quantity) sums: the one-lane staged reduction
        __builtin_amdgcn_wave_barrier();
        const int o = lane >> 3;
        const double* t = t0 + ((o >> 2) * 4 + (o & 3)) * kStageRow + (lane & 7);
        double y = t[0];
#pragma unroll
        for (int r = 1; r < 8; ++r) y += t[8 * r];
        y += dpp_bcast<0xB1>(y);    // quad_perm [1,0,3,2]
        y += dpp_bcast<0x4E>(y);    // quad_perm [2,3,0,1]
        y += dpp_bcast<0x141>(y);   // row_half_mirror
        const int ks = k - 1 + (o >> 2);
        if ((lane & 7) == 0 && ks < ns) red[((int64_t)sub * ns + ks) * 4 + (o & 3)] = y;
        __builtin_amdgcn_wave_barrier();
      }
    };
    // the phase's ring values, all read before its first step: one LDS round trip per phase
    // instead of one per step on the carried chain
    auto read_ring = [&](int q, double (&rv)[G][kPipeNV]) {
#pragma unroll
      for (int i = 0; i < G; ++i)
#pragma unroll
        for (int v = 0; v < kPipeNV; ++v) rv[i][v] = *rslot(q, i, v);
      __builtin_amdgcn_sched_barrier(0);   // keep the reads together, ahead of the chain
    };
    double stn[G];   // stale opposite-stream fluxes of the next phase
#pragma unroll
    for (int i = 0; i < G; ++i) stn[i] = stale(0, i);
    PT_STAMP(DIR, bx, wv, -1, 0);
    for (int ph = 0; ph <= nph; ++ph) {
      if (ph >= 1) {
        const int q = ph - 1;   // phase consumed now
        double stc[G];
#pragma unroll
        for (int i = 0; i < G; ++i) stc[i] = stn[i];
#pragma unroll
        for (int i = 0; i < G; ++i) stn[i] = stale(ph, i);
        double rv[G][kPipeNV];
        read_ring(q, rv);
#pragma unroll
        for (int i = 0; i < G; ++i) step(q, i, stc[i], rv[i]);
      }
      PT_STAMP(DIR, bx, wv, ph, 0);
      __syncthreads();
      PT_STAMP(DIR, bx, wv, ph, 1);
    }
  }
  TRACE_MARK(2);
  if constexpr (!TL) {   // (TL: every phase is already published)
    __syncthreads();
    for (int idx = tid; idx < ns * 4; idx += 256 * NC) {
      double s = red[idx];
      for (int w = 1; w < NC; ++w) s += red[(int64_t)w * ns * 4 + idx];
      part[part_at(idx, bx, nbx, ns * 4)] = s;
    }
  }
  TRACE_PUT(CH ? 50 + NC : TL ? 60 + NC : 20 + NC);
}

template <int DIR, int NC, int M, int PF>
__global__ __launch_bounds__(256 * NC) __attribute__((amdgpu_waves_per_eu(4)))
void sweep_pipe_kernel(FastArgs a, const FastStepS* __restrict__ ss, double* __restrict__ Fu,
                       double* __restrict__ Fd, double* __restrict__ part,
                       double* __restrict__ dtaus) {
  extern __shared__ double lds[];
  sweep_pipe_body<DIR, NC, M, PF, false>(a, ss, Fu, Fd, part, dtaus, lds, blockIdx.x, gridDim.x);
}

template <int DIR, int NC, int M, int PF>
static void launch_pipe_t(const FastArgs& a, int nblocks, hipStream_t st) {
  const size_t shm = (size_t)pipe_lds_doubles(NC, M, a.n_steps) * sizeof(double);
  // (the record scratch reuses the LDS ring, which holds far more than 2 n_layers + n_tnodes)
  // dynamic LDS above 64 KiB needs the kernel's opt-in, raised whenever a launch needs more
  // (deeper atmospheres: the partial-sum rows grow with the step count)
  static size_t attr = 0;
  if (shm > attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&sweep_pipe_kernel<DIR, NC, M, PF>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
    attr = shm;
  }
  hipLaunchKernelGGL((sweep_pipe_kernel<DIR, NC, M, PF>),
                     dim3(nblocks, a.n_atm > 1 ? a.n_atm : 1), dim3(256 * NC), shm, st, a,
                     a.ssteps, a.F_up, a.F_down, a.part, a.dtaus);
}

template <int NC, int PF>
static void launch_pipe_nc(int dir, const FastArgs& a, int nblocks, hipStream_t st) {
  if (dir == kEmit) launch_pipe_t<kEmit, NC, 2, PF>(a, nblocks, st);
  else launch_pipe_t<kAbsorb, NC, 2, PF>(a, nblocks, st);
}

// NC consumers (64 NC wavelengths) per block, M = 2 steps per producer and phase (M = 4 needs
// more than the 128 VGPRs of 4 waves per SIMD and spills), table rows PF phases ahead.
void launch_sweep_pipe(int dir, int NC, int PF, const FastArgs& a, int nblocks,
                       hipStream_t st) {
  if (PF == 2) {
    if (NC == 4) launch_pipe_nc<4, 2>(dir, a, nblocks, st);
    else if (NC == 2) launch_pipe_nc<2, 2>(dir, a, nblocks, st);
    else launch_pipe_nc<1, 2>(dir, a, nblocks, st);
  } else {
    if (NC == 4) launch_pipe_nc<4, 1>(dir, a, nblocks, st);
    else if (NC == 2) launch_pipe_nc<2, 1>(dir, a, nblocks, st);
    else launch_pipe_nc<1, 1>(dir, a, nblocks, st);
  }
}

size_t pipe_lds_bytes(int NC, int M, int ns) {
  return (size_t)pipe_lds_doubles(NC, M, ns) * sizeof(double);
}

// ---------------------------------------------------------------- P2P exchange
// System-scope stores of a value and then its flag into every rank's mailbox (P2PPush): the
// release fence orders the value stores before the flag stores for any observer; the
// explicit wait keeps the compiler from dropping the fence's completion wait (gfx950 hazard,
// MI355X_MICROARCH.md "Compiler hazard").
__device__ __forceinline__ void p2p_push_values(const P2PPush& p, int64_t idx, const double* v,
                                                int nv) {
  const int par = (int)(p.seq & 1);
  for (int r = 0; r < p.nranks; ++r) {
    uint64_t* dst = reinterpret_cast<uint64_t*>(p.peers[r] + mbox_val(par, p.rank, p.nranks, p.n));
    for (int k = 0; k < nv; ++k)
      __hip_atomic_store(dst + idx + k, __builtin_bit_cast(uint64_t, v[k]), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_SYSTEM);
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  // The system-scope release orders the value stores before the flag stores for any observer.
  // (The payload is only the write-through system-scope stores above, so the completion wait
  // alone would order them too; without the fence: measured no different,
  // profiles/r02_p2p_after_fix.txt, so the canonical release stays.)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  for (int r = 0; r < p.nranks; ++r) {
    uint64_t* fl = reinterpret_cast<uint64_t*>(p.peers[r]) + mbox_flag(par, p.rank, p.nranks, p.n);
    for (int k = 0; k < nv; ++k)
      __hip_atomic_store(fl + idx + k, p.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// Wait until rank r's value idx of this sweep is published (flag == seq) or the timeout
// passes (then *err = 1 and the value is used as is: the run is reported failed, not hung).
__device__ __forceinline__ void p2p_wait(const P2PWait& w, int r, int64_t idx, long long t0) {
  const int par = (int)(w.seq & 1);
  const uint64_t* fl =
      reinterpret_cast<const uint64_t*>(w.mbox) + mbox_flag(par, r, w.nranks, w.n) + idx;
  while (__hip_atomic_load(fl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != w.seq) {
    // after one timeout every later wait gives up at once (the run is already failed)
    if (wall_clock64() - t0 > w.timeout_ticks ||
        __hip_atomic_load(w.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
      __hip_atomic_store(w.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      break;
    }
    __builtin_amdgcn_s_sleep(1);
  }
}

// The acquire that pairs with p2p_push_values' system-scope release: issued after the flag
// waits and before any p2p_value, so the value loads cannot be performed (by the compiler or
// the memory system) ahead of the flag loads that observed this sweep's sequence number.
__device__ __forceinline__ void p2p_acquire() { __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, ""); }

// Rank r's value idx of this sweep (after p2p_wait + p2p_acquire); the mailbox is uncached
// and the load is system-scope, so it reads memory.
__device__ __forceinline__ double p2p_value(const P2PWait& w, int r, int64_t idx) {
  const int par = (int)(w.seq & 1);
  const uint64_t* vp =
      reinterpret_cast<const uint64_t*>(w.mbox + mbox_val(par, r, w.nranks, w.n)) + idx;
  return __builtin_bit_cast(double,
                            __hip_atomic_load(vp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
}

__global__ void p2p_handshake_kernel(P2PPush push, P2PWait wait) {
  if (threadIdx.x != 0) return;
  const double one = 1.0;
  p2p_push_values(push, 0, &one, 1);
  const long long t0 = wall_clock64();
  for (int r = 0; r < wait.nranks; ++r) p2p_wait(wait, r, 0, t0);
  p2p_acquire();
}

void launch_p2p_handshake(const P2PPush& push, const P2PWait& wait, hipStream_t st) {
  hipLaunchKernelGGL(p2p_handshake_kernel, dim3(1), dim3(64), 0, st, push, wait);
}

// ---------------------------------------------------------------- partial sums
// Threads of the partial-sum stage (reduce_kernel and the fused update): each thread adds every
// kRedThreads-th block column, then the wave butterflies and the wave sums in wave order — the
// same fixed tree in both kernels (bit-identical).  1024 threads (four times the loads in
// flight) measured no faster at 62.5k or 500k (profiles/r02_ab_red_threads.txt).
constexpr int kRedThreads = 256;
constexpr int kRedWaves = kRedThreads / 64;

__global__ __launch_bounds__(kRedThreads) void reduce_kernel(const double* __restrict__ part,
                                                     int nblocks, double* __restrict__ Fb,
                                                     const int* conv, int force,
                                                     int64_t part_stride, int64_t fb_stride,
                                                     P2PPush push) {
  part += blockIdx.y * part_stride;   // atmosphere of a batched launch
  Fb += blockIdx.y * fb_stride;
  conv += blockIdx.y;
  if (!force && *conv) return;
  __shared__ double sh[kRedWaves];
  const int ns4 = gridDim.x;   // one reduce block per (step, quantity)
  double acc = 0.0;
  for (int b = threadIdx.x; b < nblocks; b += kRedThreads)
    acc += part[part_at(blockIdx.x, b, nblocks, ns4)];
  // fixed-order butterfly inside each wave, then the wave sums in order: deterministic
  acc = butterfly_sum(acc, threadIdx.x & 63);   // = the xor-32 ... 1 shfl butterfly
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    double v = sh[0];
    for (int w = 1; w < kRedWaves; ++w) v += sh[w];
    if (push.peers) p2p_push_values(push, blockIdx.x, &v, 1);
    else Fb[blockIdx.x] = v;
  }
}

// ln(p_l / p_{l+1}) per layer, the top entry with emit's extrapolated p_2 (twostream.py:
// 359, 180-187): constant over a run, so the update kernel's dT chain starts after it.
__global__ void log_ratio_kernel(const double* __restrict__ p, double p_top2, int nL,
                                 double* __restrict__ lnp) {
  const int l = blockIdx.x * blockDim.x + threadIdx.x;
  if (l < nL) lnp[l] = log(p[l] / (l == nL - 1 ? p_top2 : p[l + 1]));
}

void launch_log_ratio(const double* p, double p_top2, int nL, double* lnp, hipStream_t st) {
  hipLaunchKernelGGL(log_ratio_kernel, dim3((nL + 255) / 256), dim3(256), 0, st, p, p_top2,
                     nL, lnp);
}

// ---------------------------------------------------------------- setup (T -> terms)
// Shared-bracket step record k of direction `dir` from temperatures T and pressures P (every
// field but the mixing ratios): twostream.py:356-363 (T_1, T_2, p_2 of the top layer), :227-231
// (dm), opacity.py:250-263 (the T bracket and weights).  Used by setup_sweep and by the sweeps
// that form their own records (stage_records).
__device__ __forceinline__ void step_s_core(const SetupArgs& u, const double* T, const double* P,
                                            const double* tnodes, const SpecMeta& sm,
                                            const PMeta& pm, int dir, int k, FastStepS& f) {
  const int nL = u.n_layers;
  const int i = step_layer(dir, k, nL);
  const int top = (dir == kEmit && i == nL - 1) ? 1 : 0;
  f.layer = i;
  f.top = top;
  f.iT1 = 1.0 / T[i];
  f.iT2 = top ? f.iT1 : 1.0 / T[i + 1];
  const double p2 = top ? u.p_top2 : P[i + 1];
  f.dm = (P[i] - p2) / u.g;
  int64_t off;
  double wlo, whi;
  fast_term(sm, pm, tnodes, T[i], off, wlo, whi);
  f.off = off;
  f.wlo = wlo;
  f.whi = whi;
}
// Step records [kb, ke) of the sweep in direction `dir` from temperatures T (only the layers
// of those steps and the ones above them are read), written by the threads tid = 0, 1, ...
// of the caller's group (nthr of them).  pmeta / mmr of species s at layer i are read at
// s * mstride + (i - mbase): [S][n_layers] arrays (mstride n_layers, mbase 0) or one layer's
// values staged per species (mstride 1, mbase = that layer).
__device__ void setup_sweep(const SetupArgs& u, const double* T, const double* P,
                            const double* tnodes, const SpecMeta* spec, const PMeta* pmeta,
                            const double* mmr, int dir, int kb, int ke, int tid, int nthr,
                            int mstride, int mbase) {
  const int nS = u.n_species;
  const int nL = u.n_layers;
  auto MI = [&](int s, int i) { return (int64_t)s * mstride + (i - mbase); };
  // mixing ratio of species s at layer i: the chemistry table at the layer's current T
  // (kappa's chemistry(T, p) call, opacity.py:246-248), else the fixed per-layer arrays
  auto MMR = [&](int s, int i) {
    return u.chem.tab ? chem_mmr_at(u.chem, s, u.chem.pj[i], u.chem.pz[i], T[i])
                      : mmr[MI(s, i)];
  };
  if (u.fast && u.shared) {
    for (int k = kb + tid; k < ke; k += nthr) {
      const int i = step_layer(dir, k, nL);
      FastStepS* f = u.ssteps + k;
      step_s_core(u, T, P, tnodes, spec[0], pmeta[MI(0, i)], dir, k, *f);
      for (int s = 0; s < kMaxFastS; ++s) f->mmr[s] = s < nS ? MMR(s, i) : 0.0;
    }
    return;
  }
  if (u.fast) {
    for (int k = kb + tid; k < ke; k += nthr) {
      const int i = step_layer(dir, k, nL);
      FastStep* f = u.fsteps + k;
      const int top = (dir == kEmit && i == nL - 1) ? 1 : 0;
      f->layer = i;
      f->top = top;
      f->iT1 = 1.0 / T[i];
      f->iT2 = top ? f->iT1 : 1.0 / T[i + 1];
      const double p2 = top ? u.p_top2 : P[i + 1];
      f->dm = (P[i] - p2) / u.g;
    }
    for (int idx = tid; idx < (ke - kb) * kMaxFastS; idx += nthr) {
      const int k = kb + idx / kMaxFastS, s = idx % kMaxFastS;
      FastStep* f = u.fsteps + k;
      if (s >= nS) {
        if (!(u.kvalid && s == 1)) f->off[s] = 0;   // (lazy K3: off[1] is species 0's mask)
        f->wlo[s] = f->whi[s] = f->mmr[s] = 0.0;
        continue;
      }
      const int i = step_layer(dir, k, nL);
      int64_t off;
      double wlo, whi;
      fast_term(spec[s], pmeta[MI(s, i)], tnodes, T[i], off, wlo, whi);
      f->off[s] = off;
      f->wlo[s] = wlo;
      f->whi[s] = whi;
      f->mmr[s] = MMR(s, i);
      if (u.kvalid && s == 0) {   // lazy K3 (contracted table, nS = 1): rows still to contract
        int64_t mask = 0;
        if (wlo != 0.0 || whi != 0.0) {   // (outside the hull: zero weights on row 0, zeroed)
          const int64_t r = off / u.kpitch;
          mask = (u.kvalid[r] ? 0 : 1) | (u.kvalid[r + 1] ? 0 : 2);
        }
        f->off[1] = mask;
      }
    }
    return;
  }
  for (int k = kb + tid; k < ke; k += nthr) {   // generic kernel's step records
    const int i = step_layer(dir, k, nL);
    StepP sp;
    sp.layer = i;
    sp.top = (dir == kEmit && i == nL - 1) ? 1 : 0;
    sp.iT1 = 1.0 / T[i];
    sp.iT2 = sp.top ? sp.iT1 : 1.0 / T[i + 1];                         // twostream.py:358-363
    const double p2 = sp.top ? u.p_top2 : P[i + 1];
    sp.dm = (P[i] - p2) / u.g;
    sp.pad = 0;
    u.steps[k] = sp;
  }
  for (int idx = tid; idx < (ke - kb) * nS; idx += nthr) {
    const int k = kb + idx / nS, s = idx % nS;
    const int i = step_layer(dir, k, nL);
    u.terms[(int64_t)k * nS + s] = make_term(spec[s], pmeta[MI(s, i)], tnodes, u.tperm, MMR(s, i),
                             T[i], u.fast);
  }
}

// Atmosphere m of a batched context: per-atmosphere state pointers and gravity.
__device__ inline void atm_view(SetupArgs& u, int m) {
  u.T += m * u.bs.layers;
  u.steps += m * u.bs.steps;
  u.fsteps += m * u.bs.steps;
  u.ssteps += m * u.bs.steps;
  if (u.bs.g) u.g = u.bs.g[m];
}

__device__ inline void atm_view(UpdateArgs& a, int m) {
  atm_view(a.su, m);
  const AtmStride& b = a.su.bs;
  a.Fb += m * b.fb;
  a.Tb += m * b.layers;
  a.Ta += m * b.layers;
  a.hist += m * b.hist;
  a.flips += m * b.layers;
  a.prev_sign += m * b.layers;
  a.ndiff += m * b.layers;
  a.iter += m;
  a.conv += m;
  if (a.dT_out) a.dT_out += m * b.layers;
  if (a.bol_out) a.bol_out += m * b.layers * 4;
}

__global__ void setup_kernel(SetupArgs u, int dir) {
  atm_view(u, blockIdx.x);
  setup_sweep(u, u.T, u.p, u.tnodes, u.spec, u.pmeta, u.mmr, dir, 0, u.n_layers - 1,
              threadIdx.x, blockDim.x, u.n_layers, 0);
}

// ---------------------------------------------------------------- K4/K5: update
// layer_dT in two parts: everything that depends only on the layer's T and p (formed while
// the sweep's partial sums are still being loaded), then the flux-dependent tail.  The same
// operations in the same order as one expression: bit-identical.
struct LayerPre {
  double dz, cp, dF_conv, dt_rad, dt_conv, rho0, cp0;
  bool conv;
};

__device__ __forceinline__ LayerPre layer_pre(double T1, double T2, double p1, double p2,
                                              double lnp, double g, double m_bar,
                                              double alpha) {
  LayerPre r;
  // div_bol_net_flux (twostream.py:190-205); lnp = log(p1 / p2) (log_ratio_kernel)
  r.dz = (kKB * T1) / (m_bar * g) * lnp;                         // :180-187
  r.cp = (2 + 5) / (2 * m_bar) * kKB;                            // :220-224
  const double rho = ((p1 - p2) / g) / r.dz;                     // :234-238
  const double dg = (T1 - T2) / r.dz - g / r.cp;                 // :241-266
  r.conv = dg > 0;
  r.dF_conv = 0.0;                                               // :273-287
  r.dt_conv = 0.0;
  if (r.conv) {
    const double lmix = alpha * kKB * T1 / (m_bar * g);
    r.dF_conv = rho * r.cp * (lmix * lmix) * sqrt(g / T1) * pow(dg, 1.5);
    r.dt_conv = sqrt(T1 / g / dg);
  }
  // delta_t_i (:23-43): the radiative timescale
  r.dt_rad = r.cp * p1 / kSigmaSB / g / pow(T1, 3.0);
  // delta_temperature with the default m_bar (:208-217, Q7)
  const double m0 = kMbarDefault;
  const double dz0 = (kKB * T1) / (m0 * g) * lnp;
  r.rho0 = ((p1 - p2) / g) / dz0;
  r.cp0 = (2 + 5) / (2 * m0) * kKB;
  return r;
}

__device__ __forceinline__ double layer_dT_post(const double* Fb, const LayerPre& r) {
  const double dF_rad = (Fb[0] - Fb[1]) - (Fb[2] - Fb[3]);
  const double div = (dF_rad + r.dF_conv) / r.dz;
  const double x = div * r.dz;
  const double f = (x != 0) ? 1e5 / pow(fabs(x), 0.9) : 1.0;
  const double dt = r.conv ? f * fmin(r.dt_rad, r.dt_conv) : f * r.dt_rad;
  return 1 / r.rho0 / r.cp0 * div * dt;
}

__device__ double layer_dT(const double* Fb, double T1, double T2, double p1, double p2,
                           double lnp, double g, double m_bar, double alpha) {
  return layer_dT_post(Fb, layer_pre(T1, T2, p1, p2, lnp, g, m_bar, alpha));
}

// One workgroup.  Phase 0 issues every global read the kernel needs at once (T, p, sorted
// T nodes, the all-gathered partial sums, the T-P history state and — when it fits — the
// per-(species, layer) interpolation metadata) into LDS; the dT physics, the convergence
// bookkeeping and the next sweep's bracket searches then run from LDS.

__global__ __launch_bounds__(256) void update_kernel(UpdateArgs a) {
  atm_view(a, blockIdx.x);  // identity for one atmosphere
  if (!a.force && *a.conv) return;
  extern __shared__ __attribute__((aligned(16))) double sh[];
  __shared__ int all_conv;
  const int nL = a.su.n_layers;
  const int ns = nL - 1;
  const int dir = a.dir;
  const int S = a.su.n_species;
  const int ntn = a.su.n_tnodes;
  double* sT = sh;             // [nL] temperatures (old, then new)
  double* sdT = sT + nL;       // [nL] dT
  double* sP = sdT + nL;       // [nL] pressures
  double* sTb = sP + nL;       // [nL] T entering the absorb sweep
  double* sTa = sTb + nL;      // [nL] T after the previous absorb
  double* sLn = sTa + nL;      // [nL] log(p_l / p_{l+1}), top entry for emit
  double* sTn = sLn + nL;      // [ntn] sorted T nodes of every species
  double* sFb = sTn + ntn;     // [ns * 4] rank-summed bolometric partials
  int* sFl = reinterpret_cast<int*>(sFb + ns * 4);  // flips, prev sign, n diffs
  int* sPv = sFl + nL;
  int* sNd = sPv + nL;
  const bool meta = a.meta_in_lds;
  char* mb = reinterpret_cast<char*>(sh) + (((reinterpret_cast<char*>(sNd + nL) -
                                              reinterpret_cast<char*>(sh)) + 15) & ~15);
  PMeta* sPm = reinterpret_cast<PMeta*>(mb);
  double* sMm = reinterpret_cast<double*>(sPm + (meta ? S * nL : 0));
  SpecMeta* sSp = reinterpret_cast<SpecMeta*>(sMm + (meta ? S * nL : 0));
  if (threadIdx.x == 0) all_conv = 1;
  for (int l = threadIdx.x; l < nL; l += blockDim.x) {
    sT[l] = a.su.T[l];
    sdT[l] = 0.0;
    sP[l] = a.su.p[l];
    sLn[l] = a.lnp[l];
    if (a.track) {
      sTb[l] = a.Tb[l];
      sTa[l] = a.Ta[l];
      sFl[l] = a.flips[l];
      sPv[l] = a.prev_sign[l];
      sNd[l] = a.ndiff[l];
    }
  }
  for (int q = threadIdx.x; q < ntn; q += blockDim.x) sTn[q] = a.su.tnodes[q];
  if (a.p2p.mbox) {   // P2P: wait for every rank's sums of this sweep, add in rank order
    const long long t0 = wall_clock64();
    for (int q = threadIdx.x; q < ns * 4; q += blockDim.x)
      for (int r = 0; r < a.p2p.nranks; ++r) p2p_wait(a.p2p, r, q, t0);
    p2p_acquire();
    for (int q = threadIdx.x; q < ns * 4; q += blockDim.x) {
      double v = p2p_value(a.p2p, 0, q);
      for (int r = 1; r < a.p2p.nranks; ++r) v += p2p_value(a.p2p, r, q);
      sFb[q] = v;
    }
    __syncthreads();
    if (threadIdx.x == 0 && a.p2p.wait_ticks)
      atomicAdd(a.p2p.wait_ticks, (unsigned long long)(wall_clock64() - t0));
  } else {
    for (int q = threadIdx.x; q < ns * 4; q += blockDim.x) {
      double v = a.Fb[q];
      for (int r = 1; r < a.nranks; ++r) v += a.Fb[(int64_t)r * ns * 4 + q];  // rank order
      sFb[q] = v;
    }
  }
  if (meta) {
    for (int q = threadIdx.x; q < S * nL; q += blockDim.x) {
      sPm[q] = a.su.pmeta[q];
      sMm[q] = a.su.mmr[q];
    }
    for (int q = threadIdx.x; q < S; q += blockDim.x) sSp[q] = a.su.spec[q];
  }
  __syncthreads();
  for (int k = threadIdx.x; k < ns; k += blockDim.x) {
    const int i = step_layer(dir, k, nL);
    const double* Fb = sFb + k * 4;
    if (a.bol_out)
      for (int q = 0; q < 4; ++q) a.bol_out[(int64_t)i * 4 + q] = Fb[q];
    const bool top = (dir == kEmit && i == nL - 1);
    const double T1 = sT[i];
    const double T2 = top ? T1 : sT[i + 1];
    const double p2 = top ? a.su.p_top2 : sP[i + 1];
    sdT[i] = layer_dT(Fb, T1, T2, sP[i], p2, sLn[i], a.su.g, a.m_bar, a.alpha);
  }
  __syncthreads();
  // T <- T - dT for every layer (untouched layers have dT = 0, Q6)
  const int it = *a.iter;
  for (int l = threadIdx.x; l < nL; l += blockDim.x) {
    const double dT = sdT[l];
    const double Tnew = sT[l] - dT;
    if (a.dT_out) a.dT_out[l] = dT;
    if (a.track) {
      if (dir == kEmit) {
        a.Tb[l] = Tnew;  // temperature entering the absorb sweep
      } else {
        const double Tb = sTb[l];
        // absorb history column pair [T_before, T_after] (core.py:303-307)
        if (it < a.hist_cap) {
          a.hist[((int64_t)it * 2 + 0) * nL + l] = Tb;
          a.hist[((int64_t)it * 2 + 1) * nL + l] = Tnew;
        }
        // incremental sign-flip count over the concatenated history (core.py:308-311)
        int flips = sFl[l], prev = sPv[l], nd = sNd[l];
        const double d0 = Tb - sTa[l], d1 = Tnew - Tb;
        for (int q = (it > 0 ? 0 : 1); q < 2; ++q) {
          const double d = q == 0 ? d0 : d1;
          const int sgn = (d > 0) - (d < 0);
          if (nd > 0 && sgn != prev) ++flips;
          prev = sgn;
          ++nd;
        }
        a.flips[l] = flips;
        a.prev_sign[l] = prev;
        a.ndiff[l] = nd;
        a.Ta[l] = Tnew;
        const bool c = (flips > a.n_zero_crossings) || (fabs(dT) < a.convergence_dT);
        if (!c) atomicAnd(&all_conv, 0);
      }
    }
    a.su.T[l] = Tnew;
    sT[l] = Tnew;
  }
  __syncthreads();
  if (threadIdx.x == 0 && a.track && dir == kAbsorb) {
    *a.iter = it + 1;
    if (all_conv && a.stop_on_conv) *a.conv = 1;
  }
  if (a.next_dir >= 0)
    setup_sweep(a.su, sT, sP, sTn, meta ? sSp : a.su.spec, meta ? sPm : a.su.pmeta,
                meta ? sMm : a.su.mmr, a.next_dir, 0, ns, threadIdx.x, blockDim.x, nL, 0);
}

// ---------------------------------------------------------------- reduce + update, fused
// One workgroup per layer l: the per-block partial sums of the steps whose
// layers are l and l + 1 (the two dT values the next sweep's step record of layer l needs),
// summed in reduce_kernel's order; with P2P, wave 1 pushes the workgroup's own step's sums
// while wave 0 takes the peers' (rank order, own rank from registers); dT (layer_dT) in wave
// 0; then thread 0 does layer l's bookkeeping as in update_kernel and writes its new T into
// T_out (the other temperature buffer: neighbouring workgroups still read T_in) while wave 1
// writes the next sweep's record of layer l.  Every input is loaded at the start.  The
// convergence AND over layers rides on one arrival counter: each workgroup adds
// 1 + 65536 * (layer not converged); the last to arrive sets iter / conv and rearms it.
//
// Chained (a.epoch set): the update runs as the leading workgroups of the NEXT sweep's launch
// (sweep_chain_kernel), whose sweep blocks poll what it publishes instead of waiting for a
// kernel boundary: each layer's new T by one write-through (sc1) store — the buffer holds
// kPoisonT until then (the sweep that deferred this update filled it) — and the layer's
// granule epoch[l] = (epoch_val << 2) | (run already converged << 1) | (layer converged), from
// which every sweep block forms the convergence decision itself (the same AND over layers the
// last-arriving workgroup makes for iter / conv), with no arrival round trip in between.
__device__ __forceinline__ void publish_T(const UpdateArgs& a, int l, double T, int conv0,
                                          bool c) {
  if (a.epoch) {
    __hip_atomic_store(reinterpret_cast<unsigned long long*>(a.T_out) + l,
                       __builtin_bit_cast(unsigned long long, T), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(a.epoch + l,
                       (a.epoch_val << 2) | (conv0 ? 2ull : 0ull) | (c ? 1ull : 0ull),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  } else {
    a.T_out[l] = T;
  }
}
// The convergence AND over layers (absorb with tracking: the reference's convergence test)
// rides on one arrival counter: each of the nU workgroups adds 1 + 65536 * (layer not
// converged); the last to arrive sets iter / conv and rearms it.
__device__ __forceinline__ void update_arrive(const UpdateArgs& a, int nU, int it, bool nc1) {
  if (!(a.track && a.dir == kAbsorb)) return;
  const unsigned old = __hip_atomic_fetch_add(a.done, 1u + (nc1 ? 65536u : 0u),
                                              __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if ((old & 0xffffu) != (unsigned)nU - 1) return;   // not the last layer in
  const unsigned nc = (old >> 16) + (nc1 ? 1u : 0u);
  *a.iter = it + 1;
  if (nc == 0 && a.stop_on_conv) *a.conv = 1;
  __hip_atomic_store(a.done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Layer lr of nU update workgroups, run by kRedThreads threads (tid) — part h of a 512- or
// 1024-thread block in a chained launch (each part its own LDS: sh, and the [h] arrays below).  A
// half past the last layer (lr >= n_layers, odd layer counts) computes the last layer again
// with every side effect suppressed, so both halves meet the same block barriers.
// sh: dynamic LDS of (2 n_layers + n_tnodes) doubles.
// U: partial-sum strides loaded per batch (the standalone update kernel; a chained launch's
// update blocks share the sweep's register budget and keep U = 1)
template <int U = 1>
__device__ void update_fused_body(const UpdateArgs& a, int lr, int nU, int tid, int h,
                                  double* sh) {
  TRACE_DECL;
  const int nL = a.su.n_layers;
  const bool on = lr < nL;
  const int l = on ? lr : nL - 1;
  const int dir = a.dir;
  const double* Tin = a.su.T;
  double* sTn = sh;                 // [nL] new T of layers l, l + 1 (the setup's T view)
  double* sP = sTn + nL;            // [nL] p of layers l, l + 1 (the setup's p view)
  double* sNodes = sP + nL;         // [n_tnodes] sorted T nodes
  __shared__ double wsum_[4][kRedWaves][8];
  __shared__ double tot_[4][8];        // this rank's sums of steps k0 (0..3) and k1 (4..7)
  __shared__ PMeta sPm_[4][kMaxFastS];  // layer l's metadata per species (setup)
  __shared__ SpecMeta sSp_[4][kMaxFastS];
  __shared__ double sMm_[4][kMaxFastS];
  auto& wsum = wsum_[h];
  double* tot = tot_[h];
  PMeta* sPm = sPm_[h];
  SpecMeta* sSp = sSp_[h];
  double* sMm = sMm_[h];
  const int k0 = layer_step(dir, l, nL);
  const int k1 = l + 1 < nL ? layer_step(dir, l + 1, nL) : -1;
  const int kn = a.next_dir >= 0 ? layer_step(a.next_dir, l, nL) : -1;
  const int S = a.su.n_species;
  const bool stage = S <= kMaxFastS;
  // ---- every input up front: unconditional loads at clamped indices (no branch between a
  // load and the next one), consumed after the partial sums have landed
  const int conv = *a.conv;
  const int it = *a.iter;
  const int ntn = a.su.n_tnodes;
  const double rNode = a.su.tnodes[tid < ntn ? tid : ntn - 1];
  const int li = min(l + (tid & 1), nL - 1);
  const int li1 = min(li + 1, nL - 1);
  const int kd = (tid & 1) ? k1 : k0;
  const bool top = (dir == kEmit && li == nL - 1);
  const double T1 = Tin[li];
  const double rT2 = Tin[li1];
  const double p1 = a.su.p[li];
  const double rp2 = a.su.p[li1];
  const double lnp = a.lnp[li];
  const double Tb = a.Tb[l], Ta = a.Ta[l];
  int flips = a.flips[l], prev = a.prev_sign[l], nd = a.ndiff[l];
  const int sm = min(max(tid - 64, 0), S - 1);
  const PMeta rPm = a.su.pmeta[(int64_t)sm * nL + l];
  const SpecMeta rSp = a.su.spec[sm];
  const double rMm = a.su.mmr[(int64_t)sm * nL + l];
  const double T2 = top ? T1 : rT2;
  const double p2 = top ? a.su.p_top2 : rp2;
  const double Tl = T1;              // lanes with (tid & 1) == 0: layer l
  // dT's flux-independent part while the partial sums load (lanes 0, 1: layers l, l + 1)
  LayerPre pre{};
  if (tid < 2 && kd >= 0) pre = layer_pre(T1, T2, p1, p2, lnp, a.su.g, a.m_bar, a.alpha);
  // ---- this rank's sums, reduce_kernel's order (strided per thread, wave butterfly, waves),
  // loaded before the convergence test below (one round trip less on the update's critical
  // path; a converged run's update only discards them)
  if (k0 >= 0 || k1 >= 0) {
    const double* pj[8];
    for (int j = 0; j < 8; ++j) {
      const int k = (j < 4) ? (k0 >= 0 ? k0 : k1) : (k1 >= 0 ? k1 : k0);
      pj[j] = a.part + part_at(k * 4 + (j & 3), 0, a.nblocks, 4 * (nL - 1));
    }
    // element of block b in row j: pj[j][b * bs]
    const int64_t bs = part_at(0, 1, a.nblocks, 4 * (nL - 1));
    double acc[8];
    for (int j = 0; j < 8; ++j) acc[j] = 0.0;
    // U strided partials of all 8 rows loaded before any is added (one round trip per batch,
    // not per two strides: the previous trip's adds no longer gate the next loads), then
    // added in the same order as before — per thread b = tid, tid + 256, ... — so the sums
    // keep reduce_kernel's bits.  Past the end the loads repeat the last block (in bounds)
    // and are not added.  (500k: 1954 blocks, 8 strides, 64 loads in flight per thread.)
    constexpr int kU = U;
    const int nb = a.nblocks;
    if constexpr (U == 1) {
#pragma unroll 2
      for (int b = tid; b < nb; b += kRedThreads)
        for (int j = 0; j < 8; ++j) acc[j] += pj[j][b * bs];
    } else
    for (int b0 = tid; b0 < nb; b0 += kU * kRedThreads) {
      double v[kU][8];
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        const int b = min(b0 + u * kRedThreads, nb - 1);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[u][j] = pj[j][b * bs];
      }
#pragma unroll
      for (int u = 0; u < kU; ++u)
        if (b0 + u * kRedThreads < nb)
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[j] += v[u][j];
    }
    for (int j = 0; j < 8; ++j)
      acc[j] = butterfly_sum(acc[j], tid & 63);   // = the xor-32 ... 1 shfl butterfly
    if ((tid & 63) == 0)
      for (int j = 0; j < 8; ++j) wsum[tid >> 6][j] = acc[j];
  }
  if (!a.force && conv) {    // converged: carry T into the output buffer (no barrier passed)
    if (tid == 0 && on) publish_T(a, l, Tl, conv, true);
    return;
  }
  // stage the setup's inputs in LDS (their loads were issued at the start)
  if (tid < ntn) sNodes[tid] = rNode;
  for (int q = tid + kRedThreads; q < ntn; q += kRedThreads) sNodes[q] = a.su.tnodes[q];
  if (kn >= 0) {
    const int s = tid - 64;
    if (stage && s >= 0 && s < S) {
      sPm[s] = rPm;
      sSp[s] = rSp;
      sMm[s] = rMm;
    }
    if (tid < 2 && l + tid < nL) sP[l + tid] = p1;   // lane 1: layer l + 1
    if (tid == 1 && l + 1 < nL) sTn[l + 1] = T1;      // layer l + 1 before its update
  }
  __syncthreads();
  TRACE_MARK(1);
  if (tid < 8) {
    double t = wsum[0][tid];
    for (int w = 1; w < kRedWaves; ++w) t += wsum[w][tid];
    tot[tid] = t;
  }
  __syncthreads();
  const long long t0 = wall_clock64();
  if (a.p2p.mbox && tid == 64 && k0 >= 0 && on)
    p2p_push_values(a.push, (int64_t)k0 * 4, tot, 4);
  if (tid < 64) {
    // all ranks' sums in rank order (lanes 0..7), then dT of layers l, l + 1 (lanes 0, 1)
    double v = 0.0;
    const int k = tid < 4 ? k0 : k1;
    if (tid < 8 && k >= 0) {
      v = tot[tid];
      if (a.p2p.mbox) {
        const double own = v;
        const int64_t idx = (int64_t)k * 4 + (tid & 3);
        for (int r = 0; r < a.p2p.nranks; ++r)
          if (r != a.push.rank) p2p_wait(a.p2p, r, idx, t0);
        p2p_acquire();
        for (int r = 0; r < a.p2p.nranks; ++r) {
          const double x = (r == a.push.rank) ? own : p2p_value(a.p2p, r, idx);
          v = (r == 0) ? x : v + x;
        }
      }
    }
    const int base = (tid & 1) * 4;
    double F[4];
    for (int q = 0; q < 4; ++q) F[q] = __shfl(v, base + q, 64);
    if (tid < 4 && k0 >= 0 && a.bol_out && on) a.bol_out[(int64_t)l * 4 + tid] = v;
    if (tid == 0 && lr == 0 && a.p2p.mbox && a.p2p.wait_ticks)
      atomicAdd(a.p2p.wait_ticks, (unsigned long long)(wall_clock64() - t0));
    double d = 0.0;
    if (tid < 2 && kd >= 0) {
      d = layer_dT_post(F, pre);
      sTn[li] = T1 - d;
    }
    if (tid == 0 && on) {
      // layer l's bookkeeping (update_kernel's expressions)
      const double dT = d;
      const double Tnew = Tl - dT;
      if (a.dT_out) a.dT_out[l] = dT;
      bool c = true;
      if (a.track) {
        if (dir == kEmit) {
          a.Tb[l] = Tnew;
        } else {
          if (it < a.hist_cap) {
            a.hist[((int64_t)it * 2 + 0) * nL + l] = Tb;
            a.hist[((int64_t)it * 2 + 1) * nL + l] = Tnew;
          }
          const double d0 = Tb - Ta, d1 = Tnew - Tb;
          for (int q = (it > 0 ? 0 : 1); q < 2; ++q) {
            const double dd = q == 0 ? d0 : d1;
            const int sgn = (dd > 0) - (dd < 0);
            if (nd > 0 && sgn != prev) ++flips;
            prev = sgn;
            ++nd;
          }
          a.flips[l] = flips;
          a.prev_sign[l] = prev;
          a.ndiff[l] = nd;
          a.Ta[l] = Tnew;
          c = (flips > a.n_zero_crossings) || (fabs(dT) < a.convergence_dT);
        }
      }
      publish_T(a, l, Tnew, conv, c);
      if (kd < 0) sTn[l] = Tnew;
      update_arrive(a, nU, it, !c);
    }
  }
  TRACE_MARK(2);
  __syncthreads();   // sTn of layers l, l + 1
  if (a.su.kvalid && tid == 64 && on && k0 >= 0) {
    // lazy K3: the sweep that just ran contracted every row its records masked, so layer l's
    // rows at the temperature that sweep used (T_in) are complete now; marked by the thread
    // that forms layer l's next record below (it reads them back in program order)
    int64_t off;
    double wlo, whi;
    fast_term(rSp, rPm, sNodes, Tl, off, wlo, whi);   // (thread 64: species 0, layer l)
    if (wlo != 0.0 || whi != 0.0) {
      const int64_t r = off / a.su.kpitch;
      a.su.kvalid[r] = 1;
      a.su.kvalid[r + 1] = 1;
    }
  }
  if (kn >= 0 && tid >= 64 && on) {
    if (stage)
      setup_sweep(a.su, sTn, sP, sNodes, sSp, sPm, sMm, a.next_dir, kn, kn + 1, tid - 64,
                  kRedThreads - 64, 1, l);
    else
      setup_sweep(a.su, sTn, sP, sNodes, a.su.spec, a.su.pmeta, a.su.mmr, a.next_dir, kn,
                  kn + 1, tid - 64, kRedThreads - 64, nL, 0);
  }
  TRACE_PUT(30);
}

// The barriers of update_fused_body for the threads of a chained launch's update block that
// update no layer (the producer/consumer form's 1024-thread blocks: threads 0..255 update one
// layer, the other 768 only meet the body's block barriers).  The body has three barriers, none
// on its converged path; *a.conv is read before the first, and it is only written by the last
// layer to arrive, after every block has passed its second barrier — so both reads agree.
__device__ __forceinline__ void update_shadow(const UpdateArgs& a) {
  if (!a.force && *a.conv) return;
  __syncthreads();
  __syncthreads();
  __syncthreads();
}

__global__ __launch_bounds__(kRedThreads) void update_fused_kernel(UpdateArgs a) {
  extern __shared__ __attribute__((aligned(16))) double sh[];
  update_fused_body<8>(a, blockIdx.x, gridDim.x, threadIdx.x, 0, sh);
}

// Chained launch: workgroups [0, nU) run the previous sweep's fused update (u; with 8-wave
// blocks each workgroup's two 256-thread halves take a layer each), the rest sweep.  One
// atmosphere.  Forward progress: the update workgroups wait for nothing in this launch (only
// for the other ranks' sums, over P2P), so the sweep blocks' bounded polls always end.
template <int DIR, int Q, int NW>
__global__ __launch_bounds__(64 * NW) void sweep_chain_kernel(
    FastArgs a, UpdateArgs u, const FastStepS* __restrict__ ss, double* __restrict__ Fu,
    double* __restrict__ Fd, double* __restrict__ part, double* __restrict__ dtaus) {
  static_assert(kRedThreads == 256, "update halves of 256 threads");
  extern __shared__ double red[];
  const int nL = u.su.n_layers;
  constexpr int kHalves = NW / 4;
  const int nU = (nL + kHalves - 1) / kHalves;
  if ((int)blockIdx.x < nU) {
    const int h = threadIdx.x >> 8;
    update_fused_body(u, blockIdx.x * kHalves + h, nL, threadIdx.x & 255, h,
                      red + (int64_t)h * (2 * nL + u.su.n_tnodes));
    return;
  }
  sweep_group_body<DIR, Q, NW, true>(a, ss, Fu, Fd, part, dtaus, red, blockIdx.x - nU,
                                     gridDim.x - nU);
}

// The producer/consumer form chained: 1024-thread blocks, one layer per update block (its first
// 256 threads; the other 768 only meet the update's barriers, update_shadow) — four layers per
// block measured slower: the partial-sum loads of four layers queue on one CU.
template <int DIR, int PF>
__global__ __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(4)))
void sweep_pipe_chain_kernel(FastArgs a, UpdateArgs u, const FastStepS* __restrict__ ss,
                             double* __restrict__ Fu, double* __restrict__ Fd,
                             double* __restrict__ part, double* __restrict__ dtaus) {
  static_assert(kRedThreads == 256, "update parts of 256 threads");
  extern __shared__ double lds[];
  const int nL = u.su.n_layers;
  if ((int)blockIdx.x < nL) {
    if (threadIdx.x < 256) update_fused_body(u, blockIdx.x, nL, threadIdx.x, 0, lds);
    else update_shadow(u);
    return;
  }
  sweep_pipe_body<DIR, 4, 2, PF, true>(a, ss, Fu, Fd, part, dtaus, lds, blockIdx.x - nL,
                                       gridDim.x - nL);
}

// The producer/consumer sweep (4 consumers per block) chained to the previous sweep's update u.
void launch_sweep_pipe_chain(int dir, int PF, const FastArgs& a, const UpdateArgs& u,
                             int nblocks, hipStream_t st) {
  const int nL = u.su.n_layers;
  size_t shm = pipe_lds_bytes(4, 2, a.n_steps);
  const size_t ushm = (size_t)(2 * nL + u.su.n_tnodes) * sizeof(double);
  if (ushm > shm) shm = ushm;
  auto go = [&](auto kernel) {
    static std::unordered_map<const void*, size_t> optin;
    size_t& have = optin[reinterpret_cast<const void*>(kernel)];
    if (shm > have) {
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kernel),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
      have = shm;
    }
    hipLaunchKernelGGL(kernel, dim3(nL + nblocks), dim3(1024), shm, st, a, u,
                       a.ssteps, a.F_up, a.F_down, a.part, a.dtaus);
  };
  if (PF == 2) {
    if (dir == kEmit) go(sweep_pipe_chain_kernel<kEmit, 2>);
    else go(sweep_pipe_chain_kernel<kAbsorb, 2>);
  } else {
    if (dir == kEmit) go(sweep_pipe_chain_kernel<kEmit, 1>);
    else go(sweep_pipe_chain_kernel<kAbsorb, 1>);
  }
}

// ---------------------------------------------------------------- trailing update (round 6)
// The producer/consumer sweep (four consumers per block) with its own fused update as trailing
// workgroups of the same launch: blocks [0, nbx) sweep and publish each phase's partial sums as
// soon as the phase is done (sweep_pipe_body<TL>); blocks [nbx, nbx + nT) each run four
// 256-thread update slots over the layers in the order the sweep finishes them, slot h of block t
// in round r taking position (r nT + t) 4 + h (emit: layer = position; absorb: n_layers - 1 -
// position).  A layer's reduction waits only for the steps it reads (twostream.py:396-407: dT_l
// needs layer l's four bolometric sums), so all but the last layers' updates run while the
// sweep is still in flight, and the next sweep waits for one kernel boundary instead of two.
// Forward progress: the sweep blocks wait for nothing; the update blocks come after them in
// dispatch order (launched only while the device has a free CU per update block, so they are
// resident beside the sweep) and wait only for sweep blocks of their own launch and, over P2P,
// for the other ranks' update blocks.  The update blocks also put the previous launch's
// partials (`clear`, the other of two buffers) back to kPoisonT for the next launch, by
// write-through stores (a plain store would leave the line in this XCD's L2, where the next
// launch's polls of it would find the stale kPoisonT).
//
// One layer of the update (tail_update_slot): update_fused_body's computation in the same
// order — the same summation tree over the sweep blocks (thread t adds blocks t, t + 256, ...;
// the xor butterfly per wave; the waves in order), the same layer_dT of layers l and l + 1, the
// same bookkeeping and the same step record — restricted to the case the trailing update serves
// (one atmosphere, contracted table with shared brackets, fixed mixing ratios, fused exchange)
// and ordered so that only the partial sums are live while they are polled: the 128 VGPRs of a
// 16-wave block hold it without spills (update_fused_body, which loads every input up front,
// spilled 544 B per lane here and took 3-5x its standalone time, profiles/r06/tail/).
// A trailing block's copy of every per-layer input of the update, loaded once at its start (none
// of them is written in the launch by anyone but the layer's own slot): the slots' dT and
// bookkeeping then wait on no global load (round 6: loading them after the poll put three
// dependent global round trips, ~5 us, behind every layer's sums).
struct TailIn {
  double *T, *p, *Tb, *Ta, *mmr, *nodes;
  int *flips, *prev, *nd;
  PMeta* pm;
  LayerPre* pre;   // [n_layers] layer_pre of every layer (formed at the block's start)
};
__host__ __device__ inline size_t tail_in_bytes(int nL, int ntn) {
  return (size_t)nL * (sizeof(PMeta) + sizeof(LayerPre)) + (size_t)(5 * nL + ntn) * sizeof(double) +
         (size_t)3 * nL * sizeof(int);
}
__device__ __forceinline__ TailIn tail_in_layout(double* lds, int nL, int ntn) {
  TailIn t;
  t.pre = reinterpret_cast<LayerPre*>(lds);
  t.pm = reinterpret_cast<PMeta*>(t.pre + nL);
  double* d = reinterpret_cast<double*>(t.pm + nL);
  t.T = d;
  t.p = d + nL;
  t.Tb = d + 2 * nL;
  t.Ta = d + 3 * nL;
  t.mmr = d + 4 * nL;
  t.nodes = d + 5 * nL;
  int* q = reinterpret_cast<int*>(t.nodes + ntn);
  t.flips = q;
  t.prev = q + nL;
  t.nd = q + 2 * nL;
  return t;
}

#ifdef FREI_TRACE
__shared__ unsigned long long g_tail_done[4];
__shared__ unsigned g_tail_pass[4];
#endif
__device__ __forceinline__ void tail_update_slot(const UpdateArgs& a, int lr, int tid, int h,
                                                 double (&wsum)[kRedWaves][8],
                                                 const TailIn& in, int conv, int it) {
  TRACE_DECL;
  const int nL = a.su.n_layers;
  const bool on = lr < nL;
  const int l = on ? lr : nL - 1;
  const int dir = a.dir;
  const int k0 = layer_step(dir, l, nL);
  const int k1 = l + 1 < nL ? layer_step(dir, l + 1, nL) : -1;
  const bool skip = !a.force && conv;   // converged: the sweep published nothing
  const bool sums = !skip && (k0 >= 0 || k1 >= 0);
  const int nb = a.nblocks;   // <= 256 (a trailing launch leaves free CUs)
  // ---- thread t polls sweep block t's partial sums of steps k0 (values 0..3) and k1 (4..7),
  // then update_fused_body's tree: the xor butterfly per wave, the waves in order (a block t +
  // 256, ... never exists here)
  if (sums) {
    const double* pj[8];
    for (int j = 0; j < 8; ++j) {
      const int k = (j < 4) ? (k0 >= 0 ? k0 : k1) : (k1 >= 0 ? k1 : k0);
      pj[j] = a.part + (int64_t)(k * 4 + (j & 3)) * nb;
    }
    const int b = min(tid, nb - 1);
    unsigned long long x[8];
    auto load_all = [&]() {
      bool m = false;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        x[j] = __hip_atomic_load((const gu64*)(pj[j] + b), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        m |= x[j] == kPoisonT;
      }
      return m;
    };
    bool miss = load_all();
#ifdef FREI_TRACE
    int passes = 1;
#endif
    if (__any(miss)) {
      const long long t0 = wall_clock64();
      do {   // (every value re-read each pass: no data-dependent load)
        __builtin_amdgcn_s_sleep(1);
        miss = load_all();
#ifdef FREI_TRACE
        ++passes;
#endif
        const int e = __hip_atomic_load(a.poll_err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (__any(miss) && (e || wall_clock64() - t0 > a.poll_timeout)) {
          if (!e) __hip_atomic_store(a.poll_err, 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
      } while (__any(miss));
    }
#ifdef FREI_TRACE
    // the slot's last poll to finish, and the most passes any lane needed (trace builds)
    atomicMax(&g_tail_done[h], (unsigned long long)wall_clock64());
    atomicMax(&g_tail_pass[h], (unsigned)passes);
#endif
    double acc[8];
    for (int j = 0; j < 8; ++j) acc[j] = tid < nb ? 0.0 + __builtin_bit_cast(double, x[j]) : 0.0;
    for (int j = 0; j < 8; ++j) acc[j] = butterfly_sum(acc[j], tid & 63);
    if ((tid & 63) == 0)
      for (int j = 0; j < 8; ++j) wsum[tid >> 6][j] = acc[j];
  }
  __syncthreads();
  TRACE_MARK(2);
#ifdef FREI_TRACE
  if (sums) {   // the block's last poll (over its four slots) and the most passes
    unsigned long long dm = 0;
    unsigned pm = 0;
    for (int q = 0; q < 4; ++q) dm = max(dm, g_tail_done[q]), pm = max(pm, g_tail_pass[q]);
    tr_[1] = (long long)(dm & ((1ull << 40) - 1)) | ((long long)pm << 40);
  }
  __syncthreads();
  if (tid == 0) g_tail_done[h] = 0, g_tail_pass[h] = 0;
#endif
  if (skip) {   // carry T into the output buffer
    if (tid == 0 && on) publish_T(a, l, in.T[l], conv, true);
    return;
  }
  // this rank's sums in wave order (lanes 0..7: k0's four, then k1's)
  auto own = [&](int q) {
    double t = wsum[0][q];
    for (int w = 1; w < kRedWaves; ++w) t += wsum[w][q];
    return t;
  };
  // (the push's system-scope release writes back this XCD's L2 while the sweep may still run:
  // cheap because the trailing-update sweep stores its fluxes write-through — with plain flux
  // stores the releases cost 230 against 83 us per T-P iteration, profiles/r06/tail/)
  if (a.p2p.mbox && tid == 64 && k0 >= 0 && on) {   // push while wave 0 waits for the peers
    double t4[4];
    for (int q = 0; q < 4; ++q) t4[q] = own(q);
    p2p_push_values(a.push, (int64_t)k0 * 4, t4, 4);
  }
  if (tid >= 64) return;
  const int li = min(l + (tid & 1), nL - 1);
  const int kd = (tid & 1) ? k1 : k0;
  double v = 0.0;
  const int k = tid < 4 ? k0 : k1;
  if (tid < 8 && k >= 0) {
    v = own(tid);
    if (a.p2p.mbox) {   // all ranks' sums in rank order (own rank from registers)
      const double mine = v;
      const int64_t idx = (int64_t)k * 4 + (tid & 3);
      const long long t0 = wall_clock64();
      for (int r = 0; r < a.p2p.nranks; ++r)
        if (r != a.push.rank) p2p_wait(a.p2p, r, idx, t0);
      p2p_acquire();
      for (int r = 0; r < a.p2p.nranks; ++r) {
        const double xr = (r == a.push.rank) ? mine : p2p_value(a.p2p, r, idx);
        v = (r == 0) ? xr : v + xr;
      }
    }
  }
  const int base = (tid & 1) * 4;
  double F[4];
  for (int q = 0; q < 4; ++q) F[q] = __shfl(v, base + q, 64);
  if (tid < 4 && k0 >= 0 && a.bol_out && on) a.bol_out[(int64_t)l * 4 + tid] = v;
  // dT of layers l (lane 0) and l + 1 (lane 1): layer_dT's expressions
  const double T1 = in.T[li];
  double d = 0.0;
  if (tid < 2 && kd >= 0) d = layer_dT_post(F, in.pre[li]);
  const double Tn = T1 - d;               // lane 0: layer l, lane 1: layer l + 1
  const double Tl0 = __shfl(Tn, 0, 64);   // layer l's new temperature (lane 1)
  // lane 1: the next sweep's step record of layer l (setup_sweep's shared-bracket record, S = 1)
  // while lane 0 does the bookkeeping and the convergence arrival (round trips in parallel)
  const int kn = a.next_dir >= 0 ? layer_step(a.next_dir, l, nL) : -1;
  if (tid == 1 && on && kn >= 0) {
    const int tp = (a.next_dir == kEmit && l == nL - 1) ? 1 : 0;
    FastStepS f{};
    f.layer = l;
    f.top = tp;
    f.iT1 = 1.0 / Tl0;
    f.iT2 = tp ? f.iT1 : 1.0 / Tn;
    const double p2 = tp ? a.su.p_top2 : in.p[l + 1];
    f.dm = (in.p[l] - p2) / a.su.g;
    int64_t off;
    double wlo, whi;
    fast_term(a.su.spec[0], in.pm[l], in.nodes, Tl0, off, wlo, whi);
    f.off = off;
    f.wlo = wlo;
    f.whi = whi;
    for (int q = 0; q < kMaxFastS; ++q) f.mmr[q] = q < 1 ? in.mmr[l] : 0.0;
    a.su.ssteps[kn] = f;
  }
  if (tid != 0 || !on) return;
  // layer l's bookkeeping (update_kernel's expressions)
  const double dT = d;
  const double Tnew = Tn;
  if (a.dT_out) a.dT_out[l] = dT;
  bool c = true;
  if (a.track) {
    if (dir == kEmit) {
      a.Tb[l] = Tnew;
    } else {
      const double Tb = in.Tb[l], Ta = in.Ta[l];
      int flips = in.flips[l], prev = in.prev[l], nd = in.nd[l];
      if (it < a.hist_cap) {
        a.hist[((int64_t)it * 2 + 0) * nL + l] = Tb;
        a.hist[((int64_t)it * 2 + 1) * nL + l] = Tnew;
      }
      const double d0 = Tb - Ta, d1 = Tnew - Tb;
      for (int q = (it > 0 ? 0 : 1); q < 2; ++q) {
        const double dd = q == 0 ? d0 : d1;
        const int sgn = (dd > 0) - (dd < 0);
        if (nd > 0 && sgn != prev) ++flips;
        prev = sgn;
        ++nd;
      }
      a.flips[l] = flips;
      a.prev_sign[l] = prev;
      a.ndiff[l] = nd;
      a.Ta[l] = Tnew;
      c = (flips > a.n_zero_crossings) || (fabs(dT) < a.convergence_dT);
    }
  }
  publish_T(a, l, Tnew, conv, c);
  update_arrive(a, nL, it, !c);
  TRACE_PUT(31);
}

template <int DIR, int PF>
__global__ __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(4)))
void sweep_pipe_tail_kernel(FastArgs a, UpdateArgs u, const FastStepS* __restrict__ ss,
                            double* __restrict__ Fu, double* __restrict__ Fd,
                            double* __restrict__ dtaus, double* __restrict__ clear,
                            int64_t n_clear) {
  static_assert(kRedThreads == 256, "update slots of 256 threads");
  extern __shared__ double lds[];
  const int nbx = u.nblocks;
  if ((int)blockIdx.x < nbx) {
    sweep_pipe_body<DIR, 4, 2, PF, false, true>(a, ss, Fu, Fd, nullptr, dtaus, lds, blockIdx.x,
                                                nbx);
    return;
  }
  __shared__ double wsum[4][kRedWaves][8];
  const int t = blockIdx.x - nbx, nT = gridDim.x - nbx;
  const int nL = u.su.n_layers, ntn = u.su.n_tnodes;
  const int tid = threadIdx.x;
  const TailIn in = tail_in_layout(lds, nL, ntn);
  // every per-layer input once (issued before the refill below, which waits on nothing)
  for (int q = tid; q < nL; q += 1024) {
    const double Tq = u.su.T[q], pq = u.su.p[q];
    in.T[q] = Tq;
    in.p[q] = pq;
    in.mmr[q] = u.su.mmr[q];
    // dT's flux-independent part of layer q (layer_dT's first half, update_fused_body's inputs)
    const bool top = (u.dir == kEmit && q == nL - 1);
    const int q1 = min(q + 1, nL - 1);
    in.pre[q] = layer_pre(Tq, top ? Tq : u.su.T[q1], pq, top ? u.su.p_top2 : u.su.p[q1], u.lnp[q],
                          u.su.g, u.m_bar, u.alpha);
    in.pm[q] = u.su.pmeta[q];
    if (u.track) {
      in.Tb[q] = u.Tb[q];
      in.Ta[q] = u.Ta[q];
      in.flips[q] = u.flips[q];
      in.prev[q] = u.prev_sign[q];
      in.nd[q] = u.ndiff[q];
    }
  }
  for (int q = tid; q < ntn; q += 1024) in.nodes[q] = u.su.tnodes[q];
  const int conv = *u.conv, it = *u.iter;
  // the previous launch's partials back to "not published" (write-through: see above)
  for (int64_t i = (int64_t)t * 1024 + tid; i < n_clear; i += (int64_t)nT * 1024)
    __hip_atomic_store((gu64*)clear + i, kPoisonT, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  const int h = tid >> 8;
  for (int r = 0;; ++r) {
    const int p0 = (r * nT + t) * 4;
    if (p0 >= nL) break;
    const int p = p0 + h;
    const int lr = p >= nL ? nL : (u.dir == kEmit ? p : nL - 1 - p);
    tail_update_slot(u, lr, tid & 255, h, wsum[h], in, conv, it);
    __syncthreads();   // the next round's slots rewrite wsum and the stage
  }
}

size_t pipe_tail_lds_bytes(int ns, int n_tnodes) {
  return std::max(pipe_lds_bytes(4, 2, ns), tail_in_bytes(ns + 1, n_tnodes));
}

void launch_sweep_pipe_tail(int dir, int PF, const FastArgs& a, const UpdateArgs& u,
                            int nbx, int n_tail, double* clear, hipStream_t st) {
  const size_t shm = pipe_tail_lds_bytes(a.n_steps, u.su.n_tnodes);
  const int64_t n_clear = (int64_t)nbx * a.n_steps * 4;
  auto go = [&](auto kernel) {
    static std::unordered_map<const void*, size_t> optin;
    size_t& have = optin[reinterpret_cast<const void*>(kernel)];
    if (shm > have) {
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kernel),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
      have = shm;
    }
    hipLaunchKernelGGL(kernel, dim3(nbx + n_tail), dim3(1024), shm, st, a, u, a.ssteps, a.F_up,
                       a.F_down, a.dtaus, clear, n_clear);
  };
  if (PF == 2) {
    if (dir == kEmit) go(sweep_pipe_tail_kernel<kEmit, 2>);
    else go(sweep_pipe_tail_kernel<kAbsorb, 2>);
  } else {
    if (dir == kEmit) go(sweep_pipe_tail_kernel<kEmit, 1>);
    else go(sweep_pipe_tail_kernel<kAbsorb, 1>);
  }
}

// Fill n 8-byte slots with kPoisonT ("not published"): the trailing update's partial buffers
// (write-through stores: no copy of the line stays in this XCD's L2 for a later poll to find).
__global__ void poison_kernel(unsigned long long* x, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    __hip_atomic_store((gu64*)x + i, kPoisonT, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
void launch_poison(double* x, int64_t n, hipStream_t st) {
  const int nb = (int)std::min<int64_t>((n + 255) / 256, 4096);
  hipLaunchKernelGGL(poison_kernel, dim3(nb > 0 ? nb : 1), dim3(256), 0, st,
                     reinterpret_cast<unsigned long long*>(x), n);
}

// The one-lane form chained (contracted single table, step records formed in the block).
template <int DIR, int PD, int PF>
__global__ __launch_bounds__(kBlock, 1) void sweep_fast_chain_kernel(
    FastArgs a, UpdateArgs u, const FastStepS* __restrict__ ss, double* __restrict__ Fu,
    double* __restrict__ Fd, double* __restrict__ part, double* __restrict__ dtaus) {
  static_assert(kRedThreads == kBlock, "update workgroups of the sweep's block size");
  extern __shared__ double red[];
  const int nL = u.su.n_layers;
  if ((int)blockIdx.x < nL) {
    update_fused_body(u, blockIdx.x, nL, threadIdx.x, 0, red);
    return;
  }
  sweep_fast_body<DIR, 1, PD, false, true, true, PF, true>(a, nullptr, ss, Fu, Fd, part, dtaus,
                                                          red, blockIdx.x - nL, gridDim.x - nL);
}

template <int PD, int PF>
static void launch_fast_chain_t(int dir, const FastArgs& a, const UpdateArgs& u, int nblocks,
                                size_t shm, hipStream_t st) {
  const int nL = u.su.n_layers;
  const auto kernel = dir == kEmit ? sweep_fast_chain_kernel<kEmit, PD, PF>
                                   : sweep_fast_chain_kernel<kAbsorb, PD, PF>;
  hipLaunchKernelGGL(kernel, dim3(nL + nblocks), dim3(kBlock),
                     sweep_shm(reinterpret_cast<const void*>(kernel), a, shm), st, a, u,
                     a.ssteps, a.F_up, a.F_down, a.part, a.dtaus);
}

// The one-lane sweep chained to the previous sweep's fused update u: depth 2 or 4 steps in
// flight, loads pf (8, 16; 0: the depth) steps ahead, as launch_sweep_fast chooses them.
void launch_sweep_fast_chain(int dir, int depth, int pf, const FastArgs& a, const UpdateArgs& u,
                             int nblocks, hipStream_t st) {
  size_t shm = (size_t)red_lds_doubles(a.red_rows, a.n_steps) * sizeof(double) +
               (size_t)a.n_steps * sizeof(FastStepS) +
               (size_t)rec_scratch_doubles(a) * sizeof(double);
  const size_t ushm = (size_t)(2 * u.su.n_layers + u.su.n_tnodes) * sizeof(double);
  if (ushm > shm) shm = ushm;
  if (depth >= 4) {
    if (pf >= 16) launch_fast_chain_t<4, 16>(dir, a, u, nblocks, shm, st);
    else if (pf >= 8) launch_fast_chain_t<4, 8>(dir, a, u, nblocks, shm, st);
    else launch_fast_chain_t<4, 4>(dir, a, u, nblocks, shm, st);
  } else {
    if (pf >= 16) launch_fast_chain_t<2, 16>(dir, a, u, nblocks, shm, st);
    else if (pf >= 8) launch_fast_chain_t<2, 8>(dir, a, u, nblocks, shm, st);
    else launch_fast_chain_t<2, 2>(dir, a, u, nblocks, shm, st);
  }
}

// The chained launch of a grouped-lane sweep: the update workgroups of u ahead of nblocks sweep
// blocks, dynamic LDS for the larger of the two.
void launch_sweep_chain(int dir, int Q, int NW, const FastArgs& a, const UpdateArgs& u,
                        int nblocks, hipStream_t st) {
  const int nL = u.su.n_layers;
  const int nU = (nL + NW / 4 - 1) / (NW / 4);
  size_t shm = (size_t)red_lds_doubles(a.red_rows, a.n_steps, NW) * sizeof(double) +
               (size_t)a.n_steps * sizeof(FastStepS) +
               (size_t)rec_scratch_doubles(a) * sizeof(double);
  const size_t ushm = (size_t)(NW / 4) * (2 * nL + u.su.n_tnodes) * sizeof(double);
  if (ushm > shm) shm = ushm;
  auto go = [&](auto kernel) {
    const size_t s = sweep_shm(reinterpret_cast<const void*>(kernel), a, shm);
    hipLaunchKernelGGL(kernel, dim3(nU + nblocks), dim3(64 * NW), s, st, a, u, a.ssteps,
                       a.F_up, a.F_down, a.part, a.dtaus);
  };
  if (NW == 8) {
    if (Q == 4) {
      if (dir == kEmit) go(sweep_chain_kernel<kEmit, 4, 8>);
      else go(sweep_chain_kernel<kAbsorb, 4, 8>);
    } else {
      if (dir == kEmit) go(sweep_chain_kernel<kEmit, 2, 8>);
      else go(sweep_chain_kernel<kAbsorb, 2, 8>);
    }
  } else if (Q == 4) {
    if (dir == kEmit) go(sweep_chain_kernel<kEmit, 4, 4>);
    else go(sweep_chain_kernel<kAbsorb, 4, 4>);
  } else {
    if (dir == kEmit) go(sweep_chain_kernel<kEmit, 2, 4>);
    else go(sweep_chain_kernel<kAbsorb, 2, 4>);
  }
}

// ---------------------------------------------------------------- standalone kernels
__global__ void propagate_kernel(int64_t n, const double* c1, const double* lk,
                                 const double* F1u, const double* F2d, double T1, double T2,
                                 const double* dtau, const double* w0, const double* g0,
                                 double* F2u, double* F1d) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  double u, d;
  const double hcl = kHC / lk[j];   // as the sweeps' host-side constant
  const double B1 = planck(c1[j], hcl, 1.0 / T1), B2 = planck(c1[j], hcl, 1.0 / T2);
  if (g0)
    two_stream_g(w0[j], g0[j], dtau[j], B1, B2, F1u[j], F2d[j], u, d);
  else
    two_stream(w0[j], dtau[j], B1, B2, F1u[j], F2d[j], u, d);
  F2u[j] = u;
  F1d[j] = d;
}

__global__ void kappa_kernel(int64_t n, const TermP* terms, int nS, const double* sig,
                             double* k) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  k[j] = kappa_at<1, false>(terms, nS, j, sig[j]);
}

__global__ void gen_table_kernel(double* tab, const double* base, const double* fp,
                                 const double* fT, int n_p, int n_T, int64_t n_lam,
                                 int64_t stride, double lo, double hi) {
  const int64_t total = (int64_t)n_p * n_T * n_lam;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int64_t l = idx % n_lam;
    const int64_t pt = idx / n_lam;
    const int t = (int)(pt % n_T);
    const int p = (int)(pt / n_T);
    const double v = (fp[p] * fT[t]) * base[l];
    tab[pt * stride + l] = fmin(fmax(v, lo), hi);  // np.clip
  }
}

// Species contraction of the shared-bracket tables: for every layer l
// and T node t, eff[prow_l][t][:] = sum_s mmr[s][l] * tab_s[prow_l][t][:] in species
// order (no FMA).  The sweep then interpolates this one table (mmr = 1), reading 2 rows
// per layer instead of 2 S.
struct ContractArgs {
  const double* tab[kMaxFastS];
  const double* mmr;      // [S][n_layers]
  const int32_t* prow;    // [n_layers] table pressure row of each layer
  double* eff;
  int S, n_layers, n_T;
  int64_t pitch;
};

// S is a template parameter so every species' load is issued at once (kernel-argument table
// pointers at constant indices); two adjacent columns per lane (16-B loads and stores).  The
// sum keeps the species order: eff = mmr_0 tab_0, then eff + mmr_s tab_s.
typedef double dbl2k3 __attribute__((ext_vector_type(2)));
template <int S>
__global__ __launch_bounds__(256) void contract_kernel(ContractArgs a) {
  const int64_t j = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 2;
  if (j >= a.pitch) return;   // the pitch is a multiple of 64
  const int l = blockIdx.y, t = blockIdx.z;
  const int64_t idx = ((int64_t)a.prow[l] * a.n_T + t) * a.pitch + j;
  dbl2k3 v[S];
#pragma unroll
  for (int s = 0; s < S; ++s) v[s] = *reinterpret_cast<const dbl2k3*>(a.tab[s] + idx);
  dbl2k3 acc = a.mmr[l] * v[0];
#pragma unroll
  for (int s = 1; s < S; ++s) acc = acc + a.mmr[(int64_t)s * a.n_layers + l] * v[s];
  *reinterpret_cast<dbl2k3*>(a.eff + idx) = acc;
}

void launch_contract(const double* const* tabs, int S, const double* mmr, const int32_t* prow,
                     int n_layers, int n_T, int64_t pitch, double* eff, hipStream_t st) {
  ContractArgs a{};
  for (int s = 0; s < S && s < kMaxFastS; ++s) a.tab[s] = tabs[s];
  a.mmr = mmr;
  a.prow = prow;
  a.eff = eff;
  a.S = S;
  a.n_layers = n_layers;
  a.n_T = n_T;
  a.pitch = pitch;
  dim3 grid((unsigned)((pitch / 2 + 255) / 256), (unsigned)n_layers, (unsigned)n_T);
  switch (S) {
#define K3(n) case n: hipLaunchKernelGGL(contract_kernel<n>, grid, dim3(256), 0, st, a); break;
    K3(1) K3(2) K3(3) K3(4) K3(5) K3(6) K3(7)
    default: hipLaunchKernelGGL(contract_kernel<8>, grid, dim3(256), 0, st, a);
#undef K3
  }
}

// ---------------------------------------------------------------- post-processing
// numpy's interp search (npy_interp binary_search_with_guess, LIKELY_IN_CACHE_SIZE 8) for a
// scalar key over arr(l), l < len: bit-for-bit the index numpy returns, unsorted arrays
// included (effective_temperature_milne interpolates on unsorted transmissions).
template <typename Arr>
__device__ int np_search(double key, int len, int guess, const Arr& arr) {
  int imin = 0, imax = len;
  if (key > arr(len - 1)) return len;
  if (key < arr(0)) return -1;
  if (len <= 4) {
    int i = 1;
    for (; i < len && key >= arr(i); ++i) {
    }
    return i - 1;
  }
  if (guess > len - 3) guess = len - 3;
  if (guess < 1) guess = 1;
  if (key < arr(guess)) {
    if (key < arr(guess - 1)) {
      imax = guess - 1;
      if (guess > 8 && key >= arr(guess - 8)) imin = guess - 8;
    } else {
      return guess - 1;
    }
  } else {
    if (key < arr(guess + 1)) return guess;
    if (key < arr(guess + 2)) return guess + 1;
    imin = guess + 2;
    if (guess < len - 8 - 1 && key < arr(guess + 8)) imax = guess + 8;
  }
  while (imin < imax) {
    const int imid = imin + ((imax - imin) >> 1);
    if (key >= arr(imid)) imin = imid + 1;
    else imax = imid;
  }
  return imin - 1;
}

// effective_temperature_milne, per wavelength (core.py:392-395):
// p_milne[j] = np.interp(2/3, exp(-dtaus[:, j]), p_bar) with numpy's search and formula.
__global__ __launch_bounds__(256) void milne_kernel(const double* __restrict__ dtaus, int nL,
                                                    int64_t n, const double* __restrict__ fp,
                                                    double* __restrict__ out) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  auto X = [&](int l) { return exp(-dtaus[(int64_t)l * n + j]); };
  const double key = 2.0 / 3.0;
  const int k = np_search(key, nL, 0, X);
  double r;
  if (k == -1) {
    r = fp[0];
  } else if (k == nL || k == nL - 1) {
    r = fp[k == nL ? nL - 1 : k];
  } else {
    const double xk = X(k);
    if (xk == key) {
      r = fp[k];
    } else {
      const double xk1 = X(k + 1);
      const double slope = (fp[k + 1] - fp[k]) / (xk1 - xk);
      r = slope * (key - xk) + fp[k];
      if (isnan(r)) {
        r = slope * (key - xk1) + fp[k + 1];
        if (isnan(r) && fp[k] == fp[k + 1]) r = fp[k];
      }
    }
  }
  out[j] = r;
}

// Contribution function (plot.py:63-79) per wavelength, layers top-first (the reference's
// reversed arrays): tau = cumsum of dtau; cf = ((exp(-tau) * dtau) * ratio) * nu^3 /
// expm1((hc/k * nu) / T), ratio = p / dP; then cf /= sum over layers (sequential, top
// first).  Written bottom-first (cf[::-1], as plotted).
__global__ __launch_bounds__(256) void contribution_kernel(
    const double* __restrict__ dtaus, int nL, int64_t n, const double* __restrict__ nu,
    const double* __restrict__ ratio, const double* __restrict__ T, double hcperk,
    double* __restrict__ cf) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  const double v = nu[j];
  const double v3 = pow(v, 3.0);
  const double hv = hcperk * v;
  double tau = 0.0, sum = 0.0;
  for (int m = 0; m < nL; ++m) {
    const int l = nL - 1 - m;
    const double d = dtaus[(int64_t)l * n + j];
    tau = (m == 0) ? d : tau + d;
    const double c = (((exp(-tau) * d) * ratio[l]) * v3) / expm1(hv / T[l]);
    cf[(int64_t)l * n + j] = c;
    sum = (m == 0) ? c : sum + c;
  }
  for (int l = 0; l < nL; ++l) cf[(int64_t)l * n + j] = cf[(int64_t)l * n + j] / sum;
}

void launch_milne(const double* dtaus, int nL, int64_t n, const double* fp, double* out,
                  hipStream_t st) {
  hipLaunchKernelGGL(milne_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, dtaus,
                     nL, n, fp, out);
}

void launch_contribution(const double* dtaus, int nL, int64_t n, const double* nu,
                         const double* ratio, const double* T, double hcperk, double* cf,
                         hipStream_t st) {
  hipLaunchKernelGGL(contribution_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st,
                     dtaus, nL, n, nu, ratio, T, hcperk, cf);
}

// K7: batched species contraction on fp64 MFMA (§8(f) #2).  A batched context holds n_atm
// atmospheres, each with its own mixing ratios, on shared tables.  For every layer l
// (pressure row prow_l) and every column c of that row's [n_T][pitch] block:
//   eff[m][prow_l][c] = sum_s mmr[m][s][l] * tab_s[prow_l][c],
// i.e. per layer the dense product [n_atm x S] . [S x n_T*pitch].  v_mfma_f64_16x16x4f64:
// A = 16 atmospheres x 4 species (mixing ratios), B = 4 species x 16 columns (table values),
// D = 16 atmospheres x 16 columns; K = S in steps of 4.  Each wave owns 64 columns (four
// column tiles) for all atmosphere tiles, so every table value is read once from HBM.
//
// The stores are the traffic (n_atm contracted tables against one read of the S tables), so
// they are shaped for HBM: a D tile leaves each lane 4 atmospheres x 1 column, i.e. 4-row x
// 128-B pieces per store instruction; instead each wave parks its 16 x 64 D block in LDS
// (rows padded to 80 doubles: the two lane halves of a ds_write_b64 hit disjoint banks) and
// stores it back row by row, one atmosphere's 64 contiguous columns (512 B) per instruction.
typedef double dbl4 __attribute__((ext_vector_type(4)));

struct ContractBatchArgs {
  const double* tab[kMaxFastS];
  const double* mmr;      // [n_atm][S][n_layers]
  const int32_t* prow;    // [n_layers]
  double* eff;            // [n_atm] x tab_stride
  int S, n_layers, n_T, n_atm;
  int64_t pitch, tab_stride;
};

// 128 columns per wave, 16 B per lane per store: each store instruction writes one
// atmosphere's 128 contiguous columns (1 KiB); the 16 x 128 D block goes through LDS in two
// halves of 8 atmospheres (rows padded to 144 doubles: 1152 B = 128 B mod 256).  (64 columns
// with 8-B stores, and non-temporal stores: measured slower, profiles/r04/c5/.)
constexpr int kK7Cols = 128;
constexpr int kK7Row = kK7Cols + 16;
constexpr int kK7Rows = 8;
constexpr int kK7Tiles = kK7Cols / 16;
typedef double dbl2 __attribute__((ext_vector_type(2)));

template <int S>
__global__ __launch_bounds__(256) void contract_batch_kernel(ContractBatchArgs a) {
  __shared__ double tile[4][kK7Rows * kK7Row];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int l = blockIdx.y;
  const int64_t ncol = (int64_t)a.n_T * a.pitch;   // a multiple of 64 (pitch is)
  const int64_t col0 = ((int64_t)blockIdx.x * 4 + wv) * kK7Cols;
  const int64_t rowbase = (int64_t)a.prow[l] * ncol;
  const int ci = lane & 15, kq = lane >> 4;   // column in the tile, species in the K step
  // S is a template parameter: the species' table pointers are kernel-argument constants and
  // every load is unconditional (clamped column, zero weight for padded species), so all of
  // them are in flight at once — a runtime-indexed pointer array made each load a dependent
  // round trip (kernarg load, then the data, vmcnt(0) after each)
  constexpr int kSteps = (S + 3) / 4;
  const double* tp[kSteps];
#pragma unroll
  for (int ks = 0; ks < kSteps; ++ks) {
    const double* p = a.tab[0];
#pragma unroll
    for (int q = 0; q < 4; ++q)
      if (4 * ks + q < S && kq == q) p = a.tab[4 * ks + q];
    tp[ks] = p;
  }
  double b[kK7Tiles][kSteps];
#pragma unroll
  for (int t = 0; t < kK7Tiles; ++t)
#pragma unroll
    for (int ks = 0; ks < kSteps; ++ks) {
      const int64_t c = min(col0 + 16 * t + ci, ncol - 1);
      const double v = tp[ks][rowbase + c];
      b[t][ks] = (4 * ks + kq < S) ? v : 0.0;
    }
  double* my = tile[wv];
  for (int m0 = 0; m0 < a.n_atm; m0 += 16) {
    const int am = m0 + ci;                     // A operand row: atmosphere
    double av[kSteps];
#pragma unroll
    for (int ks = 0; ks < kSteps; ++ks) {
      const int s = 4 * ks + kq;
      av[ks] = (am < a.n_atm && s < S) ? a.mmr[((int64_t)am * S + s) * a.n_layers + l] : 0.0;
    }
    dbl4 acc[kK7Tiles];
#pragma unroll
    for (int t = 0; t < kK7Tiles; ++t) {
      acc[t] = dbl4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int ks = 0; ks < kSteps; ++ks)
        acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[ks], b[t][ks], acc[t], 0, 0, 0);
    }
    // D: this lane holds rows kq + 4 r (atmospheres) of column 16 t + ci
#pragma unroll
    for (int h = 0; h < 16 / kK7Rows; ++h) {
#pragma unroll
      for (int t = 0; t < kK7Tiles; ++t)
#pragma unroll
        for (int rr = 0; rr < kK7Rows / 4; ++rr)
          my[(kq + 4 * rr) * kK7Row + 16 * t + ci] = acc[t][h * (kK7Rows / 4) + rr];
      __syncthreads();
      const int mlo = m0 + h * kK7Rows;
      const int mrows = max(0, min(kK7Rows, a.n_atm - mlo));
      if (col0 + 2 * lane < ncol)
        for (int m = 0; m < mrows; ++m)
          *reinterpret_cast<dbl2*>(a.eff + (int64_t)(mlo + m) * a.tab_stride + rowbase + col0 +
                                   2 * lane) =
              *reinterpret_cast<const dbl2*>(my + m * kK7Row + 2 * lane);
      __syncthreads();   // the next half / atmosphere tile overwrites this wave's LDS block
    }
  }
}

// K7, VALU form: one lane per pair of adjacent columns (16-B loads and stores, 1 KiB per
// wave-instruction), the S table values held in registers and every atmosphere's sum formed in
// K3's species order — eff = mmr_0 tab_0, then eff + mmr_s tab_s — so each atmosphere's
// contracted table is bit for bit the one K3 builds for that atmosphere alone; the mixing
// ratios are wave-uniform (scalar loads).  The contraction is 0.125 flop per byte: HBM, not the
// arithmetic, bounds it, and this form reaches the store probe's rate (tools/store_probe.hip).
constexpr int kK7Chunk = 64;   // atmospheres whose mixing ratios are staged in LDS at a time

template <int S>
__global__ __launch_bounds__(256) void contract_batch_valu_kernel(ContractBatchArgs a) {
  __shared__ double smm[kK7Chunk * S];   // [atmosphere][species] of this layer
  const int l = blockIdx.y;
  const int64_t ncol = (int64_t)a.n_T * a.pitch;   // even (pitch is a multiple of 64)
  const int64_t c = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 2;
  const bool live = c < ncol;
  const int64_t at = (int64_t)a.prow[l] * ncol + (live ? c : 0);
  dbl2 v[S];
#pragma unroll
  for (int s = 0; s < S; ++s) v[s] = *reinterpret_cast<const dbl2*>(a.tab[s] + at);
  for (int m0 = 0; m0 < a.n_atm; m0 += kK7Chunk) {
    const int nm = min(kK7Chunk, a.n_atm - m0);
    if (m0 > 0) __syncthreads();   // the previous chunk's ratios are no longer read
    for (int q = threadIdx.x; q < nm * S; q += 256) {
      const int m = q / S, s = q - m * S;
      smm[q] = a.mmr[((int64_t)(m0 + m) * S + s) * a.n_layers + l];
    }
    __syncthreads();
    if (live)
      for (int m = 0; m < nm; ++m) {
        const double* mm = smm + m * S;
        dbl2 acc = mm[0] * v[0];
#pragma unroll
        for (int s = 1; s < S; ++s) acc = acc + mm[s] * v[s];
        *reinterpret_cast<dbl2*>(a.eff + (int64_t)(m0 + m) * a.tab_stride + at) = acc;
      }
  }
}

void launch_contract_batch_valu(const double* const* tabs, int S, const double* mmr,
                                const int32_t* prow, int n_layers, int n_T, int64_t pitch,
                                int n_atm, int64_t tab_stride, double* eff, hipStream_t st) {
  ContractBatchArgs a{};
  for (int s = 0; s < S && s < kMaxFastS; ++s) a.tab[s] = tabs[s];
  a.mmr = mmr;
  a.prow = prow;
  a.eff = eff;
  a.S = S;
  a.n_layers = n_layers;
  a.n_T = n_T;
  a.n_atm = n_atm;
  a.pitch = pitch;
  a.tab_stride = tab_stride;
  const int64_t ncol = (int64_t)n_T * pitch;
  dim3 grid((unsigned)((ncol / 2 + 255) / 256), (unsigned)n_layers);
  switch (S) {
#define K7V(n) case n: hipLaunchKernelGGL(contract_batch_valu_kernel<n>, grid, dim3(256), 0, st, a); break;
    K7V(1) K7V(2) K7V(3) K7V(4) K7V(5) K7V(6) K7V(7)
    default: hipLaunchKernelGGL(contract_batch_valu_kernel<8>, grid, dim3(256), 0, st, a);
#undef K7V
  }
}

void launch_contract_batch(const double* const* tabs, int S, const double* mmr,
                           const int32_t* prow, int n_layers, int n_T, int64_t pitch,
                           int n_atm, int64_t tab_stride, double* eff, hipStream_t st) {
  ContractBatchArgs a{};
  for (int s = 0; s < S && s < kMaxFastS; ++s) a.tab[s] = tabs[s];
  a.mmr = mmr;
  a.prow = prow;
  a.eff = eff;
  a.S = S;
  a.n_layers = n_layers;
  a.n_T = n_T;
  a.n_atm = n_atm;
  a.pitch = pitch;
  a.tab_stride = tab_stride;
  const int64_t ncol = (int64_t)n_T * pitch;
  dim3 grid((unsigned)((ncol + 4 * kK7Cols - 1) / (4 * kK7Cols)), (unsigned)n_layers);
  switch (S) {
#define K7M(n) case n: hipLaunchKernelGGL(contract_batch_kernel<n>, grid, dim3(256), 0, st, a); break;
    K7M(1) K7M(2) K7M(3) K7M(4) K7M(5) K7M(6) K7M(7)
    default: hipLaunchKernelGGL(contract_batch_kernel<8>, grid, dim3(256), 0, st, a);
#undef K7M
  }
}

__global__ void fill_kernel(double* x, int64_t n, double v) {
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < n;
       idx += (int64_t)gridDim.x * blockDim.x)
    x[idx] = v;
}

// ---------------------------------------------------------------- launchers
template <int DIR, int S, bool FAST>
static void launch_sweep_t(const SweepArgs& a, int nblocks, hipStream_t st) {
  const size_t shm = (size_t)(kBlock / 64) * a.n_steps * 4 * sizeof(double);
  hipLaunchKernelGGL((sweep_kernel<DIR, S, FAST>), dim3(nblocks), dim3(kBlock), shm, st, a);
}

template <int DIR>
static void launch_sweep_dir(const SweepArgs& a, int nblocks, bool, hipStream_t st) {
  launch_sweep_t<DIR, 1, false>(a, nblocks, st);
}

void launch_sweep(int dir, const SweepArgs& a, int nblocks, bool fast, hipStream_t st) {
  if (dir == kEmit) launch_sweep_dir<kEmit>(a, nblocks, fast, st);
  else launch_sweep_dir<kAbsorb>(a, nblocks, fast, st);
}

template <int DIR, int S, int PD, bool NC, bool SH, bool MM1 = false, int PF = PD>
static void launch_fast_t(const FastArgs& a, int nblocks, hipStream_t st) {
  const size_t shm = (size_t)red_lds_doubles(a.red_rows, a.n_steps) * sizeof(double) +
                     (SH ? (size_t)a.n_steps * sizeof(FastStepS) +
                               (size_t)rec_scratch_doubles(a) * sizeof(double)
                         : 0);
  const auto kernel = sweep_fast_kernel<DIR, S, PD, NC, SH, MM1, PF>;
  hipLaunchKernelGGL(kernel, dim3(nblocks, a.n_atm > 1 ? a.n_atm : 1), dim3(kBlock),
                     sweep_shm(reinterpret_cast<const void*>(kernel), a, shm), st, a, a.steps,
                     a.ssteps, a.F_up, a.F_down, a.part, a.dtaus);
}

// the contracted one-table sweep (S = 1, unit mmr) with prefetch distance pf (0: = PD)
template <int DIR, int PD, bool SH>
static void launch_fast_pf(int pf, const FastArgs& a, int nblocks, hipStream_t st) {
  if (pf >= 16) return launch_fast_t<DIR, 1, PD, false, SH, true, 16>(a, nblocks, st);
  if (pf >= 8) return launch_fast_t<DIR, 1, PD, false, SH, true, 8>(a, nblocks, st);
  return launch_fast_t<DIR, 1, PD, false, SH, true, PD>(a, nblocks, st);
}

template <int DIR, int PD, bool NC, bool SH>
static void launch_fast_dir(int S, const FastArgs& a, int nblocks, hipStream_t st) {
  switch (S) {
    case 1:
      if (a.unit_mmr && !NC) return launch_fast_t<DIR, 1, PD, false, SH, true>(a, nblocks, st);
      return launch_fast_t<DIR, 1, PD, NC, SH>(a, nblocks, st);
    case 2: return launch_fast_t<DIR, 2, PD, NC, SH>(a, nblocks, st);
    case 3: return launch_fast_t<DIR, 3, PD, NC, SH>(a, nblocks, st);
    case 4: return launch_fast_t<DIR, 4, PD, NC, SH>(a, nblocks, st);
    case 5: return launch_fast_t<DIR, 5, PD, NC, SH>(a, nblocks, st);
    case 6: return launch_fast_t<DIR, 6, PD, NC, SH>(a, nblocks, st);
    case 7: return launch_fast_t<DIR, 7, PD, NC, SH>(a, nblocks, st);
    default: return launch_fast_t<DIR, 8, PD, NC, SH>(a, nblocks, st);
  }
}

template <int PD, bool NC, bool SH>
static void launch_fast_pd(int dir, int S, const FastArgs& a, int nblocks, hipStream_t st) {
  if (dir == kEmit) launch_fast_dir<kEmit, PD, NC, SH>(S, a, nblocks, st);
  else launch_fast_dir<kAbsorb, PD, NC, SH>(S, a, nblocks, st);
}

template <bool SH>
static void launch_fast_sh(int dir, int S, int depth, int pf, bool nan_check, const FastArgs& a,
                           int nblocks, hipStream_t st) {
  if (pf > depth && S == 1 && a.unit_mmr && !nan_check && depth >= 2) {
    // the contracted table with loads issued pf steps ahead
    if (depth >= 4) {
      if (dir == kEmit) launch_fast_pf<kEmit, 4, SH>(pf, a, nblocks, st);
      else launch_fast_pf<kAbsorb, 4, SH>(pf, a, nblocks, st);
    } else {
      if (dir == kEmit) launch_fast_pf<kEmit, 2, SH>(pf, a, nblocks, st);
      else launch_fast_pf<kAbsorb, 2, SH>(pf, a, nblocks, st);
    }
    return;
  }
  if (depth == 1 && pf == 2 && S == 1 && a.unit_mmr && !nan_check) {
    // one step per coefficient block, loads two steps ahead (fewer registers: 5 waves per SIMD)
    if (dir == kEmit) launch_fast_t<kEmit, 1, 1, false, SH, true, 2>(a, nblocks, st);
    else launch_fast_t<kAbsorb, 1, 1, false, SH, true, 2>(a, nblocks, st);
    return;
  }
  if (depth >= 4 && S == 1 && !nan_check) {  // 4 steps in flight: small slices, one table
    if (a.unit_mmr) {
      if (dir == kEmit) launch_fast_t<kEmit, 1, 4, false, SH, true>(a, nblocks, st);
      else launch_fast_t<kAbsorb, 1, 4, false, SH, true>(a, nblocks, st);
    } else {
      if (dir == kEmit) launch_fast_t<kEmit, 1, 4, false, SH>(a, nblocks, st);
      else launch_fast_t<kAbsorb, 1, 4, false, SH>(a, nblocks, st);
    }
  } else if (depth >= 2) {
    if (nan_check) launch_fast_pd<2, true, SH>(dir, S, a, nblocks, st);
    else launch_fast_pd<2, false, SH>(dir, S, a, nblocks, st);
  } else {
    if (nan_check) launch_fast_pd<1, true, SH>(dir, S, a, nblocks, st);
    else launch_fast_pd<1, false, SH>(dir, S, a, nblocks, st);
  }
}

void launch_sweep_fast(int dir, int S, int depth, int pf, bool nan_check, bool shared,
                       const FastArgs& a, int nblocks, hipStream_t st) {
  if (shared) launch_fast_sh<true>(dir, S, depth, pf, nan_check, a, nblocks, st);
  else launch_fast_sh<false>(dir, S, depth, pf, nan_check, a, nblocks, st);
}

__global__ void nan_scan_kernel(const double* __restrict__ x, int64_t n, int* flag) {
  int found = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    found |= isnan(x[i]) ? 1 : 0;
  if (__any(found) && (threadIdx.x & 63) == 0) atomicOr(flag, 1);
}

void launch_nan_scan(const double* x, int64_t n, int* flag, hipStream_t st) {
  hipLaunchKernelGGL(nan_scan_kernel, dim3(2048), dim3(256), 0, st, x, n, flag);
}

void launch_reduce(const double* part, int nblocks, double* Fb, int n_idx, const int* conv,
                   int force, hipStream_t st, int n_atm, int64_t part_stride,
                   int64_t fb_stride, const P2PPush* push) {
  P2PPush p{};
  if (push) p = *push;
  hipLaunchKernelGGL(reduce_kernel, dim3(n_idx, n_atm), dim3(kRedThreads), 0, st, part, nblocks, Fb,
                     conv, force, part_stride, fb_stride, p);
}

void launch_setup(const SetupArgs& u, int dir, hipStream_t st, int n_atm) {
  hipLaunchKernelGGL(setup_kernel, dim3(n_atm), dim3(256), 0, st, u, dir);
}

void launch_update(const UpdateArgs& a, hipStream_t st, int n_atm) {
  const size_t shm = update_lds_bytes(a.su.n_layers, a.su.n_tnodes, a.su.n_species,
                                      a.meta_in_lds != 0);
  hipLaunchKernelGGL(update_kernel, dim3(n_atm), dim3(256), shm, st, a);
}

void launch_update_fused(const UpdateArgs& a, hipStream_t st) {
  const size_t shm = (2 * (size_t)a.su.n_layers + a.su.n_tnodes) * sizeof(double);
  hipLaunchKernelGGL(update_fused_kernel, dim3(a.su.n_layers), dim3(kRedThreads), shm, st, a);
}

void launch_propagate(int64_t n, const double* c1, const double* lk, const double* F1u,
                      const double* F2d, double T1, double T2, const double* dtau,
                      const double* w0, const double* g0, double* F2u, double* F1d,
                      hipStream_t st) {
  const int nb = (int)((n + 255) / 256);
  hipLaunchKernelGGL(propagate_kernel, dim3(nb), dim3(256), 0, st, n, c1, lk, F1u, F2d, T1,
                     T2, dtau, w0, g0, F2u, F1d);
}

void launch_kappa(int64_t n, const TermP* terms, int nS, const double* sig, double* k,
                  hipStream_t st) {
  const int nb = (int)((n + 255) / 256);
  hipLaunchKernelGGL(kappa_kernel, dim3(nb), dim3(256), 0, st, n, terms, nS, sig, k);
}

void launch_gen_table(double* tab, const double* base, const double* fp, const double* fT,
                      int n_p, int n_T, int64_t n_lam, int64_t stride, double lo, double hi,
                      hipStream_t st) {
  hipLaunchKernelGGL(gen_table_kernel, dim3(4096), dim3(256), 0, st, tab, base, fp, fT, n_p,
                     n_T, n_lam, stride, lo, hi);
}

void launch_fill(double* x, int64_t n, double v, hipStream_t st) {
  const int nb = (int)std::min<int64_t>((n + 255) / 256, 4096);
  hipLaunchKernelGGL(fill_kernel, dim3(nb > 0 ? nb : 1), dim3(256), 0, st, x, n, v);
}

}  // namespace frei

#ifdef FREI_TRACE
// Diagnostic builds only: copy out (and reset) the trace ring.  rec: n_max x 8 int64
// (kind, block, 4 wall-clock marks, 2 shader-cycle stamps at entry and exit); *n: records
// written since the last reset.
extern "C" int frei_trace_fetch(long long* rec, int n_max, int* n) {
  unsigned cnt = 0;
  if (hipMemcpyFromSymbol(&cnt, HIP_SYMBOL(frei::g_trace_n), sizeof(cnt)) != hipSuccess) return -1;
  const unsigned m = cnt < (unsigned)n_max ? cnt : (unsigned)n_max;
  if (m && hipMemcpyFromSymbol(rec, HIP_SYMBOL(frei::g_trace), m * sizeof(frei::TraceRec)) !=
               hipSuccess)
    return -1;
  *n = (int)cnt;
  const unsigned zero = 0;
  return hipMemcpyToSymbol(HIP_SYMBOL(frei::g_trace_n), &zero, sizeof(zero)) == hipSuccess ? 0 : -1;
}
// the producer/consumer sweep's per-phase stamps: [dir][8 sampled blocks][16 waves][1 + 24][2]
extern "C" int frei_ptrace_fetch(long long* out, int n_max) {
  const size_t n = sizeof(frei::g_ptrace) / sizeof(long long);
  if ((size_t)n_max < n) return -1;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(frei::g_ptrace), sizeof(frei::g_ptrace)) == hipSuccess
             ? (int)n
             : -1;
}
#endif
