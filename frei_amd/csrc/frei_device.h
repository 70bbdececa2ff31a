// frei_device.h — shared host/device definitions of the frei MI355X engine.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <string>

// The sweeps' coefficient form (frei_kernels.hip StepCoef): 1 = premultiplied by 1/chi and
// pi_w (two fma per flux update), 0 = the reference's literal association.
namespace frei {

// CODATA 2018 (astropy 4.3.1, the reference's unit backend), cgs.
constexpr double kH = 6.62607015e-27;
constexpr double kC = 29979245800.0;
constexpr double kHC = kH * kC;                       // h*c, as the reference forms it
constexpr double kKB = 1.380649e-16;
constexpr double kMP = 1.67262192369e-24;
constexpr double kMbarDefault = 2.4 * kMP;            // twostream.py:23 default m_bar
constexpr double kSigmaSB = 5.6703744191844314e-05;   // astropy sigma_sb in cgs
constexpr double kPi = 3.141592653589793;

constexpr int kEmit = 0;
constexpr int kAbsorb = 1;
constexpr int kBlock = 256;  // 4 wave64 per workgroup
constexpr int kMaxLayers = 1024;

// Sweep step k -> layer index (emit: twostream.py:356, absorb: :491).
__host__ __device__ inline int step_layer(int dir, int k, int nL) {
  return dir == kEmit ? k + 1 : nL - 2 - k;
}
// The step of direction `dir` whose layer is i (inverse of step_layer), -1 if layer i has none
// (emit: layer 0; absorb: the top layer).
__host__ __device__ inline int layer_step(int dir, int i, int nL) {
  const int k = dir == kEmit ? i - 1 : nL - 2 - i;
  return (k >= 0 && k < nL - 1) ? k : -1;
}

// Per sweep step, wave-uniform.
struct StepP {
  double iT1, iT2;  // 1 / T of the step's two layers, K^-1 (the Planck exponent hc/(lam k) * (1/T))
  double dm;      // (p1 - p2) / g, g cm^-2 (twostream.py:227-231)
  int32_t layer;  // i
  int32_t top;    // emit top layer: F_2_down = F_TOA, F_2_up not stored (Q3)
  int64_t pad;
};

// Fast-path sweep step (every species: on-node pressure, >= 2 T nodes, S <= kMaxFastS):
// two T-bracket rows per species, row_hi = row_lo + n_lam (T axis stored ascending).
constexpr int kMaxFastS = 8;
struct FastStep {
  double iT1, iT2, dm;     // 1 / T of the step's two layers (K^-1), (p1 - p2) / g
  int32_t layer, top;
  double wlo[kMaxFastS], whi[kMaxFastS], mmr[kMaxFastS];
  int64_t off[kMaxFastS];  // element offset of the T_lo row in species s's table
};

// Shared-bracket fast step: every species has the same pressure and temperature nodes (the
// usual case: tables binned onto the grid), so one row offset and one weight pair serve all
// species; 15 uniform values per step fit SGPRs and are prefetched with the table rows.
struct FastStepS {
  double iT1, iT2, dm, wlo, whi;   // 1 / T of the two layers (K^-1), ...
  int64_t off;             // element offset of the T_lo row (same in every species table)
  int32_t layer, top;
  double mmr[kMaxFastS];
};
static_assert(sizeof(FastStepS) % sizeof(double) == 0, "FastStepS is staged as doubles");

// Interpolation term of one species at one layer (opacity.py:250-263).
struct TermP {
  const double* row[4];  // table rows (device pointers), corner order of scipy interpn
  double w[4];           // weights (1 * w_p) * w_T
  double mmr;            // mass mixing ratio
  double x1, dx;         // single-T mode: p - p_lo, p_hi - p_lo (scipy interp1d)
  int32_t nrow;          // rows used (0 = outside the hull); -1 = single-T mode
  int32_t pad;
};

// Per species metadata.
struct SpecMeta {
  const double* tab;  // [n_p][n_T][n_lam] device, rows padded to n_lam (row pitch)
  int64_t n_lam;      // row pitch in elements
  int32_t n_p, n_T;
  int32_t t_off;      // offset of this species' sorted T nodes in tnodes/tperm
  int32_t one_T;      // single unique temperature -> pressure-only interpolation
};

// Pressure bracket of one species at one layer (T independent, computed at load time).
struct PMeta {
  int32_t p_lo, p_hi;    // table pressure rows (memory index) of the bracket
  double wp_lo, wp_hi;   // scipy weights (1 - y, y)
  double x1, dx;         // interp1d form for single-T tables
  int32_t oob;           // outside the pressure hull -> fill 0
  int32_t pad;
};

// scipy RegularGridInterpolator._find_indices on an ascending grid (searchsorted left).
__host__ __device__ inline void bracket(const double* g, int n, double x, int& i, double& y,
                                        int& oob) {
  int lo = 0, hi = n;  // number of nodes < x
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (g[mid] < x) lo = mid + 1; else hi = mid;
  }
  i = lo - 1;
  if (i < 0) i = 0;
  if (i > n - 2) i = n - 2;
  y = (x - g[i]) / (g[i + 1] - g[i]);
  oob = (x < g[0] || x > g[n - 1]) ? 1 : 0;
}

// Build the interpolation term at temperature T.  With `fast`, the result always has
// two rows (the T bracket in the on-node pressure slab), OOB encoded as zero weights.
__host__ __device__ inline TermP make_term(const SpecMeta& sm, const PMeta& pm,
                                           const double* tnodes, const int32_t* tperm,
                                           double mmr, double T, int fast) {
  TermP t;
  for (int r = 0; r < 4; ++r) { t.row[r] = sm.tab; t.w[r] = 0.0; }
  t.mmr = mmr;
  t.x1 = 0.0;
  t.dx = 1.0;
  t.nrow = 0;
  t.pad = 0;
  const int64_t rowlen = sm.n_lam;
  if (sm.one_T) {
    if (pm.oob) return t;
    const int tp = tperm[sm.t_off];
    t.row[0] = sm.tab + ((int64_t)pm.p_lo * sm.n_T + tp) * rowlen;
    t.row[1] = sm.tab + ((int64_t)pm.p_hi * sm.n_T + tp) * rowlen;
    t.x1 = pm.x1;
    t.dx = pm.dx;
    t.nrow = -1;
    return t;
  }
  int it, oobT;
  double yt;
  bracket(tnodes + sm.t_off, sm.n_T, T, it, yt, oobT);
  if (pm.oob || oobT) {
    if (fast) t.nrow = 2;  // zero weights on valid rows
    return t;
  }
  const int tlo = tperm[sm.t_off + it], thi = tperm[sm.t_off + it + 1];
  const int pr[2] = {pm.p_lo, pm.p_hi};
  const double wp[2] = {pm.wp_lo, pm.wp_hi};
  const int tr[2] = {tlo, thi};
  const double wt[2] = {1.0 - yt, yt};
  int n = 0;
  for (int a = 0; a < 2; ++a) {
    if (wp[a] == 0.0) continue;  // on-node pressure: the other slab has weight 0
    for (int b = 0; b < 2; ++b) {
      t.row[n] = sm.tab + ((int64_t)pr[a] * sm.n_T + tr[b]) * rowlen;
      t.w[n] = (1.0 * wp[a]) * wt[b];
      ++n;
    }
  }
  t.nrow = n;
  return t;
}

// Fast-path term (on-node pressure, >= 2 T nodes): T_lo row offset and the two weights.
// Same arithmetic as make_term (weights (1.0 * wp) * wT), no runtime-indexed arrays.
__host__ __device__ inline void fast_term(const SpecMeta& sm, const PMeta& pm,
                                          const double* tnodes, double T, int64_t& off,
                                          double& wlo, double& whi) {
  int it, oobT;
  double yt;
  bracket(tnodes + sm.t_off, sm.n_T, T, it, yt, oobT);
  off = 0;
  wlo = whi = 0.0;
  if (pm.oob || oobT) return;  // fill 0: zero weights on valid rows
  const int prow = (pm.wp_lo != 0.0) ? pm.p_lo : pm.p_hi;
  const double wp = (pm.wp_lo != 0.0) ? pm.wp_lo : pm.wp_hi;
  off = ((int64_t)prow * sm.n_T + it) * sm.n_lam;  // T axis stored ascending
  wlo = (1.0 * wp) * (1.0 - yt);
  whi = (1.0 * wp) * yt;
}

// Per-atmosphere element strides of the batched engine (one context holding n_atm
// atmospheres on a shared wavelength/pressure grid and shared opacity tables, each with its
// own temperatures, gravity, mixing ratios and fluxes; §8(f) #2).  All zero (and g null)
// for a single atmosphere, so every kernel's atmosphere view is the identity there.
struct AtmStride {
  int64_t layers;    // [n_layers] state: T, Tb, Ta, flips, prev sign, n diffs
  int64_t steps;     // step tables [n_layers - 1]
  int64_t fb;        // reduced bolometric partials [n_steps * 4]
  int64_t hist;      // T history [hist_cap][2][n_layers]
  int64_t flux;      // F_up / F_down / dtaus [n_layers][n_lam]
  int64_t tab;       // contracted opacity table
  int64_t part;      // block partial sums [n_steps * 4][blocks]
  int64_t ftoa;      // per-atmosphere F_TOA [n_lam] (0: one F_TOA shared by all)
  const double* g;   // per-atmosphere gravity (nullptr: SetupArgs.g)
};

// Temperature-dependent chemistry (the reference calls chemistry(T, p) inside every kappa,
// opacity.py:246-248): mass mixing ratios tabulated on (T, p) nodes, interpolated at each
// sweep step's layer (T_i, p_i) when the update kernel writes the next sweep's step table —
// linear in T and in log10 p, clamped to the node range.  tab == nullptr: the fixed
// per-layer mmr arrays of frei_set_mmr.
struct ChemArgs {
  const double* tab;       // [n_species][n_T][n_p]
  const double* T;         // [n_T] ascending (K)
  const int32_t* pj;       // [n_layers] pressure bracket of each layer (node index)
  const double* pz;        // [n_layers] weight of node pj + 1 (log10 p)
  int n_T, n_p;
};

// Bracket of x on ascending nodes g[n] clamped to [g0, g_{n-1}]: node i <= n - 2 and the
// weight y of node i + 1 (0 when n == 1).
__host__ __device__ inline void chem_bracket(const double* g, int n, double x, int& i,
                                             double& y) {
  i = 0;
  y = 0.0;
  if (n < 2) return;
  const double xc = x < g[0] ? g[0] : (x > g[n - 1] ? g[n - 1] : x);
  int lo = 0, hi = n - 2;   // largest i in [0, n-2] with g[i] <= xc
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (g[mid] <= xc) lo = mid; else hi = mid - 1;
  }
  i = lo;
  y = (xc - g[i]) / (g[i + 1] - g[i]);
}

// mmr of species s at layer i (pressure bracket pj[i], pz[i]) and temperature T:
// ((v00 (1 - z) + v01 z) (1 - y) + (v10 (1 - z) + v11 z) y), exact order (oracle/frei_oracle.py
// ChemistryTable restates it).
__host__ __device__ inline double chem_mmr_at(const ChemArgs& c, int s, int j, double z,
                                              double T) {
  int it;
  double y;
  chem_bracket(c.T, c.n_T, T, it, y);
  const double* v = c.tab + ((int64_t)s * c.n_T + it) * c.n_p;
  auto row = [&](const double* r) { return c.n_p > 1 ? r[j] * (1.0 - z) + r[j + 1] * z : r[0]; };
  const double a = row(v);
  return c.n_T > 1 ? a * (1.0 - y) + row(v + c.n_p) * y : a;
}

struct SetupArgs {
  ChemArgs chem;           // T-dependent chemistry (chem.tab == nullptr: fixed mmr)
  int n_layers, n_species, fast;
  int n_tnodes;            // total sorted T nodes over species (tnodes length)
  double* T;               // device temperatures [n_layers]
  const double* p;         // device pressures (dyn cm^-2)
  double p_top2, g;
  const SpecMeta* spec;
  const PMeta* pmeta;      // [n_species][n_layers]
  const double* tnodes;
  const int32_t* tperm;
  const double* mmr;       // [n_species][n_layers]
  StepP* steps;            // [n_layers - 1]
  TermP* terms;            // [n_layers - 1][n_species]
  FastStep* fsteps;        // [n_layers - 1] (fast path)
  FastStepS* ssteps;       // [n_layers - 1] (fast path, shared brackets)
  int shared;              // all species share p and T nodes
  AtmStride bs;            // batched atmospheres (blockIdx.x of setup/update kernels)
  // Lazy K3 (round 6): [n_p * n_T] 1 where the contracted row (pressure row, T node) holds
  // its values (nullptr: the whole table was contracted up front).  Records written from T get
  // the mask of their two rows not yet contracted in off[1] (bit 0: T_lo row, bit 1: T_hi row);
  // an update marks the rows the sweep before it used.  kpitch: the tables' row pitch.
  int32_t* kvalid;
  int64_t kpitch;
};

struct FastArgs {
  int64_t n_lam;
  int64_t pitch;           // table row pitch (elements), even
  int n_steps, force;
  int live_only;           // skip flux stores no later sweep reads (T-P loop only)
  const double *c1, *hcl, *sig, *wtr, *ftoa;   // hcl = hc / (lam k_B)
  const double* tab[kMaxFastS];
  const FastStep* steps;
  const FastStepS* ssteps;
  double* F_up;
  double* F_down;
  double* dtaus;
  double* part;
  const int* conv;
  AtmStride bs;            // batched atmospheres (blockIdx.y of the sweep kernels)
  int n_atm;               // atmospheres in the launch (0 or 1: a single atmosphere)
  int red_rows;            // one-lane sweep: per-row partial sums in LDS (fits: few layers)
  int unit_mmr;            // S = 1 with mmr = 1 everywhere (the contracted table, K3)
  // rec_on: the sweep forms its own step records from the current temperatures in its
  // prologue (contracted table, shared brackets, fixed mmr) instead of reading the ones the
  // previous update kernel wrote; rec holds the setup inputs (T of this sweep).
  int rec_on;
  SetupArgs rec;
  int min_lds;             // minimum dynamic LDS bytes per block (caps blocks per CU; launch only)
  // Chained launch (sweep_chain_kernel: its leading workgroups run the previous sweep's fused
  // update): the sweep blocks poll rec.T — kPoisonT until that update publishes each value —
  // and *ch_epoch for its convergence decision, instead of waiting for a kernel boundary.
  const unsigned long long* ch_epoch;   // [n_layers] the update's granules; nullptr: not chained
  unsigned long long ch_val;            // epoch value this launch waits for
  int ch_can_conv;                      // the update is the convergence test (tracked absorb)
  long long ch_timeout;                 // wall_clock64 ticks before a wait gives up
  int* ch_err;                          // set to 1 when a wait gave up
  // the deferred update's output temperatures: block 0 fills them with kPoisonT (nullptr: none)
  double* poison;
  // Lazy K3 (sweep_pair_kernel): a step whose record masks rows not yet contracted (off[1])
  // contracts them for the lane's own wavelengths first — K3's sum, same order — into tab[0]
  // (kmmr == nullptr: every row is contracted)
  const double* ktab[kMaxFastS];
  const double* kmmr;      // [n_species][n_layers]
  int kS, kNL;
  // Trailing update (sweep_pipe_tail_kernel, round 6): the sweep blocks publish each phase's
  // per-block partial sums into tail_part as soon as the phase is done (write-through stores,
  // every slot kPoisonT until then), so the launch's trailing update workgroups can start a
  // layer's reduction while the sweep is still in flight (nullptr: partials into `part` at the
  // end, as every other form)
  double* tail_part;
};
// "not yet published" pattern of a chained temperature: a signalling NaN, which no arithmetic
// produces (results are quiet NaNs), so a diverged run's NaN temperature is still a value
constexpr unsigned long long kPoisonT = 0xFFF4F4F4F4F4F4F4ull;

struct SweepArgs {
  int64_t n_lam;
  int n_steps, n_species, force;
  int live_only;
  const double *c1, *hcl, *sig, *wtr, *ftoa;   // hcl = hc / (lam k_B)
  const StepP* steps;
  const TermP* terms;
  double* F_up;
  double* F_down;
  double* dtaus;           // optional [n_layers][n_lam]
  double* part;            // [n_steps*4][nblocks]
  const int* conv;
};

// P2P exchange of the per-sweep bolometric partial sums over xGMI, no RCCL and no host in the
// loop.  Every rank owns a mailbox in uncached device memory that every other
// rank has mapped through an IPC handle; per sweep each rank pushes its n sums into slot
// [rank] of every mailbox, then a sequence flag per value, and polls its own mailbox until
// every rank's flags carry the sweep's sequence number, summing the ranks in rank order (the
// fused update kernel does both, one workgroup per layer; with fused_update 0 the reduce
// kernel pushes and the update kernel waits).  Two parity slots: a rank can run at most one sweep ahead of another
// (its next update needs everyone's next sums), so slot seq & 1 is never overwritten while a
// slower rank still reads it.
struct P2PPush {
  double* const* peers;    // [nranks] every rank's mailbox (own included), device pointers
  int nranks, rank;
  int64_t n;               // sums per rank (n_steps * 4)
  uint64_t seq;            // this sweep's sequence number (> 0); nullptr peers: no push
};
struct P2PWait {
  const double* mbox;      // this rank's mailbox (nullptr: no P2P exchange)
  int nranks;
  int64_t n;
  uint64_t seq;
  int64_t timeout_ticks;   // wall_clock64 ticks before a missing peer is reported
  int* err;                // set to 1 when a peer never published (timeout)
  unsigned long long* wait_ticks;  // accumulated ticks thread 0 spent waiting (diagnostic)
};
// mailbox layout: values [2][nranks][n] doubles, then flags [2][nranks][n] uint64
__host__ __device__ inline int64_t mbox_val(int par, int r, int R, int64_t n) {
  return ((int64_t)par * R + r) * n;
}
__host__ __device__ inline int64_t mbox_flag(int par, int r, int R, int64_t n) {
  return 2 * (int64_t)R * n + ((int64_t)par * R + r) * n;
}
__host__ __device__ inline size_t mbox_bytes(int R, int64_t n) { return (size_t)4 * R * n * 8; }

struct UpdateArgs {
  SetupArgs su;
  P2PWait p2p;
  int dir, next_dir, nranks, force, track, stop_on_conv, n_zero_crossings, hist_cap;
  int meta_in_lds;         // per-(species, layer) metadata staged in LDS (small grids)
  double m_bar, alpha, convergence_dT;
  const double* Fb;        // [nranks][n_steps*4]
  const double* lnp;       // [n_layers] log(p_l / p_{l+1}) (top: emit's p_2)
  double* dT_out;          // [n_layers] optional
  double* bol_out;         // [n_layers][4] optional
  double *Tb, *Ta, *hist;
  int32_t *flips, *prev_sign, *ndiff;
  int* iter;
  int* conv;
  // fused reduce + update (launch_update_fused): the sweep's per-block partials, the P2P push
  // of this rank's sums, the output temperature buffer (T_in is su.T) and the arrival counter
  const double* part;      // [n_steps*4][nblocks]
  int nblocks;
  P2PPush push;
  double* T_out;
  unsigned* done;
  // chained into the next sweep's launch (sweep_chain_kernel): T_out published by sc1 stores,
  // and per layer l the granule epoch[l] = (epoch_val << 2) | (converged before << 1) |
  // (layer converged) (nullptr: a launch of its own)
  unsigned long long* epoch;
  unsigned long long epoch_val;
  // trailing update in the sweep's own launch (sweep_pipe_tail_kernel): the partials are polled
  // until no slot holds kPoisonT (each 8-byte value is its own ready flag), bounded by
  // poll_timeout wall_clock64 ticks, after which *poll_err is set and the value is used as is
  int poll;
  long long poll_timeout;
  int* poll_err;
};

// LDS bytes of the update kernel (K4/K5): T, dT, p, T before/after absorb, ln p ratios,
// sorted T nodes, rank-summed partials, 3 int state arrays; then (meta) the per-(species,
// layer) pressure brackets and mixing ratios and the species metadata.
__host__ __device__ inline size_t update_lds_bytes(int nL, int ntn, int S, bool meta) {
  size_t b = (size_t)(8 * nL + ntn + 4 * (nL - 1)) * sizeof(double) + 3 * (size_t)nL * sizeof(int);
  b = (b + 15) & ~(size_t)15;
  if (meta) b += (size_t)S * nL * (sizeof(PMeta) + sizeof(double)) + (size_t)S * sizeof(SpecMeta);
  return b;
}

// Per-block partial sums of a sweep, [blocks][steps x 4]: each block writes its ns x 4 values
// as whole cache lines; an update workgroup reads its layer's 8 values of every block, one
// 64-byte span each (round 4; rounds 1-3 stored [steps x 4][blocks]).
__host__ __device__ inline int64_t part_at(int idx, int bx, int nbx, int ns4) {
  (void)nbx;
  return (int64_t)bx * ns4 + idx;
}

// launchers (frei_kernels.hip)
void launch_sweep(int dir, const SweepArgs& a, int nblocks, bool fast, hipStream_t st);
void launch_sweep_fast(int dir, int S, int depth, int pf, bool nan_check, bool shared,
                       const FastArgs& a, int nblocks, hipStream_t st);
// The contracted one-lane sweep with two adjacent wavelengths per lane (even n_lam, global step
// records, staged partial sums: a.red_rows = 2); nblocks = ceil(n_lam / (2 kBlock)).
void launch_sweep_pair(int dir, const FastArgs& a, int nblocks, hipStream_t st);
// Grouped-lane sweep (Q = 2 or 4 lanes per wavelength, NW = 4 or 8 waves per block, 64 NW / Q
// wavelengths per block):
// contracted single table, step table in LDS; for slices with about one wave per SIMD.
void launch_sweep_group(int dir, int Q, int NW, const FastArgs& a, int nblocks, hipStream_t st);
// The grouped-lane sweep chained to the previous sweep's fused update u (one launch: u's
// workgroups first, then the sweep blocks, which poll the new temperatures; single atmosphere).
void launch_sweep_chain(int dir, int Q, int NW, const FastArgs& a, const UpdateArgs& u,
                        int nblocks, hipStream_t st);
// The producer/consumer sweep (NC = 4) chained likewise.
void launch_sweep_pipe_chain(int dir, int PF, const FastArgs& a, const UpdateArgs& u,
                             int nblocks, hipStream_t st);
// The one-lane contracted sweep (step records formed in the block) chained likewise.
void launch_sweep_fast_chain(int dir, int depth, int pf, const FastArgs& a, const UpdateArgs& u,
                             int nblocks, hipStream_t st);
// producer/consumer sweep: NC consumer waves (64 NC wavelengths) per block, table rows PF
// phases ahead
void launch_sweep_pipe(int dir, int NC, int PF, const FastArgs& a, int nblocks, hipStream_t st);
size_t pipe_lds_bytes(int NC, int M, int ns);
// The producer/consumer sweep (NC = 4) with its fused update u as n_tail trailing workgroups of
// the same launch (u.poll: the update polls each phase's partials as the sweep publishes them
// into a.tail_part; the trailing workgroups refill `clear` — the previous launch's partials —
// with kPoisonT).  nbx sweep blocks; single atmosphere.
void launch_sweep_pipe_tail(int dir, int PF, const FastArgs& a, const UpdateArgs& u, int nbx,
                            int n_tail, double* clear, hipStream_t st);
size_t pipe_tail_lds_bytes(int ns, int n_tnodes);
void launch_poison(double* x, int64_t n, hipStream_t st);
void launch_nan_scan(const double* x, int64_t n, int* flag, hipStream_t st);
void launch_reduce(const double* part, int nblocks, double* Fb, int n_idx, const int* conv,
                   int force, hipStream_t st, int n_atm = 1, int64_t part_stride = 0,
                   int64_t fb_stride = 0, const P2PPush* push = nullptr);
// One tiny launch that publishes flag value `seq` for this rank in every mailbox and waits
// for every rank's (the P2P handshake at communicator setup).
void launch_p2p_handshake(const P2PPush& push, const P2PWait& wait, hipStream_t st);
void launch_setup(const SetupArgs& u, int dir, hipStream_t st, int n_atm = 1);
void launch_log_ratio(const double* p, double p_top2, int nL, double* lnp, hipStream_t st);
void launch_update(const UpdateArgs& a, hipStream_t st, int n_atm = 1);
// Reduce + update in one launch for one atmosphere, local or P2P exchange: one workgroup per
// layer sums the partials of the (at most two) steps its layer pair needs, pushes its own
// step's sums to the peers, takes theirs, and writes its layer's T (into a.T_out), history
// and next-sweep step record; the last workgroup to arrive (a.done) settles the convergence
// flag.  Bitwise identical to launch_reduce + launch_update.
void launch_update_fused(const UpdateArgs& a, hipStream_t st);
void launch_propagate(int64_t n, const double* c1, const double* lk, const double* F1u,
                      const double* F2d, double T1, double T2, const double* dtau,
                      const double* w0, const double* g0, double* F2u, double* F1d,
                      hipStream_t st);
void launch_kappa(int64_t n, const TermP* terms, int nS, const double* sig, double* k,
                  hipStream_t st);
void launch_gen_table(double* tab, const double* base, const double* fp, const double* fT,
                      int n_p, int n_T, int64_t n_lam, int64_t stride, double lo, double hi,
                      hipStream_t st);
void launch_fill(double* x, int64_t n, double v, hipStream_t st);
void launch_milne(const double* dtaus, int nL, int64_t n, const double* fp, double* out,
                  hipStream_t st);
void launch_contribution(const double* dtaus, int nL, int64_t n, const double* nu,
                         const double* ratio, const double* T, double hcperk, double* cf,
                         hipStream_t st);
void launch_contract_batch(const double* const* tabs, int S, const double* mmr,
                           const int32_t* prow, int n_layers, int n_T, int64_t pitch,
                           int n_atm, int64_t tab_stride, double* eff, hipStream_t st);
void launch_contract_batch_valu(const double* const* tabs, int S, const double* mmr,
                           const int32_t* prow, int n_layers, int n_T, int64_t pitch,
                           int n_atm, int64_t tab_stride, double* eff, hipStream_t st);
void launch_contract(const double* const* tabs, int S, const double* mmr, const int32_t* prow,
                     int n_layers, int n_T, int64_t pitch, double* eff, hipStream_t st);

// Error reporting shared by the runtime and the binning module (frei_last_error()).
int set_error(const std::string& msg);
}  // namespace frei
struct frei_xsec;
namespace frei {
// K6 (frei_binning.hip): bin one species into table rows d_tab + row_off[kp * n_T + kt].
int bin_into_table(frei_xsec* x, int mode, const double* wl_bins, const double* lam,
                   int64_t n_bins, int64_t lam_lo, int64_t n_out, const double* T_t, int n_T,
                   const double* p_t, int n_p, const int64_t* row_off, double* d_tab,
                   int device);

}  // namespace frei
