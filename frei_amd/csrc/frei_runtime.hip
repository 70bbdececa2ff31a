// frei_runtime.hip — native runtime and C ABI (include/frei_hip.h) of the frei MI355X engine.
//
// Owns device memory, the HIP stream, the device-resident T-P loop driver (frei_run:
// core.py:233-338), and the optional RCCL exchange of per-sweep bolometric partial sums
// (one ncclAllGather of n_layers*4 doubles per sweep).
#include <dlfcn.h>

#include <algorithm>
#include <cctype>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <string>
#include <vector>

#include "../../include/frei_hip.h"
#include "frei_device.h"

using namespace frei;

namespace {

thread_local std::string g_err;

int fail(const std::string& msg) {
  g_err = msg;
  return -1;
}

}  // namespace

namespace frei {
int set_error(const std::string& msg) { return fail(msg); }
}  // namespace frei

namespace {

#define HIP_TRY(expr)                                                              \
  do {                                                                             \
    hipError_t _e = (expr);                                                        \
    if (_e != hipSuccess)                                                          \
      return fail(std::string(#expr) + ": " + hipGetErrorString(_e));              \
  } while (0)

#define TRY(expr)                 \
  do {                            \
    int _r = (expr);              \
    if (_r != 0) return _r;       \
  } while (0)

// ---------------------------------------------------------------- RCCL (dlopen)
struct Rccl {
  void* h = nullptr;
  typedef int (*GetId)(void*);
  typedef int (*InitRank)(void**, int, /*ncclUniqueId by value*/ struct Id128, int);
  int (*getUniqueId)(void*) = nullptr;
  int (*commInitRank)(void**, int, struct Id128, int) = nullptr;
  int (*allGather)(const void*, void*, size_t, int, void*, hipStream_t) = nullptr;
  int (*commDestroy)(void*) = nullptr;
  const char* (*errStr)(int) = nullptr;
};
struct Id128 { char b[128]; };

Rccl* rccl() {
  static Rccl r;
  static bool tried = false;
  if (!tried) {
    tried = true;
    r.h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!r.h) r.h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (r.h) {
      r.getUniqueId = (int (*)(void*))dlsym(r.h, "ncclGetUniqueId");
      r.commInitRank = (int (*)(void**, int, Id128, int))dlsym(r.h, "ncclCommInitRank");
      r.allGather = (int (*)(const void*, void*, size_t, int, void*, hipStream_t))dlsym(
          r.h, "ncclAllGather");
      r.commDestroy = (int (*)(void*))dlsym(r.h, "ncclCommDestroy");
      r.errStr = (const char* (*)(int))dlsym(r.h, "ncclGetErrorString");
    }
  }
  return (r.h && r.getUniqueId && r.commInitRank && r.allGather) ? &r : nullptr;
}
constexpr int kNcclFloat64 = 8;

struct Species {
  double* d_tab = nullptr;
  int n_p = 0, n_T = 0;
  int has_nan = 1;     // set by a device scan after upload/generation
  int64_t stride = 0;  // row pitch in elements (n_lam rounded up to 64, zero padded)
  std::vector<double> p_nodes, T_nodes;
};

}  // namespace

struct frei_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  int nL = 0, S = 0;
  int64_t nlam = 0;
  int nblocks = 0;
  // grid
  double *d_c1 = nullptr, *d_hcl = nullptr, *d_sig = nullptr, *d_ftoa = nullptr,
         *d_wtr = nullptr, *d_p = nullptr, *d_lnp = nullptr;
  std::vector<double> p;
  double p_top2 = 0, g = 0, m_bar = 0;
  bool grid_set = false;
  // state
  double *d_Fu = nullptr, *d_Fd = nullptr, *d_T = nullptr, *d_dT = nullptr,
         *d_dtaus = nullptr, *d_bol = nullptr;
  // the fused reduce + update writes the new temperatures into the other buffer and the two
  // swap (d_T is always the current one); d_done: its arrival counter
  double* d_T_alt = nullptr;
  double* d_T3 = nullptr;               // third temperature buffer (chained launches)
  double* d_T_home = nullptr;           // the buffer d_T names after a host upload
  // Chained launches (FREI_CHAIN): a sweep's fused update is deferred and runs as the leading
  // workgroups of the next sweep's launch (launch_sweep_chain)
  int chain = 1;                        // FREI_CHAIN
  bool has_pend = false;                // an update deferred to the next launch
  UpdateArgs pend{};
  unsigned long long* d_epoch = nullptr;  // [n_layers] the chained update's per-layer granules
  unsigned long long chain_seq = 0;
  int* d_chain_err = nullptr;           // a chained sweep block's wait gave up
  unsigned* d_done = nullptr;
  int fused_update = 1;                 // FREI_FUSED_UPDATE=0: separate reduce and update kernels
  // T-P iterations replayed from a captured hipGraph (frei_iterate / frei_run, timing off,
  // single rank): g_key holds the hashes of one iteration's kernel arguments; any change
  // (pointers, options, loop parameters) re-captures.  Off by default (FREI_GRAPH=1 turns it
  // on): measured no faster than stream launches, whose dispatch already overlaps the
  // previous kernel (profiles/r02_ab_graph.txt).
  int use_graph = 0;
  int graph_iters = 4;                  // iterations per captured graph
  hipGraphExec_t g_exec = nullptr;
  std::vector<uint64_t> g_key;
  int g_captures = 0, g_replays = 0;     // frei_graph_info
  int64_t n_chained = 0;                // chained sweep launches so far (frei_chain_info)
  // Trailing update (FREI_TAIL, round 6): the producer/consumer sweep's launch carries its own
  // fused update as trailing workgroups that reduce each layer as soon as the sweep has
  // published its steps (launch_sweep_pipe_tail).  Two partial-sum buffers used alternately:
  // a launch publishes into one and its update workgroups put the other back to kPoisonT.
  int tail = 1;                         // FREI_TAIL: 1 when it applies, 0 off
  double* d_tpart = nullptr;            // [2][tpart_n]
  int64_t tpart_n = 0;
  int tpart_parity = 0;
  bool tpart_fill = true;               // both buffers must be (re)filled with kPoisonT
  int64_t n_tail = 0;                   // trailing-update launches so far (frei_tail_info)
  bool shared_device = false;           // ranks share this GPU: no chained launches
  std::vector<uint64_t>* keys = nullptr;  // collecting run_sweep's argument hashes
  bool dry = false;                       // run_sweep computes hashes only (no launches)
  // tables
  std::vector<Species> sp;
  std::vector<double> mmr;
  bool meta_dirty = true;
  bool mmr_dirty = false;               // only the mixing ratios changed (per-sweep provider)
  int fast = 1;
  SpecMeta* d_smeta = nullptr;
  PMeta* d_pmeta = nullptr;
  double* d_tnodes = nullptr;
  int32_t* d_tperm = nullptr;
  double* d_mmr = nullptr;
  std::vector<SpecMeta> smeta;
  std::vector<PMeta> pmeta;
  std::vector<double> tnodes;
  std::vector<int32_t> tperm;
  // sweep scratch
  StepP* d_steps = nullptr;
  TermP* d_terms = nullptr;
  FastStep* d_fsteps = nullptr;
  FastStepS* d_ssteps = nullptr;
  int shared = 0;   // fast path with one bracket for all species (identical nodes)
  // Species-contracted table (K3): with shared nodes, no NaN and fixed per-layer mmr the
  // sweep reads eff[p][t][:] = sum_s mmr_s(l) tab_s[p][t][:] (2 rows per layer, not 2 S).
  // FREI_PRECONTRACT=0 keeps the per-species sum inside the sweep.
  int eff = 0, eff_mode = -1;
  double* d_eff = nullptr;
  // Lazy K3 (FREI_LAZY_K3, round 6): with the two-wavelength sweep, the setup contracts no row;
  // a sweep contracts the rows its records mask as missing (the lane's own wavelengths), and the
  // update after it marks them (d_kvalid).  A run touches a fraction of the table's T nodes (C3
  // to radiative equilibrium: 191 of 960 rows).  Any other sweep form first contracts the
  // whole table (eff_complete).
  int lazy_k3 = 1;
  bool lazy_on = false;
  bool eff_complete = true;
  int32_t* d_kvalid = nullptr;
  size_t eff_cap = 0;
  SpecMeta* d_smeta_eff = nullptr;
  double* d_ones = nullptr;
  int32_t* d_prow = nullptr;
  bool dtaus_valid = false;  // d_dtaus holds the last frei_run's final-emit dtaus
  // Batched atmospheres (frei_ctx_create_batch): n_atm atmospheres share the wavelength and
  // pressure grids and the opacity tables; every per-atmosphere buffer is n_atm blocks.
  int n_atm = 1;
  double* d_g = nullptr;      // [n_atm] gravity (batched)
  size_t eff_stride = 0;      // elements per atmosphere of d_eff
  int* h_conv = nullptr;      // pinned [2][n_atm] convergence flags (frei_run_batch)
  double *d_part = nullptr, *d_Fb = nullptr, *d_Fb_all = nullptr;
  // T-P loop state
  int* d_conv = nullptr;
  int* d_iter = nullptr;
  double *d_Tb = nullptr, *d_Ta = nullptr, *d_hist = nullptr;
  int hist_cap = 0;
  int32_t *d_flips = nullptr, *d_prev = nullptr, *d_ndiff = nullptr;
  int* h_flag = nullptr;  // pinned [2]
  int* h_err = nullptr;   // pinned [2]: the chained-poll and P2P error flags (check_comm)
  // pinned staging of the per-sweep host round trip of a chemistry provider stepping the loop
  // (frei_get_temperatures, frei_sweep's dT / bolometric sums, frei_set_mmr's upload): one
  // stream synchronisation per read, none for the upload (pageable copies add their own)
  double* h_T = nullptr;     // [n_layers * n_atm]
  double* h_dT = nullptr;    // [n_layers]
  double* h_bol = nullptr;   // [n_layers * 4]
  double* h_mmr = nullptr;   // [n_species * n_layers * n_atm]
  hipEvent_t mmr_ev = nullptr;   // the last upload from h_mmr
  bool mmr_ev_set = false;
  int64_t chain_checked = 0;   // n_chained at the last check_comm
  hipEvent_t flag_ev[2] = {nullptr, nullptr};
  // comm
  void* comm = nullptr;
  int nranks = 1, rank = 0;
  int prefetch_depth = 0;               // 0 = automatic (FREI_PREFETCH_DEPTH overrides)
  int k7_mfma = 1;                      // FREI_K7_MFMA: batched contraction on MFMA (1) or VALU (0)
  int prefetch_steps = 0;               // FREI_PREFETCH_STEPS: contracted one-lane sweep's load
                                        // distance in steps (0 = automatic, 8 / 16 = deeper)
  // Shared-bracket kernel (step table staged in LDS): used when every species shares its
  // nodes AND the slice is small (nblocks <= shared_max_blocks, about one resident round of
  // blocks), where each CU runs ~1 block and the per-step scalar loads would miss the K$.
  // FREI_SHARED=0/1 forces it off/on; FREI_SHARED_MAX_BLOCKS moves the threshold.
  int shared_mode = -1;
  int shared_max_blocks = 640;          // <= 164k lambda (125k: LDS 4 % faster; 164k tie; 250k: global 1 % faster)
  // Grouped-lane sweep (2 or 4 lanes per wavelength): contracted table, LDS step table and
  // at most this many 256-wavelength blocks, i.e. about one wave per SIMD or less.
  int pair_max_blocks = 420;            // FREI_PAIR_MAX_BLOCKS (<= 107k lambda per GPU)
  int quad_max_blocks = 208;            // FREI_QUAD_MAX_BLOCKS (<= 53k lambda per GPU)
  int group_q = 0;                      // FREI_GROUP_Q forces 1, 2 or 4 lanes per wavelength
  int pipe_nc = -1;                     // FREI_PIPE: producer/consumer sweep, 1/2/4 consumers per
                                        // block, 0 off, -1 by slice size (pipe_*_blocks; the
                                        // default again since its roles were balanced over the
                                        // SIMDs: -2 % per T-P iteration at 62.5k with P2P vs
                                        // the chained grouped-lane form, profiles/r03/chain/)
  int pipe_min_blocks = 208;            // FREI_PIPE_MIN_BLOCKS / _MAX_BLOCKS: 256-wavelength
  int pipe_max_blocks = -1;             // blocks per GPU where the auto choice takes NC = 4
                                        // (-1: the CU count, one 16-wave block per CU)
  int n_cu = 256;                       // hipDeviceProp multiProcessorCount
  int rec_sweep = -1;                   // FREI_REC_SWEEP: sweeps form their own step records
                                        // (1 every form, 0 never, -1 single-atmosphere contexts
                                        // without the producer/consumer sweep)
  bool rec_skipped = false;             // the last update wrote no records (the sweep did)
  int pipe_m = 2;                       // steps per producer and phase
  int pipe_pf = 1;                      // FREI_PIPE_PF: phases the producers load ahead (1, 2)
  int red_rows = 1;                     // FREI_RED_ROWS=0: full wave sums per step
  int red_stage = 1;                    // FREI_RED_STAGE=0: no staged sums (one-lane sweep)
  int lam2 = -1;                        // FREI_LAM2: two wavelengths per lane in the contracted
                                        // one-lane sweep (1 on, 0 off, -1 large slices)
  int sweep_lds_kb = 0;                 // FREI_SWEEP_LDS_KB: minimum LDS per sweep block (KiB)
  int group_waves = 4;                  // FREI_GROUP_WAVES: waves per grouped-lane sweep block
  int depth4_max_blocks = 0;            // FREI_DEPTH4_MAX_BLOCKS (4 steps in flight: off, measured no faster)
  size_t lds_per_block = 64 * 1024;     // hipDeviceProp sharedMemPerBlock
  size_t lds_optin = 64 * 1024;         // with the dynamic-LDS opt-in (gfx950: 160 KiB)
  bool ftoa_per_atm = false;            // batched: one F_TOA per atmosphere (frei_set_ftoa_batch)
  double setup_ms[5] = {0, 0, 0, 0, 0};  // last metadata build, by phase (frei_setup_timing)
  double contract_ms = 0.0;     // last K3 / K7 kernel, HIP events (frei_contract_timing)
  double contract_bytes = 0.0;  // its algorithmic HBM bytes
  // T-dependent chemistry (frei_set_chemistry): mmr tables on (T, p) nodes
  bool chem_on = false;
  int chem_nT = 0, chem_np = 0;
  std::vector<double> chem_tab, chem_T, chem_logp;   // host copies (frei_kappa)
  double *d_chem_tab = nullptr, *d_chem_T = nullptr, *d_chem_pz = nullptr;
  int32_t* d_chem_pj = nullptr;
  // P2P exchange over xGMI (frei_comm_p2p_*): own mailbox (uncached device memory), the
  // mapped mailboxes of every rank (own included) and the per-sweep sequence number
  double* d_mbox = nullptr;
  double** d_peers = nullptr;
  std::vector<void*> peer_mapped;        // IPC mappings to close
  uint64_t p2p_seq = 0;
  int* d_comm_err = nullptr;             // set by a kernel when a peer never published
  unsigned long long* d_wait_ticks = nullptr;
  double p2p_timeout_s = 30.0;           // FREI_P2P_TIMEOUT_S
  frei_allgather_fn host_ag = nullptr;  // host all-gather callback (alternative to RCCL)
  void* host_ag_user = nullptr;
  double* h_ag = nullptr;               // pinned [nranks + 1][n_steps * 4]
  // timing
  bool timing = false;
  std::vector<hipEvent_t> ev_pool;
  size_t ev_used = 0;
  std::vector<hipEvent_t> xev_pool;     // around the rank exchange (all-gather) of each sweep
  size_t xev_used = 0;
};

namespace {

int set_device(frei_ctx* c) {
  HIP_TRY(hipSetDevice(c->device));
  return 0;
}

template <typename T>
int dalloc(T** p, size_t n) {
  if (n == 0) n = 1;
  HIP_TRY(hipMalloc((void**)p, n * sizeof(T)));
  // FREI_ALLOC_FILL (diagnostic): fill every new device buffer with a byte value, so a read of
  // memory the engine never wrote shows up as changed results
  static const int fill = [] {
    const char* e = getenv("FREI_ALLOC_FILL");
    return e ? atoi(e) : -1;
  }();
  if (fill >= 0) {   // (the null-stream memset must finish before the context's stream uses p)
    HIP_TRY(hipMemset((void*)*p, fill, n * sizeof(T)));
    HIP_TRY(hipDeviceSynchronize());
  }
  return 0;
}

template <typename T>
void dfree(T*& p) {
  if (p) (void)hipFree((void*)p);
  p = nullptr;
}

template <typename T>
int h2d(T* d, const T* h, size_t n, hipStream_t st) {
  HIP_TRY(hipMemcpyAsync(d, h, n * sizeof(T), hipMemcpyHostToDevice, st));
  // the sources are often temporaries (pageable, freed at the caller's scope exit): wait for
  // the copy (setup and per-run uploads only, never inside the T-P loop)
  HIP_TRY(hipStreamSynchronize(st));
  return 0;
}

// Species contraction (K3) when every species shares its nodes (one bracket per layer), no
// table holds a NaN (the reference's nansum, Q8, is per species) and S >= 2.
// two wavelengths per lane from this many one-lane blocks per launch (all atmospheres of a
// batched launch): about 1.1 rounds of the one-lane form at five waves per SIMD
constexpr int kLam2MinBlocks = 1400;
bool lam2_blocks(const frei_ctx* c) {
  return (int64_t)c->nblocks * (c->n_atm > 1 ? c->n_atm : 1) >= kLam2MinBlocks;
}

// Staged partial sums (red_rows 2): the per-wave LDS tile plus one row per wave and the step
// table within 48 KiB (deep atmospheres, above ~160 steps, do not fit).
bool staged_sums_fit(int ns) {
  return ((size_t)(kBlock / 64) * ns * 4 + (size_t)(kBlock / 64) * 2 * 4 * 72) * sizeof(double) +
             (size_t)ns * sizeof(FastStepS) <= 48 * 1024;
}
// Prefetch depth of the one-lane sweep: below ~2 waves per SIMD (small per-GPU slices, e.g. 500k
// lambda over 8 GPUs) a second layer in flight hides HBM latency; at full occupancy one suffices.
// With one table (K3) and few blocks per CU, four steps in flight add the instruction-level
// parallelism that occupancy cannot (FREI_DEPTH4_MAX_BLOCKS).
int sweep_depth(const frei_ctx* c, int S_run) {
  return c->prefetch_depth > 0 ? c->prefetch_depth
         : (S_run == 1 && c->nblocks <= c->depth4_max_blocks) ? 4 : 2;
}
// Loads issued pf steps ahead (the contracted table only; 0: the coefficient block's depth;
// prefetch_steps 2 with depth 1: one step per coefficient block, loads two steps ahead).
int sweep_pf(const frei_ctx* c, bool eff, int S_run, int depth) {
  return (eff && S_run == 1 && (depth >= 2 || c->prefetch_steps == 2)) ? c->prefetch_steps : 0;
}
// The two-wavelength sweep's requirements besides the contracted NaN-free table, one lane per
// wavelength, global step records and no chained launch: an even slice, enough one-lane blocks
// (or FREI_LAM2=1), a depth-2 coefficient block loading at most two steps ahead, and the staged
// partial sums.  run_sweep (fast_form), frei_ctx_path and the batched step-table choice
// (build_meta) all decide by it.
bool lam2_static(const frei_ctx* c, int depth, int pf) {
  return c->lam2 != 0 && c->nlam % 2 == 0 && (c->lam2 > 0 || lam2_blocks(c)) && depth == 2 &&
         pf <= 2 && c->red_stage && staged_sums_fit(c->nL - 1);
}

bool lam2_form(const frei_ctx* c);   // (below: fast_form)

template <typename Lap>
int build_contracted(frei_ctx* c, bool shared_fast, Lap&& lap) {
  const int nL = c->nL, S = c->S;
  c->lazy_on = false;        // (decided below, with the contracted table)
  c->eff_complete = true;
  const bool batch = c->n_atm > 1;
  // (a T-dependent chemistry changes mmr every sweep: the species sum stays in the sweep)
  bool on = shared_fast && (S >= 2 || batch) && (c->eff_mode != 0 || batch) && !c->chem_on;
  for (int s = 0; s < S && on; ++s) on = !c->sp[s].has_nan;
  std::vector<int32_t> prow(nL, 0);
  if (on) {
    std::vector<int> owner((size_t)c->sp[0].n_p, -1);
    for (int l = 0; l < nL && on; ++l) {
      const PMeta& pm = c->pmeta[l];  // species 0 (shared nodes)
      prow[l] = (pm.wp_lo != 0.0) ? pm.p_lo : pm.p_hi;
      if (owner[prow[l]] >= 0) {  // two layers on one pressure row: mmr must agree
        for (size_t m = 0; m < (size_t)c->n_atm && on; ++m)
          for (int s = 0; s < S && on; ++s)
            on = c->mmr[(m * S + s) * nL + l] == c->mmr[(m * S + s) * nL + owner[prow[l]]];
      }
      owner[prow[l]] = l;
    }
  }
  c->eff = on ? 1 : 0;
  if (!on) {
    if (batch)
      return fail("a batched context needs tables on shared on-node p/T nodes without NaN "
                  "(one contracted table per atmosphere)");
    return 0;
  }
  const Species& q0 = c->sp[0];
  const size_t per = (size_t)q0.n_p * q0.n_T * (size_t)q0.stride + 64;
  const size_t need = per * c->n_atm;
  if (c->eff_cap < need) {
    HIP_TRY(hipStreamSynchronize(c->stream));   // no queued sweep still reads the old table
    dfree(c->d_eff);
    c->eff_cap = 0;
    TRY(dalloc(&c->d_eff, need));
    c->eff_cap = need;
  }
  lap(2);
  c->eff_stride = per;
  // the contraction writes every column (padding included) of the pressure rows the layers
  // use; only the other rows and each atmosphere's 64-element tail are zero-filled here (a
  // fill of the whole table would double the setup's HBM writes: 24.6 GB at C5)
  {
    const size_t rowblk = (size_t)q0.n_T * q0.stride;
    std::vector<char> used((size_t)q0.n_p, 0);
    for (int l = 0; l < nL; ++l) used[prow[l]] = 1;
    for (size_t m = 0; m < (size_t)c->n_atm; ++m) {
      double* base = c->d_eff + m * per;
      for (int p = 0; p < q0.n_p;) {
        if (used[p]) {
          ++p;
          continue;
        }
        int e = p;
        while (e < q0.n_p && !used[e]) ++e;
        HIP_TRY(hipMemsetAsync(base + (size_t)p * rowblk, 0,
                               (size_t)(e - p) * rowblk * sizeof(double), c->stream));
        p = e;
      }
      HIP_TRY(hipMemsetAsync(base + (size_t)q0.n_p * rowblk, 0, 64 * sizeof(double),
                             c->stream));
    }
  }
  lap(3);
  if (!c->d_ones) {
    std::vector<double> ones(nL, 1.0);
    TRY(dalloc(&c->d_ones, nL));
    TRY(h2d(c->d_ones, ones.data(), nL, c->stream));
  }
  dfree(c->d_prow);
  TRY(dalloc(&c->d_prow, nL));
  TRY(h2d(c->d_prow, prow.data(), nL, c->stream));
  const double* tabs[kMaxFastS];
  for (int s = 0; s < S; ++s) tabs[s] = c->sp[s].d_tab;
  // lazy K3: the sweeps that read this table take two wavelengths per lane (the form run_sweep
  // launches for a loop's sweeps), one atmosphere
  c->lazy_on = c->lazy_k3 && !batch && lam2_form(c);
  c->eff_complete = !c->lazy_on;
  if (c->lazy_on) {
    dfree(c->d_kvalid);
    TRY(dalloc(&c->d_kvalid, (size_t)q0.n_p * q0.n_T));
    HIP_TRY(hipMemsetAsync(c->d_kvalid, 0, (size_t)q0.n_p * q0.n_T * sizeof(int32_t),
                           c->stream));
    // a layer outside the hull reads rows 0 and 1 with zero weights: finite (zero) until then
    HIP_TRY(hipMemsetAsync(c->d_eff, 0, 2 * (size_t)q0.stride * sizeof(double), c->stream));
    c->contract_ms = 0.0;
    c->contract_bytes = 0.0;
    lap(4);
    SpecMeta m = c->smeta[0];
    m.tab = c->d_eff;
    if (!c->d_smeta_eff) TRY(dalloc(&c->d_smeta_eff, 1));
    TRY(h2d(c->d_smeta_eff, &m, 1, c->stream));
    return 0;
  }
  hipEvent_t k0 = nullptr, k1 = nullptr;   // the contraction kernel alone (frei_contract_timing)
  if (hipEventCreate(&k0) != hipSuccess || hipEventCreate(&k1) != hipSuccess)
    return fail("hipEventCreate failed");
  HIP_TRY(hipEventRecord(k0, c->stream));
  if (batch && c->k7_mfma)  // K7: [n_atm x S] . [S x n_T*pitch] per layer on fp64 MFMA
    launch_contract_batch(tabs, S, c->d_mmr, c->d_prow, nL, q0.n_T, q0.stride, c->n_atm,
                          (int64_t)per, c->d_eff, c->stream);
  else if (batch)           // K7 on the VALU, K3's species order
    launch_contract_batch_valu(tabs, S, c->d_mmr, c->d_prow, nL, q0.n_T, q0.stride,
                               c->n_atm, (int64_t)per, c->d_eff, c->stream);
  else
    launch_contract(tabs, S, c->d_mmr, c->d_prow, nL, q0.n_T, q0.stride, c->d_eff, c->stream);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipEventRecord(k1, c->stream));
  lap(4);
  {
    float ms = 0.f;
    HIP_TRY(hipEventSynchronize(k1));
    HIP_TRY(hipEventElapsedTime(&ms, k0, k1));
    c->contract_ms = ms;
    // bytes the launch must move: the S tables' used rows read once, n_atm tables written
    // (every column of the used rows, padding included)
    std::vector<char> used((size_t)q0.n_p, 0);
    for (int l = 0; l < nL; ++l) used[prow[l]] = 1;
    size_t rows = 0;
    for (char u : used) rows += u;
    const double rowbytes = (double)q0.n_T * q0.stride * sizeof(double);
    c->contract_bytes = rows * rowbytes * (S + c->n_atm);
    (void)hipEventDestroy(k0);
    (void)hipEventDestroy(k1);
  }
  SpecMeta m = c->smeta[0];
  m.tab = c->d_eff;
  if (!c->d_smeta_eff) TRY(dalloc(&c->d_smeta_eff, 1));
  TRY(h2d(c->d_smeta_eff, &m, 1, c->stream));
  return 0;
}

// Build the per-(species, layer) pressure brackets and upload all table metadata.
double now_ms() {
  return std::chrono::duration<double, std::milli>(
             std::chrono::steady_clock::now().time_since_epoch()).count();
}

int build_meta(frei_ctx* c) {
  if (!c->meta_dirty) {
    if (c->mmr_dirty) {   // new mixing ratios only: up on the stream, ahead of the next sweep
      // (through pinned staging, no synchronisation: the previous upload from it has finished
      // once its event has)
      if (c->mmr_ev_set) HIP_TRY(hipEventSynchronize(c->mmr_ev));
      std::memcpy(c->h_mmr, c->mmr.data(), c->mmr.size() * sizeof(double));
      HIP_TRY(hipMemcpyAsync(c->d_mmr, c->h_mmr, c->mmr.size() * sizeof(double),
                             hipMemcpyHostToDevice, c->stream));
      HIP_TRY(hipEventRecord(c->mmr_ev, c->stream));
      c->mmr_ev_set = true;
      c->mmr_dirty = false;
    }
    return 0;
  }
  if (!c->grid_set) return fail("frei_set_grid must be called before using tables");
  double t_prev = now_ms();
  auto lap = [&](int k) {   // frei_setup_timing phases (host wall clock, stream synced)
    (void)hipStreamSynchronize(c->stream);
    const double t = now_ms();
    c->setup_ms[k] += t - t_prev;
    t_prev = t;
  };
  for (double& x : c->setup_ms) x = 0.0;
  const int nL = c->nL, S = c->S;
  c->smeta.assign(S, SpecMeta{});
  c->pmeta.assign((size_t)S * nL, PMeta{});
  c->tnodes.clear();
  c->tperm.clear();
  int fast = 1;
  for (int s = 0; s < S; ++s) {
    const Species& q = c->sp[s];
    if (!q.d_tab) return fail("opacity table of species " + std::to_string(s) + " not set");
    SpecMeta m{};
    m.tab = q.d_tab;
    m.n_lam = q.stride;
    m.n_p = q.n_p;
    m.n_T = q.n_T;
    m.t_off = (int32_t)c->tnodes.size();
    // sorted temperature nodes (xarray sortby) + permutation to memory rows
    std::vector<int32_t> perm(q.n_T);
    std::iota(perm.begin(), perm.end(), 0);
    std::stable_sort(perm.begin(), perm.end(),
                     [&](int a, int b) { return q.T_nodes[a] < q.T_nodes[b]; });
    int n_unique = q.n_T > 0 ? 1 : 0;
    for (int k = 1; k < q.n_T; ++k)
      if (q.T_nodes[perm[k]] != q.T_nodes[perm[k - 1]]) ++n_unique;
    m.one_T = (n_unique <= 1) ? 1 : 0;
    if (!m.one_T && n_unique != q.n_T)
      return fail("duplicate temperature nodes (drop_duplicates first, opacity.py:339)");
    for (int k = 0; k < q.n_T; ++k) {
      c->tnodes.push_back(q.T_nodes[perm[k]]);
      c->tperm.push_back(perm[k]);
    }
    if (m.one_T) fast = 0;
    if (S > kMaxFastS) fast = 0;
    c->smeta[s] = m;
    // sorted pressure nodes + bracket of every layer pressure
    std::vector<int32_t> pp(q.n_p);
    std::iota(pp.begin(), pp.end(), 0);
    std::stable_sort(pp.begin(), pp.end(),
                     [&](int a, int b) { return q.p_nodes[a] < q.p_nodes[b]; });
    std::vector<double> ps(q.n_p);
    for (int k = 0; k < q.n_p; ++k) ps[k] = q.p_nodes[pp[k]];
    for (int l = 0; l < nL; ++l) {
      PMeta pm{};
      const double x = c->p[l];
      if (m.one_T) {
        // scipy interp1d: searchsorted(left) clipped to [1, n-1]
        int jx = (int)(std::lower_bound(ps.begin(), ps.end(), x) - ps.begin());
        jx = std::max(1, std::min(jx, q.n_p - 1));
        pm.p_lo = pp[jx - 1];
        pm.p_hi = pp[jx];
        pm.x1 = x - ps[jx - 1];
        pm.dx = ps[jx] - ps[jx - 1];
        pm.oob = (x < ps[0] || x > ps[q.n_p - 1]) ? 1 : 0;
      } else {
        int i, oob;
        double y;
        bracket(ps.data(), q.n_p, x, i, y, oob);
        pm.p_lo = pp[i];
        pm.p_hi = pp[i + 1];
        pm.wp_lo = 1.0 - y;
        pm.wp_hi = y;
        pm.oob = oob;
        if (!oob && pm.wp_lo != 0.0 && pm.wp_hi != 0.0) fast = 0;  // off-node pressure
      }
      c->pmeta[(size_t)s * nL + l] = pm;
    }
  }
  c->fast = fast;
  lap(0);
  // One bracket serves every species when their nodes, shapes and row pitch coincide.
  int shared = 1;
  for (int s = 1; s < S; ++s) {
    const Species &q0 = c->sp[0], &q = c->sp[s];
    shared = shared && q.n_p == q0.n_p && q.n_T == q0.n_T && q.stride == q0.stride &&
             q.p_nodes == q0.p_nodes && q.T_nodes == q0.T_nodes;
  }
  // batched launches with many blocks in all take the two-wavelength sweep, which reads the
  // step records from global memory (C5, 32 x 100k lambda: -9 % per step, profiles/r04/c5/)
  // (a batched context always has the contracted table without NaN, or fails in build_contracted)
  const int bdepth = sweep_depth(c, 1);
  const bool lam2_batch = c->n_atm > 1 && lam2_static(c, bdepth, sweep_pf(c, true, 1, bdepth));
  const bool small = c->nblocks <= c->shared_max_blocks && !lam2_batch;
  // the LDS-staged step table plus one partial-sum row per wave must leave room for several
  // blocks per CU (deep atmospheres: > ~260 layers read the step table from global memory)
  const size_t ns_l = (size_t)nL - 1;
  const bool lds_fits =
      (size_t)(kBlock / 64) * ns_l * 4 * sizeof(double) + ns_l * sizeof(FastStepS) <= 64 * 1024;
  c->shared = (c->shared_mode == 1 || (c->shared_mode < 0 && small)) && lds_fits ? shared : 0;
  HIP_TRY(hipStreamSynchronize(c->stream));   // queued kernels may still read the metadata
  dfree(c->d_smeta);
  dfree(c->d_pmeta);
  dfree(c->d_tnodes);
  dfree(c->d_tperm);
  TRY(dalloc(&c->d_smeta, S));
  TRY(dalloc(&c->d_pmeta, (size_t)S * nL));
  TRY(dalloc(&c->d_tnodes, c->tnodes.size()));
  TRY(dalloc(&c->d_tperm, c->tperm.size()));
  TRY(h2d(c->d_smeta, c->smeta.data(), S, c->stream));
  TRY(h2d(c->d_pmeta, c->pmeta.data(), (size_t)S * nL, c->stream));
  TRY(h2d(c->d_tnodes, c->tnodes.data(), c->tnodes.size(), c->stream));
  TRY(h2d(c->d_tperm, c->tperm.data(), c->tperm.size(), c->stream));
  if (c->mmr.size() != (size_t)S * nL * c->n_atm) return fail("frei_set_mmr must be called");
  TRY(h2d(c->d_mmr, c->mmr.data(), (size_t)S * nL * c->n_atm, c->stream));
  lap(1);
  TRY(build_contracted(c, fast && shared, lap));
  HIP_TRY(hipStreamSynchronize(c->stream));
  c->meta_dirty = false;
  c->mmr_dirty = false;
  return 0;
}

AtmStride atm_stride(frei_ctx* c);

// Lanes per wavelength of the sweep: the grouped-lane kernel (2 or 4 lanes) when the slice
// leaves about one wave per SIMD or less (contracted table, LDS step table), else 1.
int group_lanes(const frei_ctx* c) {
  if (!(c->fast && c->eff && c->shared)) return 1;
  if (c->group_q > 0) return c->group_q;
  const int64_t blocks = (int64_t)c->nblocks * c->n_atm;   // 256-wavelength blocks
  if (blocks <= c->quad_max_blocks) return 4;
  if (blocks <= c->pair_max_blocks) return 2;
  return 1;
}

// Consumers per block of the producer/consumer sweep (0: not used).  Contracted table and the
// FastStepS records (the LDS-step-table path); the block's LDS must fit the device.
int pipe_consumers(const frei_ctx* c) {
  if (!(c->fast && c->eff && c->shared) || c->pipe_nc == 0) return 0;
  int nc = c->pipe_nc;
  if (nc < 0) {   // by slice size: one 256-wavelength block per CU or fewer
    const int64_t blocks = (int64_t)c->nblocks * c->n_atm;
    const int64_t mx = c->pipe_max_blocks < 0 ? c->n_cu : c->pipe_max_blocks;
    if (blocks <= c->pipe_min_blocks || blocks > mx) return 0;
    nc = 4;
  }
  if (pipe_lds_bytes(nc, c->pipe_m, c->nL - 1) > c->lds_optin) return 0;
  return nc;
}

SetupArgs setup_args(frei_ctx* c);

// Sweeps form their own step records in their prologue (and the update kernels skip writing
// them) when the sweep reads the shared-bracket records from LDS — every form on the contracted
// table with shared brackets — and the mixing ratios are fixed (no T-dependent chemistry).
bool records_in_sweep(frei_ctx* c) {
  if (!(c->rec_sweep && c->fast && c->eff && c->shared && !c->chem_on)) return false;
  // auto: not for batched contexts (every (block, atmosphere) would form the records: C5 -2 %,
  // profiles/r02_ab_rec_sweep.txt), nor for the producer/consumer sweep unless its launches
  // are chained (neutral to slower on their own; a chained sweep must form its records)
  return c->rec_sweep > 0 || (c->n_atm == 1 && (pipe_consumers(c) == 0 || c->chain == 2));
}

SetupArgs setup_args(frei_ctx* c) {
  SetupArgs u{};
  u.n_layers = c->nL;
  u.n_species = c->eff ? 1 : c->S;
  u.fast = c->fast;
  u.T = c->d_T;
  u.p = c->d_p;
  u.p_top2 = c->p_top2;
  u.g = c->g;
  u.spec = c->eff ? c->d_smeta_eff : c->d_smeta;
  u.pmeta = c->d_pmeta;
  u.tnodes = c->d_tnodes;
  u.n_tnodes = (int)c->tnodes.size();
  u.tperm = c->d_tperm;
  u.mmr = c->eff ? c->d_ones : c->d_mmr;
  u.steps = c->d_steps;
  u.terms = c->d_terms;
  u.fsteps = c->d_fsteps;
  u.ssteps = c->d_ssteps;
  u.shared = c->shared;
  u.bs = atm_stride(c);
  u.kvalid = c->lazy_on ? c->d_kvalid : nullptr;
  u.kpitch = c->sp.empty() ? 0 : c->sp[0].stride;
  if (c->chem_on) {
    u.chem.tab = c->d_chem_tab;
    u.chem.T = c->d_chem_T;
    u.chem.pj = c->d_chem_pj;
    u.chem.pz = c->d_chem_pz;
    u.chem.n_T = c->chem_nT;
    u.chem.n_p = c->chem_np;
  }
  return u;
}

hipEvent_t next_event_in(std::vector<hipEvent_t>& pool, size_t& used) {
  if (used == pool.size()) {
    hipEvent_t e;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    pool.push_back(e);
  }
  return pool[used++];
}
hipEvent_t next_event(frei_ctx* c) { return next_event_in(c->ev_pool, c->ev_used); }

struct SweepOpts {
  int dir = kEmit;
  int next_dir = -1;   // setup for the next sweep inside update
  int force = 0;       // ignore the convergence flag
  int track = 0;       // T-P history / convergence bookkeeping
  int stop_on_conv = 0;
  int n_zero_crossings = 2;
  double convergence_dT = 3.0;
  double alpha = 1.0;
  double* dtaus = nullptr;    // device
  double* dT_out = nullptr;   // device
  double* bol_out = nullptr;  // device
  int live_only = 0;          // T-P loop: skip stores no later sweep reads
};

// Temperature buffers: d_T is the current one; an update writes a buffer that is neither d_T
// (its input) nor `busy` (the input of an update still running in the same launch), which
// then becomes d_T.
void rotate_T(frei_ctx* c, double* out) {
  double* b[3] = {c->d_T, c->d_T_alt, c->d_T3};
  double* rest[2];
  int n = 0;
  for (double* x : b)
    if (x != out && n < 2) rest[n++] = x;
  c->d_T = out;
  c->d_T_alt = rest[0];
  c->d_T3 = rest[1];
}
double* free_T(frei_ctx* c, const double* busy) { return c->d_T_alt != busy ? c->d_T_alt : c->d_T3; }

// Drop a deferred update that will never run (an error part-way through a run).  The sweep that
// deferred it already made its output buffer the current temperatures, filled with kPoisonT
// ("not published"), so the current temperatures go back to that update's input: a later sweep
// or read that skips frei_state_init sees the last published temperatures, not poison.
void drop_pending(frei_ctx* c) {
  if (!c->has_pend) return;
  c->has_pend = false;
  rotate_T(c, c->pend.su.T);
}

// reduce + update fused into one launch: one atmosphere, exchange local or P2P (RCCL and the
// host hook need the rank's sums in memory between the two kernels)
bool fused_ok(frei_ctx* c) {
  return c->fused_update && c->n_atm == 1 && !c->comm && !(c->nranks > 1 && c->host_ag) &&
         (2 * (size_t)c->nL + c->tnodes.size()) * sizeof(double) <= 32 * 1024;
}

// This sweep can run chained: a grouped-lane or one-lane (two or more steps in flight) sweep
// of the contracted table forming its own step records, fused update, stream launches (no graph
// capture).
// Not while per-sweep HIP events are on (frei_timing): events around a chained launch would also
// cover the deferred update it runs, including its wait for the peers' sums, so a timed run
// launches sweep and update separately and the events time the sweep alone.  Not when ranks
// share this device (frei_comm_shared_device): a chained launch's sweep blocks
// spin on the update workgroups, which wait for every rank's sums, and could hold the CUs
// another rank's kernels need.
bool chain_ready(frei_ctx* c) {
  if (!(c->chain && c->fast && c->eff && c->shared && records_in_sweep(c) && fused_ok(c) &&
        !c->use_graph && !c->keys && !c->timing && !c->shared_device))
    return false;
  const int nc = pipe_consumers(c);
  // producer/consumer, four consumers per block; the chained kernel adds the update body's
  // static LDS (4.3 KiB) to the sweep's, which must still fit the CU (deep atmospheres do not)
  // — only on request (FREI_CHAIN=2): chained, its 1024-thread update blocks take 6 µs where
  // the separate update kernel takes 3 (profiles/r03/chain/ab_pipe.txt)
  if (nc > 0)
    return c->chain == 2 && nc == 4 &&
           pipe_lds_bytes(4, c->pipe_m, c->nL - 1) + 6 * 1024 <= c->lds_optin;
  if (group_lanes(c) > 1) return true;      // grouped-lane
  // one-lane (two or more steps in flight): measured neutral to slower at 125k-500k
  // (profiles/r03/chain/ab_onelane.txt), so only on request (FREI_CHAIN=2)
  return c->chain == 2 && c->prefetch_depth != 1;
}

// Update workgroups of a trailing-update launch (0: not used): the producer/consumer sweep with
// four consumers, the fused update (one atmosphere, local or P2P exchange), stream launches
// without per-sweep events (they would time the update with the sweep), not chained, ranks not
// sharing the device, and — so that they are resident beside the sweep, never waiting behind
// it — at least two CUs left free by the sweep's one block per CU (eight update blocks at most).
int tail_blocks(const frei_ctx* c, int nb_sweep) {
  if (!(c->tail && c->fast && c->eff && c->shared && c->n_atm == 1 && !c->use_graph && !c->keys &&
        !c->timing && !c->shared_device && !c->chem_on))
    return 0;
  if (!(c->fused_update && !c->comm && !(c->nranks > 1 && c->host_ag) &&
        (2 * (size_t)c->nL + c->tnodes.size()) * sizeof(double) <= 32 * 1024))
    return 0;
  if (pipe_consumers(c) != 4 || records_in_sweep(const_cast<frei_ctx*>(c))) return 0;
  if (pipe_tail_lds_bytes(c->nL - 1, (int)c->tnodes.size()) + 6 * 1024 > c->lds_optin) return 0;
  const int free_cu = c->n_cu - nb_sweep;
  return free_cu >= 2 ? std::min(free_cu, 8) : 0;
}

// Launch a deferred update on its own (the next sweep cannot take it, or the caller needs its
// results now).  Its output buffer holds kPoisonT until the update writes it.
int flush_update(frei_ctx* c) {
  if (!c->has_pend) return 0;
  c->has_pend = false;
  launch_update_fused(c->pend, c->stream);
  HIP_TRY(hipGetLastError());
  return 0;
}

// FNV-1a over an argument block (zero-initialised structs: padding bytes are zero)
template <typename T>
uint64_t arg_hash(uint64_t h, const T& x) {
  const unsigned char* b = reinterpret_cast<const unsigned char*>(&x);
  for (size_t i = 0; i < sizeof(T); ++i) h = (h ^ b[i]) * 1099511628211ull;
  return h;
}

// The sweep form run_sweep launches for the contracted / per-species tables (c->fast), in one
// place, so that frei_ctx_path reports what runs.  merge: the launch also runs a deferred update.
struct FastForm {
  int S_run, depth, pf, Q, NW, NC, red_rows;
  bool nan_check, lam2;
};
FastForm fast_form(const frei_ctx* c, bool merge) {
  FastForm m{};
  const int ns = c->nL - 1;
  m.S_run = c->eff ? 1 : c->S;
  // per-row partials while the one-lane sweep's LDS stays within 48 KiB (3+ blocks per CU)
  m.red_rows = c->red_rows &&
               (size_t)16 * ns * 4 * sizeof(double) + (size_t)ns * sizeof(FastStepS) <= 48 * 1024;
  m.depth = sweep_depth(c, m.S_run);
  m.pf = sweep_pf(c, c->eff != 0, m.S_run, m.depth);
  m.nan_check = false;
  for (int q = 0; q < c->S; ++q) m.nan_check = m.nan_check || c->sp[q].has_nan;
  m.Q = group_lanes(c);
  // staged partial sums (mode 2): the one-lane sweep with two steps in flight, and the
  // grouped-lane sweep (two groups in flight)
  if ((m.Q > 1 || m.depth == 2 || (m.depth == 1 && m.pf == 2)) && c->red_stage &&
      staged_sums_fit(ns))
    m.red_rows = 2;
  m.NW = c->group_waves;
  m.NC = pipe_consumers(c);
  // two wavelengths per lane: the one-lane contracted sweep on slices that need more than
  // about one round of one-lane blocks (1280 resident at five waves per SIMD on 256 CUs)
  m.lam2 = c->eff && m.S_run == 1 && !c->shared && !m.nan_check && m.Q == 1 && m.NC == 0 &&
           !merge && m.red_rows == 2 && lam2_static(c, m.depth, m.pf);
  return m;
}

bool lam2_form(const frei_ctx* c) { return fast_form(c, false).lam2; }

// Lazy K3: contract every row not contracted yet (any sweep form other than the two-wavelength
// one, which contracts its masked rows itself, or an update that does not mark them).
int complete_contraction(frei_ctx* c) {
  if (c->eff_complete) return 0;
  const Species& q0 = c->sp[0];
  const double* tabs[kMaxFastS];
  for (int s = 0; s < c->S; ++s) tabs[s] = c->sp[s].d_tab;
  std::vector<int32_t> prow(c->nL);
  for (int l = 0; l < c->nL; ++l) {
    const PMeta& pm = c->pmeta[l];
    prow[l] = (pm.wp_lo != 0.0) ? pm.p_lo : pm.p_hi;
  }
  launch_contract(tabs, c->S, c->d_mmr, c->d_prow, c->nL, q0.n_T, q0.stride, c->d_eff, c->stream);
  HIP_TRY(hipGetLastError());
  std::vector<int32_t> ones((size_t)q0.n_p * q0.n_T, 0);
  for (int l = 0; l < c->nL; ++l)
    for (int t = 0; t < q0.n_T; ++t) ones[(size_t)prow[l] * q0.n_T + t] = 1;
  TRY(h2d(c->d_kvalid, ones.data(), ones.size(), c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));   // (the host vector)
  c->eff_complete = true;
  return 0;
}

// One sweep: K1 -> fused reduce + update (+ next setup; P2P exchange inside), or K1 ->
// reduce -> [RCCL / host all-gather] -> K4/K5 (batched contexts, RCCL, host hook,
// fused_update 0).  Asynchronous.
// With c->dry it only appends the hash of every launch's arguments to c->keys and applies
// the host-side state changes (temperature buffer swap), launching nothing.
int run_sweep(frei_ctx* c, const SweepOpts& o, bool defer = false) {
  const int ns = c->nL - 1;
  // chained: this sweep's launch also runs the deferred update (merge), and this sweep's own
  // update may be deferred to the next launch (defer_own)
  const bool chain = !c->dry && chain_ready(c);
  if (c->has_pend && !chain) TRY(flush_update(c));
  const bool merge = chain && c->has_pend;
  const bool defer_own = chain && defer;
  // the output buffer of this sweep's update: not d_T, and not the merged update's input
  double* T_next = chain ? free_T(c, merge ? c->pend.su.T : nullptr) : c->d_T_alt;
  SweepArgs a{};
  a.n_lam = c->nlam;
  a.n_steps = ns;
  a.n_species = c->S;
  a.force = o.force;
  a.live_only = o.live_only;
  a.c1 = c->d_c1;
  a.hcl = c->d_hcl;
  a.sig = c->d_sig;
  a.wtr = c->d_wtr;
  a.ftoa = c->d_ftoa;
  a.steps = c->d_steps;
  a.terms = c->d_terms;
  a.F_up = c->d_Fu;
  a.F_down = c->d_Fd;
  a.dtaus = o.dtaus;
  a.part = c->d_part;
  a.conv = c->d_conv;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  if (c->timing) {
    e0 = next_event(c);
    e1 = next_event(c);
    if (!e0 || !e1) return fail("hipEventCreate failed");
    HIP_TRY(hipEventRecord(e0, c->stream));
  }
  int nb_run = c->nblocks;  // partial-sum columns written by this sweep
  FastArgs tail_f{};        // a trailing-update launch: the sweep's arguments (launched below)
  int tail_nT = 0;          // its update workgroups (0: not a trailing-update launch)
  const bool rec_on = c->fast && records_in_sweep(c);
  // a sweep that reads the update's records after one whose update skipped them (an option or
  // the tables changed mid-run): write this sweep's records first
  if (!rec_on && c->rec_skipped && !c->dry) {
    launch_setup(setup_args(c), o.dir, c->stream, c->n_atm);
    HIP_TRY(hipGetLastError());
  }
  c->rec_skipped = false;
  if (c->fast) {
    FastArgs f{};
    f.n_lam = c->nlam;
    f.pitch = c->sp[0].stride;
    f.n_steps = ns;
    f.force = o.force;
    f.live_only = o.live_only;
    f.c1 = c->d_c1;
    f.hcl = c->d_hcl;
    f.sig = c->d_sig;
    f.wtr = c->d_wtr;
    f.ftoa = c->d_ftoa;
    const FastForm m = fast_form(c, merge);
    // lazy K3: only the two-wavelength sweep with the fused update (which marks the rows it
    // used) contracts on the way; any other form gets the whole table first
    if (c->lazy_on && !c->eff_complete && !c->dry && !(m.lam2 && fused_ok(c)))
      TRY(complete_contraction(c));
    const int S_run = m.S_run;
    for (int q = 0; q < kMaxFastS; ++q) f.tab[q] = q < c->S ? c->sp[q].d_tab : nullptr;
    if (c->eff) f.tab[0] = c->d_eff;
    if (c->lazy_on && !c->eff_complete) {   // the two-wavelength sweep contracts masked rows
      for (int q = 0; q < kMaxFastS; ++q) f.ktab[q] = q < c->S ? c->sp[q].d_tab : nullptr;
      f.kmmr = c->d_mmr;
      f.kS = c->S;
      f.kNL = c->nL;
    }
    f.steps = c->d_fsteps;
    f.ssteps = c->d_ssteps;
    f.F_up = c->d_Fu;
    f.F_down = c->d_Fd;
    f.dtaus = o.dtaus;
    f.part = c->d_part;
    f.conv = c->d_conv;
    f.bs = atm_stride(c);
    f.n_atm = c->n_atm;
    f.unit_mmr = c->eff ? 1 : 0;
    f.rec_on = rec_on ? 1 : 0;
    f.min_lds = c->sweep_lds_kb * 1024;
    if (merge) {   // this launch's leading workgroups run the deferred update
      f.ch_epoch = c->d_epoch;
      f.ch_val = ++c->chain_seq;
      f.ch_can_conv = c->pend.track && c->pend.dir == kAbsorb && c->pend.stop_on_conv;
      f.ch_timeout = (long long)(c->p2p_timeout_s * 1e8);   // wall_clock64: 100 MHz
      f.ch_err = c->d_chain_err;
    }
    if (defer_own) f.poison = T_next;
    if (f.rec_on) f.rec = setup_args(c);   // T of this sweep: c->d_T now
    f.red_rows = m.red_rows;
    const int depth = m.depth, pf = m.pf, Q = m.Q, NW = m.NW, NC = m.NC;
    const bool nan_check = m.nan_check, lam2 = m.lam2;
    if (Q > 1) nb_run = (int)((c->nlam + 64 * NW / Q - 1) / (64 * NW / Q));
    if (NC > 0) nb_run = (int)((c->nlam + 64 * NC - 1) / (64 * NC));
    if (lam2) nb_run = (int)((c->nlam + 2 * kBlock - 1) / (2 * kBlock));
    if (c->keys) {
      uint64_t h = arg_hash(1469598103934665603ull, f);
      const int cfg[11] = {o.dir, Q, S_run, depth, (nan_check && !c->eff) ? 1 : 0, c->shared,
                           NC, c->pipe_pf, pf, NW, lam2 ? 1 : 0};
      c->keys->push_back(arg_hash(h, cfg));
    }
    if (c->dry) {
    } else if (NC > 0 && merge) {
      UpdateArgs u = c->pend;
      u.epoch = c->d_epoch;
      u.epoch_val = c->chain_seq;
      c->has_pend = false;
      launch_sweep_pipe_chain(o.dir, c->pipe_pf, f, u, nb_run, c->stream);
      ++c->n_chained;
    } else if (NC > 0 && (tail_nT = tail_blocks(c, nb_run)) > 0) {
      tail_f = f;   // launched with its update (which needs the P2P arguments below)
    } else if (NC > 0) {
      launch_sweep_pipe(o.dir, NC, c->pipe_pf, f, nb_run, c->stream);
    } else if (Q > 1 && merge) {
      UpdateArgs u = c->pend;
      u.epoch = c->d_epoch;
      u.epoch_val = c->chain_seq;
      c->has_pend = false;
      launch_sweep_chain(o.dir, Q, NW, f, u, nb_run, c->stream);
      ++c->n_chained;
    } else if (Q > 1) {
      launch_sweep_group(o.dir, Q, NW, f, nb_run, c->stream);
    } else if (merge) {   // the one-lane contracted sweep, records formed in the block
      UpdateArgs u = c->pend;
      u.epoch = c->d_epoch;
      u.epoch_val = c->chain_seq;
      c->has_pend = false;
      launch_sweep_fast_chain(o.dir, depth, pf, f, u, c->nblocks, c->stream);
      ++c->n_chained;
    } else if (lam2) {
      launch_sweep_pair(o.dir, f, nb_run, c->stream);
    } else {
      launch_sweep_fast(o.dir, S_run, depth, pf, nan_check && !c->eff, c->shared != 0, f,
                        c->nblocks, c->stream);
    }
  } else {
    if (c->keys) c->keys->push_back(arg_hash(arg_hash(1469598103934665603ull, a), o.dir));
    if (!c->dry) launch_sweep(o.dir, a, c->nblocks, false, c->stream);
  }
  HIP_TRY(hipGetLastError());
  if (c->timing) HIP_TRY(hipEventRecord(e1, c->stream));
  P2PPush push{};
  P2PWait wait{};
  if (c->d_mbox && !c->dry) {   // P2P: each rank's sums are pushed and waited for on device
    const uint64_t seq = ++c->p2p_seq;
    push.peers = c->d_peers;
    push.nranks = c->nranks;
    push.rank = c->rank;
    push.n = (int64_t)ns * 4;
    push.seq = seq;
    wait.mbox = c->d_mbox;
    wait.nranks = c->nranks;
    wait.n = push.n;
    wait.seq = seq;
    wait.timeout_ticks = (int64_t)(c->p2p_timeout_s * 1e8);   // wall_clock64: 100 MHz
    wait.err = c->d_comm_err;
    wait.wait_ticks = c->timing ? c->d_wait_ticks : nullptr;
  }
  // one launch for reduce + update: one atmosphere, exchange local or P2P (RCCL and the host
  // hook need the rank's sums in memory between the two kernels)
  const bool fused = fused_ok(c);
  if (!fused && c->dry) {   // not graph-replayable (the check in iterate() sees the marker)
    if (c->keys) c->keys->push_back(0);
    return 0;
  }
  if (!fused) {
    const AtmStride bs = atm_stride(c);
    launch_reduce(c->d_part, nb_run, c->d_Fb, ns * 4, c->d_conv, o.force, c->stream,
                  c->n_atm, bs.part, bs.fb, c->d_mbox ? &push : nullptr);
  }
  HIP_TRY(hipGetLastError());
  const double* Fb = c->d_Fb;
  hipEvent_t x1 = nullptr;
  if (c->timing && (c->comm || (c->nranks > 1 && c->host_ag))) {   // exchange timing
    hipEvent_t x0 = next_event_in(c->xev_pool, c->xev_used);
    x1 = next_event_in(c->xev_pool, c->xev_used);
    if (!x0 || !x1) return fail("hipEventCreate failed");
    HIP_TRY(hipEventRecord(x0, c->stream));
  }
  if (c->nranks > 1 && c->host_ag) {
    const size_t n = (size_t)ns * 4;
    HIP_TRY(hipMemcpyAsync(c->h_ag, c->d_Fb, n * sizeof(double), hipMemcpyDeviceToHost,
                           c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (c->host_ag(c->h_ag, c->h_ag + n, (int64_t)n, c->host_ag_user) != 0)
      return fail("host all-gather callback failed");
    HIP_TRY(hipMemcpyAsync(c->d_Fb_all, c->h_ag + n, c->nranks * n * sizeof(double),
                           hipMemcpyHostToDevice, c->stream));
    Fb = c->d_Fb_all;
  } else if (c->comm) {  // RCCL (also a forced 1-rank communicator, FREI_FORCE_RCCL=1)
    Rccl* r = rccl();
    if (!r || !c->comm) return fail("RCCL communicator not initialised");
    int rc = r->allGather(c->d_Fb, c->d_Fb_all, (size_t)ns * 4, kNcclFloat64, c->comm,
                          c->stream);
    if (rc != 0)
      return fail(std::string("ncclAllGather: ") + (r->errStr ? r->errStr(rc) : "error"));
    Fb = c->d_Fb_all;
  }
  if (x1) HIP_TRY(hipEventRecord(x1, c->stream));
  UpdateArgs u{};
  u.su = setup_args(c);
  u.p2p = wait;
  u.dir = o.dir;
  u.next_dir = o.next_dir;
  if (c->fast && records_in_sweep(c) && o.next_dir >= 0) {   // the next sweep forms its own
    u.next_dir = -1;
    c->rec_skipped = true;
  }
  u.nranks = c->nranks;
  u.force = o.force;
  u.track = o.track;
  u.stop_on_conv = o.stop_on_conv;
  u.n_zero_crossings = o.n_zero_crossings;
  u.hist_cap = c->hist_cap;
  u.m_bar = c->m_bar;
  u.alpha = o.alpha;
  u.convergence_dT = o.convergence_dT;
  u.Fb = Fb;
  u.lnp = c->d_lnp;
  u.dT_out = o.dT_out;
  u.bol_out = o.bol_out;
  u.Tb = c->d_Tb;
  u.Ta = c->d_Ta;
  u.hist = c->d_hist;
  u.flips = c->d_flips;
  u.prev_sign = c->d_prev;
  u.ndiff = c->d_ndiff;
  u.iter = c->d_iter;
  u.conv = c->d_conv;
  // metadata in LDS when the update's whole allocation (the launch's own formula) fits the
  // 64 KiB a workgroup may request
  const int S_meta = c->eff ? 1 : c->S;
  u.meta_in_lds = update_lds_bytes(c->nL, (int)c->tnodes.size(), S_meta, true) <=
                  std::min<size_t>(c->lds_per_block, 64 * 1024);
  if (fused) {
    u.part = c->d_part;
    u.nblocks = nb_run;
    u.push = push;
    u.T_out = T_next;
    u.done = c->d_done;
    if (c->keys) c->keys->push_back(arg_hash(1469598103934665603ull, u));
    if (defer_own) {   // runs at the head of the next sweep's launch, or flush_update
      c->pend = u;
      c->has_pend = true;
    } else if (tail_nT > 0) {   // the sweep and this update in one launch
      const int64_t need = (int64_t)nb_run * ns * 4;
      if (c->tpart_n < need) {
        dfree(c->d_tpart);
        c->tpart_n = 0;
        TRY(dalloc(&c->d_tpart, 2 * (size_t)need));
        c->tpart_n = need;
        c->tpart_fill = true;
      }
      if (c->tpart_fill) {
        launch_poison(c->d_tpart, 2 * c->tpart_n, c->stream);
        c->tpart_fill = false;
        c->tpart_parity = 0;
      }
      double* cur = c->d_tpart + c->tpart_parity * c->tpart_n;
      double* other = c->d_tpart + (1 - c->tpart_parity) * c->tpart_n;
      c->tpart_parity ^= 1;
      tail_f.tail_part = cur;
      u.part = cur;
      u.poll = 1;
      u.poll_timeout = (long long)(c->p2p_timeout_s * 1e8);   // wall_clock64: 100 MHz
      u.poll_err = c->d_chain_err;
      launch_sweep_pipe_tail(o.dir, c->pipe_pf, tail_f, u, nb_run, tail_nT, other, c->stream);
      ++c->n_tail;
    } else if (!c->dry) {
      launch_update_fused(u, c->stream);
    }
    HIP_TRY(hipGetLastError());
    rotate_T(c, T_next);
    return 0;
  }
  launch_update(u, c->stream, c->n_atm);
  HIP_TRY(hipGetLastError());
  return 0;
}

// A host upload overwrites the current temperatures, so the fused update's ping-pong can
// restart from the same buffer (every run then issues identical launch arguments).
void home_temperatures(frei_ctx* c) {
  if (c->d_T != c->d_T_home) rotate_T(c, c->d_T_home);
}

int reset_loop_state(frei_ctx* c) {
  const size_t A = c->n_atm;
  HIP_TRY(hipMemsetAsync(c->d_conv, 0, sizeof(int) * A, c->stream));
  HIP_TRY(hipMemsetAsync(c->d_iter, 0, sizeof(int) * A, c->stream));
  HIP_TRY(hipMemsetAsync(c->d_flips, 0, sizeof(int32_t) * c->nL * A, c->stream));
  HIP_TRY(hipMemsetAsync(c->d_prev, 0, sizeof(int32_t) * c->nL * A, c->stream));
  HIP_TRY(hipMemsetAsync(c->d_ndiff, 0, sizeof(int32_t) * c->nL * A, c->stream));
  return 0;
}

int ensure_hist(frei_ctx* c, int cap) {
  if (cap <= c->hist_cap) return 0;
  HIP_TRY(hipStreamSynchronize(c->stream));   // queued update kernels may still write it
  dfree(c->d_hist);
  TRY(dalloc(&c->d_hist, (size_t)cap * 2 * c->nL * c->n_atm));
  c->hist_cap = cap;
  return 0;
}

// Per-atmosphere strides of a batched context (all zero for one atmosphere).
AtmStride atm_stride(frei_ctx* c) {
  AtmStride b{};
  if (c->n_atm <= 1) return b;
  const int64_t nL = c->nL, ns = nL - 1;
  b.layers = nL;
  b.steps = ns;
  b.fb = ns * 4;
  b.hist = (int64_t)c->hist_cap * 2 * nL;
  b.flux = nL * c->nlam;
  b.tab = (int64_t)c->eff_stride;
  b.part = ns * 4 * (int64_t)(4 * c->nblocks);
  b.ftoa = c->ftoa_per_atm ? c->nlam : 0;
  b.g = c->d_g;
  return b;
}

int ensure_dtaus(frei_ctx* c) {
  if (!c->d_dtaus) TRY(dalloc(&c->d_dtaus, (size_t)c->nL * c->nlam));
  launch_fill(c->d_dtaus, c->nlam, 1.0, c->stream);  // row 0 placeholder (Q12)
  HIP_TRY(hipGetLastError());
  return 0;
}

bool ready(frei_ctx* c) { return c && c->grid_set; }

// Tuning knobs (frei_set_option and FREI_<NAME> environment variables); each takes effect at
// the next metadata build (the tables' sweep path is re-derived).
const char* const kOptionNames[] = {"prefetch_depth", "shared", "shared_max_blocks",
                                    "precontract", "depth4_max_blocks", "pair_max_blocks",
                                    "quad_max_blocks", "red_rows", "red_stage", "group_q",
                                    "fused_update", "graph", "pipe", "pipe_pf", "pipe_min_blocks", "rec_sweep",
                                    "pipe_max_blocks", "prefetch_steps", "k7_mfma", "sweep_lds_kb", "group_waves", "chain",
                                    "lam2", "tail", "lazy_k3", nullptr};
int set_option(frei_ctx* c, const std::string& k, int v) {
  if (k == "prefetch_depth") c->prefetch_depth = v;
  else if (k == "shared") c->shared_mode = v < 0 ? -1 : (v ? 1 : 0);
  else if (k == "shared_max_blocks") c->shared_max_blocks = v;
  else if (k == "precontract") c->eff_mode = v < 0 ? -1 : (v ? 1 : 0);
  else if (k == "depth4_max_blocks") c->depth4_max_blocks = v;
  else if (k == "pair_max_blocks") c->pair_max_blocks = v;
  else if (k == "quad_max_blocks") c->quad_max_blocks = v;
  else if (k == "red_rows") c->red_rows = v != 0;
  else if (k == "red_stage") c->red_stage = v != 0;
  else if (k == "group_q") c->group_q = (v == 1 || v == 2 || v == 4) ? v : 0;
  else if (k == "fused_update") c->fused_update = v != 0;
  else if (k == "graph") c->use_graph = v != 0;
  else if (k == "pipe") c->pipe_nc = (v == 1 || v == 2 || v == 4 || v == -1) ? v : 0;
  else if (k == "pipe_min_blocks") c->pipe_min_blocks = v;
  else if (k == "rec_sweep") c->rec_sweep = v < 0 ? -1 : (v ? 1 : 0);
  else if (k == "pipe_max_blocks") c->pipe_max_blocks = v;
  else if (k == "pipe_pf") c->pipe_pf = v == 1 ? 1 : 2;
  else if (k == "k7_mfma") c->k7_mfma = v != 0;
  else if (k == "group_waves") c->group_waves = v == 8 ? 8 : 4;
  else if (k == "chain") c->chain = v < 0 ? 0 : (v > 2 ? 2 : v);
  else if (k == "lam2") c->lam2 = v < 0 ? -1 : (v ? 1 : 0);
  else if (k == "tail") c->tail = v != 0;
  else if (k == "lazy_k3") c->lazy_k3 = v != 0;
  else if (k == "sweep_lds_kb") c->sweep_lds_kb = v < 0 ? 0 : (v > 160 ? 160 : v);
  else if (k == "prefetch_steps") c->prefetch_steps = v >= 16 ? 16 : v >= 8 ? 8 : v == 2 ? 2 : 0;
  else return fail("unknown option '" + k + "'");
  c->meta_dirty = true;
  return 0;
}

// After a stream synchronize: did a chained sweep's poll or a P2P wait time out (a rank never
// published its sums)?  The flags are read only when they can have been set — a chained launch
// since the last check, a P2P communicator — and into pinned memory on the context's stream: a
// pageable hipMemcpy here cost ~20 ms the first time (its staging buffer), which left the GPU
// idle right before a timed loop (bench.py's warm-up synchronize) and changed how the power
// management clocked the loop that followed (profiles/r04/bisect/README.md).
int check_comm(frei_ctx* c) {
  const bool chain = c->d_chain_err && c->n_chained + c->n_tail != c->chain_checked;
  const bool comm = c->d_comm_err != nullptr;
  if (!chain && !comm) return 0;
  if (chain)
    HIP_TRY(hipMemcpyAsync(&c->h_err[0], c->d_chain_err, sizeof(int), hipMemcpyDeviceToHost,
                           c->stream));
  if (comm)
    HIP_TRY(hipMemcpyAsync(&c->h_err[1], c->d_comm_err, sizeof(int), hipMemcpyDeviceToHost,
                           c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  c->chain_checked = c->n_chained + c->n_tail;
  if (chain && c->h_err[0]) {   // reported once: rearm it so later runs are not failed by it
    drop_pending(c);
    c->tpart_fill = true;       // a trailing update gave up: its buffers are in no known state
    const int code = c->h_err[0];
    c->h_err[0] = 0;
    HIP_TRY(hipMemsetAsync(c->d_chain_err, 0, sizeof(int), c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    // (the first wait to give up: 1 a chained sweep block's temperatures, 3 a trailing update
    // slot's partial sums)
    return fail("chained sweep / trailing update: a wait for values another workgroup "
                "publishes gave up (FREI_P2P_TIMEOUT_S; wait " + std::to_string(code) + ")");
  }
  if (comm && c->h_err[1])
    return fail("P2P exchange timed out: a peer rank did not publish its partial sums "
                "(FREI_P2P_TIMEOUT_S)");
  return 0;
}

}  // namespace

// ==================================================================== C ABI
extern "C" {

int frei_version(void) { return 20000; }

const char* frei_last_error(void) { return g_err.c_str(); }

int frei_device_count(int* n) {
  if (!n) return fail("null argument");
  HIP_TRY(hipGetDeviceCount(n));
  return 0;
}

static int ctx_create(frei_ctx** out, int device, int n_layers, int64_t n_lam, int n_species,
                      int n_atm) {
  if (!out) return fail("null argument");
  *out = nullptr;
  if (n_atm < 1 || n_atm > 65535) return fail("n_atm must be in [1, 65535]");
  if (n_layers < 4 || n_layers > kMaxLayers)
    return fail("n_layers must be in [4, 1024] (the emit top layer uses p[-3])");
  if (n_lam < 2) return fail("n_lam must be >= 2");
  if (n_species < 1 || n_species > 64) return fail("n_species must be in [1, 64]");
  frei_ctx* c = new frei_ctx();
  c->device = device;
  c->nL = n_layers;
  c->nlam = n_lam;
  c->S = n_species;
  c->n_atm = n_atm;
  c->sp.resize(n_species);
  c->nblocks = (int)((n_lam + kBlock - 1) / kBlock);
  // tuning knobs: FREI_<NAME> in the environment, or frei_set_option(ctx, "<name>", v)
  for (const char* const* k = kOptionNames; *k; ++k) {
    std::string env = "FREI_";
    for (const char* q = *k; *q; ++q) env += (char)std::toupper((unsigned char)*q);
    if (const char* e = getenv(env.c_str())) (void)set_option(c, *k, atoi(e));
  }
  auto bail = [&](int rc) {
    frei_ctx_destroy(c);
    return rc;
  };
  int rc;
  if ((rc = set_device(c))) return bail(rc);
  {
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) == hipSuccess && prop.sharedMemPerBlock > 0) {
      c->lds_per_block = prop.sharedMemPerBlock;
      c->lds_optin = std::max(c->lds_per_block, (size_t)prop.sharedMemPerBlockOptin);
      if (prop.multiProcessorCount > 0) c->n_cu = prop.multiProcessorCount;
    }
  }
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess)
    return bail(fail("hipStreamCreate failed"));
  const size_t NL = n_layers, NS = n_species, ns = n_layers - 1, A = n_atm;
  const size_t F = NL * (size_t)n_lam * A;   // per-atmosphere buffers are n_atm blocks
  if ((rc = dalloc(&c->d_c1, n_lam)) || (rc = dalloc(&c->d_hcl, n_lam)) ||
      (rc = dalloc(&c->d_sig, n_lam)) || (rc = dalloc(&c->d_ftoa, n_lam)) ||
      (rc = dalloc(&c->d_wtr, n_lam)) || (rc = dalloc(&c->d_p, NL)) || (rc = dalloc(&c->d_lnp, NL)) ||
      (rc = dalloc(&c->d_Fu, F)) || (rc = dalloc(&c->d_Fd, F)) ||
      (rc = dalloc(&c->d_T, NL * A)) || (rc = dalloc(&c->d_T_alt, NL * A)) ||
      (rc = dalloc(&c->d_T3, NL * A)) || (rc = dalloc(&c->d_epoch, NL)) ||
      (rc = dalloc(&c->d_chain_err, 1)) ||
      (rc = dalloc(&c->d_done, 1)) || (rc = dalloc(&c->d_dT, NL * A)) ||
      (rc = dalloc(&c->d_bol, NL * 4 * A)) || (rc = dalloc(&c->d_mmr, NS * NL * A)) ||
      (rc = dalloc(&c->d_steps, ns * A)) || (rc = dalloc(&c->d_terms, ns * NS * A)) ||
      (rc = dalloc(&c->d_fsteps, ns * A)) || (rc = dalloc(&c->d_ssteps, ns * A)) ||
      (rc = dalloc(&c->d_part, ns * 4 * (size_t)(4 * c->nblocks) * A)) ||
      (rc = dalloc(&c->d_Fb, ns * 4 * A)) || (rc = dalloc(&c->d_Fb_all, ns * 4)) ||
      (rc = dalloc(&c->d_conv, A)) || (rc = dalloc(&c->d_iter, A)) ||
      (rc = dalloc(&c->d_Tb, NL * A)) || (rc = dalloc(&c->d_Ta, NL * A)) ||
      (rc = dalloc(&c->d_flips, NL * A)) || (rc = dalloc(&c->d_prev, NL * A)) ||
      (rc = dalloc(&c->d_ndiff, NL * A)) || (A > 1 && (rc = dalloc(&c->d_g, A))))
    return bail(rc);
  c->d_T_home = c->d_T;
  if (hipHostMalloc((void**)&c->h_flag, 2 * sizeof(int)) != hipSuccess ||
      hipHostMalloc((void**)&c->h_err, 2 * sizeof(int)) != hipSuccess)
    return bail(fail("hipHostMalloc failed"));
  c->h_err[0] = c->h_err[1] = 0;
  for (int k = 0; k < 2; ++k)
    if (hipEventCreateWithFlags(&c->flag_ev[k], hipEventDisableTiming) != hipSuccess)
      return bail(fail("hipEventCreate failed"));
  // stream-ordered (the context's stream does not synchronise with the null stream)
  if (hipMemsetAsync(c->d_Fu, 0, F * sizeof(double), c->stream) != hipSuccess ||
      hipMemsetAsync(c->d_Fd, 0, F * sizeof(double), c->stream) != hipSuccess ||
      hipMemsetAsync(c->d_conv, 0, sizeof(int) * A, c->stream) != hipSuccess ||
      hipMemsetAsync(c->d_done, 0, sizeof(unsigned), c->stream) != hipSuccess ||
      hipMemsetAsync(c->d_epoch, 0, sizeof(unsigned long long) * NL, c->stream) != hipSuccess ||
      hipMemsetAsync(c->d_chain_err, 0, sizeof(int), c->stream) != hipSuccess ||
      hipStreamSynchronize(c->stream) != hipSuccess)
    return bail(fail("hipMemsetAsync failed"));
  if (A > 1 && hipHostMalloc((void**)&c->h_conv, 2 * A * sizeof(int)) != hipSuccess)
    return bail(fail("hipHostMalloc failed"));
  if (hipHostMalloc((void**)&c->h_T, NL * A * sizeof(double)) != hipSuccess ||
      hipHostMalloc((void**)&c->h_dT, NL * sizeof(double)) != hipSuccess ||
      hipHostMalloc((void**)&c->h_bol, NL * 4 * sizeof(double)) != hipSuccess ||
      hipHostMalloc((void**)&c->h_mmr, (size_t)n_species * NL * A * sizeof(double)) != hipSuccess ||
      hipEventCreateWithFlags(&c->mmr_ev, hipEventDisableTiming) != hipSuccess)
    return bail(fail("hipHostMalloc failed"));
  *out = c;
  return 0;
}

int frei_ctx_create(frei_ctx** out, int device, int n_layers, int64_t n_lam, int n_species) {
  return ctx_create(out, device, n_layers, n_lam, n_species, 1);
}

int frei_ctx_create_batch(frei_ctx** out, int device, int n_layers, int64_t n_lam,
                          int n_species, int n_atm) {
  return ctx_create(out, device, n_layers, n_lam, n_species, n_atm);
}

int frei_ctx_destroy(frei_ctx* c) {
  if (!c) return 0;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  if (c->comm) {
    Rccl* r = rccl();
    if (r && r->commDestroy) r->commDestroy(c->comm);
  }
  if (c->g_exec) (void)hipGraphExecDestroy(c->g_exec);
  c->g_exec = nullptr;
  for (void* p : c->peer_mapped) (void)hipIpcCloseMemHandle(p);
  c->peer_mapped.clear();
  dfree(c->d_peers);
  dfree(c->d_mbox);
  dfree(c->d_comm_err);
  dfree(c->d_wait_ticks);
  dfree(c->d_epoch);
  dfree(c->d_chain_err);
  dfree(c->d_tpart);
  dfree(c->d_kvalid);
  for (auto& s : c->sp) dfree(s.d_tab);
  dfree(c->d_eff);
  dfree(c->d_smeta_eff);
  dfree(c->d_chem_tab);
  dfree(c->d_chem_T);
  dfree(c->d_chem_pz);
  dfree(c->d_chem_pj);
  dfree(c->d_ones);
  dfree(c->d_prow);
  double* dd[] = {c->d_c1, c->d_hcl, c->d_sig, c->d_ftoa, c->d_wtr, c->d_p, c->d_lnp,
                  c->d_Fu, c->d_Fd, c->d_T, c->d_T_alt, c->d_T3, c->d_dT, c->d_dtaus, c->d_bol, c->d_tnodes, c->d_mmr, c->d_part,
                  c->d_Fb, c->d_Fb_all, c->d_Tb, c->d_Ta, c->d_hist};
  for (double* p : dd)
    if (p) (void)hipFree(p);
  void* vv[] = {c->d_smeta, c->d_pmeta, c->d_tperm, c->d_steps, c->d_terms, c->d_fsteps,
                c->d_ssteps, c->d_conv, c->d_iter, c->d_flips, c->d_prev, c->d_ndiff,
                c->d_done};
  for (void* p : vv)
    if (p) (void)hipFree(p);
  if (c->h_flag) (void)hipHostFree(c->h_flag);
  if (c->h_err) (void)hipHostFree(c->h_err);
  if (c->h_conv) (void)hipHostFree(c->h_conv);
  for (double* h : {c->h_T, c->h_dT, c->h_bol, c->h_mmr})
    if (h) (void)hipHostFree(h);
  if (c->mmr_ev) (void)hipEventDestroy(c->mmr_ev);
  dfree(c->d_g);
  if (c->h_ag) (void)hipHostFree(c->h_ag);
  for (auto e : c->flag_ev)
    if (e) (void)hipEventDestroy(e);
  for (auto e : c->xev_pool) (void)hipEventDestroy(e);
  for (auto e : c->ev_pool) (void)hipEventDestroy(e);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
  return 0;
}

int frei_set_grid(frei_ctx* c, const double* c1, const double* lk, const double* sigma,
                  const double* f_toa, const double* trapz_w, const double* p, double g,
                  double m_bar) {
  if (!c || !c1 || !lk || !sigma || !f_toa || !trapz_w || !p) return fail("null argument");
  if (!(g > 0) || !(m_bar > 0)) return fail("g and m_bar must be positive");
  TRY(set_device(c));
  const int64_t n = c->nlam;
  c->p.assign(p, p + c->nL);
  for (int l = 1; l < c->nL; ++l)
    if (!(c->p[l] < c->p[l - 1])) return fail("pressures must be strictly descending (BOA first)");
  // emit's top layer: p_2 = p[-1] * p[-2] / p[-3] (twostream.py:359)
  c->p_top2 = c->p[c->nL - 1] * c->p[c->nL - 2] / c->p[c->nL - 3];
  c->g = g;
  c->m_bar = m_bar;
  if (c->n_atm > 1) {  // default gravity of every atmosphere (frei_set_gravity overrides)
    std::vector<double> gv(c->n_atm, g);
    TRY(h2d(c->d_g, gv.data(), gv.size(), c->stream));
  }
  TRY(h2d(c->d_c1, c1, n, c->stream));
  {   // the Planck exponent's per-wavelength factor hc / (lam k_B) (kernels: times 1 / T)
    std::vector<double> hcl(n);
    for (int64_t j = 0; j < n; ++j) hcl[j] = kHC / lk[j];
    TRY(h2d(c->d_hcl, hcl.data(), n, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));   // hcl is a temporary
  }
  TRY(h2d(c->d_sig, sigma, n, c->stream));
  TRY(h2d(c->d_ftoa, f_toa, n, c->stream));
  c->ftoa_per_atm = false;   // one F_TOA for every atmosphere again
  TRY(h2d(c->d_wtr, trapz_w, n, c->stream));
  TRY(h2d(c->d_p, c->p.data(), c->nL, c->stream));
  launch_log_ratio(c->d_p, c->p_top2, c->nL, c->d_lnp, c->stream);
  HIP_TRY(hipStreamSynchronize(c->stream));
  c->grid_set = true;
  c->meta_dirty = true;
  return 0;
}

// Ascending order of the temperature nodes: tables are stored with the T axis sorted so
// that the upper bracket row is always the next row (row_hi = row_lo + n_lam).
static std::vector<int32_t> t_order(const double* T_nodes, int n_T) {
  std::vector<int32_t> perm(n_T);
  std::iota(perm.begin(), perm.end(), 0);
  std::stable_sort(perm.begin(), perm.end(),
                   [&](int a, int b) { return T_nodes[a] < T_nodes[b]; });
  return perm;
}

static int set_table_common(frei_ctx* c, int s, const double* p_nodes, int n_p,
                            const double* T_nodes, int n_T) {
  if (s < 0 || s >= c->S) return fail("species index out of range");
  if (n_p < 2) return fail("a table needs at least 2 pressure nodes");
  if (n_T < 1) return fail("a table needs at least 1 temperature node");
  Species& q = c->sp[s];
  const int64_t stride = (c->nlam + 63) / 64 * 64;
  const size_t need = (size_t)n_p * n_T * (size_t)stride + 64;
  // queued sweeps of the old tables must finish before they are overwritten or freed
  HIP_TRY(hipStreamSynchronize(c->stream));
  if (!q.d_tab || (size_t)q.n_p * q.n_T != (size_t)n_p * n_T) {
    dfree(q.d_tab);
    TRY(dalloc(&q.d_tab, need));
  }
  // finite padding; on the context's stream, ordered before the table upload / generation.
  // (A null-stream hipMemset is not ordered with the non-blocking stream: it could still be
  // zeroing the table while gen_table_kernel writes it — the intermittent C5 results of round 2.)
  HIP_TRY(hipMemsetAsync(q.d_tab, 0, need * sizeof(double), c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));   // before frei_set_table's blocking host copies
  q.stride = stride;
  q.n_p = n_p;
  q.n_T = n_T;
  q.p_nodes.assign(p_nodes, p_nodes + n_p);
  const std::vector<int32_t> perm = t_order(T_nodes, n_T);
  q.T_nodes.resize(n_T);
  for (int t = 0; t < n_T; ++t) q.T_nodes[t] = T_nodes[perm[t]];  // stored ascending
  c->meta_dirty = true;
  return 0;
}

// Device NaN scan of species s's table: the sweep drops the per-species NaN skip of the
// reference's nansum (Q8) when no table can produce a NaN.
static int scan_nan(frei_ctx* c, int s) {
  Species& q = c->sp[s];
  int* d_flag = nullptr;
  TRY(dalloc(&d_flag, 1));
  HIP_TRY(hipMemsetAsync(d_flag, 0, sizeof(int), c->stream));
  launch_nan_scan(q.d_tab, (int64_t)q.n_p * q.n_T * q.stride, d_flag, c->stream);
  HIP_TRY(hipGetLastError());
  int h = 1;
  HIP_TRY(hipMemcpyAsync(&h, d_flag, sizeof(int), hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  dfree(d_flag);
  q.has_nan = h;
  return 0;
}

int frei_set_table(frei_ctx* c, int s, const double* values, const double* p_nodes, int n_p,
                   const double* T_nodes, int n_T) {
  if (!c || !values || !p_nodes || !T_nodes) return fail("null argument");
  TRY(set_device(c));
  TRY(set_table_common(c, s, p_nodes, n_p, T_nodes, n_T));
  const std::vector<int32_t> perm = t_order(T_nodes, n_T);
  bool ident = true;
  for (int t = 0; t < n_T; ++t) ident = ident && perm[t] == t;
  const size_t row = (size_t)c->nlam;
  const size_t pitch = (size_t)c->sp[s].stride * sizeof(double);
  if (ident) {
    HIP_TRY(hipMemcpy2D(c->sp[s].d_tab, pitch, values, row * sizeof(double),
                        row * sizeof(double), (size_t)n_p * n_T, hipMemcpyHostToDevice));
  } else {
    for (int p = 0; p < n_p; ++p)
      for (int t = 0; t < n_T; ++t)
        HIP_TRY(hipMemcpy(c->sp[s].d_tab + ((size_t)p * n_T + t) * c->sp[s].stride,
                          values + ((size_t)p * n_T + perm[t]) * row, row * sizeof(double),
                          hipMemcpyHostToDevice));
  }
  return scan_nan(c, s);
}

int frei_set_table_separable(frei_ctx* c, int s, const double* base, const double* fp,
                             const double* fT, double lo, double hi, const double* p_nodes,
                             int n_p, const double* T_nodes, int n_T) {
  if (!c || !base || !fp || !fT || !p_nodes || !T_nodes) return fail("null argument");
  TRY(set_device(c));
  TRY(set_table_common(c, s, p_nodes, n_p, T_nodes, n_T));
  const std::vector<int32_t> perm = t_order(T_nodes, n_T);
  std::vector<double> fT_sorted(n_T);
  for (int t = 0; t < n_T; ++t) fT_sorted[t] = fT[perm[t]];
  fT = fT_sorted.data();
  double *d_base = nullptr, *d_fp = nullptr, *d_fT = nullptr;
  TRY(dalloc(&d_base, c->nlam));
  TRY(dalloc(&d_fp, n_p));
  TRY(dalloc(&d_fT, n_T));
  TRY(h2d(d_base, base, c->nlam, c->stream));
  TRY(h2d(d_fp, fp, n_p, c->stream));
  TRY(h2d(d_fT, fT, n_T, c->stream));
  launch_gen_table(c->sp[s].d_tab, d_base, d_fp, d_fT, n_p, n_T, c->nlam, c->sp[s].stride, lo,
                   hi, c->stream);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipStreamSynchronize(c->stream));
  dfree(d_base);
  dfree(d_fp);
  dfree(d_fT);
  return scan_nan(c, s);
}

int frei_set_table_binned(frei_ctx* c, int s, frei_xsec* x, int mode, const double* wl_bins,
                          const double* lam, int64_t n_bins, int64_t lam_lo,
                          const double* T_nodes, int n_T, const double* p_nodes, int n_p) {
  if (!c || !x || !wl_bins || !lam || !T_nodes || !p_nodes) return fail("null argument");
  TRY(set_device(c));
  std::vector<double> p_cgs(n_p > 0 ? n_p : 0);
  for (int k = 0; k < n_p; ++k) p_cgs[k] = p_nodes[k] * 1e6;  // bar -> dyn cm^-2
  TRY(set_table_common(c, s, p_cgs.data(), n_p, T_nodes, n_T));
  // destination row of node (kp, kt): the T axis is stored ascending
  const std::vector<int32_t> perm = t_order(T_nodes, n_T);
  std::vector<int32_t> rank(n_T);
  for (int t = 0; t < n_T; ++t) rank[perm[t]] = t;
  std::vector<int64_t> row_off((size_t)n_p * n_T);
  for (int kp = 0; kp < n_p; ++kp)
    for (int kt = 0; kt < n_T; ++kt)
      row_off[(size_t)kp * n_T + kt] = ((int64_t)kp * n_T + rank[kt]) * c->sp[s].stride;
  TRY(bin_into_table(x, mode, wl_bins, lam, n_bins, lam_lo, c->nlam, T_nodes, n_T, p_nodes,
                     n_p, row_off.data(), c->sp[s].d_tab, c->device));
  return scan_nan(c, s);
}

int frei_set_mmr(frei_ctx* c, const double* mmr) {
  if (!c || !mmr) return fail("null argument");
  const size_t n = (size_t)c->S * c->nL * c->n_atm;
  // A chemistry provider evaluated between sweeps (T-dependent, frei_amd Engine) sets new mixing
  // ratios before every sweep.  When the metadata is built and the sweep sums the species itself
  // (no contraction K3 formed from the old ratios), nothing else depends on them: they only go up
  // to the device before the next sweep forms its step records — not a metadata rebuild (bracket
  // searches, uploads and stream synchronizations) per sweep.
  const bool light = !c->meta_dirty && !c->eff && c->mmr.size() == n && c->d_mmr != nullptr;
  c->mmr.assign(mmr, mmr + n);
  if (light) c->mmr_dirty = true;
  else c->meta_dirty = true;
  return 0;
}

int frei_set_ftoa_batch(frei_ctx* c, const double* f_toa) {
  if (!c || !f_toa) return fail("null argument");
  if (c->n_atm < 2) return fail("frei_set_ftoa_batch needs a batched context (frei_set_grid sets F_TOA)");
  if (!c->grid_set) return fail("frei_set_grid must be called first");
  TRY(set_device(c));
  const size_t n = (size_t)c->nlam * c->n_atm;
  double* d = nullptr;
  TRY(dalloc(&d, n));
  if (h2d(d, f_toa, n, c->stream) || hipStreamSynchronize(c->stream) != hipSuccess) {
    dfree(d);
    return fail("F_TOA upload failed");
  }
  dfree(c->d_ftoa);
  c->d_ftoa = d;
  c->ftoa_per_atm = true;
  return 0;
}

int frei_set_chemistry(frei_ctx* c, const double* values, const double* T_nodes, int n_T,
                       const double* p_nodes, int n_p) {
  if (!c) return fail("null argument");
  if (!c->grid_set) return fail("frei_set_grid must be called first");
  TRY(set_device(c));
  if (!values) {   // back to the fixed per-layer mmr arrays
    c->chem_on = false;
    c->meta_dirty = true;
    return 0;
  }
  if (c->n_atm > 1) return fail("a chemistry table is per atmosphere: not for batched contexts");
  if (!T_nodes || !p_nodes || n_T < 1 || n_p < 1) return fail("chemistry table needs nodes");
  for (int k = 1; k < n_T; ++k)
    if (!(T_nodes[k] > T_nodes[k - 1])) return fail("chemistry T nodes must ascend");
  for (int k = 0; k < n_p; ++k)
    if (!(p_nodes[k] > 0) || (k > 0 && !(p_nodes[k] > p_nodes[k - 1])))
      return fail("chemistry p nodes must be positive and ascend");
  const int nL = c->nL;
  const size_t nv = (size_t)c->S * n_T * n_p;
  c->chem_tab.assign(values, values + nv);
  c->chem_T.assign(T_nodes, T_nodes + n_T);
  c->chem_logp.resize(n_p);
  for (int k = 0; k < n_p; ++k) c->chem_logp[k] = std::log10(p_nodes[k]);
  std::vector<int32_t> pj(nL);
  std::vector<double> pz(nL);
  for (int l = 0; l < nL; ++l)   // layer pressures are fixed: their log10 p brackets once
    chem_bracket(c->chem_logp.data(), n_p, std::log10(c->p[l]), pj[l], pz[l]);
  dfree(c->d_chem_tab);
  dfree(c->d_chem_T);
  dfree(c->d_chem_pj);
  dfree(c->d_chem_pz);
  TRY(dalloc(&c->d_chem_tab, nv));
  TRY(dalloc(&c->d_chem_T, n_T));
  TRY(dalloc(&c->d_chem_pj, nL));
  TRY(dalloc(&c->d_chem_pz, nL));
  TRY(h2d(c->d_chem_tab, c->chem_tab.data(), nv, c->stream));
  TRY(h2d(c->d_chem_T, c->chem_T.data(), n_T, c->stream));
  TRY(h2d(c->d_chem_pj, pj.data(), nL, c->stream));
  TRY(h2d(c->d_chem_pz, pz.data(), nL, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  c->chem_nT = n_T;
  c->chem_np = n_p;
  c->chem_on = true;
  c->meta_dirty = true;   // the species contraction (K3) no longer applies
  return 0;
}

int frei_set_gravity(frei_ctx* c, const double* g) {
  if (!c || !g) return fail("null argument");
  if (c->n_atm < 2) return fail("frei_set_gravity needs a batched context (frei_set_grid sets g)");
  for (int m = 0; m < c->n_atm; ++m)
    if (!(g[m] > 0)) return fail("g must be positive");
  TRY(set_device(c));
  TRY(h2d(c->d_g, g, c->n_atm, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return 0;
}

int frei_set_fluxes(frei_ctx* c, const double* up, const double* down) {
  if (!c) return fail("null argument");
  TRY(set_device(c));
  const size_t F = (size_t)c->nL * c->nlam * c->n_atm;
  if (up) TRY(h2d(c->d_Fu, up, F, c->stream));
  if (down) TRY(h2d(c->d_Fd, down, F, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return 0;
}

int frei_get_fluxes(frei_ctx* c, double* up, double* down) {
  if (!c) return fail("null argument");
  TRY(set_device(c));
  const size_t F = (size_t)c->nL * c->nlam * c->n_atm;
  HIP_TRY(hipStreamSynchronize(c->stream));
  if (up) HIP_TRY(hipMemcpy(up, c->d_Fu, F * sizeof(double), hipMemcpyDeviceToHost));
  if (down) HIP_TRY(hipMemcpy(down, c->d_Fd, F * sizeof(double), hipMemcpyDeviceToHost));
  return 0;
}

int frei_get_spectrum(frei_ctx* c, double* spec) {
  if (!c || !spec) return fail("null argument");
  if (c->n_atm > 1) return fail("frei_get_spectrum is per atmosphere: use frei_run_batch");
  TRY(set_device(c));
  HIP_TRY(hipStreamSynchronize(c->stream));
  HIP_TRY(hipMemcpy(spec, c->d_Fu + (size_t)(c->nL - 1) * c->nlam, c->nlam * sizeof(double),
                    hipMemcpyDeviceToHost));
  return 0;
}

int frei_set_temperatures(frei_ctx* c, const double* T) {
  if (!c || !T) return fail("null argument");
  const size_t n = (size_t)c->nL * c->n_atm;
  for (size_t l = 0; l < n; ++l)
    if (!(T[l] > 0)) return fail("temperatures must be positive");
  TRY(set_device(c));
  home_temperatures(c);
  TRY(h2d(c->d_T, T, n, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return 0;
}

int frei_get_temperatures(frei_ctx* c, double* T) {
  if (!c || !T) return fail("null argument");
  TRY(set_device(c));
  const size_t n = (size_t)c->nL * c->n_atm;
  HIP_TRY(hipMemcpyAsync(c->h_T, c->d_T, n * sizeof(double), hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  std::memcpy(T, c->h_T, n * sizeof(double));
  return 0;
}

int frei_sweep(frei_ctx* c, int direction, double alpha, double* dT, double* bol,
               double* dtaus) {
  if (c && c->n_atm > 1) return fail("frei_sweep is per atmosphere: use frei_iterate / frei_run_batch");
  if (!ready(c)) return fail("context not ready (frei_set_grid)");
  if (direction != FREI_EMIT && direction != FREI_ABSORB) return fail("bad direction");
  TRY(set_device(c));
  TRY(build_meta(c));
  SweepOpts o;
  o.dir = direction;
  o.force = 1;
  o.alpha = alpha;
  o.dT_out = c->d_dT;
  o.bol_out = c->d_bol;
  if (dtaus) {
    TRY(ensure_dtaus(c));
    o.dtaus = c->d_dtaus;
  }
  c->dtaus_valid = false;
  launch_setup(setup_args(c), direction, c->stream);
  HIP_TRY(hipGetLastError());
  TRY(run_sweep(c, o));
  // the small results through pinned staging, ordered on the stream: one synchronisation
  if (dT) HIP_TRY(hipMemcpyAsync(c->h_dT, c->d_dT, c->nL * sizeof(double), hipMemcpyDeviceToHost,
                                 c->stream));
  if (bol) HIP_TRY(hipMemcpyAsync(c->h_bol, c->d_bol, c->nL * 4 * sizeof(double),
                                  hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  TRY(check_comm(c));
  if (dT) std::memcpy(dT, c->h_dT, c->nL * sizeof(double));
  if (bol) {
    std::memcpy(bol, c->h_bol, c->nL * 4 * sizeof(double));
    // rows of layers a sweep does not visit are undefined on the device: zero them
    const int skip = (direction == FREI_EMIT) ? 0 : c->nL - 1;
    for (int q = 0; q < 4; ++q) bol[skip * 4 + q] = 0.0;
  }
  if (dtaus)
    HIP_TRY(hipMemcpy(dtaus, c->d_dtaus, (size_t)c->nL * c->nlam * sizeof(double),
                      hipMemcpyDeviceToHost));
  return 0;
}

int frei_state_init(frei_ctx* c, const double* T_init) {
  if (!ready(c) || !T_init) return fail("context not ready or null T_init");
  TRY(set_device(c));
  TRY(build_meta(c));
  c->has_pend = false;   // an update deferred by an interrupted run must not land on the new T
  home_temperatures(c);
  TRY(h2d(c->d_T, T_init, (size_t)c->nL * c->n_atm, c->stream));
  const size_t F = (size_t)c->nL * c->nlam * c->n_atm;
  HIP_TRY(hipMemsetAsync(c->d_Fu, 0, F * sizeof(double), c->stream));  // core.py:265-266
  HIP_TRY(hipMemsetAsync(c->d_Fd, 0, F * sizeof(double), c->stream));
  TRY(reset_loop_state(c));
  launch_setup(setup_args(c), kEmit, c->stream, c->n_atm);
  HIP_TRY(hipGetLastError());
  return 0;
}

static int iterate_steps(frei_ctx* c, int n, int nzc, double thr, double alpha, bool stop);

// An error part-way leaves no update deferred (drop_pending): a later frei_state_init + sweep
// must not flush a stale one over the freshly uploaded temperatures, and a read without
// frei_state_init sees the deferred update's input temperatures, not its poisoned output.
static int iterate_direct(frei_ctx* c, int n, int nzc, double thr, double alpha, bool stop) {
  const int rc = iterate_steps(c, n, nzc, thr, alpha, stop);
  if (rc != 0) drop_pending(c);
  return rc;
}

static int iterate_steps(frei_ctx* c, int n, int nzc, double thr, double alpha, bool stop) {
  for (int it = 0; it < n; ++it) {
    SweepOpts e;
    e.dir = kEmit;
    e.next_dir = kAbsorb;
    e.track = 1;
    e.alpha = alpha;
    e.live_only = 1;
    TRY(run_sweep(c, e, true));
    SweepOpts a = e;
    a.dir = kAbsorb;
    a.next_dir = kEmit;
    a.stop_on_conv = stop ? 1 : 0;
    a.n_zero_crossings = nzc;
    a.convergence_dT = thr;
    TRY(run_sweep(c, a, true));
  }
  return flush_update(c);   // no call returns with an update still deferred
}

// Graph replay applies when one iteration is two fused launches pairs on one rank with no
// per-launch host work (no events, no exchange), i.e. when its kernel arguments repeat.
static bool graph_ok(frei_ctx* c) {
  return c->use_graph && c->graph_iters > 0 && !c->timing && c->fused_update && c->n_atm == 1 &&
         c->nranks == 1 && !c->comm && !c->d_mbox;
}

static int iterate(frei_ctx* c, int n, int nzc, double thr, double alpha, bool stop) {
  const int G = c->graph_iters;
  if (!graph_ok(c) || n < G) return iterate_direct(c, n, nzc, thr, alpha, stop);
  // the hashes of one iteration's launches as they would be issued now
  std::vector<uint64_t> key;
  c->keys = &key;
  c->dry = true;
  // the dry pass launches nothing, so it must leave no state behind that a real sweep reads:
  // run_sweep clears / sets rec_skipped as it would for real launches
  const bool rec_skipped = c->rec_skipped;
  const int rc = iterate_direct(c, 1, nzc, thr, alpha, stop);
  c->rec_skipped = rec_skipped;
  c->dry = false;
  c->keys = nullptr;
  TRY(rc);
  // sweep, fused update, sweep, fused update (0: a launch that is not replayable)
  const bool fused_only = key.size() == 4 && std::find(key.begin(), key.end(), 0ull) == key.end();
  if (!fused_only) return iterate_direct(c, n, nzc, thr, alpha, stop);
  if (!c->g_exec || key != c->g_key) {
    if (c->g_exec) (void)hipGraphExecDestroy(c->g_exec);
    c->g_exec = nullptr;
    c->g_key.clear();
    hipGraph_t g = nullptr;
    HIP_TRY(hipStreamBeginCapture(c->stream, hipStreamCaptureModeThreadLocal));
    const int rc2 = iterate_direct(c, G, nzc, thr, alpha, stop);
    const hipError_t e = hipStreamEndCapture(c->stream, &g);
    TRY(rc2);
    if (e != hipSuccess) return fail(std::string("hipStreamEndCapture: ") + hipGetErrorString(e));
    const hipError_t ei = hipGraphInstantiate(&c->g_exec, g, nullptr, nullptr, 0);
    (void)hipGraphDestroy(g);
    if (ei != hipSuccess) {
      c->g_exec = nullptr;
      return fail(std::string("hipGraphInstantiate: ") + hipGetErrorString(ei));
    }
    c->g_key = key;
    ++c->g_captures;
    // the capture swapped the temperature buffers 2 G times: an even count, back in place
  }
  int done = 0;
  for (; done + G <= n; done += G) {
    HIP_TRY(hipGraphLaunch(c->g_exec, c->stream));
    ++c->g_replays;
  }
  return iterate_direct(c, n - done, nzc, thr, alpha, stop);
}

int frei_iterate(frei_ctx* c, int n, int n_zero_crossings, double convergence_dT,
                 double alpha) {
  if (!ready(c)) return fail("context not ready");
  TRY(set_device(c));
  TRY(ensure_hist(c, 1));
  const bool stop = n_zero_crossings >= 0;
  return iterate(c, n, stop ? n_zero_crossings : 0x7fffffff, convergence_dT, alpha, stop);
}

int frei_graph_info(frei_ctx* c, int* captures, int* replays) {
  if (!c) return fail("null argument");
  if (captures) *captures = c->g_captures;
  if (replays) *replays = c->g_replays;
  return 0;
}

int frei_comm_shared_device(frei_ctx* c, int shared) {
  if (!c) return fail("null argument");
  c->shared_device = shared != 0;
  return 0;
}

int frei_device_pci_bus_id(int device, char* buf, int len) {
  if (!buf || len < 16) return fail("null argument or buffer under 16 bytes");
  HIP_TRY(hipDeviceGetPCIBusId(buf, len, device));
  return 0;
}

int frei_tail_info(frei_ctx* c, int64_t* launches) {
  if (!c || !launches) return fail("null argument");
  *launches = c->n_tail;
  return 0;
}

int frei_chain_info(frei_ctx* c, int64_t* chained) {
  if (!c || !chained) return fail("null argument");
  *chained = c->n_chained;
  return 0;
}

int frei_synchronize(frei_ctx* c) {
  if (!c) return fail("null argument");
  TRY(set_device(c));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return check_comm(c);
}

int frei_run(frei_ctx* c, const double* T_init, int n_timesteps, int n_zero_crossings,
             double convergence_dT, double alpha, int* n_iter, double* T_final,
             double* temp_hist, double* dtaus, double* spectrum) {
  if (!ready(c) || !T_init || !n_iter) return fail("context not ready or null argument");
  if (c->n_atm > 1) return fail("batched context: use frei_run_batch");
  if (n_timesteps < 1) return fail("n_timesteps must be >= 1");
  TRY(set_device(c));
  TRY(ensure_hist(c, n_timesteps));
  TRY(frei_state_init(c, T_init));
  // device-resident loop; poll the convergence flag one chunk behind
  const int chunk = 4;
  int launched = 0, k = 0;
  while (launched < n_timesteps) {
    const int n = std::min(chunk, n_timesteps - launched);
    TRY(iterate(c, n, n_zero_crossings, convergence_dT, alpha, true));
    launched += n;
    HIP_TRY(hipMemcpyAsync(&c->h_flag[k & 1], c->d_conv, sizeof(int), hipMemcpyDeviceToHost,
                           c->stream));
    HIP_TRY(hipEventRecord(c->flag_ev[k & 1], c->stream));
    if (k > 0) {
      HIP_TRY(hipEventSynchronize(c->flag_ev[(k - 1) & 1]));
      if (c->h_flag[(k - 1) & 1]) break;
    }
    ++k;
  }
  // final emit without alpha (alpha = 1, core.py:323-333), writes dtaus
  TRY(ensure_dtaus(c));
  c->dtaus_valid = true;
  SweepOpts f;
  f.dir = kEmit;
  f.force = 1;
  f.alpha = 1.0;
  f.dtaus = c->d_dtaus;
  TRY(run_sweep(c, f));
  HIP_TRY(hipStreamSynchronize(c->stream));
  TRY(check_comm(c));
  int it = 0;
  HIP_TRY(hipMemcpy(&it, c->d_iter, sizeof(int), hipMemcpyDeviceToHost));
  *n_iter = it;
  const int nL = c->nL;
  if (T_final) HIP_TRY(hipMemcpy(T_final, c->d_T, nL * sizeof(double), hipMemcpyDeviceToHost));
  if (temp_hist && it > 0) {
    std::vector<double> h((size_t)it * 2 * nL);
    HIP_TRY(hipMemcpy(h.data(), c->d_hist, h.size() * sizeof(double), hipMemcpyDeviceToHost));
    for (int l = 0; l < nL; ++l)
      for (int col = 0; col < 2 * it; ++col) temp_hist[(size_t)l * 2 * it + col] = h[(size_t)col * nL + l];
  }
  if (dtaus)
    HIP_TRY(hipMemcpy(dtaus, c->d_dtaus, (size_t)nL * c->nlam * sizeof(double),
                      hipMemcpyDeviceToHost));
  if (spectrum)
    HIP_TRY(hipMemcpy(spectrum, c->d_Fu + (size_t)(nL - 1) * c->nlam, c->nlam * sizeof(double),
                      hipMemcpyDeviceToHost));
  return 0;
}

int frei_run_batch(frei_ctx* c, const double* T_init, int n_timesteps, int n_zero_crossings,
                   double convergence_dT, double alpha, int* n_iter, double* T_final,
                   double* spectra) {
  if (!ready(c) || !T_init || !n_iter) return fail("context not ready or null argument");
  if (n_timesteps < 1) return fail("n_timesteps must be >= 1");
  TRY(set_device(c));
  TRY(ensure_hist(c, n_timesteps));
  TRY(frei_state_init(c, T_init));
  const int A = c->n_atm;
  int* flags = c->h_conv ? c->h_conv : c->h_flag;   // pinned [2][A]
  // every atmosphere iterates until its own convergence test holds (its kernels then
  // return at once); the host polls all flags one chunk behind
  const int chunk = 4;
  int launched = 0, k = 0;
  while (launched < n_timesteps) {
    const int n = std::min(chunk, n_timesteps - launched);
    TRY(iterate(c, n, n_zero_crossings, convergence_dT, alpha, true));
    launched += n;
    HIP_TRY(hipMemcpyAsync(flags + (k & 1) * A, c->d_conv, A * sizeof(int),
                           hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipEventRecord(c->flag_ev[k & 1], c->stream));
    if (k > 0) {
      HIP_TRY(hipEventSynchronize(c->flag_ev[(k - 1) & 1]));
      bool all = true;
      for (int m = 0; m < A; ++m) all = all && flags[((k - 1) & 1) * A + m] != 0;
      if (all) break;
    }
    ++k;
  }
  // final emit of every atmosphere without alpha (alpha = 1, core.py:323-333)
  SweepOpts f;
  f.dir = kEmit;
  f.force = 1;
  f.alpha = 1.0;
  TRY(run_sweep(c, f));
  HIP_TRY(hipStreamSynchronize(c->stream));
  HIP_TRY(hipMemcpy(n_iter, c->d_iter, A * sizeof(int), hipMemcpyDeviceToHost));
  const size_t nL = c->nL;
  if (T_final)
    HIP_TRY(hipMemcpy(T_final, c->d_T, nL * A * sizeof(double), hipMemcpyDeviceToHost));
  if (spectra)  // F_up[n_layers - 1] of every atmosphere
    HIP_TRY(hipMemcpy2D(spectra, c->nlam * sizeof(double),
                        c->d_Fu + (nL - 1) * c->nlam, nL * c->nlam * sizeof(double),
                        c->nlam * sizeof(double), A, hipMemcpyDeviceToHost));
  return 0;
}

int frei_kappa(frei_ctx* c, double T, double p, double* k, double* sigma) {
  if (!ready(c) || !k) return fail("context not ready or null argument");
  if (c->n_atm > 1) return fail("frei_kappa is per atmosphere: use a single-atmosphere context");
  TRY(set_device(c));
  TRY(build_meta(c));
  std::vector<TermP> terms(c->S);
  for (int s = 0; s < c->S; ++s) {
    const Species& q = c->sp[s];
    const SpecMeta& sm = c->smeta[s];
    // pressure bracket of the query point (same rules as build_meta)
    std::vector<int32_t> pp(q.n_p);
    std::iota(pp.begin(), pp.end(), 0);
    std::stable_sort(pp.begin(), pp.end(),
                     [&](int a, int b) { return q.p_nodes[a] < q.p_nodes[b]; });
    std::vector<double> ps(q.n_p);
    for (int i = 0; i < q.n_p; ++i) ps[i] = q.p_nodes[pp[i]];
    PMeta pm{};
    if (sm.one_T) {
      int jx = (int)(std::lower_bound(ps.begin(), ps.end(), p) - ps.begin());
      jx = std::max(1, std::min(jx, q.n_p - 1));
      pm.p_lo = pp[jx - 1];
      pm.p_hi = pp[jx];
      pm.x1 = p - ps[jx - 1];
      pm.dx = ps[jx] - ps[jx - 1];
      pm.oob = (p < ps[0] || p > ps[q.n_p - 1]) ? 1 : 0;
    } else {
      int i, oob;
      double y;
      bracket(ps.data(), q.n_p, p, i, y, oob);
      pm.p_lo = pp[i];
      pm.p_hi = pp[i + 1];
      pm.wp_lo = 1.0 - y;
      pm.wp_hi = y;
      pm.oob = oob;
    }
    // mmr: the chemistry table at (T, p) when set (opacity.py:246-248), else the layer whose
    // pressure equals p, else the first layer's value
    double m = c->mmr[(size_t)s * c->nL];
    for (int l = 0; l < c->nL; ++l)
      if (c->p[l] == p) m = c->mmr[(size_t)s * c->nL + l];
    if (c->chem_on) {
      int j;
      double z;
      chem_bracket(c->chem_logp.data(), c->chem_np, std::log10(p), j, z);
      ChemArgs h{c->chem_tab.data(), c->chem_T.data(), nullptr, nullptr, c->chem_nT, c->chem_np};
      m = chem_mmr_at(h, s, j, z, T);
    }
    terms[s] = make_term(sm, pm, c->tnodes.data(), c->tperm.data(), m, T, 0);
  }
  TermP* d_terms = nullptr;
  double* d_k = nullptr;
  TRY(dalloc(&d_terms, c->S));
  TRY(dalloc(&d_k, c->nlam));
  TRY(h2d(d_terms, terms.data(), c->S, c->stream));
  launch_kappa(c->nlam, d_terms, c->S, c->d_sig, d_k, c->stream);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipStreamSynchronize(c->stream));
  HIP_TRY(hipMemcpy(k, d_k, c->nlam * sizeof(double), hipMemcpyDeviceToHost));
  if (sigma) HIP_TRY(hipMemcpy(sigma, c->d_sig, c->nlam * sizeof(double), hipMemcpyDeviceToHost));
  dfree(d_terms);
  dfree(d_k);
  return 0;
}

int frei_propagate_fluxes(int device, int64_t n, const double* c1, const double* lk,
                          const double* F_1_up, const double* F_2_down, double T_1,
                          double T_2, const double* delta_tau, const double* omega_0,
                          const double* g_0, double* F_2_up, double* F_1_down) {
  if (n <= 0) return 0;
  if (!c1 || !lk || !F_1_up || !F_2_down || !delta_tau || !omega_0 || !F_2_up || !F_1_down)
    return fail("null argument");
  HIP_TRY(hipSetDevice(device));
  // inputs c1, lk, F_1_up, F_2_down, delta_tau, omega_0 [, g_0]; outputs F_2_up, F_1_down
  const double* in[7] = {c1, lk, F_1_up, F_2_down, delta_tau, omega_0, g_0};
  const int n_in = g_0 ? 7 : 6;
  double* d[9] = {};
  hipStream_t st = nullptr;
  int rc = 0;
  if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess)
    return fail("hipStreamCreate failed");
  for (int i = 0; i < n_in + 2 && !rc; ++i) rc = dalloc(&d[i], n);
  for (int i = 0; i < n_in && !rc; ++i) rc = h2d(d[i], in[i], n, st);
  if (!rc) {
    launch_propagate(n, d[0], d[1], d[2], d[3], T_1, T_2, d[4], d[5], g_0 ? d[6] : nullptr,
                     d[n_in], d[n_in + 1], st);
    if (hipGetLastError() != hipSuccess) rc = fail("propagate kernel launch failed");
  }
  if (!rc && (hipMemcpyAsync(F_2_up, d[n_in], n * sizeof(double), hipMemcpyDeviceToHost, st) !=
                  hipSuccess ||
              hipMemcpyAsync(F_1_down, d[n_in + 1], n * sizeof(double), hipMemcpyDeviceToHost,
                             st) != hipSuccess))
    rc = fail("propagate copy failed");
  if (hipStreamSynchronize(st) != hipSuccess && !rc) rc = fail("propagate kernel failed");
  for (double*& p : d) dfree(p);
  (void)hipStreamDestroy(st);
  return rc;
}

int frei_comm_unique_id(void* id128) {
  if (!id128) return fail("null argument");
  Rccl* r = rccl();
  if (!r) return fail("librccl.so.1 not loadable");
  int rc = r->getUniqueId(id128);
  if (rc != 0) return fail("ncclGetUniqueId failed");
  return 0;
}

int frei_comm_init(frei_ctx* c, int nranks, int rank, const void* id128) {
  if (c && c->n_atm > 1)
    return fail("batched contexts shard atmospheres across ranks: no exchange");
  if (!c || !id128) return fail("null argument");
  if (nranks < 1 || rank < 0 || rank >= nranks) return fail("bad rank/nranks");
  TRY(set_device(c));
  const char* force = getenv("FREI_FORCE_RCCL");
  if (nranks == 1 && !(force && force[0] == '1')) {
    c->nranks = 1;
    c->rank = 0;
    return 0;
  }
  Rccl* r = rccl();
  if (!r) return fail("librccl.so.1 not loadable");
  Id128 id;
  std::memcpy(id.b, id128, 128);
  void* comm = nullptr;
  int rc = r->commInitRank(&comm, nranks, id, rank);
  if (rc != 0)
    return fail(std::string("ncclCommInitRank: ") + (r->errStr ? r->errStr(rc) : "error"));
  c->comm = comm;
  c->nranks = nranks;
  c->rank = rank;
  dfree(c->d_Fb_all);
  TRY(dalloc(&c->d_Fb_all, (size_t)nranks * (c->nL - 1) * 4));
  return 0;
}

int frei_comm_init_host(frei_ctx* c, int nranks, int rank, frei_allgather_fn fn, void* user) {
  if (c && c->n_atm > 1)
    return fail("batched contexts shard atmospheres across ranks: no exchange");
  if (!c || !fn) return fail("null argument");
  if (nranks < 1 || rank < 0 || rank >= nranks) return fail("bad rank/nranks");
  TRY(set_device(c));
  const size_t n = (size_t)(c->nL - 1) * 4;
  if (c->h_ag) (void)hipHostFree(c->h_ag);
  c->h_ag = nullptr;
  if (hipHostMalloc((void**)&c->h_ag, (nranks + 1) * n * sizeof(double)) != hipSuccess)
    return fail("hipHostMalloc failed");
  dfree(c->d_Fb_all);
  TRY(dalloc(&c->d_Fb_all, (size_t)nranks * n));
  c->host_ag = fn;
  c->host_ag_user = user;
  c->nranks = nranks;
  c->rank = rank;
  return 0;
}

// ---- P2P exchange: mailbox + IPC handle, then map every rank's mailbox.
int frei_comm_p2p_handle(frei_ctx* c, int nranks, int rank, void* handle64) {
  if (c && c->n_atm > 1)
    return fail("batched contexts shard atmospheres across ranks: no exchange");
  if (!c || !handle64) return fail("null argument");
  if (nranks < 1 || rank < 0 || rank >= nranks) return fail("bad rank/nranks");
  if (c->comm || c->host_ag || c->d_mbox) return fail("communicator already initialised");
  TRY(set_device(c));
  const int64_t n = (int64_t)(c->nL - 1) * 4;
  void* mb = nullptr;
  HIP_TRY(hipExtMallocWithFlags(&mb, mbox_bytes(nranks, n), hipDeviceMallocUncached));
  c->d_mbox = static_cast<double*>(mb);
  // flags 0: nothing published; complete before the handle goes to the peers
  HIP_TRY(hipMemsetAsync(c->d_mbox, 0, mbox_bytes(nranks, n), c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  hipIpcMemHandle_t h;
  HIP_TRY(hipIpcGetMemHandle(&h, c->d_mbox));
  std::memcpy(handle64, &h, sizeof(h));
  c->nranks = nranks;
  c->rank = rank;
  if (const char* e = getenv("FREI_P2P_TIMEOUT_S")) c->p2p_timeout_s = atof(e);
  return 0;
}

int frei_comm_p2p_open(frei_ctx* c, const void* handles) {
  if (!c || !handles) return fail("null argument");
  if (!c->d_mbox) return fail("frei_comm_p2p_handle first");
  if (c->d_peers) return fail("P2P mailboxes already mapped");
  TRY(set_device(c));
  const int R = c->nranks;
  std::vector<double*> ptr(R, nullptr);
  for (int r = 0; r < R; ++r) {
    if (r == c->rank) {
      ptr[r] = c->d_mbox;
      continue;
    }
    hipIpcMemHandle_t h;
    std::memcpy(&h, static_cast<const char*>(handles) + (size_t)r * sizeof(h), sizeof(h));
    void* p = nullptr;
    HIP_TRY(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess));
    c->peer_mapped.push_back(p);
    ptr[r] = static_cast<double*>(p);
  }
  TRY(dalloc(&c->d_peers, R));
  TRY(h2d(c->d_peers, ptr.data(), R, c->stream));
  TRY(dalloc(&c->d_comm_err, 1));
  TRY(dalloc(&c->d_wait_ticks, 1));
  HIP_TRY(hipMemsetAsync(c->d_comm_err, 0, sizeof(int), c->stream));
  HIP_TRY(hipMemsetAsync(c->d_wait_ticks, 0, sizeof(unsigned long long), c->stream));
  dfree(c->d_Fb_all);
  TRY(dalloc(&c->d_Fb_all, (size_t)R * (c->nL - 1) * 4));
  // handshake: every rank publishes flag 1 in every mailbox and waits for all (bounded)
  P2PPush push{};
  push.peers = c->d_peers;
  push.nranks = R;
  push.rank = c->rank;
  push.n = (int64_t)(c->nL - 1) * 4;
  push.seq = ++c->p2p_seq;
  P2PWait wait{};
  wait.mbox = c->d_mbox;
  wait.nranks = R;
  wait.n = push.n;
  wait.seq = push.seq;
  wait.timeout_ticks = (int64_t)(std::min(c->p2p_timeout_s, 20.0) * 1e8);
  wait.err = c->d_comm_err;
  launch_p2p_handshake(push, wait, c->stream);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipStreamSynchronize(c->stream));
  return check_comm(c);
}

// dtaus for post-processing: the caller's host array (uploaded) or the device copy.
static int post_dtaus(frei_ctx* c, const double* h, double** tmp, const double** d) {
  *tmp = nullptr;
  if (c->n_atm > 1) return fail("post-processing is per atmosphere: use a single context");
  if (h) {
    const size_t n = (size_t)c->nL * c->nlam;
    TRY(dalloc(tmp, n));
    TRY(h2d(*tmp, h, n, c->stream));
    *d = *tmp;
    return 0;
  }
  if (!c->dtaus_valid || !c->d_dtaus) return fail("no device dtaus: run frei_run first or pass dtaus");
  *d = c->d_dtaus;
  return 0;
}

int frei_milne_pressure(frei_ctx* c, const double* dtaus, const double* p_bar,
                        double* p_milne) {
  if (!ready(c) || !p_bar || !p_milne) return fail("context not ready or null argument");
  TRY(set_device(c));
  double *tmp = nullptr, *d_fp = nullptr, *d_out = nullptr;
  const double* d_dt = nullptr;
  int rc = post_dtaus(c, dtaus, &tmp, &d_dt);
  if (!rc) rc = dalloc(&d_fp, c->nL);
  if (!rc) rc = dalloc(&d_out, c->nlam);
  if (!rc) rc = h2d(d_fp, p_bar, c->nL, c->stream);
  if (!rc) {
    launch_milne(d_dt, c->nL, c->nlam, d_fp, d_out, c->stream);
    if (hipGetLastError() != hipSuccess) rc = fail("milne kernel launch failed");
  }
  if (!rc && hipMemcpyAsync(p_milne, d_out, c->nlam * sizeof(double), hipMemcpyDeviceToHost,
                            c->stream) != hipSuccess)
    rc = fail("milne copy failed");
  if (hipStreamSynchronize(c->stream) != hipSuccess && !rc) rc = fail("milne kernel failed");
  dfree(tmp), dfree(d_fp), dfree(d_out);
  return rc;
}

int frei_contribution(frei_ctx* c, const double* dtaus, const double* nu, const double* ratio,
                      const double* T, double hcperk, double* cf) {
  if (!ready(c) || !nu || !ratio || !T || !cf) return fail("context not ready or null argument");
  TRY(set_device(c));
  double *tmp = nullptr, *d_nu = nullptr, *d_ratio = nullptr, *d_T = nullptr, *d_cf = nullptr;
  const double* d_dt = nullptr;
  const size_t n = (size_t)c->nL * c->nlam;
  int rc = post_dtaus(c, dtaus, &tmp, &d_dt);
  if (!rc) rc = dalloc(&d_nu, c->nlam);
  if (!rc) rc = dalloc(&d_ratio, c->nL);
  if (!rc) rc = dalloc(&d_T, c->nL);
  if (!rc) rc = dalloc(&d_cf, n);
  if (!rc) rc = h2d(d_nu, nu, c->nlam, c->stream);
  if (!rc) rc = h2d(d_ratio, ratio, c->nL, c->stream);
  if (!rc) rc = h2d(d_T, T, c->nL, c->stream);
  if (!rc) {
    launch_contribution(d_dt, c->nL, c->nlam, d_nu, d_ratio, d_T, hcperk, d_cf, c->stream);
    if (hipGetLastError() != hipSuccess) rc = fail("contribution kernel launch failed");
  }
  if (!rc && hipMemcpyAsync(cf, d_cf, n * sizeof(double), hipMemcpyDeviceToHost, c->stream) !=
                 hipSuccess)
    rc = fail("contribution copy failed");
  if (hipStreamSynchronize(c->stream) != hipSuccess && !rc) rc = fail("contribution kernel failed");
  dfree(tmp), dfree(d_nu), dfree(d_ratio), dfree(d_T), dfree(d_cf);
  return rc;
}

int frei_ctx_path(frei_ctx* c, int* flags) {
  if (!ready(c) || !flags) return fail("context not ready or null argument");
  TRY(set_device(c));
  TRY(build_meta(c));
  int nan = 0;
  for (const auto& q : c->sp) nan = nan || q.has_nan;
  // the form run_sweep launches: a loop's sweeps after the first merge a deferred update when
  // chained launches apply
  const FastForm m = fast_form(c, chain_ready(c));
  const int Q = m.Q, NC = m.NC;
  const bool lam2 = c->fast && m.lam2;
  *flags = (c->fast ? 1 : 0) | (c->fast && c->shared ? 2 : 0) | (c->eff ? 4 : 0) |
           (nan ? 8 : 0) | (NC == 0 && Q == 2 ? 16 : 0) | (NC == 0 && Q == 4 ? 32 : 0) |
           (NC << 6) | (lam2 ? 512 : 0) |
           (c->fast && NC > 0 && !chain_ready(c) && tail_blocks(c, (int)((c->nlam + 255) / 256)) > 0
                ? 1024 : 0) |
           (c->lazy_on ? 2048 : 0);
  return 0;
}

int frei_set_option(frei_ctx* c, const char* name, int value) {
  if (!c || !name) return fail("null argument");
  return set_option(c, name, value);
}

int frei_setup_timing(frei_ctx* c, double* ms) {
  if (!c || !ms) return fail("null argument");
  for (int k = 0; k < 5; ++k) ms[k] = c->setup_ms[k];
  return 0;
}

int frei_contract_timing(frei_ctx* c, double* ms, double* bytes) {
  if (!c || !ms || !bytes) return fail("null argument");
  *ms = c->contract_ms;
  *bytes = c->contract_bytes;
  return 0;
}

int frei_timing_enable(frei_ctx* c, int on) {
  if (!c) return fail("null argument");
  TRY(set_device(c));
  HIP_TRY(hipStreamSynchronize(c->stream));
  c->timing = on != 0;
  c->ev_used = 0;
  c->xev_used = 0;
  if (c->d_wait_ticks)
    HIP_TRY(hipMemsetAsync(c->d_wait_ticks, 0, sizeof(unsigned long long), c->stream));
  return 0;
}

int frei_timing_read(frei_ctx* c, double* total_ms, int* n_launches) {
  if (!c || !total_ms || !n_launches) return fail("null argument");
  TRY(set_device(c));
  HIP_TRY(hipStreamSynchronize(c->stream));
  double tot = 0;
  for (size_t k = 0; k + 1 < c->ev_used; k += 2) {
    float ms = 0;
    HIP_TRY(hipEventElapsedTime(&ms, c->ev_pool[k], c->ev_pool[k + 1]));
    tot += ms;
  }
  *total_ms = tot;
  *n_launches = (int)(c->ev_used / 2);
  return 0;
}

int frei_timing_read_exchange(frei_ctx* c, double* total_ms, int* n_calls) {
  if (!c || !total_ms || !n_calls) return fail("null argument");
  TRY(set_device(c));
  HIP_TRY(hipStreamSynchronize(c->stream));
  if (c->d_mbox && c->d_wait_ticks) {   // P2P: time the update kernels spent waiting
    unsigned long long t = 0;
    HIP_TRY(hipMemcpy(&t, c->d_wait_ticks, sizeof(t), hipMemcpyDeviceToHost));
    *total_ms = (double)t * 1e-5;       // 100 MHz ticks
    *n_calls = (int)(c->ev_used / 2);   // one wait per timed sweep
    return 0;
  }
  double tot = 0;
  for (size_t k = 0; k + 1 < c->xev_used; k += 2) {
    float ms = 0;
    HIP_TRY(hipEventElapsedTime(&ms, c->xev_pool[k], c->xev_pool[k + 1]));
    tot += ms;
  }
  *total_ms = tot;
  *n_calls = (int)(c->xev_used / 2);
  return 0;
}

}  // extern "C"
