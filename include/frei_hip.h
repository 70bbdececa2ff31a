/*
 * frei_hip.h — C ABI of the MI355X (gfx950) two-stream radiative-transfer engine.
 *
 * Drop-in boundary for bmorris3/frei's hot path.  The reference
 * has no FFI: its seam is a set of Python functions, and each entry point below
 * replaces one of them (file:line in /root/reference):
 *
 *   frei_propagate_fluxes   frei/twostream.py:97-177   propagate_fluxes(...)
 *   frei_kappa              frei/opacity.py:203-269    kappa(opacities, T, p, lam, m_bar)
 *   frei_sweep              frei/twostream.py:290-421  emit(..., n_timesteps=1)
 *                           frei/twostream.py:424-550  absorb(..., n_timesteps=1)
 *   frei_run                frei/core.py:233-338       Grid.emission_spectrum(...)
 *   frei_set_table*         frei/core.py:198-231       Grid.load_opacities(opacities=...)
 *   frei_set_grid           frei/core.py:113-188,48-55 Grid(...) + F_TOA(...)
 *   frei_xsec_bin           frei/opacity.py:66-170     binned_opacity(...) (one species)
 *                           frei/interp.py:156-307     groupby_bins_agg / AggregateTrapz
 *   frei_set_table_binned   frei/core.py:198-231       Grid.load_opacities(species, path)
 *
 * Conventions (all plain pointers and sizes, no framework types):
 *   - Units are cgs: wavelength cm, pressure dyn cm^-2, T K, flux erg s^-1 cm^-3,
 *     opacity cm^2 g^-1, g cm s^-2, masses g.  Layer index 0 = bottom of atmosphere.
 *   - Every function returns 0 on success, < 0 on error; frei_last_error() then holds
 *     a message (thread-local).  The Python layer raises RuntimeError with it.
 *   - Host buffers are caller-owned and copied in/out; device buffers belong to the
 *     context.  One context per GPU; a context is not thread-safe.
 *   - A context owns the contiguous wavelength slice [lam_offset, lam_offset+n_lam)
 *     of a global grid; with nranks > 1 the per-sweep bolometric partial sums are
 *     all-gathered over RCCL (frei_comm_init) and summed in rank order, so every rank
 *     computes bitwise-identical temperatures.
 */
#ifndef FREI_HIP_H
#define FREI_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct frei_ctx frei_ctx;

enum { FREI_EMIT = 0, FREI_ABSORB = 1 };

/* Library/ABI version (major*10000 + minor*100 + patch); 2.0.0. */
int frei_version(void);
/* Message of the last failing call on this thread ("" if none). */
const char* frei_last_error(void);
/* Number of visible HIP devices. */
int frei_device_count(int* n);

/* Context for n_layers x n_lam (local slice) x n_species on `device`. */
int frei_ctx_create(frei_ctx** out, int device, int n_layers, int64_t n_lam, int n_species);
/*
 * Batched context (§8(f) #2, grid sweeps such as C5): n_atm independent atmospheres share the
 * wavelength and pressure grids and the opacity tables; each has its own temperatures,
 * gravity (frei_set_gravity) and mixing ratios (frei_set_mmr takes [n_atm][n_species]
 * [n_layers]).  The reference has no batch API: each atmosphere is the reference's
 * Grid.emission_spectrum (core.py:233-338) run independently.  Needs tables on shared
 * on-node p/T nodes without NaN; the per-atmosphere species contraction runs on fp64 MFMA
 * (K7).  State accessors (set/get fluxes and temperatures) take n_atm blocks; frei_sweep,
 * frei_run, frei_kappa, post-processing and the rank exchange are single-atmosphere only
 * (batched runs shard atmospheres across ranks with no exchange).
 */
int frei_ctx_create_batch(frei_ctx** out, int device, int n_layers, int64_t n_lam,
                          int n_species, int n_atm);
int frei_set_gravity(frei_ctx* ctx, const double* g);
/* Batched: one F_TOA per atmosphere, f_toa[n_atm][n_lam] (core.py:48-55 with each planet's
 * T_star and a/R_star; replaces frei_set_grid's shared F_TOA until the next frei_set_grid). */
int frei_set_ftoa_batch(frei_ctx* ctx, const double* f_toa);
/* Every atmosphere iterates to its own convergence (core.py:273-318), then the final emit;
 * n_iter[n_atm], T_final[n_atm][n_layers] and spectra[n_atm][n_lam] (F_up[n_layers-1]). */
int frei_run_batch(frei_ctx* ctx, const double* T_init, int n_timesteps, int n_zero_crossings,
                   double convergence_dT, double alpha, int* n_iter, double* T_final,
                   double* spectra);
int frei_ctx_destroy(frei_ctx* ctx);

/*
 * Grid and per-wavelength constants (frei/core.py:113-188, 48-55; twostream.py:46-67).
 *   c1[n_lam]     2 h c^2 / lam^5                (Planck prefactor, BB)
 *   lk[n_lam]     lam * k_B   (BB exponent h c / (lk T), formed as (h c / lk) * (1 / T))
 *   sigma[n_lam]  Rayleigh H2 + He, cm^2 g^-1    (opacity.py:173-200, 233)
 *   f_toa[n_lam]  stellar flux at TOA            (core.py:48-55)
 *   trapz_w[n_lam] per-point trapezoid weights of the GLOBAL grid (cm), sliced
 *   p[n_layers]   layer pressures, dyn cm^-2, descending (tp.py:10-33)
 *   g, m_bar      planet gravity and mean molecular mass (core.py:65-106)
 */
int frei_set_grid(frei_ctx* ctx, const double* c1, const double* lk, const double* sigma,
                  const double* f_toa, const double* trapz_w, const double* p,
                  double g, double m_bar);

/*
 * Opacity table of species s (Grid.load_opacities(opacities=...), core.py:198-231):
 * values[n_p][n_T][n_lam] (row-major, this context's wavelength slice), cm^2 g^-1,
 * on nodes p_nodes[n_p] (dyn cm^-2) x T_nodes[n_T] (K), any order.  Linear
 * interpolation with fill 0 outside the node hull (opacity.py:241-263); a table with
 * one unique T is interpolated in pressure only (opacity.py:256-259).
 */
int frei_set_table(frei_ctx* ctx, int s, const double* values, const double* p_nodes, int n_p,
                   const double* T_nodes, int n_T);
/*
 * Same, but the table is generated on the device (no host copy of n_p*n_T*n_lam values):
 * values[p][t][l] = min(max((fp[p] * fT[t]) * base[l], lo), hi).  Synthetic separable
 * tables for benchmarks and parity tests.
 */
int frei_set_table_separable(frei_ctx* ctx, int s, const double* base, const double* fp,
                             const double* fT, double lo, double hi, const double* p_nodes,
                             int n_p, const double* T_nodes, int n_T);
/* Per-species, per-layer mass mixing ratios mmr[n_species][n_layers] (chemistry.py:114-205;
 * the reference's mock gives a constant VMR).  CIA-like tables take their weights here. */
int frei_set_mmr(frei_ctx* ctx, const double* mmr);

/*
 * Temperature-dependent chemistry (chemistry(T, p) inside every kappa call,
 * opacity.py:246-248; chemistry.py:114-205): mass mixing ratios values[n_species][n_T][n_p]
 * on ascending T_nodes (K) x p_nodes (dyn cm^-2).  At every sweep step the layer's mmr is
 * interpolated at its current (T_i, p_i) — linear in T and in log10 p, clamped to the nodes —
 * when the update kernel writes the next sweep's step table; the species sum then stays in
 * the sweep (no K3 contraction).  values = NULL returns to frei_set_mmr's fixed arrays.
 * Single-atmosphere contexts; call after frei_set_grid.
 */
int frei_set_chemistry(frei_ctx* ctx, const double* values, const double* T_nodes, int n_T,
                       const double* p_nodes, int n_p);

/* Flux state [n_layers][n_lam] (this slice), caller layout row-major. */
int frei_set_fluxes(frei_ctx* ctx, const double* up, const double* down);
int frei_get_fluxes(frei_ctx* ctx, double* up, double* down);
/* The emergent spectrum F_up[n_layers - 1] of this slice (n_lam values): the row the reference's
 * Grid returns as Spectrum1D(flux=fluxes_up[-1]) (frei/core.py:335-338), without reading back
 * the whole flux state. */
int frei_get_spectrum(frei_ctx* ctx, double* spectrum);
int frei_set_temperatures(frei_ctx* ctx, const double* T);
int frei_get_temperatures(frei_ctx* ctx, double* T);

/*
 * One sweep with the current temperatures (emit: twostream.py:351-407, absorb: 486-536),
 * in place on the flux state, then T <- T - dT (Q11).  alpha = mixing-length parameter.
 * Optional outputs (NULL to skip): dT[n_layers], bol[n_layers][4] = bolometric
 * (F_2_up, F_2_down, F_1_up, F_1_down) per sweep step, dtaus[n_layers][n_lam] (row 0 = 1,
 * row k = k-th step of the sweep, Q12).
 */
int frei_sweep(frei_ctx* ctx, int direction, double alpha, double* dT, double* bol,
               double* dtaus);

/*
 * Grid.emission_spectrum (core.py:233-338): zero fluxes, T = T_init, up to n_timesteps
 * (emit, absorb) iterations with the reference convergence test (sign flips of the
 * absorb temperature history > n_zero_crossings, or |dT| < convergence_dT, for all
 * layers), then a final emit with alpha = 1.  The loop stays on the device; the host
 * polls the convergence flag once per chunk of iterations.
 * Outputs: *n_iter; T_final[n_layers]; temp_hist[n_layers][2*n_iter] (may be NULL; caller
 * sizes it for n_timesteps); dtaus[n_layers][n_lam] (may be NULL); spectrum[n_lam]
 * = F_up[n_layers-1] (may be NULL).
 */
int frei_run(frei_ctx* ctx, const double* T_init, int n_timesteps, int n_zero_crossings,
             double convergence_dT, double alpha, int* n_iter, double* T_final,
             double* temp_hist, double* dtaus, double* spectrum);

/* Benchmark/driver pieces of frei_run (all asynchronous on the context's stream). */
int frei_state_init(frei_ctx* ctx, const double* T_init);
/* n T-P iterations; convergence is tracked but never stops the work when
 * n_zero_crossings < 0 (fixed-work benchmark steps). */
int frei_iterate(frei_ctx* ctx, int n, int n_zero_crossings, double convergence_dT,
                 double alpha);
int frei_synchronize(frei_ctx* ctx);

/* kappa (opacity.py:203-269) at one (T, p) on this slice: k[n_lam] (includes sigma, Q1),
 * sigma[n_lam] (may be NULL). */
int frei_kappa(frei_ctx* ctx, double T, double p, double* k, double* sigma);

/* propagate_fluxes (twostream.py:97-177), elementwise on n points; g_0[n] is the scattering
 * asymmetry factor (NULL: g_0 = 0, as at the emit/absorb call sites twostream.py:389, 518). */
int frei_propagate_fluxes(int device, int64_t n, const double* c1, const double* lk,
                          const double* F_1_up, const double* F_2_down, double T_1,
                          double T_2, const double* delta_tau, const double* omega_0,
                          const double* g_0, double* F_2_up, double* F_1_down);

/* Multi-GPU: 128-byte RCCL unique id (rank 0 creates, others receive it out of band),
 * then every rank joins.  Per sweep: one ncclAllGather of n_layers*4 doubles. */
int frei_comm_unique_id(void* id128);
int frei_comm_init(frei_ctx* ctx, int nranks, int rank, const void* id128);

/*
 * P2P exchange over xGMI without RCCL or the host: each rank allocates a
 * mailbox in uncached device memory and exports its 64-byte IPC handle
 * (frei_comm_p2p_handle); after the handles are all-gathered out of band (rank order),
 * frei_comm_p2p_open maps every rank's mailbox and runs a bounded handshake.  Per sweep the
 * update kernel pushes this rank's n_layers*4 partial sums into every mailbox with a
 * sequence flag per value and waits for every rank's flags (a rank that never publishes is
 * reported as an error after FREI_P2P_TIMEOUT_S seconds, default 30).
 * Ranks may share one GPU (processes on the same device).
 */
int frei_comm_p2p_handle(frei_ctx* ctx, int nranks, int rank, void* handle64);
int frei_comm_p2p_open(frei_ctx* ctx, const void* handles);

/* Alternative exchange for testing and for hosts without RCCL peers (e.g. several ranks
 * sharing one GPU): per sweep the n partial sums are copied to the host and
 * fn(send[n], recv[nranks*n], n, user) must all-gather them in rank order (returns 0). */
typedef int (*frei_allgather_fn)(const double* send, double* recv, int64_t n, void* user);
int frei_comm_init_host(frei_ctx* ctx, int nranks, int rank, frei_allgather_fn fn, void* user);

/*
 * Post-processing of a converged atmosphere (§8(f) #3), per wavelength on this slice.
 * dtaus[n_layers][n_lam] is the host array frei_run returned, or NULL to use the copy the
 * last frei_run left on the device.
 *   frei_milne_pressure  core.py:392-395  p_milne[j] = np.interp(2/3, exp(-dtaus[:, j]),
 *                        p_bar) (numpy's search, unsorted transmissions included); the
 *                        weighted mean and final interpolation (core.py:397-405) stay on
 *                        the host.
 *   frei_contribution    plot.py:63-79  cf[n_layers][n_lam], rows bottom-first (cf[::-1]),
 *                        from nu[n_lam] (cm^-1), ratio[n_layers] = p / dP, T[n_layers] and
 *                        hcperk = h c / k_B (cm K).
 */
int frei_milne_pressure(frei_ctx* ctx, const double* dtaus, const double* p_bar,
                        double* p_milne);
int frei_contribution(frei_ctx* ctx, const double* dtaus, const double* nu,
                      const double* ratio, const double* T, double hcperk, double* cf);

/* Which sweep implementation the context's current tables select (after metadata build):
 * bit 0 fast path (on-node pressures, >= 2 T nodes, S <= 8), bit 1 step table staged in
 * LDS (shared brackets, small slices), bit 2 species-contracted table (K3), bit 3 tables
 * hold NaN (per-species nansum variant), bit 4 / bit 5 grouped-lane sweep with two / four
 * lanes per wavelength (small slices), bits 6-8: consumer waves per block of the
 * producer/consumer sweep (1, 2 or 4; 0 = not used), bit 9 two wavelengths per lane in the
 * contracted one-lane sweep (large slices: option "lam2"), bit 10 the producer/consumer sweep
 * runs its update as trailing workgroups of its own launch (option "tail"; loops without
 * per-sweep events), bit 11 lazy K3: the setup contracted no row, the two-wavelength sweeps
 * contract the rows their records reach first (option "lazy_k3"). */
int frei_ctx_path(frei_ctx* ctx, int* flags);

/* Tuning knobs (also FREI_<NAME> in the environment at context creation): "precontract"
 * (K3 species contraction: 1 on when it applies / 0 off / -1 automatic), "group_q" (lanes per
 * wavelength 1, 2, 4 or 0 = automatic), "shared" (LDS step table 1/0/-1), "prefetch_depth",
 * "shared_max_blocks", "pair_max_blocks", "quad_max_blocks", "depth4_max_blocks",
 * "red_rows", "red_stage" (take effect at the next metadata build), "fused_update" (1: one
 * launch for the partial-sum reduction and the T update when the exchange is local or P2P;
 * 0: two kernels; bitwise identical results; takes effect at the next sweep), "graph" (1:
 * replay T-P iterations from a captured hipGraph; 0, the default: launch kernel by kernel),
 * "tail" (1, the default: the producer/consumer sweep's fused update runs as trailing
 * workgroups of the sweep's launch, layer by layer as the sweep publishes; 0: a launch of its
 * own after the sweep; bitwise identical results), "lazy_k3" (1, the default: with the
 * two-wavelength sweep, K3 contracts no row at setup — each sweep contracts the (pressure row,
 * T node) rows its records reach for the first time, for its own wavelengths, with K3's sum;
 * 0: every row at setup; bitwise identical results). */
int frei_set_option(frei_ctx* ctx, const char* name, int value);
/* With the "graph" option on (default off), T-P iterations (frei_iterate, frei_run) are
 * replayed from a captured hipGraph of a few iterations when one rank runs with timing off:
 * the number of captures and of graph launches so far. */
int frei_graph_info(frei_ctx* ctx, int* captures, int* replays);
/* Chained sweep launches so far (FREI_CHAIN / option "chain": a sweep launch whose leading
 * workgroups run the previous sweep's deferred fused update).  Never while per-sweep HIP events
 * are on (frei_timing) or when P2P ranks share this device. */
int frei_chain_info(frei_ctx* ctx, int64_t* chained);
/* Trailing-update launches so far (FREI_TAIL / option "tail", round 6): producer/consumer sweeps
 * whose launch also ran their own fused update, layer by layer as the sweep published each
 * layer's partial sums (twostream.py:396-407: a layer's dT needs only its own four bolometric
 * sums), instead of a separate update kernel after the sweep.  Never while per-sweep HIP events
 * are on, when chained, or when ranks share this device; bitwise the separate launches. */
int frei_tail_info(frei_ctx* ctx, int64_t* launches);
/* Ranks of this communicator share the context's GPU (shared != 0): no chained launches (a
 * chained launch's sweep blocks spin on update workgroups that wait for every rank's sums, and
 * could hold the CUs another rank's kernels need).  frei_amd sets it when two ranks report the
 * same host and PCI bus id (frei_device_pci_bus_id). */
int frei_comm_shared_device(frei_ctx* ctx, int shared);
/* The PCI bus id string of a device ("0000:05:00.0"), len >= 16. */
int frei_device_pci_bus_id(int device, char* buf, int len);
/* Host wall-clock milliseconds of the last metadata build (the one-time setup before the
 * first sweep after tables/mmr change), by phase: [0] per-(species, layer) brackets on the
 * host, [1] metadata uploads, [2] contracted-table allocation, [3] its zero fill, [4] the K3
 * contraction kernel. */
int frei_setup_timing(frei_ctx* ctx, double* ms5);
/* The last species-contraction launch (K3 for one atmosphere, K7 on fp64 MFMA for a batched
 * context; part of the metadata build): its duration by HIP events on the context stream, ms,
 * and its algorithmic HBM bytes (the S tables' used pressure rows read once, one contracted
 * table per atmosphere written).  0 / 0 before any contraction.  (No reference counterpart:
 * the reference sums species inside every kappa call, opacity.py:250-268.) */
int frei_contract_timing(frei_ctx* ctx, double* ms, double* bytes);

/* Timing of the sweep kernel (HIP events on the context stream around every sweep
 * launch while enabled): total milliseconds and number of timed launches. */
int frei_timing_enable(frei_ctx* ctx, int on);
int frei_timing_read(frei_ctx* ctx, double* total_ms, int* n_launches);
/* While timing is enabled, also HIP events around each sweep's rank exchange (the RCCL
 * all-gather of the bolometric partials, or the host hook): total ms and number of calls.
 * With the P2P exchange: the time the update kernels spent waiting for peers' sums. */
int frei_timing_read_exchange(frei_ctx* ctx, double* total_ms, int* n_calls);

/*
 * Opacity binning (opacity.py:66-170).  A frei_xsec is one species' high-resolution
 * cross-section resident in HBM, in the opacity_dir_to_netcdf layout (opacity.py:395-483):
 * values[n_T][n_p][n_hi] float32 on nodes T_nodes (K) x p_nodes (bar), wavelengths
 * wl_hi[n_hi] (µm, strictly ascending).
 */
typedef struct frei_xsec frei_xsec;
enum { FREI_BIN_GROUPIES = 0, FREI_BIN_EXACT = 1 };

int frei_xsec_create(frei_xsec** out, int device, const float* values, int n_T, int n_p,
                     int64_t n_hi, const double* T_nodes, const double* p_nodes,
                     const double* wl_hi);
/* Synthetic line forest generated on the device (benchmarks; no host copy). */
int frei_xsec_create_synthetic(frei_xsec** out, int device, int n_T, int n_p, int64_t n_hi,
                               const double* T_nodes, const double* p_nodes,
                               const double* wl_hi, uint64_t seed);
int frei_xsec_destroy(frei_xsec* x);
/*
 * binned_opacity for this species onto a grid: bins wl_bins[n_bins+1] (µm, ascending) with
 * centres lam[n_bins] (µm).  Target nodes T_nodes[n_T] (K) x p_nodes[n_p] (bar) each take
 * the nearest source node (xarray interp 'nearest', extrapolating; opacity.py:26-29).
 *   mode FREI_BIN_GROUPIES (binned_opacity default, opacity.py:126-146): per bin the
 *     reference's float32 unit-step trapezoid (interp.py:176-194) x bin width x 1e-3;
 *   mode FREI_BIN_EXACT (Grid.load_opacities default, opacity.py:148-167): per non-empty
 *     bin the trapezoid integral / bin span (NaN for single-point bins) at the bin's mean
 *     wavelength, then linear interpolation/extrapolation onto lam.
 * out[n_p][n_T][n_bins] float64 on the host (NULL: leave the result on the device, for
 * timing).
 */
int frei_xsec_bin(frei_xsec* x, int mode, const double* wl_bins, const double* lam,
                  int64_t n_bins, const double* T_nodes, int n_T, const double* p_nodes,
                  int n_p, double* out);
/* HIP-event timing of the binning kernels: returns the accumulated milliseconds and calls
 * since the last reset; on = 1/0 enables/disables and resets, on = -1 only reads. */
int frei_xsec_timing(frei_xsec* x, int on, double* total_ms, int* n_calls);
/*
 * Same binning, written straight into species s of a context (no host round trip): the
 * context's wavelength slice is [lam_lo, lam_lo + n_lam) of the global grid
 * (wl_bins[n_bins+1], lam[n_bins]); the table gets nodes p_nodes (bar) x T_nodes (K).
 */
int frei_set_table_binned(frei_ctx* ctx, int s, frei_xsec* x, int mode, const double* wl_bins,
                          const double* lam, int64_t n_bins, int64_t lam_lo,
                          const double* T_nodes, int n_T, const double* p_nodes, int n_p);

#ifdef __cplusplus
}
#endif

#endif /* FREI_HIP_H */
