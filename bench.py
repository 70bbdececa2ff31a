#!/usr/bin/env python3
"""Benchmark: λ-bin·layer flux updates/s at 60 layers × 500k λ (BASELINE.json metric).

Workload: hot Jupiter, 60 layers × 500,000 wavelengths, 8 opacity
species (H2O, CO, CO2, CH4, Na, K + H2-H2/H2-He CIA), 16 T-nodes, synthetic separable
tables generated on the device.  One step = one radiative-equilibrium T–P iteration
(emit sweep + absorb sweep, each with its bolometric reduction, dT update and the
convergence test) = 2 × 59 × 500k flux updates, always fully computed (convergence is
tracked but does not stop the timed work).  With --gpus N the 500k wavelengths are
sharded over N ranks (strong scaling) with one exchange of the per-sweep partial sums (the
engine's P2P mailboxes over xGMI by default).

Run:  python bench.py [--gpus N --steps K --warmup W]
      (N > 1 either under a launcher — python -m torch.distributed.run --nproc-per-node N
      bench.py --gpus N ... — or on its own: without WORLD_SIZE in the environment the process
      starts N rank processes of itself (launch_ranks) before anything touches the GPU and prints
      rank 0's line.  Rendezvous, barriers and timing reductions go over plain sockets, the
      per-sweep exchange is the engine's own)
Prints ONE JSON line on rank 0.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_HBM = 8.0e12  # B/s, MI355X HBM3E (MI355X_MICROARCH.md)



def sweep_kernel_name(path):
    """The sweep kernel the tables' path selects (frei_ctx_path bits, engine.path())."""
    if path.get("pipe"):
        return "sweep_pipe_kernel"
    if path.get("paired") or path.get("quad"):
        return "sweep_group_kernel"
    if path.get("lam2"):
        return "sweep_pair_kernel"
    return "sweep_fast_kernel"

def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--n-lam", type=int, default=500_000)
    ap.add_argument("--n-layers", type=int, default=60)
    ap.add_argument("--n-T", type=int, default=16)
    ap.add_argument("--rad-eq-max", type=int, default=200,
                    help="max T-P iterations for the iterations-to-radiative-equilibrium run")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-lam", type=int, default=500_000)
    ap.add_argument("--cpu-workers", type=int, default=min(16, os.cpu_count() or 1),
                    help="worker processes of the all-cores CPU leg (1 = skip it; the GPU box "
                         "grants a 16-CPU share)")
    ap.add_argument("--cpu-sharded-lam", type=int, default=500_000,
                    help="wavelengths of the all-cores CPU leg's sample")
    ap.add_argument("--no-provider", action="store_true",
                    help="skip the chemistry-provider (chemistry=) measurement")
    ap.add_argument("--no-binning", action="store_true",
                    help="skip the K6 opacity-binning measurement (rank 0)")
    ap.add_argument("--binning-reps", type=int, default=5)
    ap.add_argument("--comm", choices=("p2p", "rccl", "host"), default="p2p",
                    help="N > 1 exchange: the engine's P2P mailboxes over xGMI (default; falls "
                         "back to RCCL if they cannot be set up), RCCL all-gather, or the host "
                         "hook (lets several ranks share one GPU to rehearse the multi-rank flow)")
    ap.add_argument("--lam-slice", default=None,
                    help="LO:HI — one GPU runs only this slice of the --n-lam grid (global "
                         "trapezoid weights), as one rank of a multi-GPU run would: projection")
    ap.add_argument("--balance", action="store_true",
                    help="re-split the wavelength grid across GPUs to equal measured per-rank sweep "
                         "time before timing (default: the even split)")
    ap.add_argument("--force-comm", action="store_true",
                    help="with --gpus 1: still join the exchange (a one-rank P2P mailbox or "
                         "RCCL communicator), to time its per-sweep cost on one GPU")
    ap.add_argument("--no-per-species", action="store_true",
                    help="skip the per-species (no K3 contraction) measurement")
    ap.add_argument("--per-species-steps", type=int, default=6)
    ap.add_argument("--no-chemistry", action="store_true",
                    help="skip the T-dependent chemistry measurement (one GPU only)")
    ap.add_argument("--no-c5", action="store_true",
                    help="skip the batched-atmosphere (C5) measurement")
    ap.add_argument("--c5-lam", type=int, default=100_000)
    ap.add_argument("--c5-steps", type=int, default=5)
    ap.add_argument("--launch-selftest", action="store_true",
                    help=argparse.SUPPRESS)   # ranks rendezvous and report, no GPU (CPU test)
    return ap.parse_args()


def launch_ranks(a):
    """`--gpus N` without a launcher: start N rank processes of this script (RANK, LOCAL_RANK,
    WORLD_SIZE, MASTER_ADDR / MASTER_PORT set for each; the rendezvous is frei_amd.rendezvous
    over 127.0.0.1), forward their stderr, and return rank 0's JSON line.  Runs before anything
    in this process touches the GPU (nothing is imported from frei_amd here), and the ranks are
    child processes, never an exec of this one.  Any rank failing fails the launch: the others
    are terminated and the first non-zero exit status is returned."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(a.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(a.gpus),
                   LOCAL_WORLD_SIZE=str(a.gpus), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:],
                                      env=env, stdout=subprocess.PIPE if r == 0 else
                                      subprocess.DEVNULL))
    import threading
    out = []
    reader = threading.Thread(target=lambda: out.append(procs[0].stdout.read()), daemon=True)
    reader.start()
    rc = 0
    while True:
        bad = [p.returncode for p in procs if p.poll() is not None and p.returncode != 0]
        if bad:   # one rank failed: the others would only wait for it at the next barrier
            rc = bad[0]
            for p in procs:
                if p.poll() is None:
                    p.terminate()
            break
        if all(p.poll() is not None for p in procs):
            break
        time.sleep(0.2)
    for p in procs:
        p.wait()
    reader.join(timeout=10)
    text = out[0].decode() if out else ""
    lines = [x for x in text.splitlines() if x.strip()]
    return rc, (lines[-1] if lines else None)


class Dist:
    """Rendezvous, barriers and max-over-ranks timing for one process per GPU, over plain
    sockets (frei_amd.rendezvous; no PyTorch).  The data-path exchange is the engine's own
    (P2P mailboxes over xGMI, RCCL or the host hook)."""

    def __init__(self, n):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        if self.world != n:
            raise SystemExit(f"--gpus {n} but WORLD_SIZE={self.world}")
        self.rdzv = None
        if self.world > 1:
            from frei_amd.rendezvous import from_env
            self.rdzv = from_env()

    def barrier(self):
        if self.rdzv:
            self.rdzv.barrier()

    def max(self, x):
        return self.rdzv.max(x) if self.rdzv else x

    def all_ok(self, ok):
        """True when every rank reports ok."""
        if not self.rdzv:
            return bool(ok)
        return all(v == b"1" for v in self.rdzv.all_gather(b"1" if ok else b"0"))

    def gather(self, x):
        """Every rank's float x, in rank order."""
        if not self.rdzv:
            return [float(x)]
        return [float(v) for v in self.rdzv.all_gather(repr(float(x)).encode())]


def cpu_baseline(w, n_sample, steps=1):
    """Oracle (NumPy restatement of the reference path, 1 core) on a wavelength sample of the
    same workload: `steps` T-P iterations, timed with perf_counter."""
    from oracle import frei_oracle as O
    lam = w["lam"]
    idx = np.linspace(0, lam.size - 1, n_sample).round().astype(int)
    tabs = {n: O.Table(O.SeparableValues(w["base"][s][idx], w["fp"][s], w["fT"][s]), w["p"],
                       w["T_nodes"]) for s, n in enumerate(w["names"])}
    lam_s = lam[idx]
    Ft = O.F_TOA(lam_s)
    t0 = time.perf_counter()
    O.emission_spectrum(tabs, w["T0"], w["p"], lam_s, Ft, 2478.6519476149147,
                        4.0142926168559996e-24, 1, n_timesteps=steps,
                        n_zero_crossings=10 ** 9, convergence_dT=-1.0, mmr=w["mmr"])
    dt = time.perf_counter() - t0
    updates = (2 * steps + 1) * (w["p"].size - 1) * n_sample   # incl. the final emit
    return updates / dt, dt


def cpu_baseline_sharded(w, n_lam, workers, steps=1):
    """The oracle λ-sharded over `workers` processes (SURVEY.md §8(d)'s all-cores variant):
    oracle/sharded.py runs the unchanged oracle on contiguous slices of an evenly strided
    `n_lam`-wavelength sample and exchanges the four bolometric partial sums per layer through the
    coordinator, so every slice steps the same temperatures as the one-process run.  The worker
    processes are spawned (they never touch the GPU) before the clock starts; the timed region is
    the run itself, exchanges included."""
    from oracle.sharded import ShardedOracle
    lam = w["lam"]
    idx = np.linspace(0, lam.size - 1, n_lam).round().astype(int)
    tables = {n: (w["base"][s][idx], w["fp"][s], w["fT"][s], w["T_nodes"])
              for s, n in enumerate(w["names"])}
    from oracle import frei_oracle as O
    with ShardedOracle(tables, lam[idx], w["p"], w["T0"], O.F_TOA(lam[idx]), 2478.6519476149147,
                       4.0142926168559996e-24, mmr=w["mmr"], n_workers=workers) as so:
        so.emission_spectrum(n_timesteps=1, n_zero_crossings=10 ** 9,
                             convergence_dT=-1.0)          # untimed: workers import, warm up
        t0 = time.perf_counter()
        so.emission_spectrum(n_timesteps=steps, n_zero_crossings=10 ** 9, convergence_dT=-1.0)
        dt = time.perf_counter() - t0
    updates = (2 * steps + 1) * (w["p"].size - 1) * n_lam
    return updates / dt, dt


# the reference itself (imported in the build container, 1 core), whole
# emission_spectrum path, 60 layers x 500k lambda, one species: 62.3 s for 3 sweeps
REFERENCE_MEASURED = {"value": 1.42e6, "unit": "updates/s", "cores": 1, "species": 1,
                      "source": "SURVEY.md §6 (frei's own Grid.emission_spectrum in the build "
                                "container, 60 x 500k lambda, 1 species, 1 core of a Xeon)"}


def provider_leg(a, d, w, tabs):
    """The drop-in's chemistry path (frei's chemistry passed as chemistry=): a
    T-dependent provider on the reference's signature (frei_amd.workloads.c3_provider, the
    FastChem stand-in) drives the C3 run to radiative equilibrium.  Every sweep: the layers' T
    read back (8 B per layer), the provider called on them as kappa calls it
    (opacity.py:246-248), the mixing ratios uploaded, the per-species sweep and its update.
    Reports iterations/s and where a sweep's wall time goes (sweep kernel vs the rest: update
    kernel, T readback, provider call, mixing-ratio upload, launch and synchronisation)."""
    from frei_amd.engine import Engine
    from frei_amd.workloads import c3_provider
    prov = c3_provider(w)
    n_calls = [0]

    def counted(*args, **kw):
        n_calls[0] += 1
        return prov(*args, **kw)
    pe = Engine(w["lam"], w["p"], tabs, chemistry=counted, device=d.local)
    try:
        path = pe.path()
        pe.run(w["T0"], n_timesteps=2, n_zero_crossings=2, convergence_dT=3.0, alpha=1.0,
               want_dtaus=False)                                      # warm-up
        n0 = n_calls[0]
        t0 = time.perf_counter()
        out = pe.run(w["T0"], n_timesteps=a.rad_eq_max, n_zero_crossings=2, convergence_dT=3.0,
                     alpha=1.0, want_dtaus=False)
        wall = time.perf_counter() - t0
        calls = n_calls[0] - n0
        pe.timing(True)                                               # the same run, timed
        t2 = time.perf_counter()
        pe.run(w["T0"], n_timesteps=a.rad_eq_max, n_zero_crossings=2, convergence_dT=3.0,
               alpha=1.0, want_dtaus=False)
        wall_t = time.perf_counter() - t2
        ms, n_sw = pe.timing_read()
        pe.timing(False)
        # the provider alone, on one sweep's layer temperatures (host side)
        T = out["final_T"]
        t4 = time.perf_counter()
        for _ in range(20):
            prov(T, w["p"], w["names"], m_bar=4.0142926168559996e-24)
        prov_ms = (time.perf_counter() - t4) / 20 * 1e3
    finally:
        pe.close()
    it = out["n_iter"]
    n_sweeps = 2 * it + 1
    return {"workload": f"C3 60 x {a.n_lam} lambda x {len(w['names'])} species to radiative "
                        "equilibrium, mixing ratios from a T-dependent provider (chemistry=)",
            "path": path, "iterations": it, "wall_s": wall, "iters_per_s": it / wall,
            "sweeps": n_sweeps, "provider_calls": calls,
            "ms_per_sweep": wall / n_sweeps * 1e3,
            "sweep_kernel_ms": ms / max(n_sw, 1),
            "rest_ms_per_sweep": (wall_t * 1e3 - ms) / max(n_sw, 1),
            "provider_call_ms": prov_ms,
            "note": "rest_ms_per_sweep: the timed run's wall time per sweep outside the sweep "
                    "kernel (HIP events): update kernel, T readback, the provider call, the "
                    "mixing-ratio upload, launches and stream synchronisation"}


def binning_leg(a, device, cpu=True):
    """K6 (opacity binning) on the C3 grid: one species' synthetic
    DACE-like cross-section resident in HBM, binned into the reference's output shape
    (60 x 60 (T, p) rows of 500k bins) in both modes; HIP-event kernel time, algorithmic
    bytes per launch, CPU oracle on a bounded row sample."""
    from frei_amd.binning import CrossSection
    from frei_amd.workloads import binning_bytes, binning_workload
    w = binning_workload(n_layers=a.n_layers, n_lam=a.n_lam)
    x = CrossSection.synthetic(w["T_src"], w["p_src"], w["wl_hi"], seed=3)
    out = {"workload": f"1 species, {w['T_src'].size} T x {w['p_src'].size} p source nodes x "
                       f"{w['wl_hi'].size} points (0.01 cm^-1, float32) -> "
                       f"{a.n_layers} x {a.n_layers} (T, p) rows x {a.n_lam} bins (float64)"}
    try:
        for mode, groupies in (("groupies", True), ("exact", False)):
            x.bin(w["wl_bins"], w["lam"], w["T0"], w["p"], groupies=groupies, device=device,
                  out=False)                                   # warm-up (plan + scratch)
            per = []
            for _ in range(a.binning_reps):
                x.timing(1, device)
                x.bin(w["wl_bins"], w["lam"], w["T0"], w["p"], groupies=groupies,
                      device=device, out=False)
                per.append(x.timing(0, device)[0])
            ms, n = sum(per), len(per)
            acc = binning_bytes(w, groupies)
            t = ms / n * 1e-3
            out[mode] = {"avg_launch_ms": ms / n, "launches": n,
                         "launch_ms": [round(v, 4) for v in per],
                         "table_values_per_s": acc["dest_rows"] * acc["n_bins"] / t,
                         "source_points_per_s": acc["source_rows"] * acc["points"] / t,
                         "roofline": {"bound": "hbm", "achieved": acc["bytes"] / t / 1e9,
                                      "peak": PEAK_HBM / 1e9, "unit": "GB/s",
                                      "frac": acc["bytes"] / t / PEAK_HBM,
                                      "bytes_per_launch": acc["bytes"]},
                         "source_rows": acc["source_rows"], "dest_rows": acc["dest_rows"]}
    finally:
        x.release()
    # The per-process placement mode (profiles/r05/binning/README.md): the same
    # code runs "fast" (0.69-0.73 of peak) or "slow" (0.60-0.66) in a given process, both modes
    # together, by where the buffers land in HBM.  Classified from this process's two modes' mean
    # fraction, so a driver figure says which mode it measured.
    if "groupies" in out and "exact" in out:
        m = 0.5 * (out["groupies"]["roofline"]["frac"] + out["exact"]["roofline"]["frac"])
        out["placement_mode"] = {
            "mode": "fast" if m >= 0.675 else "slow", "mean_frac": m,
            "rule": "mean of the groupies and exact fractions of HBM peak >= 0.675: fast "
                    "(measured 0.69-0.73 per mode), else slow (0.60-0.66); one process, both "
                    "modes move together (buffer placement in HBM, profiles/r05/binning/)"}
    if cpu:
        # oracle (groupies branch) on 24 random source rows of the same high-res axis and
        # bins: binned points per second, 1 core
        from oracle import frei_oracle as O
        rng = np.random.default_rng(3)
        n_rows = 24
        rows = (10 ** rng.uniform(-3, 2, (n_rows, w["wl_hi"].size))).astype(np.float32)
        start, end = O.bin_ranges(w["wl_hi"], w["wl_bins"])
        t0 = time.perf_counter()
        O.bin_groupies_rows(rows, start, end, w["wl_bins"])
        dt = time.perf_counter() - t0
        pts = n_rows * int(end[-1] - start[0])
        out["cpu_baseline"] = {"value": pts / dt, "unit": "source points binned/s (groupies)",
                               "cores": 1, "kind": "port",
                               "sample": f"oracle bin_groupies_rows, {n_rows} source rows x "
                                         f"{pts // n_rows} points -> {a.n_lam} bins, "
                                         f"{dt:.2f} s"}
        out["groupies"]["vs_cpu"] = out["groupies"]["source_points_per_s"] / (pts / dt)
    return out


def c5_leg(a, d):
    """Config C5 on this rank: 32 atmospheres (T_ref 1000..2400 K step 200 x log g 2.5..4,
    [M/H] of this rank's slot of 8) x 60 layers x 100k lambda x 8 species, as one batched
    context (256 atmospheres over 8 GPUs = 32 per GPU, weak scaling, no
    exchange).  Fixed-work T-P iterations (updates/s) and the run of every atmosphere to its
    own radiative equilibrium."""
    from frei_amd.batch import BatchEngine
    from frei_amd.opacity import SeparableTable
    from frei_amd.tp import temperature_grid
    from frei_amd.workloads import c3
    w = c3(n_layers=a.n_layers, n_lam=a.c5_lam, n_T=16)
    T_refs = np.arange(1000.0, 2401.0, 200.0)
    loggs = np.array([2.5, 3.0, 3.5, 4.0])
    mh = np.linspace(-1.0, 1.0, 8)[d.rank % 8]
    T0 = np.array([temperature_grid(w["p"], t, 0.1, 0.1) for t in T_refs for _ in loggs])
    g = np.array([10.0 ** lg for _ in T_refs for lg in loggs])
    T_nodes = np.linspace(0.8 * T0.min(), 1.2 * T0.max(), 16)
    fT = (T_nodes / 1000.0) ** 0.5
    tabs = {n: SeparableTable(w["base"][s], w["fp"][s], fT, w["p"], T_nodes)
            for s, n in enumerate(w["names"])}
    mmr = np.broadcast_to(w["mmr"] * 10.0 ** mh, (len(g),) + w["mmr"].shape)
    A = len(g)
    t_s = time.perf_counter()
    eng = BatchEngine(w["lam"], w["p"], tabs, g=g, mmr=mmr, device=d.local)
    try:
        eng.state_init(T0)       # metadata + K7 contraction (fp64 MFMA), once
        eng.synchronize()
        setup_s = time.perf_counter() - t_s
        k7 = eng.contract_timing()
        phases = eng.setup_timing()
        eng.iterate(1)
        eng.synchronize()
        d.barrier()
        t0 = time.perf_counter()
        eng.iterate(a.c5_steps)
        eng.synchronize()
        t1 = time.perf_counter()
        d.barrier()
        el = d.max(t1 - t0)
        upd = 2 * (a.n_layers - 1) * a.c5_lam * A * a.c5_steps * d.world
        eng.run(T0, n_timesteps=a.rad_eq_max, n_zero_crossings=2, convergence_dT=3.0)
        d.barrier()
        t2 = time.perf_counter()
        out = eng.run(T0, n_timesteps=a.rad_eq_max, n_zero_crossings=2, convergence_dT=3.0)
        t3 = time.perf_counter()
        d.barrier()
        rad = d.max(t3 - t2)
    finally:
        eng.close()
    return {"workload": f"C5: {A} atmospheres per GPU (T_ref 1000..2400 K x log g 2.5..4, "
                        f"[M/H] {mh:+.2f} on rank 0) x {a.n_layers} layers x {a.c5_lam} "
                        f"lambda x {len(w['names'])} species, batched, {d.world} GPU(s)",
            "updates_per_s": upd / el, "ms_per_step": el / a.c5_steps * 1e3,
            "atmospheres": A * d.world,
            "rad_eq": {"wall_s": rad, "atmospheres_per_s": A * d.world / rad,
                       "iterations_min": int(out["n_iter"].min()),
                       "iterations_max": int(out["n_iter"].max()),
                       "max_iterations": a.rad_eq_max,
                       "converged_rank0": int((out["n_iter"] < a.rad_eq_max).sum()),
                       "note": "iterations per atmosphere under the reference's convergence "
                               "test; an atmosphere at max_iterations did not meet it"},
            "setup_s": setup_s,
            "setup_phases_ms": phases,
            "k7_roofline": {"bound": "hbm", "kernel": "contract_batch_kernel",
                            "avg_launch_ms": k7["ms"], "bytes_per_launch": k7["bytes"],
                            "achieved": k7["bytes"] / (k7["ms"] * 1e-3) / 1e9,
                            "peak": PEAK_HBM / 1e9, "unit": "GB/s",
                            "frac": k7["bytes"] / (k7["ms"] * 1e-3) / PEAK_HBM,
                            "byte_model": "the S tables' used pressure rows read once + one "
                                          "contracted table per atmosphere written (n_T x "
                                          "pitch columns per used row), one launch per "
                                          "tables/mmr; HIP events on the engine stream"},
            "note": "setup_s: table generation + metadata + K7 MFMA contraction, once"}


# stdout carries exactly one line: the JSON result of rank 0.  Everything else any library
# writes to fd 1 (gloo's connection notices, RCCL, the HIP runtime) goes to stderr.
_RESULT_FD = None


def _reserve_stdout():
    global _RESULT_FD
    sys.stdout.flush()
    _RESULT_FD = os.dup(1)
    os.dup2(2, 1)


def _emit_result(line):
    os.write(_RESULT_FD, (json.dumps(line) + "\n").encode())


def build_engine(w, tabs, lo, hi, d, kind, force=False):
    """Engine for this rank's slice, joined to the other ranks over ``kind`` (p2p, rccl, host);
    ``force`` joins a one-rank exchange on a single GPU (cost measurement)."""
    from frei_amd.distributed import host_comm, p2p_comm, rccl_comm
    from frei_amd.engine import Engine
    from frei_amd.rendezvous import Rendezvous
    comm = None
    if d.world > 1 or force:
        rdzv = d.rdzv if d.rdzv is not None else Rendezvous(1, 0)
        comm = {"p2p": p2p_comm, "rccl": rccl_comm, "host": host_comm}[kind](rdzv)
    # a forced one-rank RCCL communicator is requested through FREI_FORCE_RCCL for this
    # engine's construction only (later engines of the run do not inherit it)
    forced = force and kind == "rccl"
    prev = os.environ.get("FREI_FORCE_RCCL")
    if forced:
        os.environ["FREI_FORCE_RCCL"] = "1"
    try:
        return Engine(w["lam"], w["p"], tabs, mmr=w["mmr"], device=d.local, lam_slice=(lo, hi),
                      comm=comm)
    finally:
        if forced:
            if prev is None:
                os.environ.pop("FREI_FORCE_RCCL", None)
            else:
                os.environ["FREI_FORCE_RCCL"] = prev


def build_engine_fallback(w, tabs, lo, hi, d, force, note):
    """After a failed P2P setup: RCCL on every rank, or — when RCCL cannot be set up on some
    rank either — the host all-gather over the socket rendezvous (slow, always available), so
    the run still reports a line.  Returns (engine, kind, note)."""
    eng, err = None, None
    try:
        eng = build_engine(w, tabs, lo, hi, d, "rccl", force)
    except RuntimeError as e:
        err = str(e)
    if d.all_ok(eng is not None):
        return eng, "rccl", note + "; fell back to RCCL"
    if eng is not None:
        eng.close()
    return (build_engine(w, tabs, lo, hi, d, "host", force), "host",
            note + f"; RCCL setup failed too ({err or 'on a peer rank'}): host all-gather")


def timed_iterations(eng, d, warmup, steps):
    """Fixed-work T-P iterations: warm-up, then exactly ``steps`` bracketed by a barrier and a
    stream synchronize on both sides; the max over ranks."""
    eng.iterate(warmup)
    eng.synchronize()
    d.barrier()
    t0 = time.perf_counter()
    eng.iterate(steps)
    eng.synchronize()
    t1 = time.perf_counter()
    d.barrier()
    return d.max(t1 - t0)


def sweep_kernel_time(eng, n_iter):
    """HIP events on the engine's stream around every sweep launch: (avg ms, launches,
    exchange avg ms, exchange calls)."""
    eng.timing(True)
    eng.iterate(n_iter)
    eng.synchronize()
    ms, n = eng.timing_read()
    xms, nx = eng.timing_read_exchange()
    eng.timing(False)
    return ms / max(n, 1), n, xms / max(nx, 1), nx


def main():
    _reserve_stdout()
    a = parse()
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:   # no launcher: start the ranks here
        rc, line = launch_ranks(a)
        if line is not None and rc == 0:
            os.write(_RESULT_FD, (line + "\n").encode())
        if rc == 0 and line is None:
            rc = 1
        sys.exit(rc)
    # a peer that never publishes its sums fails the run after this long instead of 30 s
    os.environ.setdefault("FREI_P2P_TIMEOUT_S", "10")
    d = Dist(a.gpus)
    if a.launch_selftest:   # the launch path alone (CPU test): rendezvous, barrier, max, line
        if os.environ.get("FREI_LAUNCH_SELFTEST_FAIL") == str(d.rank):
            sys.exit(3)
        d.barrier()
        t = d.max(float(d.rank))
        if d.rank == 0:
            _emit_result({"metric": "launch selftest", "n_gpus": d.world, "value": t,
                          "pids": [int(x) for x in d.gather(os.getpid())]})
        else:
            d.gather(os.getpid())
        return
    from frei_amd import _native as N
    from frei_amd.engine import partition
    from frei_amd.opacity import SeparableTable
    from frei_amd.workloads import bytes_per_update, c3

    n_dev = max(1, N.device_count())
    if d.world > n_dev:   # rehearsal on fewer GPUs than ranks: ranks share the GPUs there are
        d.local = d.local % n_dev
        # the producer/consumer sweep takes a whole CU per block (VGPRs and LDS); next to other
        # ranks' update kernels spinning on the same GPU for their peers' sums its blocks can
        # starve (a P2P timeout): ranks that share a GPU use the grouped-lane form instead
        os.environ.setdefault("FREI_PIPE", "0")
        # likewise a chained launch's sweep blocks wait (spinning) for its update workgroups,
        # which wait for every rank's sums: beside other ranks' kernels on the same GPU they could
        # hold the CUs those ranks need, so ranks sharing a GPU launch update and sweep separately
        os.environ.setdefault("FREI_CHAIN", "0")
    w = c3(n_layers=a.n_layers, n_lam=a.n_lam, n_T=a.n_T)
    nL, n_lam, S = a.n_layers, a.n_lam, len(w["names"])
    lo, hi = partition(n_lam, d.world, d.rank)
    if a.lam_slice:
        if d.world != 1:
            raise SystemExit("--lam-slice is a one-GPU projection option")
        lo, hi = (int(x) for x in a.lam_slice.split(":"))
    tabs = {n: SeparableTable(w["base"][s], w["fp"][s], w["fT"][s], w["p"], w["T_nodes"])
            for s, n in enumerate(w["names"])}

    def make_engine(lo, hi, kind):
        """This rank's engine for [lo, hi) over `kind`, with the fallback chain P2P -> RCCL ->
        host; then its one-time setup (metadata + K3) and, over P2P, one untimed iteration
        through the mailboxes.  Returns (engine, kind, note, tables_s, path, setup_ms, phases)."""
        comm_note = None
        t_e = time.perf_counter()
        eng, err = None, None
        try:
            eng = build_engine(w, tabs, lo, hi, d, kind, a.force_comm)
        except RuntimeError as e:   # e.g. no IPC / peer mapping: fall back to RCCL everywhere
            err = str(e)
        if not d.all_ok(eng is not None):
            if kind != "p2p":
                raise SystemExit(f"rank {d.rank}: engine setup failed: {err}")
            if eng is not None:
                eng.close()
            eng, kind, comm_note = build_engine_fallback(
                w, tabs, lo, hi, d, a.force_comm, f"p2p setup failed ({err or 'on a peer rank'})")
        tables_s = time.perf_counter() - t_e
        # one-time setup: metadata build + species contraction (K3), outside the timed steps.
        # The headline measures steady-state sweeps over the whole contracted table, as in
        # rounds 1-5 (lazy K3, the library default, moves first-touch row contractions into the
        # first sweeps that reach them: measured in the rad_eq leg, incl_setup)
        eng.set_option("lazy_k3", 0)
        t_s = time.perf_counter()
        path = eng.path()
        setup_ms = (time.perf_counter() - t_s) * 1e3
        setup_phases = eng.setup_timing()
        if kind == "p2p" and d.world > 1:
            # one untimed T-P iteration through the mailboxes: a peer whose sums never arrive
            # fails every rank within FREI_P2P_TIMEOUT_S, and the run goes on over RCCL instead
            err = None
            try:
                eng.state_init(w["T0"])
                eng.iterate(1)
                eng.synchronize()
            except RuntimeError as e:
                err = str(e)
            if not d.all_ok(err is None):
                eng.close()
                eng, kind, comm_note = build_engine_fallback(
                    w, tabs, lo, hi, d, a.force_comm,
                    f"p2p exchange failed at run time ({err or 'on a peer rank'})")
        return eng, kind, comm_note, tables_s, path, setup_ms, setup_phases

    eng, kind, comm_note, tables_s, path, setup_ms, setup_phases = make_engine(lo, hi, a.comm)
    # ---- cost-balanced slices (--balance): every rank times its sweeps on the even split and the
    # grid is re-split to equal measured cost (frei_amd.balanced_edges) before anything is
    # timed.  Off by default: at the 8-GPU slice the producer/consumer sweep's time is one
    # block's loop (one 256-wavelength block per CU), which a smaller slice does not shorten, and
    # at the 4-GPU slice a larger slice can cross a sweep-form threshold (profiles/r03/projection/
    # balanced.txt: 165 -> 191 us); the slower long-wavelength ranks stay.
    slicing = {"kind": "even", "edges": [partition(n_lam, d.world, r)[0]
                                         for r in range(d.world)] + [n_lam]}
    if d.world > 1 and a.balance:
        from frei_amd.engine import balanced_edges
        eng.state_init(w["T0"])
        eng.iterate(2)
        eng.synchronize()
        ms_even = d.gather(sweep_kernel_time(eng, 4)[0])
        edges = balanced_edges(slicing["edges"], ms_even)
        moved = edges != slicing["edges"]   # the same decision on every rank
        slicing = {"kind": "cost-balanced (per-rank sweep time on the even split)",
                   "edges": edges, "even_sweep_ms": ms_even}
        if moved:
            lo, hi = edges[d.rank], edges[d.rank + 1]
            eng.close()
            eng, kind, comm_note, tables_s, path, setup_ms, setup_phases = make_engine(
                lo, hi, kind)

    # ---- headline: timed fixed-work T-P iterations (no per-kernel events inside)
    eng.state_init(w["T0"])
    elapsed = timed_iterations(eng, d, a.warmup, a.steps)
    # ---- sweep-kernel duration: HIP events on the engine's stream around every sweep launch
    avg_sweep_ms, n_sweeps, xch_ms, n_xch = sweep_kernel_time(eng, max(2, a.steps // 2))
    exchange = None
    if d.world > 1 or a.force_comm:   # per-sweep rank exchange, max over ranks
        what = {"p2p": "P2P mailbox push over xGMI (update-kernel wait)",
                "rccl": "RCCL all-gather", "host": "host all-gather"}[kind]
        exchange = {"kind": f"{what} of {4 * (nL - 1) * 8} B per rank",
                    "avg_ms": d.max(xch_ms), "calls": n_xch,
                    "note": comm_note or ("P2P: time the update kernel waits for every rank's "
                                          "sums (includes the slowest rank's lag)"
                                          if kind == "p2p" else
                                          "stream time of the all-gather, per sweep "
                                          "(includes waiting for the slowest rank)")}
    updates_per_step = 2 * (nL - 1) * (hi - lo if a.lam_slice else n_lam)
    value = updates_per_step * a.steps / elapsed
    ms_per_step = elapsed / a.steps * 1e3

    # ---- roofline of the dominant kernel (sweep), per launch, this rank's slice
    S_run = 1 if path["contracted"] else S    # K3 sweeps read one contracted table
    bpu = bytes_per_update(S_run, live_only=True)
    bytes_launch = bpu * (nL - 1) * (hi - lo)
    achieved = bytes_launch / (avg_sweep_ms * 1e-3)
    achieved = d.max(achieved) if d.world > 1 else achieved

    # ---- iterations to radiative equilibrium (reference convergence test); the first run
    # allocates the one-time buffers (T history, the final emit's dtaus)
    t_c = time.perf_counter()
    eng.run(w["T0"], n_timesteps=a.rad_eq_max, n_zero_crossings=2, convergence_dT=3.0,
            alpha=1.0, want_dtaus=False)
    cold_s = time.perf_counter() - t_c
    d.barrier()
    t2 = time.perf_counter()
    out = eng.run(w["T0"], n_timesteps=a.rad_eq_max, n_zero_crossings=2, convergence_dT=3.0,
                  alpha=1.0, want_dtaus=False)
    t3 = time.perf_counter()
    rad_eq_wall = d.max(t3 - t2)
    n_iter = out["n_iter"]
    # one-time setup + the run, both K3 modes on this engine (buffers already allocated): the
    # metadata build and contraction (lazy: none up front, then the rows the run reaches) timed
    # with the run to radiative equilibrium from T0
    incl = {}
    for mode, lazy in (("lazy_k3", 1), ("full_k3", 0)):
        eng.set_option("lazy_k3", lazy)
        d.barrier()
        t4 = time.perf_counter()
        p_m = eng.path()
        o_m = eng.run(w["T0"], n_timesteps=a.rad_eq_max, n_zero_crossings=2, convergence_dT=3.0,
                      alpha=1.0, want_dtaus=False)
        t5 = time.perf_counter()
        wall_m = d.max(t5 - t4)
        incl[mode] = {"iterations": o_m["n_iter"], "wall_s": wall_m,
                      "iters_per_s": o_m["n_iter"] / wall_m, "lazy_active": p_m.get("lazy_k3"),
                      "setup_phases_ms": eng.setup_timing()}
    eng.set_option("lazy_k3", 0)
    eng.path()

    # ---- per-species path (no K3): the sweep sums all S species' table rows per step, the
    # form any T-dependent chemistry needs; same workload, fixed work
    per_species = None
    if not a.no_per_species:
        eng.set_option("precontract", 0)
        p2 = eng.path()
        eng.state_init(w["T0"])
        el_ps = timed_iterations(eng, d, 2, a.per_species_steps)
        ps_ms, ps_n, _, _ = sweep_kernel_time(eng, a.per_species_steps)
        bpu_ps = bytes_per_update(S, live_only=True)
        ach_ps = d.max(bpu_ps * (nL - 1) * (hi - lo) / (ps_ms * 1e-3))
        per_species = {
            "value": updates_per_step * a.per_species_steps / el_ps, "unit": "updates/s",
            "ms_per_step": el_ps / a.per_species_steps * 1e3, "steps": a.per_species_steps,
            "path": p2,
            "roofline": {"bound": "hbm", "achieved": ach_ps / 1e9, "peak": PEAK_HBM / 1e9,
                         "unit": "GB/s", "frac": ach_ps / PEAK_HBM, "kernel": sweep_kernel_name(p2),
                         "bytes_per_update": bpu_ps, "avg_launch_ms": ps_ms, "launches": ps_n},
            "byte_model": f"8 stale opposite-stream read + 8 live flux write + 16*S = {bpu_ps} B "
                          f"(SURVEY 8(d)'s 24 + 16*S = {24 + 16 * S} B less the dead store the "
                          "T-P loop skips)"}
        tp = os.path.join(ROOT, "profiles", "traffic_sweep_per_species.json")
        vp = os.path.join(ROOT, "profiles", "valu_sweep_per_species.json")
        if os.path.exists(tp):
            t = json.load(open(tp))
            if t["workload"] == {"n_lam": n_lam // d.world, "n_layers": nL, "species": S,
                                 "contracted": False}:
                per_species["roofline"].update(
                    traffic=t["hbm_B_per_launch"],
                    traffic_over_algorithmic=t["traffic_over_algorithmic"],
                    traffic_source="profiles/traffic_sweep_per_species.json")
                if os.path.exists(vp):
                    v = json.load(open(vp))
                    per_species["roofline"].update(
                        valu_busy=v["valu_busy"], valu_insts_per_64_updates=v["valu_insts_per_update"],
                        valu_source="profiles/valu_sweep_per_species.json")
        eng.set_option("precontract", -1)
        eng.path()
    cpu = None
    if d.rank == 0 and d.world == 1 and not a.no_cpu_baseline:
        rate, dt = cpu_baseline(w, min(a.cpu_lam, n_lam))
        cpu = {"value": rate, "unit": "updates/s", "cores": 1, "host_cpus": os.cpu_count(),
               "kind": "port",
               "sample": f"oracle (NumPy restatement of frei's path, single-threaded: 1 of "
                         f"{os.cpu_count()} host CPUs), {nL} layers x {min(a.cpu_lam, n_lam)} "
                         f"lambda ({'the whole grid' if a.cpu_lam >= n_lam else 'evenly strided sample of the same grid'}), "
                         f"{S} species, 1 T-P iteration + final emit, {dt:.1f} s"}
        cpu["reference_measured"] = dict(REFERENCE_MEASURED,
                                         port_over_reference=rate / REFERENCE_MEASURED["value"],
                                         note="the port's figure is 8 species (K3 not used: "
                                              "the oracle sums every species per update)")
        if a.cpu_workers > 1:
            n_s = min(a.cpu_sharded_lam, n_lam)
            rate_t, dt_t = cpu_baseline_sharded(w, n_s, a.cpu_workers)
            cpu["all_cores"] = {
                "value": rate_t, "unit": "updates/s", "cores": a.cpu_workers,
                "speedup_over_1_core": rate_t / rate,
                "sample": f"the same oracle path in {a.cpu_workers} worker processes on "
                          f"contiguous slices of a {n_s}-lambda strided sample, bolometric sums "
                          f"exchanged per layer (oracle/sharded.py: the temperatures of the "
                          f"one-process run), 1 T-P iteration + final emit, {dt_t:.1f} s"}
    eng.close()

    # ---- T-dependent chemistry (mmr tabulated on (T, p), re-interpolated on the device before
    # every sweep; per-species sweep): the same fixed work, and the run to radiative equilibrium
    chem = None
    if d.world == 1 and not a.no_chemistry and not a.force_comm:
        from frei_amd.engine import Engine
        from frei_amd.workloads import c3_chemistry
        ce = Engine(w["lam"], w["p"], tabs, mmr=c3_chemistry(w), device=d.local)
        try:
            cpath = ce.path()
            ce.state_init(w["T0"])
            el_c = timed_iterations(ce, d, 2, a.per_species_steps)
            ce.run(w["T0"], n_timesteps=a.rad_eq_max, n_zero_crossings=2, convergence_dT=3.0,
                   alpha=1.0, want_dtaus=False)
            t4 = time.perf_counter()
            cout = ce.run(w["T0"], n_timesteps=a.rad_eq_max, n_zero_crossings=2,
                          convergence_dT=3.0, alpha=1.0, want_dtaus=False)
            t5 = time.perf_counter()
        finally:
            ce.close()
        chem = {"value": updates_per_step * a.per_species_steps / el_c, "unit": "updates/s",
                "ms_per_step": el_c / a.per_species_steps * 1e3, "steps": a.per_species_steps,
                "path": cpath,
                "rad_eq": {"iterations": cout["n_iter"], "wall_s": t5 - t4,
                           "iters_per_s": cout["n_iter"] / (t5 - t4)},
                "note": "synthetic T-dependent mixing ratios (frei_amd.workloads.c3_chemistry) "
                        "re-interpolated per layer before every sweep; per-species sweep (no K3)"}

    provider = None
    if d.world == 1 and not a.no_provider and not a.force_comm:
        provider = provider_leg(a, d, w, tabs)

    # PMC traffic / VALU of the same workload (separate rocprofv3 --pmc passes, committed)
    traffic, traffic_src, valu = None, None, None
    tpath = os.path.join(ROOT, "profiles", "traffic_sweep.json")
    if os.path.exists(tpath):
        t = json.load(open(tpath))
        if t["workload"] == {"n_lam": n_lam // d.world, "n_layers": nL, "species": S,
                             "contracted": path["contracted"]}:
            traffic, traffic_src = t, "profiles/traffic_sweep.json"
    vpath = os.path.join(ROOT, "profiles", "valu_sweep.json")
    if os.path.exists(vpath) and traffic is not None:
        valu = json.load(open(vpath))

    # C5 holds one contracted table per atmosphere (~31 GB per rank at its default size): with
    # several ranks sharing one GPU (the rehearsal) it would not fit, so it is left out there
    shared_gpu = d.world > n_dev
    c5 = None if (a.no_c5 or shared_gpu) else c5_leg(a, d)
    binning = None
    if d.rank == 0 and not a.no_binning:
        binning = binning_leg(a, d.local, cpu=(d.world == 1 and not a.no_cpu_baseline))
    if d.rank == 0:
        line = {
            "metric": "lambda-bin*layer flux updates/sec at 60 layers x 500k lambda",
            "value": value,
            "unit": "updates/s",
            "n_gpus": d.world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (separable line-forest opacity tables generated on device)",
            "config": {"workload": f"C3/C4: {nL} layers x {n_lam} lambda, {S} species "
                                   f"(H2O/CO/CO2/CH4/Na/K + H2-H2/H2-He CIA), {a.n_T} T-nodes, "
                                   "1 step = 1 T-P iteration (emit+absorb)",
                       "n_layers": nL, "n_lambda": n_lam, "n_species": S, "n_T": a.n_T,
                       "parallelism": f"lambda-shard x{d.world}"
                                      + ("" if d.world == 1 and not a.force_comm
                                         else f" ({kind} exchange per sweep)"),
                       "slicing": slicing},
            "tp_iters_per_s": 1e3 / ms_per_step,
            "exchange": exchange,
            "sweep_path": dict(path, setup_ms=setup_ms, setup_phases_ms=setup_phases,
                               tables_s=tables_s,
                               note="setup_ms: one-time metadata build + species contraction "
                                    "(K3) per tables/mmr, outside the timed steps; tables_s: "
                                    "context creation + device table generation"),
            "rad_eq": {"iterations": n_iter, "max_iterations": a.rad_eq_max,
                       "wall_s": rad_eq_wall, "iters_per_s": n_iter / rad_eq_wall,
                       "setup_s": setup_ms * 1e-3,
                       "wall_incl_setup_s": incl["lazy_k3"]["wall_s"],
                       "iters_per_s_incl_setup": incl["lazy_k3"]["iters_per_s"],
                       "incl_setup": incl,
                       "first_run_s": cold_s,
                       "note": "wall_s: warm run (T-P iterations to convergence + final emit) "
                               "over the table contracted up front; incl_setup: the metadata "
                               "build and species contraction timed with the run, lazy K3 (the "
                               "library default: rows contracted by the first sweep that reaches "
                               "them) and full K3 (every row at setup); first_run_s: the first "
                               "run, with its one-time buffer allocations"},
            "roofline": {"bound": "hbm", "achieved": achieved / 1e9, "peak": PEAK_HBM / 1e9,
                         "unit": "GB/s", "frac": achieved / PEAK_HBM,
                         "traffic": traffic["hbm_B_per_launch"] if traffic else None,
                         "traffic_unit": "B/launch (rocprofv3 PMC: 2*FETCH_SIZE+WRITE_SIZE)",
                         "traffic_source": traffic_src,
                         "traffic_over_algorithmic": traffic["traffic_over_algorithmic"]
                         if traffic else None,
                         "valu_busy": valu["valu_busy"] if valu else None,
                         "valu_insts_per_64_updates": valu["valu_insts_per_update"]
                         if valu else None,
                         "valu_source": "profiles/valu_sweep.json (SQ_ACTIVE_INST_VALU)"
                         if valu else None,
                         "kernel": sweep_kernel_name(path), "bytes_per_update": bpu,
                         "bytes_per_launch": bytes_launch,
                         "avg_launch_ms": avg_sweep_ms, "launches": n_sweeps,
                         "byte_model": (f"contracted table (K3): 8 stale opposite-stream read + "
                                        f"8 live flux write + 16 (two rows of one table) = {bpu} B"
                                        if path["contracted"] else
                                        f"8 + 8 + 16*S = {bpu} B"),
                         "survey_byte_model_equivalent": {
                             "bytes_per_update": 24 + 16 * S,
                             "effective_GBps": value / d.world * (24 + 16 * S) / 1e9,
                             "note": "value x SURVEY 8(d)'s (24 + 16 S) B: the traffic the "
                                     "reference's per-species assembly would need; above the "
                                     "HBM peak because K3 hoists the species sum out of the "
                                     "loop"}},
            "per_species": per_species,
            "chemistry": chem,
            "provider": provider,
            "cpu_baseline": cpu,
            "k6_binning": binning,
            "c5_batched": c5,
        }
        _emit_result(line)


if __name__ == "__main__":
    main()
