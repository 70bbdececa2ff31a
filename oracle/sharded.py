"""The CPU oracle at BASELINE sizes — TEST INFRASTRUCTURE (a checker and bench.py's all-cores
CPU baseline; never imported by the product, frei_amd).

``oracle.frei_oracle.emission_spectrum`` is single-threaded NumPy: 60 layers x 500k λ x 8
species takes about a minute per sweep-triple on one core.  Within a sweep every wavelength is
independent except through the four bolometric sums per layer (twostream.py:16-20, 396-398),
so the oracle runs unchanged on contiguous wavelength slices in worker processes, and the
oracle's own ``bol_fn`` hook (frei_oracle._sweep) sends each slice's partial sums — built with
the global per-point trapezoid weights, so no halo — to this coordinator, which adds them in
slice order and returns the same totals to every slice.  Temperatures, convergence decisions
and iteration counts are therefore identical in every slice, and the only difference from the
one-process oracle is the summation order inside np.trapz (tests/test_distributed_cpu.py
checks that equivalence at small sizes).

Tables are the separable synthetic ones of the benchmark workloads, held lazily
(``SeparableValues``): a worker builds only the rows it interpolates.  Workers are spawned
(not forked) processes that never touch the GPU.
"""
import multiprocessing as mp
import os
from contextlib import nullcontext

import numpy as np


def default_workers():
    # the GPU box reports the whole machine's CPUs but grants a 16-CPU share
    return max(1, min(16, os.cpu_count() or 1))


def _trapz_weights(lam_cm):
    d = np.diff(lam_cm)
    w = np.zeros(lam_cm.size)
    w[:-1] += d / 2
    w[1:] += d / 2
    return w


def _worker(conn, spec):
    from oracle import frei_oracle as O
    lo, hi = spec["lo"], spec["hi"]
    lam = spec["lam"]
    tabs = {n: O.Table(O.SeparableValues(b, fp, fT), spec["p"], spec["T_nodes"][n])
            for n, (b, fp, fT) in spec["tables"].items()}
    w = spec["w"]
    try:
        while True:
            msg = conn.recv()
            if msg[0] == "stop":
                break
            _, kw, perturb = msg

            def bol(F2u, F2d, F1u, F1d):
                conn.send(("part", np.array([np.sum(w * F2u), np.sum(w * F2d),
                                             np.sum(w * F1u), np.sum(w * F1d)])))
                return conn.recv()
            if perturb:   # the one-ulp floor: tests only
                from tests.parity import perturbed_exp
            with perturbed_exp() if perturb else nullcontext():
                with np.errstate(over="ignore", divide="ignore", invalid="ignore"):
                    out = O.emission_spectrum(tabs, spec["T0"], spec["p"], lam, spec["F_toa"],
                                              spec["g"], spec["m_bar"], spec["alpha"],
                                              mmr=spec["mmr"], bol_fn=bol, **kw)
            conn.send(("done", out))
    except EOFError:
        pass
    finally:
        conn.close()


class ShardedOracle:
    """``emission_spectrum`` of the oracle over ``n_workers`` wavelength slices.

    tables: {name: (base[n_lam], fp[n_p], fT[n_T], T_nodes[n_T])} separable tables
    (clip(fp fT base, 1e-4, 1e3), frei_oracle.separable_table), p in bar, lam in µm."""

    def __init__(self, tables, lam, p, T0, F_toa, g, m_bar, mmr=None, alpha=1.0,
                 n_workers=None):
        n = lam.size
        R = min(n_workers or default_workers(), n)
        w = _trapz_weights(np.asarray(lam, dtype=float) * 1e-4)
        ctx = mp.get_context("spawn")
        self.conns, self.procs, self.slices = [], [], []
        base, rem = divmod(n, R)
        for r in range(R):
            lo = r * base + min(r, rem)
            hi = lo + base + (1 if r < rem else 0)
            spec = dict(lo=lo, hi=hi, lam=np.ascontiguousarray(lam[lo:hi]),
                        p=np.asarray(p, dtype=float), T0=np.asarray(T0, dtype=float),
                        F_toa=np.ascontiguousarray(F_toa[lo:hi]), g=float(g),
                        m_bar=float(m_bar), alpha=alpha, mmr=mmr, w=w[lo:hi],
                        tables={k: (np.ascontiguousarray(v[0][lo:hi]), v[1], v[2])
                                for k, v in tables.items()},
                        T_nodes={k: np.asarray(v[3], dtype=float) for k, v in tables.items()})
            a, b = ctx.Pipe()
            pr = ctx.Process(target=_worker, args=(b, spec), daemon=True)
            pr.start()
            b.close()
            self.conns.append(a)
            self.procs.append(pr)
            self.slices.append((lo, hi))

    def emission_spectrum(self, perturb=False, **kw):
        """-> (spectrum, final_T, temp_hist, dtaus, F_up, F_down, n_iter), as
        frei_oracle.emission_spectrum on the whole grid; ``perturb`` runs every slice under
        tests.parity.perturbed_exp (exp / expm1 one ulp high) for the one-ulp floor."""
        for c in self.conns:
            c.send(("run", kw, perturb))
        while True:
            msgs = [self._recv(i) for i in range(len(self.conns))]
            kinds = {m[0] for m in msgs}
            if kinds == {"part"}:
                tot = msgs[0][1].copy()
                for m in msgs[1:]:          # slice order: identical totals everywhere
                    tot = tot + m[1]
                t = tuple(float(x) for x in tot)
                for c in self.conns:
                    c.send(t)
                continue
            if kinds != {"done"}:
                raise RuntimeError(f"oracle slices out of step: {sorted(kinds)}")
            outs = [m[1] for m in msgs]
            break
        sp = np.concatenate([o[0] for o in outs])
        T, th, it = outs[0][1], outs[0][2], outs[0][6]
        for o in outs[1:]:
            if not (np.array_equal(o[1], T) and o[6] == it):
                raise RuntimeError("oracle slices disagree on T / iteration count")
        dt = np.concatenate([o[3] for o in outs], axis=1)
        up = np.concatenate([o[4] for o in outs], axis=1)
        dn = np.concatenate([o[5] for o in outs], axis=1)
        return sp, T, th, dt, up, dn, it

    def _recv(self, i):
        c, pr = self.conns[i], self.procs[i]
        while not c.poll(1.0):
            if not pr.is_alive():
                raise RuntimeError(f"oracle worker {i} died (exit code {pr.exitcode})")
        return c.recv()

    def close(self):
        for c in self.conns:
            try:
                c.send(("stop",))
            except (BrokenPipeError, OSError):
                pass
        for pr in self.procs:
            pr.join(timeout=30)
            if pr.is_alive():
                pr.terminate()
        self.conns, self.procs = [], []

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
