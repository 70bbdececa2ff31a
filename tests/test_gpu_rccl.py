"""RCCL plumbing on one GPU: a forced single-rank communicator (FREI_FORCE_RCCL=1) runs the
real dlopen -> ncclGetUniqueId -> ncclCommInitRank -> per-sweep ncclAllGather path; the
result must be bitwise identical to the run without a communicator (1-rank all-gather is
a copy, the rank-order sum is the identity)."""
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = r'''
import ctypes, sys, numpy as np
sys.path.insert(0, ROOT)
import frei_amd as fa
from frei_amd import _native as N
from frei_amd.engine import Engine
grid = fa.Grid(fa.Planet.from_hot_jupiter(), n_wl_bins=2000, n_layers=30, T_ref=2400)
op = fa.load_example_opacity(grid, scale_factor=1)
comm = None
if RCCL:
    buf = ctypes.create_string_buffer(128)
    N.check(N.lib().frei_comm_unique_id(buf))
    comm = ("rccl", 1, 0, buf.raw)
eng = Engine(grid.lam, grid.pressures, op, device=0, comm=comm)
out = eng.run(grid.init_temperatures, n_timesteps=30)
np.savez(OUT, spec=out["spectrum"], T=out["final_T"], n=out["n_iter"])
'''


def _run(tmp_path, rccl):
    out = str(tmp_path / f"r{int(rccl)}.npz")
    env = dict(os.environ, FREI_FORCE_RCCL="1" if rccl else "0")
    code = SCRIPT.replace("ROOT", repr(ROOT)).replace("RCCL", str(rccl)).replace("OUT", repr(out))
    subprocess.run([sys.executable, "-c", code], check=True, env=env, timeout=300)
    return np.load(out)


def test_single_rank_rccl_allgather_is_bitwise_neutral(tmp_path):
    a = _run(tmp_path, False)
    b = _run(tmp_path, True)
    assert int(a["n"]) == int(b["n"])
    assert np.array_equal(a["T"], b["T"])
    assert np.array_equal(a["spec"], b["spec"])
