import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")
    config.addinivalue_line("markers", "slow: multi-second CPU test")


_OUTCOMES = {"passed": 0, "failed": 0, "skipped": 0}


def pytest_runtest_logreport(report):
    if report.when == "call" or (report.when == "setup" and report.outcome != "passed"):
        _OUTCOMES[report.outcome] = _OUTCOMES.get(report.outcome, 0) + 1


def _provenance(session, exitstatus):
    """Which tree and run produced a parity log: the hash of the shipped source tree computed
    from the files on the machine that ran (tests/provenance.py; equal to
    ``python -m tests.provenance`` on the committed checkout), the source hash the native
    library was built from, host, time, the pytest arguments and the session's outcome
    counts."""
    import datetime
    import socket
    from tests.provenance import tree_hash
    digest, n_files = tree_hash(ROOT)
    prov = {"host": socket.gethostname(),
            "utc": datetime.datetime.now(datetime.timezone.utc).isoformat(timespec="seconds"),
            "pytest_args": [str(a) for a in session.config.invocation_params.args],
            "exitstatus": int(exitstatus), "outcomes": dict(_OUTCOMES),
            "tree_hash": digest, "tree_files": n_files}
    from frei_amd.build import read_stamp, source_hash
    prov["lib_source_hash"], compiler = read_stamp()
    prov["lib_compiler"] = (compiler or "").splitlines()[:2]
    prov["lib_matches_tree"] = prov["lib_source_hash"] == source_hash()
    return prov


def pytest_sessionfinish(session, exitstatus):
    """With FREI_PARITY_JSON set, write the observed grid-level parity errors of the session
    (tests/parity.py PARITY_LOG) there, with the provenance of the run."""
    path = os.environ.get("FREI_PARITY_JSON")
    if not path:
        return
    from tests.parity import PARITY_LOG
    if not PARITY_LOG:
        return
    import json
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    worst = {k: max((e.get(k, 0.0) for e in PARITY_LOG), default=0.0)
             for k in ("spectrum_elementwise", "F_up_rownorm", "F_down_rownorm",
                       "T_elementwise")}
    with open(path, "w") as f:
        json.dump({"provenance": _provenance(session, exitstatus),
                   "criterion": "tests/parity.py assert_grid_parity: spectrum elementwise, "
                                "F_up/F_down row-normwise <= max(1e-10, 2 x one-ulp floor); "
                                "T elementwise <= 1e-10",
                   "entries": PARITY_LOG, "worst": worst,
                   "all_within_1e-10": all(e["within_1e-10"] for e in PARITY_LOG)},
                  f, indent=1)


@pytest.fixture(scope="session")
def golden():
    import numpy as np
    d = os.path.join(ROOT, "tests", "golden")

    def load(name):
        return np.load(os.path.join(d, name), allow_pickle=False)
    return load
