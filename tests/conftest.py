import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")
    config.addinivalue_line("markers", "slow: multi-second CPU test")


def pytest_sessionfinish(session, exitstatus):
    """With FREI_PARITY_JSON set, write the observed grid-level parity errors of the session
    (tests/parity.py PARITY_LOG) there."""
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
        json.dump({"criterion": "tests/parity.py assert_grid_parity: spectrum elementwise, "
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
