"""bench.py's exchange fallback chain (host logic, no GPU): after a failed P2P setup every rank
goes to RCCL, and to the host all-gather when RCCL cannot be set up on some rank either."""
import importlib.util
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


class _Dist:
    """One rank whose all_ok is the local verdict (a single-rank world)."""
    def all_ok(self, ok):
        return bool(ok)


class _Eng:
    def __init__(self, kind):
        self.kind, self.closed = kind, False

    def close(self):
        self.closed = True


def test_fallback_to_rccl(monkeypatch):
    b = _bench()
    monkeypatch.setattr(b, "build_engine", lambda w, t, lo, hi, d, kind, force=False: _Eng(kind))
    eng, kind, note = b.build_engine_fallback(None, None, 0, 1, _Dist(), False, "p2p setup failed")
    assert (eng.kind, kind) == ("rccl", "rccl") and note.endswith("fell back to RCCL")


def test_fallback_to_host_when_rccl_fails(monkeypatch):
    b = _bench()

    def build(w, t, lo, hi, d, kind, force=False):
        if kind == "rccl":
            raise RuntimeError("ncclCommInitRank: invalid usage")
        return _Eng(kind)

    monkeypatch.setattr(b, "build_engine", build)
    eng, kind, note = b.build_engine_fallback(None, None, 0, 1, _Dist(), False, "p2p failed")
    assert (eng.kind, kind) == ("host", "host")
    assert "RCCL setup failed too" in note and "invalid usage" in note
