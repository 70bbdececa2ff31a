"""bench.py --gpus N without a launcher: the process starts N rank processes of
itself, they rendezvous over 127.0.0.1, and exactly one JSON line comes back (rank 0's).  The
`--launch-selftest` workload does the rendezvous, a barrier and the max-over-ranks reduction of
the real run, and touches no GPU."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(n, extra_env=None):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT", "MASTER_ADDR")}
    env.update(extra_env or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n),
                           "--launch-selftest"], env=env, capture_output=True, timeout=120)


def test_self_launch_two_ranks_one_line():
    r = _run(2)
    assert r.returncode == 0, r.stderr.decode()[-2000:]
    lines = [x for x in r.stdout.decode().splitlines() if x.strip()]
    assert len(lines) == 1, lines
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2
    assert line["value"] == 1.0            # max over ranks of the rank number
    pids = line["pids"]
    assert len(set(pids)) == 2             # two distinct rank processes ...
    assert all(p != os.getpid() for p in pids)


def test_self_launch_four_ranks():
    r = _run(4)
    assert r.returncode == 0, r.stderr.decode()[-2000:]
    line = json.loads(r.stdout.decode().strip())
    assert line["n_gpus"] == 4 and line["value"] == 3.0 and len(set(line["pids"])) == 4


def test_self_launch_failing_rank_fails_the_launch():
    r = _run(2, {"FREI_LAUNCH_SELFTEST_FAIL": "1"})   # rank 1 exits with status 3
    assert r.returncode != 0   # 3 (rank 1) or 1 (rank 0 losing its peer), whichever ends first
    assert r.stdout.decode().strip() == ""
