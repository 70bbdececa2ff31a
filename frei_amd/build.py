"""Build libfrei_hip.so in-tree for gfx950:  python -m frei_amd.build"""
import glob
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SOURCES = ["csrc/frei_kernels.hip", "csrc/frei_runtime.hip", "csrc/frei_binning.hip"]
FLAGS = ["-O3", "--offload-arch=gfx950", "-ffp-contract=off", "-fPIC", "-shared", "-std=c++17"]


def build(verbose=False):
    out = os.path.join(HERE, "libfrei_hip.so")
    srcs = [os.path.join(HERE, s) for s in SOURCES]
    # every header the sources include (frei_math.h holds the sweep's division/sqrt cores)
    deps = (srcs + sorted(glob.glob(os.path.join(HERE, "csrc", "*.h"))) +
            sorted(glob.glob(os.path.join(ROOT, "include", "*.h"))))
    if os.path.exists(out) and all(os.path.getmtime(out) >= os.path.getmtime(d) for d in deps):
        return out
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    cmd = [hipcc, *FLAGS, "-I" + os.path.join(ROOT, "include"), *srcs, "-o", out + ".tmp", "-ldl"]
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    os.replace(out + ".tmp", out)
    return out


if __name__ == "__main__":
    print(build(verbose="-v" in sys.argv))
