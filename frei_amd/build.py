"""Build libfrei_hip.so in-tree for gfx950:  python -m frei_amd.build

The library is rebuilt whenever the SHA-256 of its sources, headers and flags — or the compiler
that built it — differs from the stamp written beside it (``libfrei_hip.so.stamp``: the source
hash on its first line, the compiler's identity after it), not by modification times, which a
copied tree (the GPU box's snapshot) does not preserve meaningfully.  ``frei_amd._native`` checks
the source hash at load time and refuses a library built from other sources; the compiler line is
only compared at build time (loading runs no compiler) and named in the load error.
"""
import glob
import hashlib
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SOURCES = ["csrc/frei_kernels.hip", "csrc/frei_runtime.hip", "csrc/frei_binning.hip"]
FLAGS = ["-O3", "--offload-arch=gfx950", "-ffp-contract=off", "-fPIC", "-shared", "-std=c++17"]
LIB = os.path.join(HERE, "libfrei_hip.so")
STAMP = LIB + ".stamp"


def _hipcc():
    return os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def source_files():
    """Every file the library is built from (frei_math.h holds the sweep's division cores)."""
    srcs = [os.path.join(HERE, s) for s in SOURCES]
    return (srcs + sorted(glob.glob(os.path.join(HERE, "csrc", "*.h"))) +
            sorted(glob.glob(os.path.join(ROOT, "include", "*.h"))))


_COMPILER_ID = None


def compiler_id():
    """The compiler's path and its ``--version`` text (a ROCm upgrade changes the stamp)."""
    global _COMPILER_ID
    if _COMPILER_ID is None:
        try:
            out = subprocess.run([_hipcc(), "--version"], capture_output=True, text=True,
                                 timeout=120).stdout
        except (OSError, subprocess.SubprocessError):
            out = "unavailable"
        _COMPILER_ID = _hipcc() + "\n" + out
    return _COMPILER_ID


def sources_present():
    return all(os.path.exists(f) for f in source_files())


def source_hash(extra_flags=()):
    """SHA-256 over the sources' names and bytes and the build command's flags."""
    h = hashlib.sha256()
    for f in source_files():
        h.update(os.path.relpath(f, ROOT).encode() + b"\0")
        with open(f, "rb") as fh:
            h.update(fh.read())
        h.update(b"\0")
    h.update(" ".join([*FLAGS, *extra_flags, "-ldl"]).encode())
    return h.hexdigest()


def read_stamp(lib=LIB):
    """(source hash, compiler identity) recorded beside ``lib``; (None, None) without a stamp."""
    try:
        with open(lib + ".stamp") as f:
            text = f.read()
    except OSError:
        return None, None
    first, _, rest = text.partition("\n")
    return first.strip(), rest.strip()


def stamp_matches(lib=LIB):
    """True when ``lib`` exists and its stamp carries the current sources' hash (load-time check:
    runs no compiler)."""
    digest, _ = read_stamp(lib)
    return os.path.exists(lib) and digest == source_hash()


def build(verbose=False):
    if stamp_matches() and read_stamp()[1] == compiler_id().strip():
        return LIB
    digest = source_hash()
    # one object per translation unit, compiled in parallel (no relocatable device code: every
    # kernel is launched from its own unit), then linked
    compile_flags = [f for f in FLAGS if f != "-shared"]
    objs, procs = [], []
    for src in SOURCES:
        obj = os.path.join(HERE, "build_" + os.path.basename(src).replace(".hip", ".o"))
        cmd = [_hipcc(), *compile_flags, "-I" + os.path.join(ROOT, "include"), "-c",
               os.path.join(HERE, src), "-o", obj]
        if verbose:
            print(" ".join(cmd))
        procs.append(subprocess.Popen(cmd))
        objs.append(obj)
    if any(p.wait() != 0 for p in procs):
        raise subprocess.CalledProcessError(1, "hipcc")
    cmd = [_hipcc(), *FLAGS, *objs, "-o", LIB + ".tmp", "-ldl"]
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    os.replace(LIB + ".tmp", LIB)
    for o in objs:
        os.unlink(o)
    with open(STAMP + ".tmp", "w") as f:
        f.write(digest + "\n" + compiler_id().strip() + "\n")
    os.replace(STAMP + ".tmp", STAMP)
    return LIB


if __name__ == "__main__":
    print(build(verbose="-v" in sys.argv))
