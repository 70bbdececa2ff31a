"""Tree provenance for parity logs (VERDICT r04 "next" #1): a hash of the shipped source tree
computed from the files themselves, so a log written on the GPU box (whose snapshot has no
.git) names exactly what ran.  ``python -m tests.provenance`` prints the same hash here; on a
clean checkout it is the committed tree's.

Hashed: every file under frei_amd/, include/, oracle/ and tests/ plus bench.py and
__graft_entry__.py, except built artefacts (shared objects, objects, build stamps) and Python
caches; each file contributes its repo-relative path and the SHA-256 of its bytes, in sorted
path order."""
import hashlib
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DIRS = ("frei_amd", "include", "oracle", "tests")
FILES = ("bench.py", "__graft_entry__.py")
_SKIP_SUFFIX = (".so", ".o", ".a", ".stamp", ".pyc", ".hsaco", ".co")
_SKIP_DIRS = ("__pycache__", "_ref", ".pytest_cache")


def shipped_files(root=ROOT):
    out = [f for f in FILES if os.path.isfile(os.path.join(root, f))]
    for d in DIRS:
        for dirpath, dirnames, filenames in os.walk(os.path.join(root, d)):
            dirnames[:] = sorted(x for x in dirnames if x not in _SKIP_DIRS)
            for name in filenames:
                if not name.endswith(_SKIP_SUFFIX):
                    out.append(os.path.relpath(os.path.join(dirpath, name), root))
    return sorted(out)


def tree_hash(root=ROOT):
    """(hex digest, number of files) over :func:`shipped_files`."""
    h = hashlib.sha256()
    files = shipped_files(root)
    for rel in files:
        with open(os.path.join(root, rel), "rb") as f:
            h.update(rel.encode() + b"\0" + hashlib.sha256(f.read()).digest())
    return h.hexdigest(), len(files)


if __name__ == "__main__":
    digest, n = tree_hash()
    print(f"{digest} {n} files")
