"""Run tools/va_probe twice at once on GPU 0 — identical allocation sequences (same VAs), then
with rank 1's allocations offset by 1.5 GiB (the tests' workaround) — and print both processes'
counts of values that were not their own.   python tools/va_probe.py [ITERS]"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))


def pair(iters, offset_mb):
    procs = [subprocess.Popen([os.path.join(HERE, "va_probe"), str(r), str(iters),
                               str(offset_mb if r == 1 else 0)],
                              stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
             for r in (0, 1)]
    outs = [p.communicate(timeout=240)[0] for p in procs]
    return [(p.returncode, o.strip()) for p, o in zip(procs, outs)]


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
    for label, off in (("identical VAs", 0), ("rank 1 offset 1536 MB", 1536),
                       ("identical VAs (again)", 0)):
        print(f"== {label}")
        for rc, out in pair(iters, off):
            print(f"  rc {rc}: " + out.replace("\n", "\n         "))


if __name__ == "__main__":
    main()
