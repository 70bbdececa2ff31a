"""ISA histogram of the headline sweep's per-step loop (VERDICT r03 "next" #5).

    python tools/isa_hist.py [-DNAME=V ...] [--kernel MANGLED] [--out FILE]

Compiles frei_kernels.hip for gfx950 (-S, the build's flags), cuts the kernel's text, finds its
loops (a backward branch to an earlier label) and prints, for the loop with the most VALU
instructions (the step loop: one (layer, lambda) update per lane per trip), the opcode histogram
grouped by what the instructions compute.  One trip = one update per lane, so the VALU count of
the loop body is VALU per 64 updates at the static level (PMC counts it dynamically).
"""
import collections
import re
import subprocess
import sys

args = [a for a in sys.argv[1:] if a.startswith("-D")]
kern = "sweep_fast_kernelILi0ELi1ELi2ELb0ELb0ELb1ELi2EE"
outf = None
for i, a in enumerate(sys.argv):
    if a == "--kernel":
        kern = sys.argv[i + 1]
    if a == "--out":
        outf = sys.argv[i + 1]
asm = "/tmp/isa_hist.s"
subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "--offload-arch=gfx950", "-ffp-contract=off",
                "-std=c++17", "--cuda-device-only", "-S", "-Iinclude", *args,
                "frei_amd/csrc/frei_kernels.hip", "-o", asm], check=True, stderr=subprocess.DEVNULL)
s = open(asm).read()
name = re.search(r"\n(_ZN4frei\w*" + kern + r"\w*):", s).group(1)
st = s.index("\n" + name + ":")
body = s[st:s.index(".Lfunc_end", st)].split("\n")

labels = {}
for i, ln in enumerate(body):
    m = re.match(r"^(\.LBB\w+):", ln)
    if m:
        labels[m.group(1)] = i
loops = []
for i, ln in enumerate(body):
    m = re.match(r"\s+s_(?:cbranch_\w+|branch)\s+(\.LBB\w+)", ln)
    if m and m.group(1) in labels and labels[m.group(1)] < i:
        lo = labels[m.group(1)]
        ops = [re.match(r"\s+(\S+)", x).group(1) for x in body[lo:i + 1]
               if re.match(r"\s+[vsgd]\w*_", x)]
        loops.append((sum(o.startswith("v_") for o in ops), lo, i, ops))
loops.sort(reverse=True)
nvalu, lo, hi, ops = loops[0]

GROUPS = [
    ("fma/mul/add f64", r"v_(fma|mul|add|fmac|sub)_f64|v_(fma|mul|add)_f64"),
    ("div (scale/fmas/fixup)", r"v_div_"),
    ("rcp/rsq/sqrt", r"v_(rcp|rsq|sqrt)_"),
    ("exp/ldexp/frexp/fract", r"v_(exp|ldexp|frexp|fract|trig)"),
    ("compare/select", r"v_(cmp|cndmask)"),
    ("cvt/int/bit", r"v_(cvt|and|or|xor|lsh|ashr|bfe|bfi|add_u|add_co|sub_u|sub_co|addc|subb|mad_u|mul_lo|mul_hi|not|max_i|min_i|lshl)"),
    ("mov", r"v_(mov|accvgpr)"),
    ("dpp/permlane/readlane", r"v_(readlane|readfirstlane|writelane|permlane)|_dpp"),
    ("max/min f64", r"v_(max|min)_f64"),
]
hist = collections.Counter(o for o in ops if o.startswith("v_"))
grouped = collections.Counter()
for o, n in hist.items():
    for g, pat in GROUPS:
        if re.match(pat, o):
            grouped[g] += n
            break
    else:
        grouped["other VALU"] += n
lines = [f"kernel {name}", f"defines {' '.join(args) or '(build defaults)'}",
         f"step loop: lines {lo}-{hi} of the kernel text, {len(ops)} instructions, "
         f"{nvalu} VALU per trip (= per 64 updates), "
         f"{sum(o.startswith('s_') for o in ops)} SALU/branch, "
         f"{sum(o.startswith(('global_', 'buffer_', 'ds_', 'flat_')) for o in ops)} memory",
         "", "by group:"]
for g, n in grouped.most_common():
    lines.append(f"  {g:26s} {n:4d}")
lines += ["", "by opcode:"]
for o, n in hist.most_common():
    lines.append(f"  {o:26s} {n:4d}")
txt = "\n".join(lines)
print(txt)
if outf:
    open(outf, "w").write(txt + "\n")
