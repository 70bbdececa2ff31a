"""ISA histogram per flux update of the headline sweep (VERDICT r03 "next" #5).

    python tools/isa_hist.py [-DNAME=V ...] [--kernel MANGLED] [--steps-per-trip N] [--out FILE]

Compiles frei_kernels.hip for gfx950 (-S, the build's flags; the E = 1 coefficient head is the
fall-through of its wave-uniform branch, the path every wave of the C3/C4 500k sweep takes) and
walks the step loop's hot path: from the loop
header, fall through every conditional branch (LLVM lays out the likely successor as the
fall-through; the unlikely paths are out of line), follow unconditional ones, until the back
edge.  One trip of the headline loop is two steps (PF = 2), i.e. two updates per lane, so the
counts are divided by 2: VALU per 64 updates, to compare with the PMC figure
(SQ_INSTS_VALU / wave-steps, tools/pmc_valu.py), which also includes the prologue, the
epilogue and any rare path.
"""
import collections
import re
import subprocess
import sys

args = [a for a in sys.argv[1:] if a.startswith("-D")]
kern = "sweep_fast_kernelILi0ELi1ELi2ELb0ELb0ELb1ELi2EE"
steps = 2
outf = None
for i, a in enumerate(sys.argv):
    if a == "--kernel":
        kern = sys.argv[i + 1]
    if a == "--steps-per-trip":
        steps = int(sys.argv[i + 1])
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
meta = re.search(r"\.name:\s+" + name + r"\n(.*?)\.vgpr_spill_count:\s+(\d+)", s, re.S).group(0)
vgpr = re.search(r"\.vgpr_count:\s+(\d+)", meta).group(1)

labels = {re.match(r"^(\.LBB\w+):", l).group(1): i for i, l in enumerate(body)
          if re.match(r"^(\.LBB\w+):", l)}
# the step loop: the depth-1 loop with the most blocks
heads = [re.match(r"^(\.LBB\w+):", l).group(1) for l in body
         if "Loop Header: Depth=1" in l and re.match(r"^(\.LBB\w+):", l)]
tag = lambda h: "Header=" + h[1:].replace("LBB", "BB") + " "
head = max(heads, key=lambda h: sum(tag(h) in l for l in body))

i, ops = labels[head] + 1, []
for _ in range(100000):
    l = body[i]
    m = re.match(r"^(\.LBB\w+):", l)
    if m and m.group(1) == head:
        break
    mm = re.match(r"\s+([a-z]\w*)", l)
    if mm:
        ops.append(mm.group(1))
        b = re.match(r"\s+s_branch\s+(\.LBB\w+)", l)
        if b:
            if b.group(1) == head:
                break
            i = labels[b.group(1)] + 1
            continue
        b = re.match(r"\s+s_cbranch_\w+\s+(\.LBB\w+)", l)
        if b and b.group(1) == head:
            break
    i += 1

GROUPS = [
    ("f64 fma/mul/add", r"v_(fma|fmac|mul|add)_f64"),
    ("f64 rcp/rsq", r"v_(rcp|rsq|sqrt)_f64"),
    ("f64 rndne/ldexp/cvt (exp)", r"v_(rndne_f64|ldexp_f64|cvt_i32_f64|frexp|fract)"),
    ("f64 max/min", r"v_(max|min)_f64"),
    ("compare / select", r"v_(cmp|cndmask)"),
    ("DPP / permlane (sums)", r"v_mov_b32_dpp|v_permlane"),
    ("address / integer", r"v_(lshl|lshr|add_u|add3|add_co|addc|sub_|mad_u|mul_lo|mul_u|and_b|or_b|or3|bfe|xor)"),
    ("moves", r"v_(mov|accvgpr)"),
    ("lane (SGPR spill)", r"v_(readlane|writelane|readfirstlane)"),
]
valu = [o for o in ops if o.startswith("v_")]
hist = collections.Counter(valu)
grouped = collections.Counter()
for o, n in hist.items():
    for g, pat in GROUPS:
        if re.match(pat, o):
            grouped[g] += n
            break
    else:
        grouped["other VALU"] += n
per = lambda n: n / steps
mem = sum(o.startswith(("global_", "buffer_", "flat_")) for o in ops)
lds = sum(o.startswith("ds_") for o in ops)
lines = [f"kernel {name}  ({vgpr} VGPRs)",
         f"defines {' '.join(args) or '(none)'}",
         f"hot path of one loop trip ({steps} steps): {len(ops)} instructions, {len(valu)} VALU "
         f"-> {per(len(valu)):.1f} VALU per 64 updates; {per(mem):.1f} global memory and "
         f"{per(lds):.1f} LDS instructions per step",
         "", "per 64 updates, by group:"]
for g, n in grouped.most_common():
    lines.append(f"  {g:28s} {per(n):6.1f}")
lines += ["", "per 64 updates, by opcode:"]
for o, n in hist.most_common():
    lines.append(f"  {o:28s} {per(n):6.1f}")
txt = "\n".join(lines)
print(txt)
if outf:
    open(outf, "w").write(txt + "\n")
