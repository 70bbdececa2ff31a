"""Register use and VALU counts of the hot sweep kernels for a set of compile definitions.
    python tools/asm_stats.py [-DNAME=V ...]"""
import re
import subprocess
import sys

KER = {
    "emit1": "sweep_fast_kernelILi0ELi1ELi2ELb0ELb0ELb1EE",
    "absorb1": "sweep_fast_kernelILi1ELi1ELi2ELb0ELb0ELb1EE",
    "emit1sh": "sweep_fast_kernelILi0ELi1ELi2ELb0ELb1ELb1EE",
    "emit8": "sweep_fast_kernelILi0ELi8ELi2ELb0ELb0ELb0EE",
    "grp2e": "sweep_group_kernelILi0ELi2EE",
}
out = "/tmp/asm_stats.s"
subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "--offload-arch=gfx950", "-ffp-contract=off",
                "-std=c++17", "--cuda-device-only", "-S", "-Iinclude", *sys.argv[1:],
                "frei_amd/csrc/frei_kernels.hip", "-o", out], check=True,
               stderr=subprocess.DEVNULL)
s = open(out).read()
for k, pat in KER.items():
    m = re.search(r"\.name:\s+\S*" + pat + r"\S*\n(.*?)\.vgpr_spill_count:\s+(\d+)", s, re.S)
    blk = m.group(0)
    g = lambda f: re.search(r"\." + f + r":\s+(\d+)", blk).group(1)
    name = re.search(r"\.name:\s+(\S+)", blk).group(1)
    st = s.index(name + ":")
    en = s.index(".Lfunc_end", st)
    valu = len(re.findall(r"\n\s+v_", s[st:en]))
    movs = len(re.findall(r"\n\s+v_mov_b64", s[st:en]))
    print(f"{k:8s} vgpr {g('vgpr_count')} sgpr {g('sgpr_count')} sgpr_spill "
          f"{g('sgpr_spill_count')} vgpr_spill {g('vgpr_spill_count')} static_valu {valu} "
          f"mov_b64 {movs}")
