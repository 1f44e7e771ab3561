"""Instruction mix of the fast kernels in a gpd_kernels.hip build (device assembly), to compare
builds on the CPU before a GPU A/B: the register allocator's choices move VALU counts by several
percent between near-identical sources.
    python tools/isa_count.py [path/to/gpd_kernels.hip] [-DFLAG ...]"""
import collections
import os
import re
import subprocess
import sys

src = sys.argv[1] if len(sys.argv) > 1 and sys.argv[1].endswith(".hip") else \
    os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gopacket_amd/csrc/gpd_kernels.hip")
flags = [a for a in sys.argv[1:] if a.startswith("-D")]
inc = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(src))), "include")
out = "/tmp/isa_count.s"
subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-I", inc, *flags, "-S",
                "--cuda-device-only", src, "-o", out], check=True, capture_output=True)
txt = open(out).read()
want = {"4096 CS HASH w4": "rs_kernelILi4096ELb1ELb1ELi4ELb0ELb1ELb0E",
        "8192 AL": "rs_kernelILi8192ELb1ELb1ELi3ELb0ELb0ELb0ELb1ELb0E",
        "8192 plain": "rs_kernelILi8192ELb1ELb1ELi3ELb0ELb0ELb0ELb0ELb0E",
        "8192 HO": "rs_kernelILi8192ELb1ELb1ELi3ELb0ELb1ELb1E"}
for label, key in want.items():
    m = re.search(r"\n(_ZN3gpd9" + key + r"\S*):", txt)
    if not m:
        print(f"{label:16s} (not found)")
        continue
    end = txt.find(".Lfunc_end", m.end())
    body = [l.strip() for l in txt[m.end():end].splitlines()
            if l.startswith("\t") and not l.startswith("\t.") and not l.strip().startswith(";")]
    c = collections.Counter(l.split()[0] for l in body)
    valu = sum(v for k, v in c.items() if k.startswith("v_"))
    vgpr = re.search(r"\.vgpr_count:\s+(\d+)", txt[end:end + 20000])
    print(f"{label:16s} total {len(body):5d}  valu {valu:5d}  v_mov {c['v_mov_b32_e32'] + c['v_mov_b64_e32']:4d}  "
          f"ds_read {sum(v for k, v in c.items() if k.startswith('ds_read')):3d}  waitcnt {c['s_waitcnt']:3d}")
