"""Per-kernel register use of gpd_kernels.hip (hipcc -Rpass-analysis=kernel-resource-usage):
    python tools/kres.py [filter]"""
import re
import subprocess
import sys

ROOT = __file__.rsplit("/tools/", 1)[0]
r = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-I", ROOT + "/include",
                    "-c", ROOT + "/gopacket_amd/csrc/gpd_kernels.hip", "-o", "/tmp/kres.o"] + __import__("os").environ.get("GPD_EXTRA_CFLAGS", "").split() + [
                    "-Rpass-analysis=kernel-resource-usage"], capture_output=True, text=True)
cur, rows = None, []
for line in r.stderr.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = {"name": m.group(1)}
        rows.append(cur)
        continue
    m = re.search(r"(VGPRs|VGPRs Spill|Occupancy \[waves/SIMD\]|AGPRs|LDS Size \[bytes/block\]): (\d+)", line)
    if m and cur is not None:
        cur[m.group(1)] = int(m.group(2))
flt = sys.argv[1] if len(sys.argv) > 1 else "rs_kernel"
for c in rows:
    if flt in c["name"]:
        print(f"{c.get('VGPRs', '?'):>4} vgpr {c.get('VGPRs Spill', 0):>3} spill occ {c.get('Occupancy [waves/SIMD]', '?')}  {c['name']}")
