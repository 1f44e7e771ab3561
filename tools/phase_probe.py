"""Diagnostic: where the fast kernel's waves spend their clocks (wait / plan+issue / decode /
cooperative checksum / stores / loop overhead), from the GPD_PHASE_TIMING build
(gopacket_amd/libgpd_phase.so, built by `python tools/phase_probe.py --build` on the CPU).

    GPD_LIB_PATH=gopacket_amd/libgpd_phase.so python tools/phase_probe.py --config imix
"""
import argparse
import ctypes as C
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
PHASES = ["wait", "plan_issue", "decode", "coop", "store", "loop"]


def build():
    from gopacket_amd.build import HIPCC, ARCH, SOURCES, ROOT as R
    out = os.path.join(R, "gopacket_amd", "libgpd_phase.so")
    subprocess.run([HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
                    "-DGPD_PHASE_TIMING", "-I", os.path.join(R, "include"), *SOURCES, "-o", out],
                   check=True)
    print(out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--config", default="imix")
    ap.add_argument("--steps", type=int, default=10)
    a = ap.parse_args()
    if a.build:
        return build()
    import torch
    import bench
    from gopacket_amd import _lib, layers as L, parser as P
    lib = C.CDLL(_lib.LIB_PATH)
    lib.gpd_diag_phase.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
    _, n = bench.CONFIGS[a.config]
    batch = bench.make_batch(a.config, n, 0)
    db, dr = P.DeviceBatch(batch, 0), P.DeviceResult(n, 0, ext=False, hdr_off=False)
    p = P.NewDecodingLayerParser(L.LayerTypeEthernet, P.Ethernet(), P.Dot1Q(), P.IPv4(), P.IPv6(),
                                 P.IPv6ExtensionSkipper(), P.TCP(), P.UDP(), P.VXLAN(), P.Payload(),
                                 P.Fragment(), device=0)
    s = torch.cuda.current_stream(0)
    buf = (C.c_ulonglong * 8)()
    for _ in range(3):
        p.decode_device(db, dr, s)
    torch.cuda.synchronize()
    lib.gpd_diag_phase(buf, 1)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(a.steps):
        p.decode_device(db, dr, s)
    e1.record(s)
    torch.cuda.synchronize()
    lib.gpd_diag_phase(buf, 0)
    tot = sum(buf[k] for k in range(6))
    tiles = (n + 63) // 64 * a.steps
    print(json.dumps({"config": a.config, "ms": e0.elapsed_time(e1) / a.steps,
                      "clk_per_tile": {PHASES[k]: round(buf[k] / tiles, 1) for k in range(6)},
                      "frac": {PHASES[k]: round(buf[k] / tot, 3) for k in range(6)}}))


if __name__ == "__main__":
    main()
