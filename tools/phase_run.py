"""Diagnostic: per-phase shader clocks of the fast kernel's loop (waiting for a window and
copying it / planning and issuing the next / decode / cooperative checksum / stores / loop
tail), summed over waves, from a GPD_PHASE_TIMING build of libgpd.so.  Run it from a tree
whose library was built with the macro (never the product tree):

    rm -rf ab_ph && mkdir ab_ph && git archive HEAD | tar -x -C ab_ph &&
    (cd ab_ph && GPD_EXTRA_CFLAGS=-DGPD_PHASE_TIMING python -m gopacket_amd.build)
    (cd ab_ph && python tools/phase_run.py --config imix)
"""
import argparse
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="udp64")
    ap.add_argument("--steps", type=int, default=10)
    args = ap.parse_args()
    import bench
    import torch
    from gopacket_amd import layers as L
    from gopacket_amd import parser as P
    from gopacket_amd._lib import lib
    fn = lib.gpd_diag_phase  # AttributeError unless the library was built with GPD_PHASE_TIMING
    fn.restype = C.c_int
    fn.argtypes = [C.c_void_p, C.c_int]
    workload, n = bench.CONFIGS[args.config]
    batch = bench.make_batch(args.config, n, 0)
    if args.config == "pcap64":
        from gopacket_amd import pcap as NP
        batch = NP.index(batch).batch
    db, dr = P.DeviceBatch(batch, 0), P.DeviceResult(n, 0, hdr_off=False)
    p = P.NewDecodingLayerParser(L.LayerTypeEthernet, P.Ethernet(), P.Dot1Q(), P.IPv4(), P.IPv6(),
                                 P.IPv6ExtensionSkipper(), P.TCP(), P.UDP(), P.VXLAN(), P.Payload(),
                                 P.Fragment())
    p.decode_device(db, dr)
    torch.cuda.synchronize()
    buf = (C.c_ulonglong * 8)()
    fn(buf, 1)
    for _ in range(args.steps):
        p.decode_device(db, dr)
    torch.cuda.synchronize()
    fn(buf, 1)
    names = ["wait+commit", "plan+issue", "decode", "coop_csum", "stores+fallback", "loop_tail"]
    tot = sum(buf[k] for k in range(6))
    print(json.dumps({"config": args.config, "share": {names[k]: round(buf[k] / tot, 4) for k in range(6)},
                      "clocks_per_tile": {names[k]: round(buf[k] / (args.steps * ((n + 63) // 64)), 1)
                                          for k in range(6)}}))


if __name__ == "__main__":
    main()
