"""Diagnostic: where the PCIe-inclusive pcap replay spends its time (one MI355X).

    python tools/pcie_probe.py [--records 2^26]

Times, on one capture of config-2 records in registered host memory: the record walk alone
(gpd_pcap_index of 2^24 records from a record position), gpd_decode_pcap_at of the same
2^24 records (walk + raw bytes H2D + decode + results D2H), a plain H2D copy of those bytes,
and a D2H copy of 2^24 40-B results into pageable and into registered host arrays.
"""
import argparse
import json
import os
import struct
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--records", type=int, default=1 << 26)
    ap.add_argument("--threads", type=int, default=16)
    a = ap.parse_args()
    import torch
    from gopacket_amd import layers as L
    from gopacket_amd import parser as P
    from gopacket_amd import pcap as NP
    from gopacket_amd import synth
    from gopacket_amd._lib import lib
    from gopacket_amd.batch import PAD
    from gopacket_amd.results import BatchResult
    n = a.records
    cap = np.empty(24 + 80 * n + PAD, np.uint8)
    cap[:24] = np.frombuffer(struct.pack("<IHHiIII", 0xA1B2C3D4, 2, 4, 0, 0, 262144, 1), np.uint8)
    synth.udp64_native(cap[24:24 + 80 * n], 0, n, records=True, nthreads=a.threads)
    cap[24 + 80 * n:] = 0
    dl = 24 + 80 * n
    info = NP.header(cap, dl)
    p = P.NewDecodingLayerParser(L.LayerTypeEthernet, P.Ethernet(), P.IPv4(), P.UDP(), P.Payload())
    h = p.ctx().h
    assert lib.gpd_host_register(h, cap.ctypes.data, cap.nbytes) == 0
    m = 1 << 24
    pos, _, _ = NP.locate(cap, [m], data_len=dl, nthreads=a.threads)  # a chunk that starts mid-capture
    start = int(pos[0])
    out = {}
    for k in range(3):
        t0 = time.perf_counter()
        pc = NP.index(cap, max_n=m, nthreads=a.threads, data_len=dl, pos=start, info=info)
        out["walk_2^24_s"] = round(time.perf_counter() - t0, 4)
    z = lambda dt: np.zeros(m, dt)
    res = BatchResult(z(np.uint32), z(np.uint64), z(np.uint64), z(np.uint64), z(np.uint32), None, z(np.uint32))
    for k in range(3):
        t0 = time.perf_counter()
        kk, nxt, stop, err = p.DecodePcapAt(cap, info, start, m, res, a.threads, data_len=dl)
        out["decode_pcap_at_2^24_s"] = round(time.perf_counter() - t0, 4)
    assert kk == m and err is None
    regd = []
    for arr in (res.status, res.layers, res.net_hash, res.tp_hash, res.csum, res.hdr_off):
        assert lib.gpd_host_register(h, arr.ctypes.data, arr.nbytes) == 0
        regd.append(arr)
    for k in range(3):
        t0 = time.perf_counter()
        p.DecodePcapAt(cap, info, start, m, res, a.threads, data_len=dl)
        out["decode_pcap_at_2^24_registered_out_s"] = round(time.perf_counter() - t0, 4)
    ph = np.zeros(6, np.float64)
    lib.gpd_decode_pcap_last_times(ph.ctypes.data)
    out["phases_ms"] = dict(zip(["total", "walk", "walk_wait", "stage", "sync", "drain"],
                                [round(float(x), 2) for x in ph]))
    dev = torch.empty(80 * m, dtype=torch.uint8, device="cuda")
    src = torch.from_numpy(cap[start:start + 80 * m])
    for k in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        dev.copy_(src)
        torch.cuda.synchronize()
        out["h2d_1.34GB_GBps"] = round(80 * m / (time.perf_counter() - t0) / 1e9, 1)
    d40 = torch.empty(40 * m, dtype=torch.uint8, device="cuda")
    hp = np.empty(40 * m, np.uint8)
    for k in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        torch.from_numpy(hp).copy_(d40)
        out["d2h_40B_x2^24_pageable_GBps"] = round(40 * m / (time.perf_counter() - t0) / 1e9, 1)
    assert lib.gpd_host_register(h, hp.ctypes.data, hp.nbytes) == 0
    for k in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        torch.from_numpy(hp).copy_(d40)
        out["d2h_40B_x2^24_registered_GBps"] = round(40 * m / (time.perf_counter() - t0) / 1e9, 1)
    out["Mpps_decode_pcap_at"] = round(m / out["decode_pcap_at_2^24_s"] / 1e6, 1)
    out["Mpps_decode_pcap_at_registered_out"] = round(m / out["decode_pcap_at_2^24_registered_out_s"] / 1e6, 1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
