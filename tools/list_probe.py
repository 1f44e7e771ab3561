"""Diagnostic: the generic list kernel's cost per fallback packet, homogeneous vs mixed.
Batches of 2^20 frames where every frame is one traffic-mix fallback class (IPv4 options,
fragments, hop-by-hop, cut TCP, STP) or the mix of all five; prints the fast / list split
(gpd_last_launch_split, mean of 5 timed launches) per batch as JSON lines."""
import ctypes as C
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from gopacket_amd import layers as L, synth  # noqa: E402
from gopacket_amd import parser as P  # noqa: E402
from gopacket_amd._lib import check, lib  # noqa: E402
from gopacket_amd.batch import PacketBatch  # noqa: E402


def run(name, frames):
    b = PacketBatch.from_packets(frames)
    p = P.DecodingLayerParser(L.LayerTypeEthernet)
    p._mask = 0xFFF
    db, dr = P.DeviceBatch(b, 0), P.DeviceResult(b.n, 0)
    h = p.ctx().h
    for _ in range(20):
        p.decode_device(db, dr)
    check(lib.gpd_ctx_set_timing(h, 1), "timing")
    fb, f, l = C.c_uint64(), C.c_float(), C.c_float()
    fs, ls = [], []
    for _ in range(5):
        p.decode_device(db, dr)
        check(lib.gpd_last_launch_split(h, C.byref(fb), C.byref(f), C.byref(l)), "split")
        fs.append(f.value)
        ls.append(l.value)
    torch.cuda.synchronize()
    print(json.dumps({"batch": name, "n": b.n, "fallback": fb.value, "fast_ms": round(float(np.mean(fs)), 4),
                      "list_ms": round(float(np.mean(ls)), 4),
                      "list_ns_per_packet": round(float(np.mean(ls)) * 1e6 / max(1, fb.value), 2)}), flush=True)


def main():
    n = 1 << 20
    ft, fu = synth._free_ports(synth.TABLES.tcp_port), synth._free_ports(synth.TABLES.udp_port)
    classes = list(synth.MIX_FALLBACK)
    rows = {c: synth._mix_class(c, n, 0x5EED0100 + k, ft, fu) for k, c in enumerate(classes)}
    for c in classes:
        a = rows[c]
        frames = [a[i].tobytes() for i in range(n)]
        if c == "tcpcut":
            frames = [f[:50] for f in frames]
        run(c, frames)
    mixed = []
    for i in range(n):
        c = classes[i % len(classes)]
        f = rows[c][i].tobytes()
        mixed.append(f[:50] if c == "tcpcut" else f)
    run("all five, interleaved", mixed)


if __name__ == "__main__":
    main()
