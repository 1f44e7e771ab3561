"""F2 diagnostic: gpd_decode_tpv3 over a registered 256 x 1 MiB ring of config-2 (64-B) or
IMIX frames, with and without capture info, the device walk on and off; host clock per call."""
import ctypes as C
import sys
import time

import numpy as np

sys.path.insert(0, ".")
from gopacket_amd import afpacket as A  # noqa: E402
from gopacket_amd import layers as L  # noqa: E402
from gopacket_amd import parser as P  # noqa: E402
from gopacket_amd import synth  # noqa: E402
from gopacket_amd._lib import GpdResult, check, lib  # noqa: E402
from gopacket_amd.results import BatchResult  # noqa: E402


def main():
    kind = sys.argv[1] if len(sys.argv) > 1 else "udp64"
    walks = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [1, 0]
    bs, nb = 1 << 20, 256
    b = synth.make_udp64(1 << 21) if kind == "udp64" else synth.make_imix(1 << 19, seed=3)
    per = bs // (((82 + int(b.caplen.max())) + 15) // 16 * 16) - 1
    m = min(b.n, per * nb)
    arr, used = synth.make_tpv3_ring([b.packet(i) for i in range(m)], bs, nb)
    ring = A.TPv3Ring(arr, bs, nb)
    for dw in walks:
        p = P.NewDecodingLayerParser(L.LayerTypeEthernet, P.Ethernet(), P.Dot1Q(), P.IPv4(), P.IPv6(),
                                     P.TCP(), P.UDP(), P.Payload())
        p.Tuning = {"device_walk": dw}
        check(lib.gpd_host_register(p.ctx().h, arr.ctypes.data, arr.nbytes), "reg")
        out = BatchResult(np.zeros(m, np.uint32), np.zeros(m, np.uint64), np.zeros(m, np.uint64),
                          np.zeros(m, np.uint64), np.zeros(m, np.uint32), None, np.zeros(m, np.uint32))
        r = GpdResult(out.status.ctypes.data, out.layers.ctypes.data, out.net_hash.ctypes.data,
                      out.tp_hash.ctypes.data, out.csum.ctypes.data, None, out.hdr_off.ctypes.data)
        ci = A.CaptureInfo.alloc(m)
        def regs(on):
            for arr_ in (out.status, out.layers, out.net_hash, out.tp_hash, out.csum, out.hdr_off,
                         ci.offset, ci.caplen, ci.length, ci.ts_ns, ci.ifindex, ci.vlan, ci.vlan_tci):
                if on:
                    check(lib.gpd_host_register(p.ctx().h, arr_.ctypes.data, arr_.nbytes), "reg")
                else:
                    lib.gpd_host_unregister(p.ctx().h, arr_.ctypes.data)
        for label, pk in (("ci", C.byref(ci.c())), ("no-ci", None), ("ci-registered", C.byref(ci.c()))):
            if label == "ci-registered":
                regs(True)
            n, nbk = C.c_uint64(), C.c_uint32()
            def call():
                check(lib.gpd_decode_tpv3(p.ctx().h, C.byref(ring.c), 0, nb, 0, m, C.byref(r), pk,
                                          C.byref(n), C.byref(nbk), 0), "tpv3")
            call()
            t = []
            for _ in range(10):
                t0 = time.perf_counter()
                call()
                t.append(time.perf_counter() - t0)
            ms = float(np.median(t)) * 1e3
            print(f"{kind} device_walk={dw} {label}: {n.value} pkts {nbk.value} blocks "
                  f"{ms:.3f} ms/ring {n.value / ms / 1e3:.1f} Mpps {nbk.value * bs / ms / 1e6:.1f} GB/s ring "
                  f"path={lib.gpd_decode_tpv3_last_path()}", flush=True)
            if label == "ci-registered":
                regs(False)
        lib.gpd_host_unregister(p.ctx().h, arr.ctypes.data)


if __name__ == "__main__":
    main()
