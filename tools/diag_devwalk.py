"""Which packets' results differ between the pcap device walk, the host walk and the oracle
(tests/test_pcap_devwalk_gpu.py's capture), per header_once mode.  GPU diagnostic."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import oracle_ref as O  # noqa: E402
from gopacket_amd import layers as L  # noqa: E402
from gopacket_amd import pcap as NP  # noqa: E402
from gopacket_amd import synth  # noqa: E402
from gopacket_amd.batch import PacketBatch  # noqa: E402

FIELDS = ("status", "layers", "net_hash", "tp_hash", "csum", "hdr_off")


def parser(dw, ho):
    from gopacket_amd import parser as P
    p = P.NewDecodingLayerParser(L.LayerTypeEthernet, P.Ethernet(), P.Dot1Q(), P.IPv4(), P.IPv6(),
                                 P.IPv6ExtensionSkipper(), P.TCP(), P.UDP(), P.VXLAN(), P.Payload(),
                                 P.Fragment())
    p.Tuning = {"device_walk": dw, "header_once": ho}
    return p


def capture(n, seed):
    b = synth.make_imix(n, seed=seed)
    pk = [b.data[o:o + c].tobytes() for o, c in zip(b.offset.tolist(), b.caplen.tolist())]
    rng = np.random.default_rng(seed)
    for i in rng.choice(n, size=n // 200, replace=False):
        pk[i] = pk[i] + bytes(rng.integers(0, 256, size=9000 - len(pk[i]), dtype=np.uint8))
    for i in rng.choice(n, size=n // 500, replace=False):
        pk[i] = b""
    return NP.synth_capture(PacketBatch.from_packets(pk))


def report(tag, got, ref, batch):
    bad = np.zeros(batch.n, bool)
    for f in FIELDS:
        bad |= getattr(got, f)[:batch.n] != getattr(ref, f)[:batch.n]
    idx = np.nonzero(bad)[0]
    print(f"{tag}: {len(idx)} packets differ", flush=True)
    for i in idx[:12]:
        o, c = int(batch.offset[i]), int(batch.caplen[i])
        diffs = [f for f in FIELDS if getattr(got, f)[i] != getattr(ref, f)[i]]
        print(f"  i={i} off={o} off%16={o % 16} caplen={c} status={int(ref.status[i]):#x} "
              f"diff={diffs} csum got={int(got.csum[i]):#x} ref={int(ref.csum[i]):#x} "
              f"prev_caplen={int(batch.caplen[i - 1]) if i else -1} tile={i // 64} lane={i % 64}",
              flush=True)
    if len(idx):
        t = np.unique(idx // 64)
        print(f"  tiles with differences: {len(t)}; caplens in the first: "
              f"{batch.caplen[t[0] * 64:t[0] * 64 + 64].tolist()}", flush=True)
    return len(idx)


def main():
    cap = capture(1 << 18, 0x51)
    pc = NP.index(cap)
    b = pc.batch
    p0 = parser(0, -1)
    ref = O.decode(b, L.LayerTypeEthernet, p0.decoders, p0.options, ext=False, nthreads=8)
    print(f"capture {cap.nbytes} B, {b.n} records", flush=True)
    for ho in (-1, 2, 1, 0):
        for dw in (1, 0):
            p = parser(dw, ho)
            res, n, err = p.DecodePcap(cap, nthreads=8)
            assert n == b.n and err is None, (n, err)
            report(f"pcap dw={dw} ho={ho}", res, ref, b)
        p = parser(0, ho)
        res = p.DecodeBatch(b, ext=False)
        report(f"DecodeBatch ho={ho}", res, ref, b)


if __name__ == "__main__":
    main()
