"""The pcap record walk on the device (gpd_pcapwalk.hip, gpd_tuning.device_walk): every
gpd_decode_pcap(_at) result — records, their decoded words, the record count, where the walk
stops and why, the error text — equals the host walk's (gpd_pcap.cpp, itself pinned to
pcapgo's ReadPacketData loop by tests/test_pcap*.py), over captures that span several 64 MiB
chunks, records longer than a walking lane's 2 KiB segment, empty records, rejected records,
a capture cut inside a record, big-endian nanosecond headers, payloads that look like pcap
records (speculation the true walk misses), and bounded calls continued record by record."""
import ctypes as C
import struct

import numpy as np
import pytest

from gopacket_amd import layers as L
from gopacket_amd import pcap as NP
from gopacket_amd import synth
from gopacket_amd.batch import PAD, PacketBatch
from gopacket_amd.results import BatchResult

pytestmark = pytest.mark.gpu
FIELDS = ("status", "layers", "net_hash", "tp_hash", "csum", "hdr_off")


def _parser(device_walk):
    from gopacket_amd import parser as P
    p = P.NewDecodingLayerParser(L.LayerTypeEthernet, P.Ethernet(), P.Dot1Q(), P.IPv4(), P.IPv6(),
                                 P.IPv6ExtensionSkipper(), P.TCP(), P.UDP(), P.VXLAN(), P.Payload(),
                                 P.Fragment())
    p.Tuning = {"device_walk": device_walk}
    return p


def _phases():
    from gopacket_amd._lib import lib
    ph = np.zeros(6, np.float64)
    lib.gpd_decode_pcap_last_times(ph.ctypes.data)
    return ph


def _capture(n, seed, jumbo=True):
    """IMIX frames with, when asked, 9000-byte frames and empty records among them."""
    b = synth.make_imix(n, seed=seed)
    pk = [b.data[o:o + c].tobytes() for o, c in zip(b.offset.tolist(), b.caplen.tolist())]
    if jumbo:
        rng = np.random.default_rng(seed)
        for i in rng.choice(n, size=n // 200, replace=False):
            pk[i] = pk[i] + bytes(rng.integers(0, 256, size=9000 - len(pk[i]), dtype=np.uint8))
        for i in rng.choice(n, size=n // 500, replace=False):
            pk[i] = b""
    return NP.synth_capture(PacketBatch.from_packets(pk))


def _both(cap, data_len=None, register=False):
    """DecodePcap of the whole capture with the device walk and with the host walk."""
    out = []
    for dw in (1, 0):
        p = _parser(dw)
        if register:
            from gopacket_amd._lib import check, lib
            check(lib.gpd_host_register(p.ctx().h, cap.ctypes.data, cap.nbytes), "register")
        res, n, err = p.DecodePcap(cap, data_len=data_len, nthreads=8)
        ph = _phases()
        if register:
            lib.gpd_host_unregister(p.ctx().h, cap.ctypes.data)
        out.append((res, n, err, ph))
    (r1, n1, e1, ph1), (r0, n0, e0, _) = out
    assert (n1, e1) == (n0, e0)
    for f in FIELDS:
        assert np.array_equal(getattr(r1, f)[:n1], getattr(r0, f)[:n0]), f
    return n1, e1, ph1


def test_device_walk_equals_host_walk_across_chunks():
    cap = _capture(1 << 18, 0x51)  # ~100 MB: two chunks, jumbo and empty records
    assert cap.nbytes > 80 << 20
    n, err, ph = _both(cap)
    assert err is None and n == 1 << 18
    assert ph[1] == 0.0  # the whole capture went through the device walk (no host walk ran)
    n, err, ph = _both(cap, register=True)
    assert err is None and ph[1] == 0.0


def test_device_walk_stops_where_the_reader_does():
    cap = _capture(1 << 17, 0x52, jumbo=False)
    dl = cap.shape[0] - PAD
    info = NP.header(cap, dl)
    pos, _, _ = NP.locate(cap, [100000], data_len=dl, info=info)
    p0 = int(pos[0])
    # a record the reader rejects (caplen > snaplen) in the second half: the host walk takes
    # over from the chunk that holds it, with the reference's error text
    bad = cap.copy()
    bad[p0 + 8:p0 + 12] = np.frombuffer(struct.pack("<I", 300000), np.uint8)
    n, err, ph = _both(bad)
    assert n == 100000 and err.startswith("capture length exceeds snap length")
    # caplen > original length
    bad2 = cap.copy()
    bad2[p0 + 12:p0 + 16] = np.frombuffer(struct.pack("<I", 1), np.uint8)
    n, err, _ = _both(bad2)
    assert n == 100000 and err.startswith("capture length exceeds original packet length")
    # the capture cut inside a record's data, then inside a record header
    for cut in (p0 + 16 + 5, p0 + 7):
        n, err, _ = _both(cap, data_len=cut)
        assert n == 100000 and err in ("unexpected EOF", "EOF")


def test_device_walk_bounded_calls_continue_exactly():
    cap = _capture(1 << 17, 0x53)
    dl = cap.shape[0] - PAD
    info = NP.header(cap, dl)
    steps = [1, 63, 1000, 77777, 5, 40000, 1 << 20]
    seqs = []
    for dw in (1, 0):
        p = _parser(dw)
        out = BatchResult(*(np.zeros(1 << 20, t) for t in (np.uint32, np.uint64, np.uint64, np.uint64, np.uint32)),
                          None, np.zeros(1 << 20, np.uint32))
        at, seq = 24, []
        for m in steps:
            k, nxt, stop, err = p.DecodePcapAt(cap, info, at, m, out, nthreads=8, data_len=dl)
            seq.append((k, nxt, stop, err, tuple(int(getattr(out, f)[:k].astype(np.uint64).sum() % (1 << 61))
                                                 for f in FIELDS)))
            at = nxt
            if stop != NP.STOP_LIMIT:
                break
        seqs.append(seq)
    assert seqs[0] == seqs[1]
    assert seqs[0][-1][2] == NP.STOP_EOF


def test_device_walk_big_endian_nanosecond_headers():
    cap = _capture(1 << 16, 0x54)
    dl = cap.shape[0] - PAD
    pc = NP.index(cap, data_len=dl)
    be = cap.copy()
    be[:4] = np.frombuffer(struct.pack("<I", 0x4D3CB2A1), np.uint8)  # nanosecond, big-endian
    be[4:24] = np.frombuffer(struct.pack(">HHiIII", 2, 4, 0, 0, 262144, 1), np.uint8)
    hdr = pc.batch.offset.astype(np.int64) - 16
    for k in range(4):  # every header word byte-swapped in place
        idx = hdr[:, None] + 4 * k + np.arange(4)[None, :]
        be[idx] = be[idx][:, ::-1]
    n, err, ph = _both(be)
    assert err is None and n == pc.batch.n and ph[1] == 0.0


def test_device_walk_speculation_misses_fall_back():
    """Frames whose payload is itself a pcap stream of small records: a lane that starts inside
    such a payload finds a chain of plausible headers that the true walk never visits."""
    inner = NP.synth_capture(synth.make_udp64(40))[24:24 + 40 * 80].tobytes()
    eth = bytes(12) + b"\x08\x00" + bytes([0x45]) + bytes(19)
    pk = []
    for i in range(60000):
        pk.append(eth + inner if i % 3 == 0 else eth + bytes(range(40)))
    cap = NP.synth_capture(PacketBatch.from_packets(pk))
    n, err, _ = _both(cap)
    assert err is None and n == 60000


def test_device_walk_corrects_refuted_speculation_on_device():
    """Config 5's 64-B records, cut so that a 2-KiB walking segment starts 40 bytes into record
    315870771: its scan finds a false chain 8 bytes before the next header (random payload
    bytes that read as a sub-second fraction, then a view 3 bytes into every 205th record, which
    chains 16,400-byte "records" forever).  The stitch re-walks that segment from the true walk's
    position on the device (gpd_decode_pcap_last_walk_counts [6]) instead of handing the chunk to
    the host walk ([1]), and every result equals the host walk's."""
    from gopacket_amd._lib import lib
    lo, n = 315870771 - 25, 100000
    cap = np.zeros(24 + 80 * n + PAD, np.uint8)
    cap[:24] = np.frombuffer(struct.pack("<IHHiIII", 0xA1B2C3D4, 2, 4, 0, 0, 262144, 1), np.uint8)
    synth.udp64_native(cap[24:24 + 80 * n], lo, lo + n, 0x5EED0002, records=True, nthreads=8)
    p = _parser(1)
    _, k, err = p.DecodePcap(cap, nthreads=8)
    wc = np.zeros(7, np.uint32)
    lib.gpd_decode_pcap_last_walk_counts(wc.ctypes.data)
    assert err is None and k == n
    assert wc[1] == 0, wc      # no chunk went to the host walk
    assert wc[6] >= 1, wc      # ... because the stitch corrected the segment itself
    n2, err2, _ = _both(cap)
    assert err2 is None and n2 == n
