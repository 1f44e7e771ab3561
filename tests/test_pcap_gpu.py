"""pcap ingest through the GPU: a capture's raw bytes decoded in place —
gpd_decode_pcap (index + H2D of the capture bytes + decode + D2H) and gpd_decode on an
HBM-resident capture — bit-exact against the CPU oracle decoding the same records, where the
records are those of oracle/pcap_ref.py's sequential ReadPacketData loop (pcapgo/read.go)."""
import os
import struct
import sys

import numpy as np
import pytest

import golden_cases as G
import oracle_ref as O
from gopacket_amd import layers as L
from gopacket_amd import pcap as NP
from gopacket_amd import synth
from gopacket_amd.batch import PacketBatch
from test_parity_gpu import assert_same

sys.path.insert(0, os.path.join(os.path.dirname(G.HERE), "oracle"))
import pcap_ref as R  # noqa: E402

pytestmark = pytest.mark.gpu
ALL = 0x3FF


def _parser():
    from gopacket_amd import parser as P
    return P.NewDecodingLayerParser(L.LayerTypeEthernet, P.Ethernet(), P.Dot1Q(), P.IPv4(), P.IPv6(),
                                    P.IPv6ExtensionSkipper(), P.TCP(), P.UDP(), P.VXLAN(), P.Payload(),
                                    P.Fragment())


def _oracle_batch(raw: bytes):
    recs, stop, nxt, err = R.walk(raw)
    cap = NP.capture_array(raw)
    off = np.array([r[0] for r in recs], np.uint32)
    ln = np.array([r[1] for r in recs], np.uint32)
    return PacketBatch(cap, len(raw), off, ln), err


def _check_decode_pcap(raw: bytes, nthreads=8, register=False):
    p = _parser()
    cap = NP.capture_array(raw)
    if register:
        from gopacket_amd._lib import check, lib
        check(lib.gpd_host_register(p.ctx().h, cap.ctypes.data, cap.nbytes), "register")
    try:
        res, n, err = p.DecodePcap(cap, nthreads=nthreads)
    finally:
        if register:
            lib.gpd_host_unregister(p.ctx().h, cap.ctypes.data)
    b, rerr = _oracle_batch(raw)
    assert n == b.n and err == rerr
    ref = O.decode(b, L.LayerTypeEthernet, ALL, 0, ext=False, nthreads=8)
    assert_same(res, ref, b, ext=False)
    return b


@pytest.mark.parametrize("maker,n", [(synth.make_udp64, 1 << 16), (synth.make_imix, 1 << 15),
                                     (synth.make_vxlan, 1 << 15), (synth.make_mixed, 1 << 14)])
def test_decode_pcap_matches_oracle(maker, n):
    raw = NP.synth_capture(maker(n, 9))[:-NP.PAD].tobytes()
    _check_decode_pcap(raw)


def test_decode_pcap_registered_and_chunked():
    # > one 256-MB staging slot of records: several chunks in flight, read in place
    b = synth.make_imix(1 << 20, 4)
    raw = NP.synth_capture(b)[:-NP.PAD].tobytes()
    assert len(raw) > 300 << 20
    p = _parser()
    cap = NP.capture_array(raw)
    from gopacket_amd._lib import check, lib
    check(lib.gpd_host_register(p.ctx().h, cap.ctypes.data, cap.nbytes), "register")
    try:
        res, n, err = p.DecodePcap(cap)
    finally:
        lib.gpd_host_unregister(p.ctx().h, cap.ctypes.data)
    assert n == b.n and err is None
    ref = O.decode(b, L.LayerTypeEthernet, ALL, 0, ext=False, nthreads=8)
    assert_same(res, ref, b, ext=False)


@pytest.mark.parametrize("name", ["test_ethernet.pcap", "test_dns.pcap", "test_loopback.pcap"])
def test_reference_pcaps(name):
    _check_decode_pcap(open(os.path.join(G.HERE, "golden", name), "rb").read())


def test_decode_pcap_stops_where_the_reader_does():
    raw = bytearray(NP.synth_capture(synth.make_imix(5000, 2))[:-NP.PAD].tobytes())
    recs, _, _, _ = R.walk(bytes(raw))
    pos = recs[3210][0] - 16
    struct.pack_into("<I", raw, pos + 12, recs[3210][1] - 1)  # caplen > original length
    b = _check_decode_pcap(bytes(raw))
    assert b.n == 3210


def test_device_resident_capture():
    """The capture bytes in HBM as the batch buffer (unaligned records) through gpd_decode."""
    raw = NP.synth_capture(synth.make_mixed(1 << 14, 3))[:-NP.PAD].tobytes()
    pc = NP.parse_pcap(raw)
    dev = _parser().DecodeBatch(pc.batch, ext=True)
    ref = O.decode(pc.batch, L.LayerTypeEthernet, ALL, 0, ext=True, nthreads=8)
    assert_same(dev, ref, pc.batch, ext=True)
