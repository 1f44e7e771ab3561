"""F2 AF_PACKET TPACKET_V3 ingest (include/gpd_afpacket.h): the native block walk vs the
restated read loop (oracle/tpv3_ref.py) on synthetic rings and on a ring the kernel filled
on the loopback device; the GPU decode of the walked packets vs the decode oracle."""
import os
import socket
import struct
import sys
import time

import numpy as np
import pytest

import golden_cases as G
import oracle_ref as O
from conftest import ROOT
from gopacket_amd import layers as L
from gopacket_amd import synth
from gopacket_amd.batch import PacketBatch

sys.path.insert(0, os.path.join(ROOT, "oracle"))
import tpv3_ref as T  # noqa: E402


def _packets(n=400, seed=9):
    b = synth.make_mixed(n, seed)
    pk = [b.packet(i) for i in range(b.n)]
    pk += [G.case_bytes(c) for c in G.load()["cases"] if len(G.case_bytes(c)) < 4000]
    return pk


def _check_walk(ring_arr, bs, nb, first, ci, nblk, max_blocks=None, add_vlan=False):
    ref, rblk = T.read_loop(ring_arr.tobytes(), bs, nb, first, max_blocks, add_vlan)
    assert nblk == rblk and len(ci.offset) == len(ref)
    for j, r in enumerate(ref):
        assert int(ci.offset[j]) == r["offset"] and int(ci.caplen[j]) == r["snaplen"]
        assert int(ci.length[j]) == r["length"] and int(ci.ts_ns[j]) == r["ts_ns"]
        assert int(ci.ifindex[j]) == r["ifindex"] and int(ci.vlan[j]) == r["vlan"]
    return ref


@pytest.mark.parametrize("first", [0, 5, 62])
@pytest.mark.parametrize("threads", [1, 8])
def test_walk_matches_read_loop(first, threads):
    from gopacket_amd import afpacket as A
    pk = _packets()
    rng = np.random.default_rng(first)
    vlan = [(int(rng.integers(0, 1 << 16)), bool(rng.integers(0, 2))) if rng.random() < 0.3 else (0, False)
            for _ in pk]
    arr, used = synth.make_tpv3_ring(pk, 1 << 14, 64, first_block=first, vlan=vlan, empty_blocks=(1, 4),
                                     wire_extra=3)
    ring = A.TPv3Ring(arr, 1 << 14, 64)
    ring.offset = first
    ci, nblk = ring.Walk(nthreads=threads)
    assert nblk == len(used)
    ref = _check_walk(arr, 1 << 14, 64, first, ci, nblk)
    assert [r["data"] for r in ref] == pk  # every packet, in order, bytes in place
    b = ring.batch(ci)
    assert all(b.packet(j) == pk[j] for j in range(len(pk)))


def test_walk_stops_and_releases():
    from gopacket_amd import afpacket as A
    pk = _packets(300)
    arr, used = synth.make_tpv3_ring(pk, 1 << 13, 32, first_block=3, kernel_blocks=(4,))
    ring = A.TPv3Ring(arr, 1 << 13, 32)
    ring.offset = 3
    ci, nblk = ring.Walk()
    assert nblk == 4  # walk positions 0..3; position 4 is still the kernel's
    _check_walk(arr, 1 << 13, 32, 3, ci, nblk)
    ci2, nblk2 = ring.Walk(max_blocks=2)
    assert nblk2 == 2 and len(ci2.offset) < len(ci.offset)
    # max_n below a block's packet count: whole blocks only
    first_blk = int(np.frombuffer(arr[3 * 8192 + 12:3 * 8192 + 16].tobytes(), np.uint32)[0])
    ci3, nblk3 = ring.Walk(max_n=first_blk + 1)
    assert nblk3 == 1 and len(ci3.offset) == first_blk
    ring.Release(nblk)
    assert ring.offset == 7
    for k in range(3, 7):
        assert arr[k * 8192 + 8] == 0  # block_status handed back (TP_STATUS_KERNEL)
    ci4, nblk4 = ring.Walk()
    assert nblk4 == 0 and len(ci4.offset) == 0  # position 4 (block 7) is the kernel's


def test_walk_reference_quirks():
    """Behaviour the restated loop reproduces: a block whose first packet reports tp_len 0
    skips it (the retry goes through next(), afpacket.go:313-316); an empty block whose stale
    first tp_len is nonzero yields that one stale packet."""
    from gopacket_amd import afpacket as A
    pk = _packets(60)
    arr, used = synth.make_tpv3_ring(pk, 1 << 13, 16)
    bs = 1 << 13
    first = int(np.frombuffer(arr[16:20].tobytes(), np.uint32)[0])
    arr[first + 16:first + 20] = 0  # block 0, packet 0: tp_len = 0
    nb1 = used[1] * bs
    arr[nb1 + 12:nb1 + 16] = 0      # block 1: num_pkts = 0 (its stale packets stay behind)
    ring = A.TPv3Ring(arr, bs, 16)
    ci, nblk = ring.Walk()
    ref = _check_walk(arr, bs, 16, 0, ci, nblk)
    n0 = int(np.frombuffer(arr[12:16].tobytes(), np.uint32)[0])
    assert ref[0]["data"] == pk[1]  # the zero-length first packet was skipped
    assert ref[n0 - 1]["data"] == pk[n0]  # block 1 yielded exactly its stale first packet
    assert ref[n0]["offset"] // bs == used[2]


def test_walk_rejects_corrupt_block():
    from gopacket_amd import _lib, afpacket as A
    arr, used = synth.make_tpv3_ring(_packets(40), 1 << 13, 8)
    arr[16:20] = np.frombuffer(np.uint32(1 << 13).tobytes(), np.uint8)  # first packet past the block
    ring = A.TPv3Ring(arr, 1 << 13, 8)
    with pytest.raises(_lib.GpdError, match="outside the block"):
        ring.Walk()


def _live_ring(bs=1 << 16, nb=16):
    """A real TPACKET_V3 ring on the loopback device, or None where sockets are refused."""
    import mmap
    SOL_PACKET, PACKET_VERSION, PACKET_RX_RING, TPACKET_V3 = 263, 10, 5, 2
    try:
        s = socket.socket(socket.AF_PACKET, socket.SOCK_RAW, socket.htons(3))
    except (PermissionError, OSError):
        return None
    try:
        s.setsockopt(SOL_PACKET, PACKET_VERSION, TPACKET_V3)
        # struct tpacket_req3: block_size, block_nr, frame_size, frame_nr, retire_blk_tov (ms),
        # sizeof_priv, feature_req_word (afpacket.go:192-199 setUpRing)
        s.setsockopt(SOL_PACKET, PACKET_RX_RING, struct.pack("7I", bs, nb, 2048, bs // 2048 * nb, 5, 0, 0))
        m = mmap.mmap(s.fileno(), bs * nb, mmap.MAP_SHARED, mmap.PROT_READ | mmap.PROT_WRITE)
        s.bind(("lo", 0))
    except (PermissionError, OSError):
        s.close()
        return None
    return s, m


def test_walk_live_loopback_ring():
    """The kernel fills the ring (loopback UDP); the native walk and the restated read loop
    agree on a snapshot of it and every datagram sent shows up."""
    from gopacket_amd import afpacket as A
    live = _live_ring()
    if live is None:
        pytest.skip("AF_PACKET sockets are not permitted on this host")
    s, m = live
    try:
        tx = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
        rx = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
        rx.bind(("127.0.0.1", 0))
        port = rx.getsockname()[1]
        sent = [b"gpd-afpacket-%05d-" % k + bytes(k % 200) for k in range(300)]
        for d in sent:
            tx.sendto(d, ("127.0.0.1", port))
        time.sleep(0.1)  # > retire_blk_tov: the kernel hands the partly filled block over
        snap = np.frombuffer(bytes(m), np.uint8).copy()
        ring = A.TPv3Ring(snap, 1 << 16, 16)
        ci, nblk = ring.Walk()
        assert nblk >= 1 and len(ci.offset) >= len(sent)
        ref = _check_walk(snap, 1 << 16, 16, 0, ci, nblk)
        frames = [r["data"] for r in ref]
        for d in sent:  # Ethernet(14) + IPv4(20) + UDP(8) + payload on lo
            assert any(f[42:] == d for f in frames)
        tx.close()
        rx.close()
    finally:
        m.close()
        s.close()


@pytest.mark.gpu
@pytest.mark.parametrize("add_vlan", [False, True])
def test_decode_tpv3_matches_oracle(add_vlan):
    from gopacket_amd import afpacket as A
    from gopacket_amd import parser as P
    pk = _packets(3000)
    rng = np.random.default_rng(4)
    vlan = [(int(rng.integers(1, 1 << 16)), True) if rng.random() < 0.25 else (0, False) for _ in pk]
    arr, used = synth.make_tpv3_ring(pk, 1 << 16, 64, first_block=60, vlan=vlan)
    ring = A.TPv3Ring(arr, 1 << 16, 64)
    ring.offset = 60
    parser = P.NewDecodingLayerParser(L.LayerTypeEthernet, *[P.DECODER_BY_NAME[k]() for k in P.DECODER_BY_NAME])
    res, ci, nblk = parser.DecodeTPv3(ring, add_vlan_header=add_vlan)
    ref_pk, rblk = T.read_loop(arr.tobytes(), 1 << 16, 64, 60, None, add_vlan)
    assert nblk == rblk == len(used) and len(res) == len(ref_pk)
    ref = O.decode(PacketBatch.from_packets([r["data"] for r in ref_pk]), L.LayerTypeEthernet,
                   parser.decoders, 0, ext=False, nthreads=8)
    for f in ("status", "layers", "net_hash", "tp_hash", "csum", "hdr_off"):
        assert (getattr(res, f) == getattr(ref, f)).all(), f
    if add_vlan:  # tagged frames decode with the inserted Dot1Q layer
        tagged = [j for j, r in enumerate(ref_pk) if len(r["data"]) == r["snaplen"] + 4]
        assert tagged and all(res.decoded(j)[:2] == [L.LayerTypeEthernet, L.LayerTypeDot1Q] for j in tagged[:50])


@pytest.mark.gpu
@pytest.mark.parametrize("device_walk,register", [(1, False), (0, False), (1, True)])
def test_decode_tpv3_detail_matches_oracle(device_walk, register):
    """gpd_detail through gpd_decode_tpv3 (afpacket.go:300-333's ZeroCopyReadPacketData loop
    feeding DecodeLayers): one packet per reference error site and > 12-layer stacks among mixed
    traffic in a ring; the detail records and the error texts rebuilt from status + detail equal
    the oracle's — device and host block walks, staged and registered (direct) result arrays."""
    import error_sites as ES
    from gopacket_amd import _lib, afpacket as A
    from gopacket_amd import parser as P
    from test_parity_gpu import assert_detail, detail_rows
    pk = _packets(1500, seed=11)
    for k, p in enumerate(ES.packets()):
        pk.insert(23 * k + 7, p)
    arr, used = synth.make_tpv3_ring(pk, 1 << 16, 64)
    ring = A.TPv3Ring(arr, 1 << 16, 64)
    parser = P.NewDecodingLayerParser(L.LayerTypeEthernet, *[P.DECODER_BY_NAME[k]() for k in P.DECODER_BY_NAME])
    parser.Tuning = {"device_walk": device_walk}
    out = ci = None
    arrays = []
    if register:  # every result and capture-info array registered: the D2H lands in them directly
        from gopacket_amd.results import DETAIL_DTYPE, BatchResult
        m = 1 << 16
        out = BatchResult(np.zeros(m, np.uint32), np.zeros(m, np.uint64), np.zeros(m, np.uint64),
                          np.zeros(m, np.uint64), np.zeros(m, np.uint32), None, np.zeros(m, np.uint32),
                          np.zeros(m, DETAIL_DTYPE))
        ci = A.CaptureInfo.alloc(m)
        arrays = [out.status, out.layers, out.net_hash, out.tp_hash, out.csum, out.hdr_off, out.detail,
                  ci.offset, ci.caplen, ci.length, ci.ts_ns, ci.ifindex, ci.vlan, ci.vlan_tci]
        for a in arrays:
            _lib.check(_lib.lib.gpd_host_register(parser.ctx().h, a.ctypes.data, a.nbytes), "register")
    try:
        res, ci, nblk = parser.DecodeTPv3(ring, max_n=1 << 16, out=out, ci=ci, detail=True)
    finally:
        for a in arrays:
            _lib.lib.gpd_host_unregister(parser.ctx().h, a.ctypes.data)
    ref_pk, rblk = T.read_loop(arr.tobytes(), 1 << 16, 64, 0, None, False)
    assert nblk == rblk and len(res) == len(ref_pk) == len(pk)
    ref = O.decode(PacketBatch.from_packets([r["data"] for r in ref_pk]), L.LayerTypeEthernet,
                   parser.decoders, 0, ext=True, nthreads=8)
    for f in ("status", "layers", "net_hash", "tp_hash", "csum", "hdr_off"):
        assert (getattr(res, f) == getattr(ref, f)).all(), f
    rows = detail_rows(ref.status)
    assert len(rows) >= len(ES.packets())
    assert_detail(res, ref)


def _decode_both(arr, bs, nb, first, register=False, **kw):
    """DecodeTPv3 with the walk on the device and on the host: equal results, capture info,
    block counts and errors.  Returns (path of the device-walk call, packets, blocks)."""
    from gopacket_amd import _lib, afpacket as A
    from gopacket_amd import parser as P
    got = []
    for dw in (1, 0):
        parser = P.NewDecodingLayerParser(L.LayerTypeEthernet, *[P.DECODER_BY_NAME[k]() for k in P.DECODER_BY_NAME])
        parser.Tuning = {"device_walk": dw}
        ring = A.TPv3Ring(arr, bs, nb)
        ring.offset = first
        if register:
            _lib.check(_lib.lib.gpd_host_register(parser.ctx().h, arr.ctypes.data, arr.nbytes), "register")
        try:
            res, ci, nblk = parser.DecodeTPv3(ring, **kw)
            got.append((res, ci, nblk, None, _lib.lib.gpd_decode_tpv3_last_path()))
        except _lib.GpdError as e:
            got.append((None, None, None, str(e), None))
        finally:
            if register:
                _lib.lib.gpd_host_unregister(parser.ctx().h, arr.ctypes.data)
    (r1, c1, b1, e1, path), (r0, c0, b0, e0, _) = got
    assert e1 == e0
    if e1 is not None:
        return None, 0, 0
    assert b1 == b0 and len(r1) == len(r0)
    for f in ("status", "layers", "net_hash", "tp_hash", "csum", "hdr_off"):
        assert np.array_equal(getattr(r1, f), getattr(r0, f)), f
    for f in ("offset", "caplen", "length", "ts_ns", "ifindex", "vlan", "vlan_tci"):
        assert np.array_equal(getattr(c1, f), getattr(c0, f)), f
    return path, len(r1), b1


@pytest.mark.gpu
@pytest.mark.parametrize("first", [0, 61])
def test_device_walk_equals_host_walk(first):
    """The block walk in HBM (gpd_tpv3walk.hip) returns what the host walk does: wrap-around,
    empty and kernel-owned blocks, both tp_next_offset forms, VLAN flags and tags, bounds."""
    pk = _packets(3000)
    rng = np.random.default_rng(first)
    vlan = [(int(rng.integers(1, 1 << 16)), bool(rng.integers(0, 2))) if rng.random() < 0.3 else (0, False)
            for _ in pk]
    arr, used = synth.make_tpv3_ring(pk, 1 << 16, 64, first_block=first, vlan=vlan, empty_blocks=(2, 5),
                                     kernel_blocks=(9,), wire_extra=3)
    path, n, nblk = _decode_both(arr, 1 << 16, 64, first)
    assert path == 1 and 0 < n < len(pk) and nblk == 9  # walk position 9 is still the kernel's
    for kw in ({"max_blocks": 7}, {"max_n": 1000}, {"add_vlan_header": True}):
        path, n, nblk = _decode_both(arr, 1 << 16, 64, first, **kw)
        # frames carrying a tag with OptAddVLANHeader: the host path inserts it
        assert path == (0 if "add_vlan_header" in kw else 1)
    arr2, _ = synth.make_tpv3_ring(pk, 1 << 16, 64, first_block=first)  # no tags at all
    assert _decode_both(arr2, 1 << 16, 64, first, add_vlan_header=True)[0] == 1


@pytest.mark.gpu
def test_device_walk_quirks_and_corrupt_blocks():
    pk = _packets(600)
    bs = 1 << 13
    arr, used = synth.make_tpv3_ring(pk, bs, 64)
    first = int(np.frombuffer(arr[16:20].tobytes(), np.uint32)[0])
    q = arr.copy()
    q[first + 16:first + 20] = 0                  # block 0, packet 0: tp_len = 0 (skipped)
    q[used[1] * bs + 12:used[1] * bs + 16] = 0    # block 1: num_pkts = 0 (one stale packet)
    path, n, _ = _decode_both(q, bs, 64, 0)
    assert path == 1 and n == len(pk) - 1 - (int(np.frombuffer(arr[used[1] * bs + 12:used[1] * bs + 16].tobytes(),
                                                                 np.uint32)[0]) - 1)
    # a tp_next_offset that leaves the block, one that is not 4-byte aligned, a frame past
    # the block's end: the device walk declines and the host walk reports (or returns) the same
    b3 = used[3] * bs + first
    for off, val in ((b3, bs), (b3, 100 * 16 + 2), (b3 + 12, bs)):
        c = arr.copy()
        c[off:off + 4] = np.frombuffer(np.uint32(val).tobytes(), np.uint8)
        _decode_both(c, bs, 64, 0)


@pytest.mark.gpu
@pytest.mark.parametrize("register", [False, True])
def test_device_walk_several_groups(register):
    """A 256 x 1 MiB ring of IMIX frames (several 64 MiB groups in flight on both slots),
    the ring registered or not."""
    b = synth.make_imix(400000, seed=0x77)
    pk = [b.packet(i) for i in range(b.n)]
    arr, used = synth.make_tpv3_ring(pk, 1 << 20, 256)
    path, n, nblk = _decode_both(arr, 1 << 20, 256, 0, register=register, max_n=1 << 19)
    assert path == 1 and n == len(pk) and nblk == len(used) and nblk * (1 << 20) > 2 * (64 << 20)
