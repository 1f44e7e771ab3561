"""pcap ingest, CPU: the native record walk (include/gpd_pcap.h) against the
sequential restatement of pcapgo's reader in oracle/pcap_ref.py, pinned by the capture bytes
of pcapgo/read_test.go (tests/golden/pcapgo_vectors.json) and the reference's pcap files."""
import gzip
import json
import os
import struct

import numpy as np
import pytest

import golden_cases as G
from gopacket_amd import pcap as NP
from gopacket_amd import synth
from gopacket_amd.batch import PacketBatch

import sys
sys.path.insert(0, os.path.join(os.path.dirname(G.HERE), "oracle"))
import pcap_ref as R  # noqa: E402  (test infrastructure)

VEC = json.load(open(os.path.join(G.HERE, "golden", "pcapgo_vectors.json")))["cases"]


def _native(buf, nthreads=0, max_n=None):
    return NP.index(NP.capture_array(buf), max_n=max_n, nthreads=nthreads)


def _agree(buf, nthreads=0):
    """native walk == the oracle's sequential ReadPacketData loop, record by record."""
    raw = gzip.decompress(buf) if buf[:2] == b"\x1f\x8b" else buf
    recs, stop, nxt, err = R.walk(raw)
    p = _native(buf, nthreads)
    assert p.batch.n == len(recs)
    if recs:
        o, c, w, t = (np.array(x, dtype=np.uint64) for x in zip(*recs))
        assert np.array_equal(p.batch.offset, o.astype(np.uint32))
        assert np.array_equal(p.batch.caplen, c.astype(np.uint32))
        assert np.array_equal(p.length, w.astype(np.uint32))
        assert np.array_equal(p.ts_ns, t)
    assert (p.stop, p.next_pos, p.err) == (stop, nxt, err)
    return p


@pytest.mark.parametrize("c", VEC, ids=[c["name"] for c in VEC])
def test_pcapgo_read_test_vectors(c):
    buf = bytes.fromhex(c["hex"])
    e = c["expect"]
    if not e["header_ok"]:
        with pytest.raises(Exception):
            _native(buf)
        with pytest.raises(Exception):
            R.header(gzip.decompress(buf) if e.get("gzip") and len(buf) > 10 else buf)
        return
    p = _agree(buf)
    if "snaplen" in e:
        assert p.snaplen == e["snaplen"] and p.linktype == e["linktype"]
        assert p.batch.n == 0 and p.err is None and p.stop == NP.STOP_EOF
    for i, q in enumerate(e.get("packets", [])):
        assert int(p.ts_ns[i]) == q["ts_ns"]
        assert int(p.batch.caplen[i]) == q["caplen"] and int(p.length[i]) == q["length"]
        assert p.batch.packet(i).hex() == q["data"]
    for i, d in enumerate(e.get("packets_data", [])):
        assert p.batch.packet(i).hex() == d


@pytest.mark.parametrize("name", ["test_ethernet.pcap", "test_dns.pcap", "test_loopback.pcap"])
def test_reference_pcap_files(name):
    buf = open(os.path.join(G.HERE, "golden", name), "rb").read()
    p = _agree(buf, nthreads=4)
    assert p.err is None and p.stop == NP.STOP_EOF
    if name == "test_ethernet.pcap":  # pcap/pcap_test.go:64-71
        assert list(p.batch.caplen) == [74, 74, 66, 138, 66, 89, 66, 421, 66, 66]


def _big_capture(n=1 << 15, seed=3):
    b = synth.make_imix(n, seed)
    return NP.synth_capture(b)[:-NP.PAD].tobytes(), b


def test_parallel_walk_equals_sequential():
    buf, b = _big_capture()
    assert len(buf) > 8 << 20  # several 4-MiB segments: the speculative path runs
    for t in (1, 2, 3, 8):
        p = _agree(buf, nthreads=t)
        assert p.batch.n == b.n
        th, met, rew = NP.last_walk_stats()
        assert th == min(t, len(buf) // (4 << 20)) and met + rew == th - 1
    # the capture bytes are the batch: every packet is where the walk says
    p = _native(buf, 8)
    for i in range(0, b.n, 997):
        assert p.batch.packet(i) == b.packet(i)


def test_speculation_decoys():
    """Payloads made of pcap record headers (nested captures) lure the speculative walks onto
    false chains; stitching must still reproduce the sequential walk."""
    rng = np.random.default_rng(7)
    inner = []
    for _ in range(64):
        L = int(rng.integers(4, 40))
        inner.append(struct.pack("<IIII", 1, 2, L, L) + bytes(rng.integers(0, 256, L, dtype=np.uint8)))
    decoy = b"".join(inner)
    pkts = [decoy[k % 97:][:1200 + (k % 300)] for k in range(12000)]
    b = PacketBatch.from_packets(pkts, align=1)
    buf = NP.synth_capture(b)[:-NP.PAD].tobytes()
    assert len(buf) > 8 << 20
    for t in (2, 5, 8):
        p = _agree(buf, nthreads=t)
        assert p.batch.n == len(pkts)
        th, met, rew = NP.last_walk_stats()
        assert th > 1 and met + rew == th - 1


@pytest.mark.parametrize("kind", ["short_hdr", "short_data", "eof_data", "snaplen", "origlen"])
@pytest.mark.parametrize("where", ["small", "parallel"])
def test_walk_errors(kind, where):
    n = 40 if where == "small" else 1 << 15
    buf, b = _big_capture(n, seed=11)
    buf = bytearray(buf)
    recs, _, _, _ = R.walk(bytes(buf))
    k = (2 * len(recs)) // 3
    pos = recs[k][0] - 16
    if kind == "short_hdr":
        buf = buf[:pos + 7]
    elif kind == "short_data":
        buf = buf[:pos + 16 + 3]
    elif kind == "eof_data":
        buf = buf[:pos + 16]
    elif kind == "snaplen":
        struct.pack_into("<II", buf, pos + 8, 262145, 262145)
    else:
        struct.pack_into("<I", buf, pos + 12, recs[k][1] - 1)
    p = _agree(bytes(buf), nthreads=8)
    assert p.batch.n == k and p.next_pos == pos and p.err
    want = {"short_hdr": "unexpected EOF", "short_data": "unexpected EOF", "eof_data": "EOF",
            "snaplen": "capture length exceeds snap length: 262145 > 262144",
            "origlen": f"capture length exceeds original packet length: {recs[k][1]} > {recs[k][1] - 1}"}
    assert p.err == want[kind]


@pytest.mark.parametrize("be,nano", [(0, 0), (0, 1), (1, 0), (1, 1)])
def test_byte_orders_and_resolutions(be, nano):
    b = synth.make_udp64(300, 5)
    le = bytearray(NP.synth_capture(b)[:-NP.PAD].tobytes())
    magic = {(0, 0): 0xA1B2C3D4, (0, 1): 0xA1B23C4D, (1, 0): 0xD4C3B2A1, (1, 1): 0x4D3CB2A1}[(be, nano)]
    struct.pack_into("<I", le, 0, magic)
    if be:  # swap every header field after the magic, record headers too
        for off, fmt in ((4, "H"), (6, "H"), (8, "i"), (12, "I"), (16, "I"), (20, "I")):
            v = struct.unpack_from("<" + fmt, le, off)[0]
            struct.pack_into(">" + fmt, le, off, v)
        o = 24
        while o < len(le):
            f = struct.unpack_from("<IIII", le, o)
            struct.pack_into(">IIII", le, o, *f)
            o += 16 + f[2]
    p = _agree(bytes(le))
    assert p.batch.n == 300 and p.nano == bool(nano)
    assert int(p.ts_ns[7]) == 7 * (1 if nano else 1000)


def test_header_errors():
    good = bytes.fromhex(VEC[0]["hex"])
    for buf, msg in [(b"", "EOF"), (b"\xd4", "EOF"), (good[:10], "unexpected EOF"),
                     (b"\x00\x00\x00\x00" + good[4:], "Unknown magic 0"),
                     (good[:4] + b"\x03\x00" + good[6:], "Unknown major version 3"),
                     (good[:6] + b"\x05\x00" + good[8:], "Unknown minor version 5")]:
        with pytest.raises(NP.PcapError, match=msg):
            _native(buf)
        with pytest.raises(R.PcapError, match=msg):
            R.header(buf)


def test_limit_and_resume():
    buf, b = _big_capture(5000, seed=2)
    cap = NP.capture_array(buf)
    p = NP.index(cap, max_n=1234)
    assert p.batch.n == 1234 and p.stop == NP.STOP_LIMIT and p.err is None
    recs, _, _, _ = R.walk(buf)
    assert p.next_pos == recs[1234][0] - 16


# ---- bounded walks, record location and shards (config 5: one capture cut by packet index) ----
def _oracle_positions(buf):
    recs, stop, nxt, err = R.walk(buf)
    return np.array([r[0] - 16 for r in recs], dtype=np.uint64), stop, nxt


@pytest.mark.parametrize("maker", ["imix", "decoys"])
def test_bounded_walk_windows(maker):
    """A bounded walk (max_n records from any record position) goes window by window in parallel;
    every window size must give the sequential loop's records, next position and stop."""
    if maker == "imix":
        buf, _ = _big_capture(1 << 15, seed=5)
    else:
        rng = np.random.default_rng(9)
        decoy = b"".join(struct.pack("<IIII", 1, 2, L, L) + bytes(L) for L in rng.integers(4, 40, 64))
        pkts = [decoy[k % 97:][:900 + (k % 400)] for k in range(9000)]
        buf = NP.synth_capture(PacketBatch.from_packets(pkts, align=1))[:-NP.PAD].tobytes()
    pos, _, _ = _oracle_positions(buf)
    cap = NP.capture_array(buf)
    N = len(pos)
    for start in (0, 1, 777, N // 2):
        for m in (1, 300, 5000, N // 3, N - start, N - start + 10):
            p = NP.index(cap, max_n=m, nthreads=8, pos=int(pos[start]))
            k = min(m, N - start)
            assert p.batch.n == k
            assert np.array_equal(p.batch.offset.astype(np.uint64), pos[start:start + k] + 16)
            if start + k < N:
                assert p.stop == NP.STOP_LIMIT and p.next_pos == pos[start + k]
            elif m == k:
                assert p.stop == NP.STOP_LIMIT and p.next_pos == len(buf)
            else:
                assert p.stop == NP.STOP_EOF and p.next_pos == len(buf)


def test_bounded_walk_stops_at_rejected_record():
    buf, _ = _big_capture(1 << 15, seed=13)
    buf = bytearray(buf)
    pos, _, _ = _oracle_positions(bytes(buf))
    k = len(pos) * 3 // 4
    struct.pack_into("<II", buf, int(pos[k]) + 8, 262145, 262145)
    cap = NP.capture_array(bytes(buf))
    p = NP.index(cap, max_n=k - 100 + 5000, nthreads=8, pos=int(pos[100]))
    assert p.batch.n == k - 100 and p.next_pos == pos[k]
    assert p.err == "capture length exceeds snap length: 262145 > 262144"


@pytest.mark.parametrize("threads", [1, 3, 8])
def test_locate_matches_sequential_walk(threads):
    buf, _ = _big_capture(1 << 15, seed=17)
    pos, _, _ = _oracle_positions(buf)
    cap = NP.capture_array(buf)
    N = len(pos)
    targets = [0, 1, 2, 4095, 4096, 10000, N // 2, N - 1, N]
    got, n, stop = NP.locate(cap, targets, nthreads=threads)
    assert n == N and stop == NP.STOP_EOF
    want = [int(pos[t]) if t < N else len(buf) for t in targets]
    assert list(got) == want
    # from a record position inside the capture
    got2, n2, _ = NP.locate(cap, [0, 5, N - 1000], pos=int(pos[1000]), nthreads=threads)
    assert n2 == N - 1000 and list(got2) == [int(pos[1000]), int(pos[1005]), len(buf)]
    with pytest.raises(Exception, match="beyond"):
        NP.locate(cap, [N + 1], nthreads=threads)


def test_locate_stops_at_rejected_record():
    buf, _ = _big_capture(1 << 15, seed=19)
    buf = bytearray(buf)
    pos, _, _ = _oracle_positions(bytes(buf))
    k = len(pos) // 3
    struct.pack_into("<I", buf, int(pos[k]) + 12, 1)  # wire length < caplen
    got, n, stop = NP.locate(NP.capture_array(bytes(buf)), [0, k // 2, k], nthreads=8)
    assert n == k and stop == NP.STOP_ORIGLEN
    assert list(got) == [int(pos[0]), int(pos[k // 2]), int(pos[k])]


@pytest.mark.parametrize("world", [2, 3, 8])
def test_shards_partition_the_capture(world):
    """Config 5's cut: shard g = records [g*N/G, (g+1)*N/G), located in one counting pass and
    indexed from its first record; the shards are disjoint and together are the whole index."""
    buf, b = _big_capture(1 << 15, seed=23)
    cap = NP.capture_array(buf)
    whole = NP.index(cap, nthreads=8)
    N = whole.batch.n
    bounds = NP.shard_bounds(N, world)
    starts, n, _ = NP.locate(cap, [lo for lo, _ in bounds] + [N], nthreads=8)
    assert n == N
    parts = []
    for g, (lo, hi) in enumerate(bounds):
        p = NP.index(cap, max_n=hi - lo, nthreads=8, pos=int(starts[g]))
        assert p.batch.n == hi - lo and p.next_pos == starts[g + 1]
        parts.append(p.batch.offset)
    cat = np.concatenate(parts)
    assert len(np.unique(cat)) == N
    assert np.array_equal(cat, whole.batch.offset)


def test_bounded_walk_runs_windows_in_parallel():
    buf, _ = _big_capture(1 << 15, seed=29)
    pos, _, _ = _oracle_positions(buf)
    cap = NP.capture_array(buf)
    N = len(pos)
    p = NP.index(cap, max_n=N - 1, nthreads=8)
    assert p.batch.n == N - 1 and p.next_pos == pos[N - 1]
    assert np.array_equal(p.batch.offset.astype(np.uint64), pos[:N - 1] + 16)
    assert NP.last_walk_stats()[0] > 1
