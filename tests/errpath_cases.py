"""The error-path golden cases (tests/golden/errpath.json, made by tests/golden/make_errpath.py):
load them and check a BatchResult row against the hand-stated object state.

The expected result words are computed here from the case's offsets with this file's own
plain-Python FNV-1a / checksum code (flows.go:60-83,167-174; ip4.go:158-179; tcpip.go:26-88), so
the check shares no code with the C oracle or the HIP kernels.
"""
from __future__ import annotations

import json
import os

import golden_cases as G
from gopacket_amd import layers as L
from gopacket_amd.batch import PacketBatch
from gopacket_amd.results import OBJ_NAMES

HERE = os.path.dirname(os.path.abspath(__file__))
ERRPATH = os.path.join(HERE, "golden", "errpath.json")


def load():
    with open(ERRPATH) as f:
        return json.load(f)["cases"]


def tables(c):
    t = L.DispatchTables()
    for name, m in c["tables"].items():
        for k, v in m.items():
            getattr(t, name)[int(k)] = G.NAME_TO_LT[v]
    return t


def batch(c) -> PacketBatch:
    return PacketBatch.from_packets([bytes.fromhex(c["hex"])])


def _fnv(b: bytes) -> int:
    h = 14695981039346656037
    for x in b:
        h = ((h ^ x) * 1099511628211) & 0xFFFFFFFFFFFFFFFF
    return h


def _flow(ept: int, a: bytes, b: bytes) -> int:
    return ((((_fnv(a) + _fnv(b)) & 0xFFFFFFFFFFFFFFFF) ^ ept) * 1099511628211) & 0xFFFFFFFFFFFFFFFF


def _fold_not(s: int) -> int:
    s &= 0xFFFFFFFF
    while s > 0xFFFF:
        s = (s >> 16) + (s & 0xFFFF)
    return ~s & 0xFFFF


def _words(b: bytes) -> int:
    s = sum((b[i] << 8) | b[i + 1] for i in range(0, len(b) - 1, 2))
    if len(b) % 2:
        s += b[-1] << 8
    return s


def ip4_checksum(h: bytes) -> int:
    h = bytearray(h)
    h[10] = h[11] = 0
    return _fold_not(_words(bytes(h)))


def l4_checksum(pkt: bytes, a: int, b: int, net_kind: str, net_off: int, proto: int) -> int:
    if net_kind == "IPv4":
        ps = _words(pkt[net_off + 12:net_off + 20])
    else:
        ps = _words(pkt[net_off + 8:net_off + 40])
    n = b - a
    return _fold_not(ps + proto + (n & 0xFFFF) + (n >> 16) + _words(pkt[a:b]))


def expected(c):
    """The result words (status bits, hashes, checksums, hdr_off) the case states."""
    pkt = bytes.fromhex(c["hex"])
    e = c["expect"]
    out = {"net_hash": None, "tp_hash": None, "ip4": None, "l4": None}
    hn = ht = 0xFFFF
    if e["net"]:
        kind, o = e["net"]
        hn = o
        if kind == "IPv4":
            out["net_hash"] = _flow(1, pkt[o + 12:o + 16], pkt[o + 16:o + 20])
        else:
            out["net_hash"] = _flow(2, pkt[o + 8:o + 24], pkt[o + 24:o + 40])
    if e["tp"]:
        kind, o = e["tp"]
        ht = o
        out["tp_hash"] = _flow(4 if kind == "TCP" else 5, pkt[o:o + 2], pkt[o + 2:o + 4])
    if e["ip4"]:
        c0, c1 = e["ip4"]
        out["ip4"] = ip4_checksum(pkt[c0:c1]) if (c1 - c0) % 2 == 0 else None  # odd: Go panics
    if e["l4"]:
        out["l4"] = l4_checksum(pkt, *e["l4"])
    out["hdr_off"] = hn | (ht << 16)
    return out


def check(c, res, i: int = 0) -> None:
    e = c["expect"]
    name = c["name"]
    want = [G.NAME_TO_LT[x] for x in e["decoded"]]
    assert res.decoded(i) == want, f"{name}: decoded {res.decoded(i)} != {want}"
    err = res.err(i)
    assert err is not None and str(err) == e["err"], f"{name}: error {err!r} != {e['err']!r}"
    assert res.truncated(i) == e["truncated"], f"{name}: truncated {res.truncated(i)}"
    x = expected(c)
    assert res.network_flow_hash(i) == x["net_hash"], f"{name}: net_hash"
    assert res.transport_flow_hash(i) == x["tp_hash"], f"{name}: tp_hash"
    assert res.ip4_checksum(i) == x["ip4"], f"{name}: ip4 checksum {res.ip4_checksum(i)} != {x['ip4']}"
    assert res.l4_checksum(i) == x["l4"], f"{name}: l4 checksum {res.l4_checksum(i)} != {x['l4']}"
    if res.hdr_off is not None:
        assert int(res.hdr_off[i]) == x["hdr_off"], f"{name}: hdr_off {int(res.hdr_off[i]):#x}"
    if res.ext is not None:
        r = res.ext[i]
        k = OBJ_NAMES.index(e["err_obj"])
        assert int(r["err_obj"]) == k, f"{name}: err_obj {int(r['err_obj'])}"
        assert int(r["err_wrote"]) == e["err_wrote"], f"{name}: err_wrote {int(r['err_wrote'])}"
        assert int(r["err_off"]) == e["err_off"], f"{name}: err_off {int(r['err_off'])}"
        valid = (int(r["obj_valid"]) >> k) & 1
        if e["err_obj_rec"] is not None:
            (c0, c1), (p0, p1) = e["err_obj_rec"]
            o = r["obj"][k]
            got = [[int(o["contents_off"]), int(o["contents_off"]) + int(o["contents_len"])],
                   [int(o["payload_off"]), int(o["payload_off"]) + int(o["payload_len"])]]
            assert got == [[c0, c1], [p0, p1]], f"{name}: {e['err_obj']} BaseLayer {got}"
        elif not valid:
            assert int(r["obj"][k]["contents_len"]) == 0, f"{name}: stale {e['err_obj']} record"
