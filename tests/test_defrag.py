"""F4 fragment hand-off (include/gpd_defrag.h): ip4defrag's per-packet pre-steps on the GPU vs
the CPU restatement (oracle/defrag_ref.py), which is pinned by ip4defrag's own fixtures
(tests/golden/defrag_vectors.json, extracted from ip4defrag/defrag_test.go)."""
import json
import os
import struct
import sys

import numpy as np
import pytest

import oracle_ref as O
from conftest import ROOT
from gopacket_amd import layers as L
from gopacket_amd import synth
from gopacket_amd.batch import PacketBatch

sys.path.insert(0, os.path.join(ROOT, "oracle"))
import defrag_ref as D  # noqa: E402

ALL = 0xFFF
FRAGMENT_BIT = 1 << 9  # GPD_DEC_FRAGMENT
VEC = json.load(open(os.path.join(ROOT, "tests", "golden", "defrag_vectors.json")))


def _frames():
    return {k: bytes.fromhex(v["hex"]) for k, v in VEC["frames"].items()}


def ip4_frame(length, flags, fo, ident, proto=1, ihl=5, src=(1, 1, 1, 1), dst=(2, 2, 2, 2), tags=0,
              body=None, cap=None, ethertype=0x0800):
    """Ethernet [Dot1Q x tags] IPv4 with the given header fields; the IPv4 datagram carries
    Length bytes (16 payload bytes when Length is 0), cut to `cap` bytes of frame if given."""
    eth = bytes(6) + bytes([2, 0, 0, 0, 0, 1])
    for t in range(tags):
        eth += struct.pack(">HH", 0x8100 if t == 0 else 0x8100, t + 1)
    eth += struct.pack(">H", ethertype)
    hl = ihl * 4
    opts = b"\x01" * max(0, hl - 20)
    hdr = struct.pack(">BBHHHBBH4s4s", 0x40 | ihl, 0, length, ident, (flags << 13) | fo, 64, proto, 0,
                      bytes(src), bytes(dst)) + opts
    n_body = (length - len(hdr)) if length else 16
    if body is None:
        body = bytes((7 * k + ident) & 0xFF for k in range(max(0, n_body)))
    f = eth + hdr + body
    return f[:cap] if cap is not None else f


def vxlan_frame(inner):
    """Outer Ethernet/IPv4/UDP(4789)/VXLAN around an inner Ethernet frame."""
    vx = b"\x08\x00\x00\x00\x00\x00\x2a\x00" + inner
    udp = struct.pack(">HHHH", 40000, 4789, 8 + len(vx), 0) + vx
    ip = struct.pack(">BBHHHBBH4s4s", 0x45, 0, 20 + len(udp), 9, 0, 64, 17, 0, bytes([10, 0, 0, 1]),
                     bytes([10, 0, 0, 2])) + udp
    return bytes(6) + bytes([2, 0, 0, 0, 0, 2]) + b"\x08\x00" + ip


def ip6_over(inner_ip4):
    """Ethernet/IPv6 (next header 4: IPv4) around an IPv4 datagram."""
    ip6 = struct.pack(">IHBB16s16s", 0x60000000, len(inner_ip4), 4, 64, bytes(15) + b"\x01", bytes(15) + b"\x02")
    return bytes(6) + bytes([2, 0, 0, 0, 0, 3]) + b"\x86\xdd" + ip6 + inner_ip4


def struct_frames():
    """The layers.IPv4 structs ip4defrag's tests build, as frames (expected outcome per frame)."""
    out = []
    for s in VEC["structs"]:
        ihl = s["ihl"] or 5
        length = s["length"] or 20
        out.append((s, ip4_frame(length, s["flags"], s["frag_offset"], s["id"], ihl=ihl,
                                 src=VEC["struct_addrs"]["src"], dst=VEC["struct_addrs"]["dst"])))
    return out


def fuzz_frames(n=3000, seed=11):
    rng = np.random.default_rng(seed)
    out = []
    for k in range(n):
        flags = int(rng.choice([0, 1, 1, 1, 2, 3, 4, 5]))
        fo = int(rng.choice([0, 0, 1, 185, 4000, 8183, 8184, 8191]))
        ihl = int(rng.choice([5, 5, 5, 6, 15]))
        length = int(rng.choice([0, ihl * 4, ihl * 4 + 7, ihl * 4 + 8, 100, 600, 1500]))
        proto = int(rng.choice([1, 6, 17, 200]))
        tags = int(rng.choice([0, 0, 1, 2, 14]))
        ident = int(rng.integers(0, 65536))
        f = ip4_frame(length, flags, fo, ident, proto=proto, ihl=ihl, tags=tags,
                      src=tuple(rng.integers(0, 256, 4)), dst=tuple(rng.integers(0, 256, 4)))
        r = rng.random()
        if r < 0.1:
            f = f[:int(rng.integers(14, len(f) + 1))]  # truncated anywhere
        elif r < 0.2:
            f = vxlan_frame(f)
        elif r < 0.25:
            f = ip6_over(f[14 + 4 * tags:])
        elif r < 0.3:
            f = f + bytes(int(rng.integers(1, 40)))  # trailer past the IPv4 Length
        out.append(f)
    return out


# ---------------------------------------------------------------- CPU: the oracle, pinned
def test_oracle_on_reference_fragments():
    """defrag_test.go's eight ping fragments: every one is handed over for insertion, keyed
    ipv4{NetworkFlow(), Id} per ping, Id = BigEndian(frame[18:]) (TestDefragIDField), the payload
    starts at frame byte 34 and each ping's payloads make the asserted 4508-byte datagram."""
    fr = _frames()
    names = list(fr)
    batch = PacketBatch.from_packets([fr[k] for k in names])
    ref = O.decode(batch, L.LayerTypeEthernet, ALL, 0, ext=True)
    recs = D.ip4_fragments(batch, ref)
    assert len(recs) == 8 and list(recs["packet"]) == list(range(8))
    assert (recs["verdict"] == D.FRAG_INSERT).all()
    a = VEC["asserted"]
    for k, r in zip(names, recs):
        f = fr[k]
        assert r["id"] == struct.unpack(">H", f[a["id_offset_in_frame"]:a["id_offset_in_frame"] + 2])[0]
        assert int(r["net_off"]) + 4 * int(r["ihl"]) == a["payload_from"]
        assert int(r["payload_len"]) == len(f) - a["payload_from"]
    for ping in ("1", "2"):
        sel = [i for i, k in enumerate(names) if k.startswith(f"testPing{ping}")]
        keys = {(bytes(recs[i]["src"]), bytes(recs[i]["dst"]), int(recs[i]["id"])) for i in sel}
        assert len(keys) == 1
        assert sum(int(recs[i]["payload_len"]) for i in sel) == a["datagram_payload_len"]
    k1 = (bytes(recs[0]["src"]), bytes(recs[0]["dst"]), int(recs[0]["id"]))
    k2 = (bytes(recs[4]["src"]), bytes(recs[4]["dst"]), int(recs[4]["id"]))
    assert k1 != k2


def test_oracle_fields_complete_the_datagrams_in_the_asserted_order():
    """The handed-over fields drive fragmentList.insert's completion test (defrag.go:253-270:
    Highest = max(FragOffset*8 + Length-20), Current += Length-20, FinalReceived on !MF); fed in
    TestDefragPing1and2's order, ping 1 completes at testPing1Frag4 and ping 2 at testPing2Frag2."""
    fr = _frames()
    order = VEC["asserted"]["ping1_and2_order"]
    batch = PacketBatch.from_packets([fr[k] for k in order])
    recs = D.ip4_fragments(batch, O.decode(batch, L.LayerTypeEthernet, ALL, 0, ext=True))
    state, done = {}, []
    for k, r in zip(order, recs):
        key = (bytes(r["src"]), bytes(r["dst"]), int(r["id"]))
        hi, cur, fin = state.get(key, (0, 0, False))
        fl = (int(r["length"]) - 20) & 0xFFFF
        hi = max(hi, (int(r["frag_offset"]) * 8 + fl) & 0xFFFF)
        cur = (cur + fl) & 0xFFFF
        fin = fin or not (int(r["flags"]) & 1)
        if fin and hi == cur:
            done.append(k)
            state.pop(key)
        else:
            state[key] = (hi, cur, fin)
    assert done == [VEC["asserted"]["completing"]["ping1"], VEC["asserted"]["completing"]["ping2_after_ping1_and2_order"]]


def test_oracle_on_reference_struct_cases():
    """TestNotFrag / TooSmall / FragmentOffset / MaxSize: an error <=> a non-insert verdict, an
    unchanged layer <=> not handed over."""
    cases = struct_frames()
    batch = PacketBatch.from_packets([f for _, f in cases])
    recs = D.ip4_fragments(batch, O.decode(batch, L.LayerTypeEthernet, ALL, 0, ext=True))
    by_pkt = {int(r["packet"]): r for r in recs}
    for i, (s, _) in enumerate(cases):
        if s.get("unchanged"):
            assert i not in by_pkt, s["test"]
            continue
        r = by_pkt[i]
        assert (int(r["verdict"]) != D.FRAG_INSERT) == s["error"], s["test"]


def test_security_checks_restatement():
    assert D.security_verdict(27, 5, 0) == D.FRAG_TOO_SMALL
    assert D.security_verdict(28, 5, 0) == D.FRAG_INSERT
    assert D.security_verdict(512, 5, 8184) == D.FRAG_OFFSET
    assert D.security_verdict(65535, 5, 8183) == D.FRAG_INSERT  # the uint16 overrun sum wraps
    assert D.security_verdict(20, 5, 3) == D.FRAG_TOO_SMALL     # empty payload
    assert D.dont_defrag(2, 100) and D.dont_defrag(0, 0) and not D.dont_defrag(1, 0)
    assert not D.dont_defrag(0, 1) and not D.dont_defrag(4, 1)


def test_frag_struct_layout_matches_c(tmp_path):
    import subprocess
    from gopacket_amd.defrag import FRAG_DTYPE as PD
    assert PD == D.FRAG_DTYPE
    prog = tmp_path / "f.c"
    fields = ["packet", "net_off", "src", "dst", "id", "frag_offset", "length", "flags", "ihl",
              "payload_len", "verdict"]
    prog.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "gpd_defrag.h"\nint main(void){'
                    'printf("%zu' + ' %zu' * len(fields) + '\\n", sizeof(gpd_ip4_frag)' +
                    "".join(f", offsetof(gpd_ip4_frag, {f})" for f in fields) + '); return 0;}\n')
    exe = tmp_path / "f"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), str(prog), "-o", str(exe)], check=True)
    got = list(map(int, subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()))
    assert got == [PD.itemsize] + [PD.fields[f][1] for f in fields]


# ---------------------------------------------------------------- GPU: the hand-off vs the oracle
def _device_fragments(parser, batch, records=False, max_out=None):
    import torch
    from gopacket_amd import defrag as DF
    from gopacket_amd import parser as P
    db = P.DeviceBatch(batch, 0)
    dr = P.DeviceResult(batch.n, 0, records=records)
    parser.decode_device(db, dr)
    out, cnt = DF.IPv4Fragments(parser, db, dr, max_out=max_out)
    torch.cuda.synchronize()
    return DF.fragments_to_host(out, cnt, allow_partial=max_out is not None), cnt


def _all_parser(mask=ALL, ignore=False):
    from gopacket_amd import parser as P
    p = P.NewDecodingLayerParser(L.LayerTypeEthernet)
    p._mask = mask
    p.IgnoreUnsupported = ignore
    return p


def _check(batch, parser, records=False):
    ref = D.ip4_fragments(batch, O.decode(batch, L.LayerTypeEthernet, parser.decoders, parser.options,
                                          ext=True, nthreads=8))
    got, cnt = _device_fragments(parser, batch, records=records)
    assert cnt == len(ref)
    assert np.array_equal(got.view(np.uint8), ref.view(np.uint8)), (got[:4], ref[:4])
    return ref


@pytest.mark.gpu
@pytest.mark.parametrize("records", [False, True])
def test_reference_fragments_on_gpu(records):
    fr = _frames()
    pk = [fr[k] for k in VEC["asserted"]["ping1_and2_order"]] + [f for _, f in struct_frames()]
    ref = _check(PacketBatch.from_packets(pk), _all_parser(), records)
    assert len(ref) == 8 + len(VEC["structs"]) - 1  # TestNotFrag's DF layer is not handed over


@pytest.mark.gpu
@pytest.mark.parametrize("mask,ignore", [(ALL, False), (ALL & ~FRAGMENT_BIT, False),
                                         (ALL & ~FRAGMENT_BIT, True)])
def test_fragment_fuzz_matches_oracle(mask, ignore):
    """Flags x offsets x Length (0 = TSO, empty and short payloads) x IHL x tags (14 tags: more
    layers than the layers word holds) x truncation, trailers, VXLAN-inner and IPv4-in-IPv6
    fragments; Fragment registered or not (the decode then stops on LayerTypeFragment)."""
    batch = PacketBatch.from_packets(fuzz_frames())
    ref = _check(batch, _all_parser(mask, ignore))
    assert len(ref) > 500 and len(set(ref["verdict"])) >= 3


@pytest.mark.gpu
def test_fragment_traffic_mix_and_max_out():
    """2^18 frames of the traffic mix (3 % fragments among every other stack), both result
    forms; with max_out below the count the first max_out records come back, count is whole."""
    batch = synth.make_traffic_mix(1 << 18, 0x5EED0011)
    parser = _all_parser()
    ref = _check(batch, parser)
    _check(batch, parser, records=True)
    assert len(ref) > 1000
    got, cnt = _device_fragments(parser, batch, max_out=100)
    assert cnt == len(ref) and np.array_equal(got.view(np.uint8), ref[:100].view(np.uint8))


@pytest.mark.gpu
def test_fragment_empty_and_fragment_free_batches():
    parser = _all_parser()
    got, cnt = _device_fragments(parser, synth.make_udp64(5000))
    assert cnt == 0 and len(got) == 0
    from gopacket_amd import defrag as DF
    from gopacket_amd import parser as P
    db = P.DeviceBatch(PacketBatch.from_packets([]), 0)
    dr = P.DeviceResult(0, 0)
    assert DF.IPv4Fragments(parser, db, dr)[1] == 0


@pytest.mark.gpu
def test_fragment_header_past_the_offset_word():
    """An IPv4 header past byte 65534 (16,384 802.1Q tags in front of it): the header offsets
    word saturates, so the batch pass cannot rule the packet out from the header bytes and the
    record pass decides — a fragment is handed over exactly as the oracle restates it, a
    non-fragment comes back as one GPD_FRAG_WHOLE record (DefragIPv4 would return it as is)."""
    frag = ip4_frame(600, 1, 0, 0x1234, tags=16384)
    whole = ip4_frame(600, 0, 0, 0x4321, tags=16384)
    small = ip4_frame(600, 1, 10, 0x99)
    batch = PacketBatch.from_packets([small, frag, whole, small])
    parser = _all_parser()
    ref = D.ip4_fragments(batch, O.decode(batch, L.LayerTypeEthernet, parser.decoders, 0, ext=True))
    assert list(ref["packet"]) == [0, 1, 3]
    got, cnt = _device_fragments(parser, batch)
    assert cnt == 4
    assert list(got["packet"]) == [0, 1, 2, 3]
    keep = got["packet"] != 2
    assert np.array_equal(got[keep].view(np.uint8), ref.view(np.uint8))
    w = got[~keep][0]
    assert w["verdict"] == D.FRAG_WHOLE and w["net_off"] == 14 + 4 * 16384 and w["id"] == 0x4321


# ---------------------------------------------------------------- the stateful rest (host)
def _reassemble(order, recs_by_name, frames, t=1.0):
    """Feed the handed-over records in `order` to one IPv4Defragmenter; returns the outcome of
    each call (layer, error)."""
    from ip4defrag_ref import NewIPv4Defragmenter
    d = NewIPv4Defragmenter()
    return d, [d.DefragIPv4WithTimestamp(recs_by_name[k], frames[k], t) for k in order]


def _defrag_scenarios(recs_by_name):
    """ip4defrag/defrag_test.go's frame scenarios, asserted as the reference asserts them."""
    fr = _frames()
    a = VEC["asserted"]
    want1 = b"".join(fr[f"testPing1Frag{k}"][a["payload_from"]:] for k in (1, 2, 3, 4))
    want2 = b"".join(fr[f"testPing2Frag{k}"][a["payload_from"]:] for k in (1, 2, 3, 4))
    # TestDefragPing1 (:69-104), twice on one defragmenter
    order = ["testPing1Frag1", "testPing1Frag3", "testPing1Frag2", "testPing1Frag4"]
    d, outs = _reassemble(order + order, recs_by_name, fr)
    for k, (o, e) in enumerate(outs):
        assert e is None and ((o is not None) == (k % 4 == 3)), (k, o, e)
    assert len(outs[3][0].payload) == a["datagram_payload_len"] and outs[3][0].payload == want1
    assert outs[7][0].payload == outs[3][0].payload
    # TestDefragIDField (:245-259)
    assert outs[3][0].ident == struct.unpack(">H", fr["testPing1Frag1"][18:20])[0]
    # TestDefragPingMultipleFrags (:38-67): duplicates ignored, nothing left to discard
    order = ["testPing1Frag1"] * 3 + ["testPing1Frag3", "testPing1Frag2", "testPing1Frag4"]
    d, outs = _reassemble(order, recs_by_name, fr)
    assert [o is not None for o, _ in outs] == [False] * 5 + [True] and outs[5][0].payload == want1
    assert d.DiscardOlderThan(10.0) == 0
    # TestDefragPing1and2 (:106-151)
    order = a["ping1_and2_order"]
    d, outs = _reassemble(order, recs_by_name, fr)
    done = [k for k, (o, e) in zip(order, outs) if o is not None]
    assert done == [a["completing"]["ping1"], a["completing"]["ping2_after_ping1_and2_order"]]
    assert outs[order.index("testPing1Frag4")][0].payload == want1
    assert outs[order.index("testPing2Frag2")][0].payload == want2
    # TestDefragDiscard (:204-214)
    d, outs = _reassemble(["testPing1Frag1", "testPing2Frag1"], recs_by_name, fr, t=1.0)
    assert d.DiscardOlderThan(2.0) == 2


def _struct_scenarios(recs, frames):
    """TestDefragTooSmall / FragmentOffset / MaxSize (:153-243): each test's layers through one
    defragmenter, errors where the reference expects them."""
    from ip4defrag_ref import NewIPv4Defragmenter
    cases = [s for s, _ in struct_frames()]
    by_test = {}
    for k, s in enumerate(cases):
        by_test.setdefault(s["test"].split()[0], []).append(k)
    rec_of = {int(r["packet"]): r for r in recs}
    for name, ks in by_test.items():
        d = NewIPv4Defragmenter()
        for k in ks:
            if cases[k].get("unchanged"):
                assert k not in rec_of
                continue
            out, err = d.DefragIPv4WithTimestamp(rec_of[k], frames[k], 1.0)
            assert (err is not None) == cases[k]["error"], (cases[k]["test"], err)
            if cases[k]["error"]:
                assert err.startswith("defrag: fragment")


def test_defragmenter_on_oracle_records():
    """The host defragmenter over the oracle's hand-off records reproduces every outcome
    defrag_test.go asserts (payload bytes, completing fragment, duplicates, discard, Id, the
    security errors)."""
    fr = _frames()
    names = list(fr)
    batch = PacketBatch.from_packets([fr[k] for k in names])
    recs = D.ip4_fragments(batch, O.decode(batch, L.LayerTypeEthernet, ALL, 0, ext=True))
    _defrag_scenarios({k: r for k, r in zip(names, recs)})
    sf = [f for _, f in struct_frames()]
    sb = PacketBatch.from_packets(sf)
    _struct_scenarios(D.ip4_fragments(sb, O.decode(sb, L.LayerTypeEthernet, ALL, 0, ext=True)), sf)


@pytest.mark.gpu
def test_defragmenter_on_gpu_records():
    """The same scenarios fed from the GPU hand-off (gpd_ip4_fragments) end to end."""
    fr = _frames()
    names = list(fr)
    parser = _all_parser()
    got, cnt = _device_fragments(parser, PacketBatch.from_packets([fr[k] for k in names]))
    assert cnt == 8 and list(got["packet"]) == list(range(8))
    _defrag_scenarios({k: r for k, r in zip(names, got)})
    sf = [f for _, f in struct_frames()]
    got, _ = _device_fragments(parser, PacketBatch.from_packets(sf))
    _struct_scenarios(got, sf)


def _rec(off8, length, flags, ident=7, ihl=5, payload_len=None):
    """A hand-off record for the host defragmenter (packet bytes: 20-B header + payload)."""
    r = np.zeros((), D.FRAG_DTYPE)
    r["net_off"], r["ihl"], r["id"], r["frag_offset"], r["length"], r["flags"] = 0, ihl, ident, off8, length, flags
    r["src"], r["dst"] = [1, 1, 1, 1], [2, 2, 2, 2]
    r["payload_len"] = length - 4 * ihl if payload_len is None else payload_len
    r["verdict"] = D.security_verdict(length, ihl, off8)
    pkt = bytes(4 * ihl) + bytes((off8 * 8 + k) & 0xFF for k in range(int(r["payload_len"])))
    return r, pkt


def test_defragmenter_restates_the_list_rules():
    """fragmentList.insert / build (defrag.go:216-328) on crafted fragments: out-of-order
    insertion, a fragment below the highest end but past every stored offset counted and not
    stored (:222-249), an overlap, a hole (:299-304), and the flush past 8,192 fragments
    (:117-125), which no admitted sequence reaches."""
    from ip4defrag_ref import NewIPv4Defragmenter
    # out of order, then complete: payload is the bytes in offset order
    d = NewIPv4Defragmenter()
    outs = [d.DefragIPv4WithTimestamp(*_rec(o, 20 + 16, f), 1.0) for o, f in ((4, 0), (0, 1), (2, 1))]
    assert [o is None for o, _ in outs] == [True, True, False]
    assert outs[2][0].payload == bytes(range(48)) and outs[2][0].length == 48
    # counted, not stored: F1 [0, 40) MF, F2 at 16 (< highest 40, past every stored offset)
    d = NewIPv4Defragmenter()
    d.DefragIPv4WithTimestamp(*_rec(0, 60, 1), 1.0)
    d.DefragIPv4WithTimestamp(*_rec(2, 28, 1), 1.0)
    fl = next(iter(d.ip_flows.values()))
    assert len(fl.frags) == 1 and fl.highest == 40 and fl.current == 48
    # an overlap: [0, 24) then [16, 40) (MF clear): build takes bytes 24.. of the second
    d = NewIPv4Defragmenter()
    d.DefragIPv4WithTimestamp(*_rec(0, 44, 1), 1.0)
    out, err = d.DefragIPv4WithTimestamp(*_rec(2, 44, 0), 1.0)
    assert err is None and out is None  # highest 40 != current 48: not complete
    # a hole: [8, 16) final with [0, 8) never sent — highest 16, current 8: waits; the
    # reference only builds when they meet, and a hole found while building is an error
    d = NewIPv4Defragmenter()
    assert d.DefragIPv4WithTimestamp(*_rec(1, 28, 0), 1.0) == (None, None)
    fl = next(iter(d.ip_flows.values()))
    fl.current = fl.highest  # force the build: the list starts at 8, not 0
    assert fl.build(fl.frags[0]) == (None, "defrag: building - hole found")
    # the flush past 8,192 stored fragments cannot trigger: securityChecks admits offsets up to
    # 8,183 and duplicates are not stored, so a list holds at most 8,184 (Len()+1 <= 8,185)
    d = NewIPv4Defragmenter()
    errs = [d.DefragIPv4WithTimestamp(*_rec(k, 28, 1), 1.0)[1] for k in range(8184)]
    errs += [d.DefragIPv4WithTimestamp(*_rec(k, 28, 1), 1.0)[1] for k in (0, 100, 8183)]
    assert errs == [None] * 8187 and len(next(iter(d.ip_flows.values())).frags) == 8184
    # security verdicts come back as the reference's errors
    r, p = _rec(0, 27, 1)
    assert d.DefragIPv4WithTimestamp(r, p, 1.0) == (None, "defrag: fragment too small (handcrafted? 7 < 8)")
    r, p = _rec(8184, 512, 1)
    assert d.DefragIPv4WithTimestamp(r, p, 1.0) == (None, "defrag: fragment offset too big (handcrafted? 8184 > 8183)")
