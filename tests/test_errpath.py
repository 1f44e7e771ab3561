"""Layer-object state after a failed DecodeFromBytes (the reused objects of layers_decoder.go:61-78).

CPU: the oracle against the hand-stated error-path cases (tests/golden/errpath.json).
GPU: the HIP path (generic decoder with ext records, and the fast kernel + fallback list
without) against the oracle and the same cases, then a fuzz family of nested stacks whose inner
headers are broken: VXLAN over UDP and over TCP (RegisterTCPPortLayerType), IPv4-in-IPv4,
IPv6-in-IPv6, 4in6 and 6in4.
"""
import struct

import numpy as np
import pytest

import errpath_cases as E
import oracle_ref as O
from gopacket_amd import layers as L
from gopacket_amd.batch import PacketBatch

CASES = E.load()
IDS = [c["name"] for c in CASES]
ALL = 0xFFF


@pytest.mark.parametrize("c", CASES, ids=IDS)
def test_oracle_errpath_case(c):
    res = O.decode(E.batch(c), L.LayerTypeEthernet, ALL, 0, tables=E.tables(c), ext=True)
    E.check(c, res)


def test_errpath_fixture_covers_every_partial_write_site():
    """One case at least per kind of partial write the reference has (gpd.h err_wrote)."""
    seen = {(c["expect"]["err_obj"], c["expect"]["err_wrote"]) for c in CASES}
    for need in [("IPv4", 2), ("IPv6", 2), ("TCP", 1), ("TCP", 2), ("UDP", 2), ("LLC", 1), ("IPv4", 0)]:
        assert need in seen, need
    # ... and both outcomes of the kind-in-decoded rule
    assert any(c["expect"]["net"] and c["expect"]["net"][1] == c["expect"]["err_off"] for c in CASES)
    assert any(c["expect"]["err_obj"] == "IPv4" and c["expect"]["ip4"] is None for c in CASES)


def nested_stacks(n: int, seed: int) -> list:
    """Nested stacks with the INNER headers fuzzed (lengths, IHL, data offsets, options, next
    headers) and cut at random lengths."""
    rng = np.random.default_rng(seed)
    mac = bytes(range(12))

    def ip4(proto, payload, **kw):
        h = bytearray(20)
        h[0] = 0x45
        struct.pack_into(">HHHBB", h, 2, 20 + len(payload), int(rng.integers(0, 65536)),
                         kw.get("ff", 0x4000), 64, proto)
        h[12:20] = rng.integers(0, 256, 8, dtype=np.uint8).tobytes()
        return bytes(h) + payload

    def ip6(nh, payload):
        return (bytes([0x60, 0, 0, 0]) + struct.pack(">HBB", len(payload), nh, 64)
                + rng.integers(0, 256, 32, dtype=np.uint8).tobytes() + payload)

    def l4(kind):
        body = rng.integers(0, 256, int(rng.integers(0, 40)), dtype=np.uint8).tobytes()
        ports = rng.integers(1024, 65536, 2)
        if kind == 6:
            h = bytearray(20)
            struct.pack_into(">HH", h, 0, *ports)
            h[12] = 0x50
            return bytes(h) + body
        return struct.pack(">HHHH", ports[0], ports[1], 8 + len(body), 0) + body

    out = []
    for k in range(n):
        kind = k % 6
        inner_proto = int(rng.choice([6, 17, 1]))
        inner = ip4(inner_proto, l4(inner_proto))
        if kind == 0:    # VXLAN over UDP
            vx = bytes([8, 0, 0, 0, 0, 0, 7, 0]) + mac + b"\x08\x00" + inner
            pk = mac + b"\x08\x00" + ip4(17, struct.pack(">HHHH", 5555, 4789, 8 + len(vx), 0) + vx)
            lo = 14 + 20 + 8 + 8 + 14
        elif kind == 1:  # VXLAN over TCP (dst port 4789 registered to VXLAN below)
            vx = bytes([8, 0, 0, 0, 0, 0, 7, 0]) + mac + b"\x08\x00" + inner
            t = bytearray(20)
            struct.pack_into(">HH", t, 0, 40000, 4789)
            t[12] = 0x50
            pk = mac + b"\x08\x00" + ip4(6, bytes(t) + vx)
            lo = 14 + 20 + 20 + 8 + 14
        elif kind == 2:  # IPv4-in-IPv4
            pk = mac + b"\x08\x00" + ip4(4, inner)
            lo = 34
        elif kind == 3:  # IPv6-in-IPv6
            pk = mac + b"\x86\xdd" + ip6(41, ip6(int(rng.choice([6, 17, 0])), l4(6)))
            lo = 54
        elif kind == 4:  # 4in6
            pk = mac + b"\x86\xdd" + ip6(4, inner)
            lo = 54
        else:            # 6in4
            pk = mac + b"\x08\x00" + ip4(41, ip6(6, l4(6)))
            lo = 34
        b = bytearray(pk)
        # break the inner headers: their first 32 bytes (version/IHL, lengths, flags, protocol,
        # the transport's ports / length / data offset / first options) are the hot spots
        for _ in range(int(rng.integers(1, 4))):
            j = lo + int(rng.integers(0, 44))
            if j < len(b):
                b[j] = int(rng.integers(0, 256))
        if rng.random() < 0.25:
            b = b[:int(rng.integers(lo, len(b) + 1))]
        out.append(bytes(b))
    return out


def nested_tables():
    t = L.DispatchTables()
    t.tcp_port[4789] = L.LayerTypeVXLAN  # RegisterTCPPortLayerType(4789, LayerTypeVXLAN)
    return t


def test_nested_stack_fuzz_oracle_runs():
    """The fuzz family decodes under the oracle with every class of outcome present."""
    b = PacketBatch.from_packets(nested_stacks(3000, 5))
    res = O.decode(b, L.LayerTypeEthernet, ALL, 0, tables=nested_tables(), ext=True)
    cls = res.status & 3
    assert (cls == 2).sum() > 300 and (cls == 0).sum() > 300
    # the partial-write kinds all occur, and some feed outputs (kind in decoded)
    wrote = res.ext["err_wrote"][cls == 2]
    assert (wrote == 1).any() and (wrote == 2).any()
    fed = [(int(r["obj_valid"]) >> int(r["err_obj"])) & 1 for r in res.ext[cls == 2] if r["err_wrote"]]
    assert sum(fed) > 50


@pytest.mark.gpu
@pytest.mark.parametrize("c", CASES, ids=IDS)
def test_errpath_case_on_device(c):
    from test_parity_gpu import run_both
    dev = run_both(E.batch(c), L.LayerTypeEthernet, ALL, 0, tables=E.tables(c), ext=True)
    E.check(c, dev)


@pytest.mark.gpu
@pytest.mark.parametrize("options", [0, 1])
def test_nested_stack_fuzz_on_device(options):
    from test_parity_gpu import run_both
    b = PacketBatch.from_packets(nested_stacks(20000, 17 + options))
    run_both(b, L.LayerTypeEthernet, ALL, options, tables=nested_tables(), ext=True)
    run_both(b, L.LayerTypeEthernet, 0x3FF, options, tables=nested_tables(), ext=False)


@pytest.mark.gpu
def test_errpath_fragment_handoff_reads_the_failed_inner_header():
    """after IPv4-in-IPv4 whose inner header fails after ip4.go:195-210, the ip4
    object the application hands to DefragIPv4 holds the INNER flags / offset / addresses; the
    GPU hand-off (gpd_ip4_fragments) must list it as the oracle restatement does."""
    from test_defrag import _all_parser, _check
    c = [c for c in CASES if c["name"] == "ip4ip4_inner_mf_bad_option"][0]
    vx = [c for c in CASES if c["name"] == "vx_inner_ip4_bad_option"][0]
    pk = bytearray.fromhex(vx["hex"])
    pk[70:72] = b"\x20\x00"  # the failed inner IPv4 of the VXLAN case with More Fragments
    b = PacketBatch.from_packets([bytes.fromhex(c["hex"]), bytes(pk)] * 3)
    ref = _check(b, _all_parser())
    assert len(ref) == 6 and set(ref["net_off"]) == {34, 64} and set(ref["flags"]) == {1}
