"""Pin the CPU oracle against every golden vector the reference's tests hold (CPU only).

The oracle (oracle/gpd_oracle.c) is what the device path is compared with, so it
is checked first against the reference's own fixtures: tests/golden/golden.json
(packet bytes + expected results from the reference's _test.go files, see
tests/golden/make_golden.py) and the pcap files of pcap/pcap_test.go.
"""
import struct

import numpy as np
import pytest

import golden_cases as G
import oracle_ref as O
from gopacket_amd import layers as L
from gopacket_amd import synth
from gopacket_amd.batch import PacketBatch
from gopacket_amd.pcap import read_pcap

META = G.load()
CASES = META["cases"]


@pytest.mark.parametrize("c", CASES, ids=[c["name"] for c in CASES])
def test_oracle_golden_case(c):
    first, mask, opts = G.case_config(c)
    res = O.decode(G.single_batch(c), first, mask, opts)
    G.check(c, res)


def _zeroed_l4(c):
    """computeChecksum with the stored checksum field zeroed = what SerializeTo writes."""
    first, mask, opts = G.case_config(c)
    pkt = bytearray(G.case_bytes(c))
    res = O.decode(PacketBatch.from_packets([bytes(pkt)]), first, mask, opts)
    name = "TCP" if "TCP" in [L.layer_type_name(t) for t in res.decoded(0)] else "UDP"
    (c0, _), _ = res.layer(0, name)
    col = 16 if name == "TCP" else 6
    pkt[c0 + col:c0 + col + 2] = b"\0\0"
    res2 = O.decode(PacketBatch.from_packets([bytes(pkt)]), first, mask, opts)
    return res2.l4_checksum(0)


@pytest.mark.parametrize("c", [c for c in CASES if "l4_csum_zeroed" in c["expect"]],
                         ids=[c["name"] for c in CASES if "l4_csum_zeroed" in c["expect"]])
def test_oracle_serialize_form_checksum(c):
    assert _zeroed_l4(c) == c["expect"]["l4_csum_zeroed"]


def test_ip4_checksum_kats():
    # layers/ip4_test.go:104-133
    for c in CASES:
        if c["name"].startswith("ip4_checksum_kat"):
            hdr = bytes.fromhex(c["hex"])
            assert O.lib().gpo_ip4_header_checksum(hdr, len(hdr)) == c["expect"]["ip4_csum"]


def test_udp6_jumbogram_checksum_kat():
    # layers/tcpip_test.go:139-185: computeChecksum over 8 + 65536 bytes with the length>>16 term
    k = META["udp6_jumbogram_checksum_kat"]
    src, dst = bytes.fromhex(k["src"]), bytes.fromhex(k["dst"])
    seg = bytes.fromhex(k["udp_header"]) + bytes([k["payload_byte"]]) * k["payload_len"]
    cs = O.lib().gpo_pseudo_v6(src, dst) + 17 + (len(seg) & 0xFFFF) + (len(seg) >> 16)
    assert O.lib().gpo_tcpip_checksum(seg, len(seg), cs) == k["want"]


def test_fnv_and_flow_hash_properties():
    lib = O.lib()
    # FNV-1a 64 of the empty string is the offset basis (flows.go:60-70)
    assert lib.gpo_fnv_hash(b"", 0) == 14695981039346656037
    # FNV-1a test vector: "a" -> 0xaf63dc4c8601ec8c
    assert lib.gpo_fnv_hash(b"a", 1) == 0xAF63DC4C8601EC8C
    # Flow.FastHash is symmetric (doc.go:216-219, flows.go:159-174)
    a, b = bytes([10, 1, 2, 3]), bytes([192, 168, 0, 9])
    assert lib.gpo_flow_fasthash(1, a, 4, b, 4) == lib.gpo_flow_fasthash(1, b, 4, a, 4)
    assert lib.gpo_flow_fasthash(1, a, 4, b, 4) != lib.gpo_flow_fasthash(2, a, 4, b, 4)


def test_pcap_test_ethernet():
    # pcap/pcap_test.go:64-71,111-115: 10 packets, each with Ethernet, IPv4, TCP
    p = META["pcaps"]["test_ethernet.pcap"]
    pc = read_pcap(G.HERE + "/golden/test_ethernet.pcap")
    assert pc.batch.n == p["num"]
    assert list(pc.batch.caplen) == p["caplens"]
    res = O.decode(pc.batch, L.LayerTypeEthernet, 0x3FF)
    for i in range(pc.batch.n):
        d = res.decoded(i)
        for need in p["expected_layers_contain"]:
            assert L.__dict__["LayerType" + need] in d
        assert res.err(i) is None
        # observed in every packet: stored IPv4 checksum == computed; TCP ComputeChecksum == 0
        (c0, _), _ = res.layer(i, "IPv4")
        pkt = pc.batch.packet(i)
        assert res.ip4_checksum(i) == struct.unpack(">H", pkt[c0 + 10:c0 + 12])[0]
        assert res.l4_checksum(i) == 0


def test_pcap_test_dns():
    # pcap/pcap_test.go:72-80: Ethernet/IPv4/UDP/DNS -> the DLP stops at DNS (unregistered)
    pc = read_pcap(G.HERE + "/golden/test_dns.pcap")
    assert pc.batch.n == META["pcaps"]["test_dns.pcap"]["num"]
    res = O.decode(pc.batch, L.LayerTypeEthernet, 0x3FF)
    for i in range(pc.batch.n):
        assert res.decoded(i) == [L.LayerTypeEthernet, L.LayerTypeIPv4, L.LayerTypeUDP]
        assert str(res.err(i)) == "No decoder for layer type DNS"


@pytest.mark.parametrize("maker,n", [(synth.make_udp64, 4096), (synth.make_imix, 4096),
                                     (synth.make_vxlan, 4096), (synth.make_tcp64, 4096)])
def test_synthetic_configs_under_oracle(maker, n):
    b = maker(n)
    res = O.decode(b, L.LayerTypeEthernet, 0x3FF, ext=False)
    assert np.all((res.status & 3) == 0)
    bad = (np.arange(n) % 64) == 63
    if maker is synth.make_udp64:
        for i in range(n):
            assert res.decoded(i) == [17, 20, 45, 2]
        ipcs = res.csum & 0xFFFF
        stored = np.array([struct.unpack(">H", b.packet(i)[24:26])[0] for i in range(n)])
        assert np.all((ipcs == stored) == ~bad)
        assert np.all((res.csum >> 16) == 0)
    else:
        l4 = res.csum >> 16
        assert np.all((l4 == 0) == ~bad)
        if maker is synth.make_vxlan:
            for i in range(0, n, 97):
                assert res.decoded(i) == [17, 20, 45, 116, 17, 20, 44, 2]
        if maker is synth.make_tcp64:
            for i in range(0, n, 97):
                assert res.decoded(i) == [17, 20, 44, 2]
            stored = np.array([struct.unpack(">H", b.packet(i)[24:26])[0] for i in range(n)])
            assert np.array_equal(res.csum & 0xFFFF, stored)
