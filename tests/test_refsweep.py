"""Every Ethernet frame a reference layers/*_test.go decodes with NewPacket and asserts with
checkLayers (tests/golden/refsweep.json, built by tests/golden/make_refsweep.py) checked
through a DecodingLayerParser holding every decoder this engine has.

checkLayers(p, want) pins p.Layers()[i] == want[i] up to the first Payload in want
(layers/base_test.go:17-41).  For a DLP with this engine's decoder set that implies:
  * the decoded list starts with want's prefix — with IPv6HopByHop dropped right after IPv6,
    since the DLP's IPv6 consumes the hop-by-hop header itself (ip6.go:239-264);
  * at the first wanted layer this engine has no decoder for, the DLP stops and returns
    UnsupportedLayerType(that layer) (parser.go:308-314) — the same NextLayerType chose it
    in both decode paths.
Frames whose assertion lists a DecodeFailure layer, and the IPv6 jumbogram (whose DLP
decode differs from NewPacket's, golden case ipv6_jumbogram_dlp), are not derivable this
way and are skipped with that reason.
"""
import json
import os

import numpy as np
import pytest

import oracle_ref as O
from conftest import ROOT
from gopacket_amd import layers as L
from gopacket_amd.batch import PacketBatch

DATA = json.load(open(os.path.join(ROOT, "tests", "golden", "refsweep.json")))["cases"]
NAME_TO_LT = {v: k for k, v in L.LAYERTYPE_NAMES.items()}
OURS = {"Ethernet", "Dot1Q", "IPv4", "IPv6", "IPv6HopByHop", "IPv6Routing", "IPv6Fragment",
        "IPv6Destination", "TCP", "UDP", "VXLAN", "Payload", "Fragment", "ICMPv4", "LLC"}
ALL = 0xFFF


def expectation(c):
    """(decoded prefix, stop LayerType or None, exact) the assertion implies, or a skip reason."""
    want = c["asserted"]
    if "DecodeFailure" in want:
        return "asserts a DecodeFailure layer"
    if want[:3] == ["Ethernet", "IPv6", "IPv6HopByHop"] and want[3:4] == ["TCP"]:
        return "IPv6 jumbogram: DLP decode differs from NewPacket (golden ipv6_jumbogram_dlp)"
    seq = []
    for name in want:
        if name == "Payload":  # checkLayers stops matching here
            return seq, None, False
        if name == "IPv6HopByHop" and seq and seq[-1] == "IPv6":
            continue  # consumed inside the DLP's IPv6
        if name not in OURS or name == "IPv6HopByHop":
            return seq, NAME_TO_LT[name], True
        seq.append(name)
    return seq, None, False


CASES = [c for c in DATA if not isinstance(expectation(c), str)]
SKIPPED = [(c["name"], expectation(c)) for c in DATA if isinstance(expectation(c), str)]


def check(c, res, i=0):
    seq, stop, exact = expectation(c)
    got = [L.LAYERTYPE_NAMES[t] for t in res.decoded(i)]
    assert got[:len(seq)] == seq, f"{c['name']}: decoded {got}, reference asserts {c['asserted']}"
    if exact:
        assert got == seq, f"{c['name']}: decoded {got}, want {seq} then {c['asserted'][len(seq):]}"
        assert res.stop_type(i) == stop
        err = res.err(i)
        assert err is not None and str(err) == f"No decoder for layer type {L.LAYERTYPE_NAMES[stop]}"


def test_sweep_covers_the_reference_assertions():
    assert len(DATA) >= 50 and len(CASES) >= 45, (len(DATA), len(CASES), SKIPPED)


@pytest.mark.parametrize("c", CASES, ids=[c["name"] for c in CASES])
def test_oracle_matches_reference_assertion(c):
    b = PacketBatch.from_packets([bytes.fromhex(c["hex"])])
    check(c, O.decode(b, L.LayerTypeEthernet, ALL, 0, ext=True))


@pytest.mark.gpu
@pytest.mark.parametrize("ext", [True, False])
def test_device_matches_reference_assertions(ext):
    from gopacket_amd import parser as P
    b = PacketBatch.from_packets([bytes.fromhex(c["hex"]) for c in CASES])
    p = P.DecodingLayerParser(L.LayerTypeEthernet)
    p._mask = ALL
    dev = p.DecodeBatch(b, ext=ext)
    ref = O.decode(b, L.LayerTypeEthernet, ALL, 0, ext=ext, nthreads=4)
    for f in ("status", "layers", "net_hash", "tp_hash", "csum", "hdr_off"):
        assert np.array_equal(getattr(dev, f), getattr(ref, f)), f
    for i, c in enumerate(CASES):
        check(c, dev, i)
