"""Every decode-error site of the reference, pinned on the CPU oracle (no GPU).

tests/error_sites.py states, per case, the error site and the arguments its format string takes;
here the oracle must return exactly that class / code / arguments, and the texts rebuilt by
gopacket_amd.errors must be the reference's.  The GPU side of the same cases is in
tests/test_parity_gpu.py::test_error_sites_detail_and_texts.
"""
import numpy as np
import pytest

import error_sites as ES
import oracle_ref as O
from gopacket_amd import layers as L
from gopacket_amd.batch import PacketBatch
from gopacket_amd.results import st_class, st_errcode, st_nlayers


@pytest.mark.parametrize("case", ES.CASES, ids=[c[0] for c in ES.CASES])
def test_oracle_error_site(case):
    name, pkt, code, a0, a1 = case
    r = O.decode(PacketBatch.from_packets([pkt]), L.LayerTypeEthernet, 0xFFF, 0, ext=True)
    s = int(r.status[0])
    assert st_class(s) == 2, (name, r.decoded(0), r.err(0))
    assert (st_errcode(s), int(r.ext["err_arg0"][0]), int(r.ext["err_arg1"][0])) == (code, a0, a1), \
        (name, str(r.err(0)))


def test_every_error_site_is_covered():
    assert {c[2] for c in ES.CASES} == set(range(1, 32))


def test_texts_of_formatted_sites():
    """A few texts spelled out in full (the format strings at the cited reference lines)."""
    want = {
        "dot1q_2_bytes": "802.1Q tag length 2 too short",
        "ip4_ihl_15_len_40": "Invalid IP header length > IP length (15 > 40)",
        "ip4_opt_exceeds": "IP option length exceeds remaining IP header size, option type 7 length 8",
        "ip4_opt_le2_type_130": "Invalid IP option type 130 length 1. Must be greater than 2",
        "ip6ext_lt_spec": "Invalid ip6-extension header. Length 8 less than specified length 16",
        "ip6_len0_tcp": "IPv6 length 0, but next header is TCP, not HopByHop",
        "ip6_len0_udp": "IPv6 length 0, but next header is UDP, not HopByHop",
        "ip6_len0_unknown": "IPv6 length 0, but next header is UnknownIPProtocol, not HopByHop",
        "tcp_opt_exceeds": "Invalid TCP option length 8 exceeds remaining 4 bytes",
        "udp_length_5": "UDP packet too small: 5 bytes",
    }
    by = {c[0]: c[1] for c in ES.CASES}
    b = PacketBatch.from_packets([by[k] for k in want])
    r = O.decode(b, L.LayerTypeEthernet, 0xFFF, 0, ext=True)
    assert [str(r.err(i)) for i in range(b.n)] == list(want.values())


@pytest.mark.parametrize("case", ES.DEEP, ids=[c[0] for c in ES.DEEP])
def test_oracle_deep_stacks(case):
    name, pkt, n = case
    r = O.decode(PacketBatch.from_packets([pkt]), L.LayerTypeEthernet, 0xFFF, 0, ext=True)
    s = int(r.status[0])
    assert st_nlayers(s) == min(n, 31) and bool((s >> 3) & 1) == (n > 31), name
    d = r.decoded(0)
    assert d[0] == L.LayerTypeEthernet and d[1:min(n, 32) - 3] == [L.LayerTypeDot1Q] * (min(n, 32) - 4)
    # the BatchResult reads the deep list from a detail array as from ext (same 16-B prefix)
    from gopacket_amd.results import DETAIL_DTYPE
    r.detail = np.zeros(1, DETAIL_DTYPE)
    r.detail["layer_codes"] = r.ext["layer_codes"]
    r.detail["err_arg0"], r.detail["err_arg1"] = r.ext["err_arg0"], r.ext["err_arg1"]
    ext, r.ext = r.ext, None
    assert r.decoded(0) == d
    assert str(r.err(0)) == str(O.decode(PacketBatch.from_packets([pkt]), 17, 0xFFF, 0, ext=True).err(0))
    r.ext = ext
