"""DecodingLayerContainer mirror (parser.go:54-177) on the CPU: Put / Decoder semantics of the
three containers, the engine's decoder-kind mask derived from a container, and the parser's
SetDecodingLayerContainer / AddDecodingLayer bookkeeping (no GPU calls)."""
import pytest

from gopacket_amd import layers as L
from gopacket_amd import parser as P


@pytest.mark.parametrize("kind", [P.DecodingLayerSparse, P.DecodingLayerArray, P.DecodingLayerMap])
def test_put_and_decoder(kind):
    eth, ip4, ext = P.Ethernet(), P.IPv4(), P.IPv6ExtensionSkipper()
    c = kind()
    for d in (eth, ip4, ext):
        c = c.Put(d)
    assert c.Decoder(L.LayerTypeEthernet) == (eth, True)
    assert c.Decoder(L.LayerTypeIPv4) == (ip4, True)
    for t in L.LayerClassIPv6Extension:  # ip6.go:454-456: one decoder for 46..49
        assert c.Decoder(t) == (ext, True)
    assert c.Decoder(L.LayerTypeTCP) == (None, False)
    assert c.Decoder(10 ** 6) == (None, False)
    ip4b = P.IPv4()  # a later Put of the same type replaces the decoder (parser.go:84-86,121-125,153-156)
    c = c.Put(ip4b)
    assert c.Decoder(L.LayerTypeIPv4) == (ip4b, True)
    assert c.engine_mask() == P.DEC_ETHERNET | P.DEC_IPV4 | P.DEC_IPV6_EXT


def test_partial_kind_has_no_engine_equivalent():
    m = P.DecodingLayerMap().Put(P.Ethernet())
    m.dl[L.LayerTypeIPv6HopByHop] = P.IPv6ExtensionSkipper()  # 46 only, not 47..49
    with pytest.raises(ValueError, match="IPv6ExtensionSkipper"):
        m.engine_mask()


def test_parser_container_bookkeeping():
    p = P.NewDecodingLayerParser(L.LayerTypeEthernet, P.Ethernet(), P.IPv4(), P.TCP())
    assert isinstance(p._dlc, P.DecodingLayerMap)  # parser.go:226: the default container
    assert p.decoders == P.DEC_ETHERNET | P.DEC_IPV4 | P.DEC_TCP
    p.AddDecodingLayer(P.UDP())
    assert p.decoders & P.DEC_UDP and p._dlc.Decoder(L.LayerTypeUDP)[1]
    s = P.DecodingLayerSparse().Put(P.Ethernet()).Put(P.IPv6())
    p.SetDecodingLayerContainer(s)  # parser.go:236-242: replaces every decoder
    assert p.decoders == P.DEC_ETHERNET | P.DEC_IPV6
    p.AddDecodingLayer("VXLAN")
    assert p.decoders == P.DEC_ETHERNET | P.DEC_IPV6 | P.DEC_VXLAN
    assert s.Decoder(L.LayerTypeVXLAN)[1]  # AddDecodingLayer Puts into the parser's container


def test_endpoint_and_flow_constructors():
    """flows.go:53-55,89-97,151-157,214-224 on the host: NewEndpoint / NewFlow bounds (a raw
    longer than MaxEndpointSize panics in the reference), FlowFromEndpoints' type check and error
    text, LessThan's order (type first, then the raw bytes lexicographically), Reverse, String."""
    import pytest
    from gopacket_amd.results import (EndpointIPv4, EndpointTCPPort, FlowFromEndpoints, MaxEndpointSize,
                                      NewEndpoint, NewFlow)
    assert MaxEndpointSize == 16
    with pytest.raises(ValueError, match="greater than MaxEndpointSize"):
        NewEndpoint(EndpointIPv4, bytes(17))
    with pytest.raises(ValueError, match="greater than MaxEndpointSize"):
        NewFlow(EndpointIPv4, bytes(4), bytes(17))
    a, b = NewEndpoint(EndpointIPv4, bytes([10, 0, 0, 1])), NewEndpoint(EndpointIPv4, bytes([10, 0, 0, 2]))
    f, err = FlowFromEndpoints(a, b)
    assert err is None and f.Src() == a and f.Dst() == b and f.String() == "10.0.0.1->10.0.0.2"
    assert f.Reverse().Src() == b and f.Reverse().Reverse() == f
    _, err = FlowFromEndpoints(a, NewEndpoint(EndpointTCPPort, b"\x00\x50"))
    assert str(err) == "Mismatched endpoint types: 1->4"
    assert a.LessThan(b) and not b.LessThan(a) and not a.LessThan(a)
    assert b.LessThan(NewEndpoint(EndpointTCPPort, b"\x00\x01"))  # type first
    assert NewEndpoint(EndpointIPv4, b"\x0a").LessThan(a)  # a prefix sorts first (bytes.Compare)
