"""Generate tests/golden/errpath.json: nested stacks whose later layer fails after the parser's
reused objects were already filled — the error-path state of the layer objects.

    python tests/golden/make_errpath.py

Why: a DecodingLayerParser holds ONE object per layer kind (layers_decoder.go:61-78), and a
failing DecodeFromBytes assigns some fields before it returns its error:
  * IPv4 — every header field, SrcIP/DstIP and BaseLayer{Contents: data} (Payload nil) before
    the Length / IHL checks (ip4.go:195-210, errors :220-232); the header split
    (Contents = data[:IHL*4], Payload = the rest after the Length trim) before the option errors
    (:235-236, errors :257-267);
  * IPv6 — fields, SrcIP/DstIP and BaseLayer{data[:40], data[40:]} before the hop-by-hop and
    length errors (ip6.go:226-235, errors :240-267);
  * TCP — ports .. Urgent before the data-offset check (tcp.go:234-261, BaseLayer untouched);
    Contents = data, Payload = nil on the offset overrun (:264-268); the header split before
    the option errors (:270-271, errors :286-295);
  * UDP — ports, Length, Checksum and BaseLayer{Contents: data[:8]} before "too small"
    (udp.go:35-53);
  * LLC — DSAP .. Control before the second length check (llc.go:35-43).
So after e.g. [Eth, IPv4, UDP, VXLAN, Eth, IPv4(error)] the single ip4 object describes the
FAILED inner header: ip4.NetworkFlow(), checksum(ip4.Contents) and the pseudo-header of
udp.SetNetworkLayerForChecksum(&ip4) all read it.

Each case below is built from a packet the reference's own tests decode (tests/golden/
golden.json: vxlan_test.go's VXLAN/ICMP frame, decode_test.go's testSimpleTCPPacket) with one
header field changed, or assembled from plain headers.  The expectations are written out BY
HAND per case as the offsets the Go code above leaves in each object (`net`, `tp`, `ip4`, `l4`,
`err_*`); tests/errpath_cases.py turns them into result words with its own small FNV /
checksum code.  No Go toolchain exists in this image, so these are derived from the cited
source lines, not from running the reference: "derived", not reference-asserted.
"""
import json
import os
import struct

HERE = os.path.dirname(os.path.abspath(__file__))


def golden(name):
    with open(os.path.join(HERE, "golden.json")) as f:
        for c in json.load(f)["cases"]:
            if c["name"] == name:
                return bytearray.fromhex(c["hex"])
    raise KeyError(name)


def be16(p, off, v):
    p[off:off + 2] = struct.pack(">H", v)


VX = golden("vxlan_icmp_full")     # Eth 0 | IPv4 14 | UDP 34 (len 114) | VXLAN 42 | Eth 50 | IPv4 64 (len 84) | ICMPv4 84 | 148
TCP = golden("simple_tcp_dlp4")    # Eth 0 | IPv4 14 (len 420) | TCP 34 (doff 8) | payload 66 | 434
ALL = ["Ethernet", "Dot1Q", "IPv4", "IPv6", "IPv6ExtensionSkipper", "TCP", "UDP", "VXLAN",
       "Payload", "Fragment", "ICMPv4", "LLC"]
VX_DECODED_TO_INNER_ETH = ["Ethernet", "IPv4", "UDP", "VXLAN", "Ethernet"]
VX_DECODED_TO_INNER_IP4 = VX_DECODED_TO_INNER_ETH + ["IPv4"]

cases = []


def case(name, pkt, decoded, err, *, truncated=False, net=None, tp=None, ip4=None, l4=None,
         err_obj=None, err_wrote=0, err_off=0, err_obj_rec=None, tables=None, why=""):
    """net/tp: [kind, offset of the header whose addresses/ports the flow reads];
    ip4: [c0, c1] of ip4.Contents (IPv4 in decoded); l4: [a, b, net kind, net offset, proto]
    = computeChecksum(pkt[a:b]) with that network object's pseudo-header;
    err_obj_rec: [[c0, c1], [p0, p1]] of the failing object's BaseLayer when err_wrote == 2."""
    cases.append(dict(name=name, hex=bytes(pkt).hex(), first="Ethernet", decoders=ALL,
                      tables=tables or {}, why=why,
                      expect=dict(decoded=decoded, err=err, truncated=truncated, net=net, tp=tp,
                                  ip4=ip4, l4=l4, err_obj=err_obj, err_wrote=err_wrote,
                                  err_off=err_off, err_obj_rec=err_obj_rec)))


# ---- VXLAN (vxlan_test.go frame) with the INNER IPv4 header broken: the ip4 object is the
# inner header as far as the failing call got; the outer UDP checksum takes its pseudo-header
p = VX.copy(); be16(p, 66, 10)
case("vx_inner_ip4_length_lt20", p, VX_DECODED_TO_INNER_ETH,
     "Invalid (too small) IP length (10 < 20)",
     net=["IPv4", 64], tp=["UDP", 34], ip4=[64, 148], l4=[34, 148, "IPv4", 64, 17],
     err_obj="IPv4", err_wrote=2, err_off=64, err_obj_rec=[[64, 148], [148, 148]],
     why="ip4.go:210,220-221: Contents = all 84 bytes of data, Payload nil")
p = VX.copy()[:147]; be16(p, 66, 10)
case("vx_inner_ip4_length_lt20_odd", p, VX_DECODED_TO_INNER_ETH,
     "Invalid (too small) IP length (10 < 20)", truncated=True,
     net=["IPv4", 64], tp=["UDP", 34], ip4=[64, 147], l4=[34, 147, "IPv4", 64, 17],
     err_obj="IPv4", err_wrote=2, err_off=64, err_obj_rec=[[64, 147], [147, 147]],
     why="83-byte Contents: checksum(ip4.Contents) would index past the end (ip4.go:165-167), "
         "so no IPv4 checksum value; outer IPv4/UDP truncated by the cut")
p = VX.copy(); p[64] = 0x44
case("vx_inner_ip4_ihl_lt5", p, VX_DECODED_TO_INNER_ETH,
     "Invalid (too small) IP header length (4 < 5)",
     net=["IPv4", 64], tp=["UDP", 34], ip4=[64, 148], l4=[34, 148, "IPv4", 64, 17],
     err_obj="IPv4", err_wrote=2, err_off=64, err_obj_rec=[[64, 148], [148, 148]])
p = VX.copy(); p[64] = 0x4F; be16(p, 66, 40)
case("vx_inner_ip4_ihl_gt_length", p, VX_DECODED_TO_INNER_ETH,
     "Invalid IP header length > IP length (15 > 40)",
     net=["IPv4", 64], tp=["UDP", 34], ip4=[64, 148], l4=[34, 148, "IPv4", 64, 17],
     err_obj="IPv4", err_wrote=2, err_off=64, err_obj_rec=[[64, 148], [148, 148]])
p = VX.copy()[:114]; p[64] = 0x4F; be16(p, 66, 200)
case("vx_inner_ip4_hdr_trunc", p, VX_DECODED_TO_INNER_ETH,
     "Not all IP header bytes available", truncated=True,
     net=["IPv4", 64], tp=["UDP", 34], ip4=[64, 114], l4=[34, 114, "IPv4", 64, 17],
     err_obj="IPv4", err_wrote=2, err_off=64, err_obj_rec=[[64, 114], [114, 114]],
     why="ip4.go:229-232: 50 bytes < IHL*4 = 60")
p = VX.copy(); p[64] = 0x46; p[84] = 0x88; p[85] = 0x00
case("vx_inner_ip4_bad_option", p, VX_DECODED_TO_INNER_ETH,
     "Invalid IP option type 136 length 0. Must be greater than 2",
     net=["IPv4", 64], tp=["UDP", 34], ip4=[64, 88], l4=[34, 148, "IPv4", 64, 17],
     err_obj="IPv4", err_wrote=2, err_off=64, err_obj_rec=[[64, 88], [88, 148]],
     why="ip4.go:235-236 before :266-267: the header split stands")
# ---- the inner transport broken
p = VX.copy(); p[73] = 17; be16(p, 88, 5)
case("vx_inner_udp_len_too_small", p, VX_DECODED_TO_INNER_IP4, "UDP packet too small: 5 bytes",
     net=["IPv4", 64], tp=["UDP", 84], ip4=[64, 84], l4=[84, 92, "IPv4", 64, 17],
     err_obj="UDP", err_wrote=2, err_off=84, err_obj_rec=[[84, 92], [92, 92]],
     why="udp.go:35-41,52-53: the udp object holds the inner ports and Contents = data[:8]")
p = VX.copy(); p[73] = 6; p[96] = 0x30
case("vx_inner_tcp_doff_lt5_not_decoded", p, VX_DECODED_TO_INNER_IP4, "Invalid TCP data offset 3 < 5",
     net=["IPv4", 64], tp=["UDP", 34], ip4=[64, 84], l4=[34, 148, "IPv4", 64, 17],
     err_obj="TCP", err_wrote=1, err_off=84,
     why="TCP is not in decoded: its object feeds no output (its BaseLayer would be stale)")


# ---- VXLAN carried over TCP (RegisterTCPPortLayerType(4789, VXLAN)): TCP in decoded, then
# the inner TCP fails — the tcp object mixes inner ports with outer (or inner) BaseLayer
def tcp_vxlan(inner_tcp: bytes) -> bytearray:
    eth = bytes(TCP[:12]) + b"\x08\x00"
    inner_ip = bytearray(TCP[14:34]); be16(inner_ip, 2, 20 + len(inner_tcp))
    inner = bytes(TCP[:14]) + bytes(inner_ip) + inner_tcp
    vx = bytes([0x08, 0, 0, 0, 0, 0, 0x2A, 0])
    outer_tcp = bytearray(20); be16(outer_tcp, 0, 40000); be16(outer_tcp, 2, 4789)
    outer_tcp[12] = 0x50; outer_tcp[13] = 0x18
    outer_ip = bytearray(TCP[14:34]); be16(outer_ip, 2, 20 + 20 + 8 + len(inner))
    return bytearray(eth + bytes(outer_ip) + bytes(outer_tcp) + vx + inner)


# Eth 0 | IPv4 14 | TCP 34 (doff 5) | VXLAN 54 | Eth 62 | IPv4 76 | TCP 96 | ...
VXT = {"tcp_port": {"4789": "VXLAN"}}
INNER = bytes(TCP[34:66]) + b"GET / HTTP/1.1\r\n"  # inner TCP header 32 B + 16 B payload
TV_DECODED = ["Ethernet", "IPv4", "TCP", "VXLAN", "Ethernet", "IPv4"]
t = bytearray(INNER); t[12] = 0x30
p = tcp_vxlan(bytes(t))
case("tcpvx_inner_tcp_doff_lt5", p, TV_DECODED, "Invalid TCP data offset 3 < 5", tables=VXT,
     net=["IPv4", 76], tp=["TCP", 96], ip4=[76, 96], l4=[34, len(p), "IPv4", 76, 6],
     err_obj="TCP", err_wrote=1, err_off=96,
     why="tcp.go:234-261: inner ports, outer Contents/Payload: TransportFlow and ComputeChecksum "
         "read different packets' TCP headers")
t = bytearray(INNER); t[12] = 0xF0
p = tcp_vxlan(bytes(t))
case("tcpvx_inner_tcp_doff_overrun", p, TV_DECODED, "TCP data offset greater than packet length",
     truncated=True, tables=VXT,
     net=["IPv4", 76], tp=["TCP", 96], ip4=[76, 96], l4=[96, len(p), "IPv4", 76, 6],
     err_obj="TCP", err_wrote=2, err_off=96, err_obj_rec=[[96, len(p)], [len(p), len(p)]],
     why="tcp.go:264-268: Contents = data, Payload = nil")
t = bytearray(INNER); t[12] = 0x60; t[20] = 2; t[21] = 1
p = tcp_vxlan(bytes(t))
case("tcpvx_inner_tcp_bad_option", p, TV_DECODED, "Invalid TCP option length 1 < 2", tables=VXT,
     net=["IPv4", 76], tp=["TCP", 96], ip4=[76, 96], l4=[96, len(p), "IPv4", 76, 6],
     err_obj="TCP", err_wrote=2, err_off=96, err_obj_rec=[[96, 120], [120, len(p)]],
     why="tcp.go:270-271 before :291-292")
t = bytearray(INNER); t[12] = 0x60; t[20] = 3; t[21] = 9
p = tcp_vxlan(bytes(t))
case("tcpvx_inner_tcp_option_exceeds", p, TV_DECODED, "Invalid TCP option length 9 exceeds remaining 4 bytes",
     truncated=True, tables=VXT,
     net=["IPv4", 76], tp=["TCP", 96], ip4=[76, 96], l4=[96, len(p), "IPv4", 76, 6],
     err_obj="TCP", err_wrote=2, err_off=96, err_obj_rec=[[96, 120], [120, len(p)]])


# ---- IPv4-in-IPv4 (IPProtocol 4 -> IPv4) and IPv6-in-IPv6 (41 -> IPv6)
def ip4ip4(inner: bytes) -> bytearray:
    outer = bytearray(TCP[14:34]); outer[9] = 4; be16(outer, 2, 20 + len(inner))
    return bytearray(bytes(TCP[:14]) + bytes(outer) + inner)


inner = bytearray(TCP[14:]); be16(inner, 2, 10)
p = ip4ip4(bytes(inner))
case("ip4ip4_inner_length_lt20", p, ["Ethernet", "IPv4"], "Invalid (too small) IP length (10 < 20)",
     net=["IPv4", 34], ip4=[34, len(p)], err_obj="IPv4", err_wrote=2, err_off=34,
     err_obj_rec=[[34, len(p)], [len(p), len(p)]])
# a More-Fragments inner header with a bad option: the ip4 object the application would hand to
# ip4defrag is the inner one (DefragIPv4(&ip4) sees the inner flags and offset)
inner = bytearray(24 + 8)
inner[0] = 0x46; be16(inner, 2, 32); be16(inner, 4, 0x1234); be16(inner, 6, 0x2000 | 5)
inner[8] = 64; inner[9] = 17; inner[12:16] = bytes([10, 0, 0, 1]); inner[16:20] = bytes([10, 0, 0, 2])
inner[20] = 0x88; inner[21] = 0
p = ip4ip4(bytes(inner))
case("ip4ip4_inner_mf_bad_option", p, ["Ethernet", "IPv4"],
     "Invalid IP option type 136 length 0. Must be greater than 2",
     net=["IPv4", 34], ip4=[34, 58], err_obj="IPv4", err_wrote=2, err_off=34,
     err_obj_rec=[[34, 58], [58, 66]])


def ip6(nh: int, length: int, src: int, dst: int) -> bytes:
    return (bytes([0x60, 0, 0, 0]) + struct.pack(">HBB", length, nh, 64) + bytes([0x20, 0x01] + [0] * 13 + [src])
            + bytes([0x20, 0x01] + [0] * 13 + [dst]))


ETH6 = bytes(TCP[:12]) + b"\x86\xdd"
body = bytes(TCP[34:54])
p = bytearray(ETH6 + ip6(41, 40 + 20, 1, 2) + ip6(6, 0, 3, 4) + body)
case("ip6ip6_inner_len0", p, ["Ethernet", "IPv6"], "IPv6 length 0, but next header is TCP, not HopByHop",
     net=["IPv6", 54], err_obj="IPv6", err_wrote=2, err_off=54, err_obj_rec=[[54, 94], [94, 114]],
     why="ip6.go:226-235 then :266-267")
p = bytearray(ETH6 + ip6(41, 40 + 8, 1, 2) + ip6(0, 8, 5, 6) + bytes([6, 3, 0, 0, 0, 0, 0, 0]))
case("ip6ip6_inner_hbh_short", p, ["Ethernet", "IPv6"],
     "Invalid ip6-extension header. Length 8 less than specified length 32",
     net=["IPv6", 54], err_obj="IPv6", err_wrote=2, err_off=54, err_obj_rec=[[54, 94], [94, 102]],
     why="the hop-by-hop error comes after ip6.go:226-235")
outer6 = ip6(4, 40, 1, 2)
inner4 = bytearray(TCP[14:34]); be16(inner4, 2, 12)
p = bytearray(ETH6 + outer6 + bytes(inner4) + bytes(20))
case("ip4in6_inner_bad_not_decoded", p, ["Ethernet", "IPv6"], "Invalid (too small) IP length (12 < 20)",
     net=["IPv6", 14], err_obj="IPv4", err_wrote=2, err_off=54, err_obj_rec=[[54, 94], [94, 94]],
     why="IPv4 is not in decoded: no IPv4 checksum; the net flow stays the IPv6 one")

# ---- the failing object is not in decoded at all (ext records only)
p = bytearray(TCP[:34 + 20]); p[16:18] = struct.pack(">H", 40); p[23] = 17; be16(p, 38, 5)
case("udp_len_too_small_top", p, ["Ethernet", "IPv4"], "UDP packet too small: 5 bytes",
     net=["IPv4", 14], ip4=[14, 34], err_obj="UDP", err_wrote=2, err_off=34,
     err_obj_rec=[[34, 42], [42, 42]])
p = bytearray(TCP[:34 + 20]); p[16:18] = struct.pack(">H", 40); p[46] = 0x30
case("tcp_doff_lt5_top", p, ["Ethernet", "IPv4"], "Invalid TCP data offset 3 < 5",
     net=["IPv4", 14], ip4=[14, 34], err_obj="TCP", err_wrote=1, err_off=34)
p = bytearray(bytes(TCP[:12]) + b"\x00\x03" + bytes([0x42, 0x42, 0x00]))
case("llc_two_byte_control_short", p, ["Ethernet"], "LLC header too small",
     err_obj="LLC", err_wrote=1, err_off=14, why="llc.go:35-43: DSAP .. Control assigned, then the error")
p = bytearray(bytes(TCP[:12]) + b"\x08\x00" + bytes(12))
case("ip4_too_short_writes_nothing", p, ["Ethernet"], "Invalid ip4 header. Length 12 less than 20",
     truncated=True, err_obj="IPv4", err_wrote=0, err_off=14, why="ip4.go:189-191 precede every assignment")

with open(os.path.join(HERE, "errpath.json"), "w") as f:
    json.dump({"generated_by": "tests/golden/make_errpath.py", "cases": cases}, f, indent=1)
print(f"{len(cases)} cases")
