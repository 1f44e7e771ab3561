"""Generate tests/golden/golden.json and copy the pcap fixtures.

Run in the build container only (it reads /root/reference as text):
    python tests/golden/make_golden.py [/root/reference]

What it writes is DATA: the packet bytes the reference's own tests decode
(extracted from the byte literals / hex strings of its _test.go files), the
pcap files its pcap tests read, and the expected results those tests assert.
Each case records `source` (where the bytes live) and `pinned_by` (the
reference assertion that fixes the expectation).  Where the reference only
asserts a NewPacket result, the DecodingLayerParser expectation is derived from
the cited decoder lines and the case says `derived: ...` — DESIGN.md §Oracle
lists which expectations are asserted by the reference and which are derived.
"""
import json
import os
import re
import shutil
import sys

REF = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))


def go_bytes_at(path, anchor):
    """Bytes of the first `[]byte{...}` literal at/after the line containing `anchor`."""
    src = open(os.path.join(REF, path)).read()
    i = src.index(anchor)
    j = src.index("[]byte{", i) + len("[]byte{")
    depth, k = 1, j
    while depth:
        if src[k] == "{":
            depth += 1
        elif src[k] == "}":
            depth -= 1
        k += 1
    body = re.sub(r"//[^\n]*", "", src[j:k - 1])
    return bytes(int(t, 16) for t in re.findall(r"0x([0-9a-fA-F]{1,2})", body))


def line_of(path, anchor):
    src = open(os.path.join(REF, path)).read()
    return src[:src.index(anchor)].count("\n") + 1


def go_string_bytes(path, anchor):
    """A Go interpreted string literal ("\\x00..." form) assigned at `anchor`."""
    src = open(os.path.join(REF, path)).read()
    i = src.index(anchor)
    q0 = src.index('"', i)
    k = q0 + 1
    out = bytearray()
    while src[k] != '"':
        c = src[k]
        if c == "\\":
            n = src[k + 1]
            if n == "x":
                out.append(int(src[k + 2:k + 4], 16))
                k += 4
                continue
            out.append({"n": 10, "t": 9, "\\": 92, '"': 34, "'": 39, "r": 13}[n])
            k += 2
            continue
        out.append(ord(c))
        k += 1
    return bytes(out)


cases = []


def case(name, data, source, decoders, expect, pinned_by, first="Ethernet", ignore_unsupported=False,
         tail_repeat=None):
    c = {"name": name, "source": source, "first": first, "decoders": decoders,
         "ignore_unsupported": ignore_unsupported, "expect": expect, "pinned_by": pinned_by}
    c["hex"] = data.hex()
    if tail_repeat:
        c["tail_repeat"] = tail_repeat  # {"hex": ..., "count": n}: bytes appended after `hex`
    cases.append(c)


DLP4 = ["Ethernet", "IPv4", "TCP", "Payload"]
FULL = ["Ethernet", "Dot1Q", "IPv4", "IPv6", "IPv6ExtensionSkipper", "TCP", "UDP", "VXLAN",
        "Payload", "Fragment"]

# 1. testSimpleTCPPacket
p = go_bytes_at("layers/decode_test.go", "var testSimpleTCPPacket")
src = f"layers/decode_test.go:{line_of('layers/decode_test.go', 'var testSimpleTCPPacket')}"
case("simple_tcp_dlp4", p, src, DLP4,
     {"decoded": ["Ethernet", "IPv4", "TCP", "Payload"], "err": None, "truncated": False,
      "ip4_csum": 0x555A, "l4_csum": 0, "l4_csum_zeroed": 0x9A8F,
      "ipv4": {"off": 14, "contents": [14, 34], "payload": [34, len(p)], "Length": 420, "Id": 14815,
               "Flags": 2, "TTL": 64, "Protocol": 6, "Checksum": 0x555A,
               "SrcIP": "172.17.81.73", "DstIP": "173.222.254.225"},
      "tcp": {"contents": [34, 66], "payload": [66, len(p)], "SrcPort": 50679, "DstPort": 80,
              "Seq": 0xC57E0E48, "Ack": 0x49074232, "DataOffset": 8, "Window": 0x73,
              "Checksum": 0x9A8F, "options": [[1, 1], [1, 1], [8, 10]]}},
     "layers/decode_test.go:1033-1043 (4 layers, nil err); :406-481 (fields); :484 testSerialization "
     "with ComputeChecksums re-creates the bytes, pinning ip4 checksum 0x555a and TCP 0x9a8f")
case("simple_tcp_full", p, src, FULL,
     {"decoded": ["Ethernet", "IPv4", "TCP", "Payload"], "err": None, "truncated": False,
      "ip4_csum": 0x555A, "l4_csum": 0},
     "same as simple_tcp_dlp4 (the extra registered decoders are never reached)")
case("simple_tcp_no_payload_decoder", p, src, ["Ethernet", "IPv4", "TCP"],
     {"decoded": ["Ethernet", "IPv4", "TCP"], "err": "No decoder for layer type Payload",
      "truncated": False},
     "derived: tcp.go:308-314 next=Payload; parser.go:308-314 UnsupportedLayerType; error text "
     "parser.go:324-326")

# 2. small TCP packet with Ethernet trailer
p = go_bytes_at("layers/decode_test.go", "func TestDecodeSmallTCPPacketHasEmptyPayload")
case("small_tcp_trailer", p,
     f"layers/decode_test.go:{line_of('layers/decode_test.go', 'func TestDecodeSmallTCPPacketHasEmptyPayload')}",
     DLP4, {"decoded": ["Ethernet", "IPv4", "TCP"], "err": None, "truncated": False,
            "ip4_csum": 0x3F9F, "l4_csum": 0, "l4_csum_zeroed": 0xC308},
     "layers/decode_test.go:532-547 (no Payload layer; serialization with checksums re-creates "
     "the bytes); DLP stops on empty payload, layers_decoder.go:71-73")

# 3. VLAN
p = go_bytes_at("layers/decode_test.go", "func TestDecodeVLANPacket")
case("vlan_tcp", p, f"layers/decode_test.go:{line_of('layers/decode_test.go', 'func TestDecodeVLANPacket')}",
     ["Ethernet", "Dot1Q", "IPv4", "TCP", "Payload"],
     {"decoded": ["Ethernet", "Dot1Q", "IPv4", "TCP"], "err": None, "truncated": False,
      "dot1q": {"VLANIdentifier": 0x1F7, "Priority": 0, "DropEligible": False}},
     "layers/decode_test.go:570-571 checkLayers [Ethernet Dot1Q IPv4 TCP]")

# 4. UDP too small (truncated)
p = go_bytes_at("layers/decode_test.go", "func TestDecodeUDPPacketTooSmall")
case("udp_truncated", p,
     f"layers/decode_test.go:{line_of('layers/decode_test.go', 'func TestDecodeUDPPacketTooSmall')}",
     ["Ethernet", "Dot1Q", "IPv4", "UDP", "Payload"],
     {"decoded": ["Ethernet", "Dot1Q", "IPv4", "UDP", "Payload"], "err": None, "truncated": True},
     "layers/decode_test.go:1026-1030 (layers + Truncated)")

# 5. UDP DNS
p = go_bytes_at("layers/udp_test.go", "var testUDPPacketDNS")
src = f"layers/udp_test.go:{line_of('layers/udp_test.go', 'var testUDPPacketDNS')}"
case("udp_dns_unsupported", p, src, ["Ethernet", "IPv4", "UDP", "Payload"],
     {"decoded": ["Ethernet", "IPv4", "UDP"], "err": "No decoder for layer type DNS", "stop": 107,
      "truncated": False,
      "udp": {"SrcPort": 53, "DstPort": 35181, "Length": 210, "Checksum": 30026,
              "contents": [34, 42], "payload": [42, len(p)]}},
     "layers/udp_test.go:61-95 (UDP fields, DNS next layer); ports.go:106 53->DNS; parser.go:308-314")
case("udp_dns_ignore_unsupported", p, src, ["Ethernet", "IPv4", "UDP", "Payload"],
     {"decoded": ["Ethernet", "IPv4", "UDP"], "err": None, "stop": 107, "truncated": False},
     "parser.go:310-312 IgnoreUnsupported => nil", ignore_unsupported=True)

# 6. VXLAN
p = go_bytes_at("layers/vxlan_test.go", "var testPacketVXLAN")
src = f"layers/vxlan_test.go:{line_of('layers/vxlan_test.go', 'var testPacketVXLAN')}"
case("vxlan_icmp_inner", p, src, ["Ethernet", "IPv4", "UDP", "VXLAN", "Payload"],
     {"decoded": ["Ethernet", "IPv4", "UDP", "VXLAN", "Ethernet", "IPv4"],
      "err": "No decoder for layer type ICMPv4", "stop": 19, "truncated": False,
      "vxlan": {"contents": [42, 50], "VNI": 255, "ValidIDFlag": True},
      "inner_ipv4_contents": [64, 84]},
     "layers/vxlan_test.go:53-80 (layer sequence through ICMPv4, VNI 255, I flag); DLP stops at the "
     "unregistered ICMPv4 (parser.go:308-314) with the inner IPv4 in the ip4 object (A11)")

# 7. TCP options MSS + EOL
p = go_bytes_at("layers/tcp_test.go", "var testPacketTCPOptionDecode")
case("tcp_option_mss_eol", p,
     f"layers/tcp_test.go:{line_of('layers/tcp_test.go', 'var testPacketTCPOptionDecode')}", DLP4,
     {"decoded": ["Ethernet", "IPv4", "TCP", "Payload"], "err": None, "truncated": False,
      "tcp": {"options": [[2, 4], [0, 1]], "contents": [34, 62], "payload": [62, 66]}},
     "layers/tcp_test.go:78-103 (options MSS(4)+EOL)")

# 8. IPv4 options / padding and invalid option length (first layer = IPv4)
src_opts = open(os.path.join(REF, "layers/ip4_test.go")).read()
m = re.search(r"func TestIPv4Options", src_opts)
hexes = re.findall(r'packet:\s*"([0-9a-f]+)"', src_opts[m.start():])
ln = line_of("layers/ip4_test.go", "func TestIPv4Options")
blocks = src_opts[m.start():src_opts.index("} {", m.start())].split("packet:")[1:]


def _opts_of(block):
    """(type, length) of every IPv4Option literal in one test-table entry, and its padding."""
    ob = block[block.index("options:"):]
    opts = [[int(t), int(l)] for t, l in
            re.findall(r"OptionType:\s*(\d+),.*?OptionLength:\s*(\d+)", ob.split("padding:")[0], re.S)]
    pad = b""
    if "padding:" in block:
        body = block[block.index("padding:"):]
        body = body[body.index("{") + 1:body.index("}")]
        pad = bytes(int(t, 0) for t in re.findall(r"0x[0-9a-fA-F]+|\d+", body))
    return opts, pad.hex()


expect_opts = [_opts_of(b) for b in blocks]
for k, hx in enumerate(hexes):
    case(f"ipv4_options_{k}", bytes.fromhex(hx), f"layers/ip4_test.go:{ln}", ["IPv4"],
         {"decoded": ["IPv4"], "err": None, "truncated": True,
          "ipv4": {"options": expect_opts[k][0], "padding": expect_opts[k][1]}},
         "layers/ip4_test.go:148-224 (no error, options and padding); Length 40 > data => "
         "Truncated (ip4.go:229-230); empty payload ends the loop", first="IPv4")
hx = re.search(r'hex\.DecodeString\("([0-9a-f]+)"\)', src_opts[src_opts.index("func TestIPv4InvalidOptionLength"):]).group(1)
case("ipv4_invalid_option_length", bytes.fromhex(hx),
     f"layers/ip4_test.go:{line_of('layers/ip4_test.go', 'func TestIPv4InvalidOptionLength')}", ["IPv4"],
     {"decoded": [], "err": "Invalid IP option type 136 length 0. Must be greater than 2",
      "truncated": True},
     "layers/ip4_test.go:135-146 (error expected); text ip4.go:267; Truncated from ip4.go:229-230",
     first="IPv4")

# 9. IPv4 header checksum KATs (also decoded with first = IPv4)
m = re.search(r"func TestChecksum", src_opts)
kats = re.findall(r'header:\s*"([0-9a-f]+)",\s*want:\s*"([0-9a-f]+)"', src_opts[m.start():])
for k, (hdr, want) in enumerate(kats):
    case(f"ip4_checksum_kat_{k}", bytes.fromhex(hdr),
         f"layers/ip4_test.go:{line_of('layers/ip4_test.go', 'func TestChecksum')}", ["IPv4"],
         {"decoded": ["IPv4"], "err": None, "truncated": True, "ip4_csum": int(want, 16)},
         "layers/ip4_test.go:104-133 (checksum KAT)", first="IPv4")

# 10. IPv4 fragment
p = go_bytes_at("layers/decode_test.go", "var testPacketIPv4Fragmented")
case("ipv4_fragment", p,
     f"layers/decode_test.go:{line_of('layers/decode_test.go', 'var testPacketIPv4Fragmented')}",
     ["Ethernet", "IPv4", "UDP", "Fragment", "Payload"],
     {"decoded": ["Ethernet", "IPv4", "Fragment"], "err": None, "truncated": False,
      "ip4_csum": 0xAF37},
     "layers/decode_test.go:1350-1356 (layers; serialization with checksums re-creates the bytes)")

# 11. IPv6 hop-by-hop via DLP with IgnoreUnsupported
p = go_bytes_at("layers/icmp6hopbyhop_test.go", "var icmp6HopByHopData")
case("ipv6_hopbyhop_icmp6", p,
     f"layers/icmp6hopbyhop_test.go:{line_of('layers/icmp6hopbyhop_test.go', 'var icmp6HopByHopData')}",
     ["Ethernet", "IPv6", "Payload"],
     {"decoded": ["Ethernet", "IPv6"], "err": None, "stop": 57, "truncated": True,
      "ipv6": {"contents": [14, 54], "payload": [62, len(p)]}},
     "layers/icmp6hopbyhop_test.go:55-85 (DLP, IgnoreUnsupported, nil error; HBH consumed inside "
     "IPv6, next header ICMPv6 = 58); ICMPv6 is outside this engine's decoder set, so the loop "
     "stops at it (parser.go:310-312). Truncated is derived (the test does not read it): Length 136 "
     "counts the 8-byte HBH header that ip6.go:262 already skipped, so pEnd > len(Payload) at "
     "ip6.go:270-273", ignore_unsupported=True)

# 12. IPv6 jumbogram (payload "payload" x 9996)
head = go_string_bytes("layers/decode_test.go", "dataStr := ")
src = f"layers/decode_test.go:{line_of('layers/decode_test.go', 'func TestDecodeIPv6Jumbogram')}"
rep = {"hex": b"payload".hex(), "count": 9996}
case("ipv6_jumbogram_dlp", head, src, ["Ethernet", "IPv6", "IPv6ExtensionSkipper", "TCP", "Payload"],
     {"decoded": ["Ethernet", "IPv6"], "err": "Invalid TCP data offset 0 < 5", "truncated": False},
     "derived: ip6.go:249-256 keeps the DLP payload starting at the hop-by-hop header (NewPacket, "
     "which the reference test uses, reads the HBH layer's payload instead), so TCP decodes the "
     "HBH bytes and fails at tcp.go:260-261", tail_repeat=rep)
case("ipv6_jumbogram_dlp_truncated", head, src,
     ["Ethernet", "IPv6", "IPv6ExtensionSkipper", "TCP", "Payload"],
     {"decoded": ["Ethernet", "IPv6"], "err": "Invalid TCP data offset 0 < 5", "truncated": True,
      "drop_last": 1},
     "layers/decode_test.go:1010-1015 (one byte short => Truncated, ip6.go:251-253); rest derived "
     "as ipv6_jumbogram_dlp", tail_repeat=rep)

# 13. UDP checksum constants (tcpip_test.go), packets as the tests serialize them
def ip4_csum(h):
    s = sum((h[i] << 8) | h[i + 1] for i in range(0, len(h), 2))
    while s > 0xFFFF:
        s = (s >> 16) + (s & 0xFFFF)
    return (~s) & 0xFFFF


ip = bytearray(bytes.fromhex("4500001c00000000401100" "00" "c0000201c6336401"))
ip[10:12] = b"\x00\x00"
ip[10:12] = ip4_csum(bytes(ip)).to_bytes(2, "big")
udp = bytes.fromhex("3039270f0008bc5f")
case("udp4_checksum_kat", bytes(ip) + udp,
     f"layers/tcpip_test.go:{line_of('layers/tcpip_test.go', 'func TestIPv4UDPChecksum')}",
     ["IPv4", "UDP", "Payload"],
     {"decoded": ["IPv4", "UDP"], "err": None, "truncated": False, "l4_csum": 0,
      "l4_csum_zeroed": 0xBC5F},
     "layers/tcpip_test.go:16,55-93 (Wireshark-confirmed UDP checksum 0xbc5f for 192.0.2.1 -> "
     "198.51.100.1, 12345 -> 9999, TTL 64, empty payload)", first="IPv4")
v6 = bytes.fromhex("60000000" "0010" "3c" "40" "20010db8000000000000000000000001"
                   "20010db8000000000000000000000002")
dst = bytes.fromhex("1100010400000000")
udp = bytes.fromhex("3039270f00084d21")
case("udp6_dstopts_checksum_kat", v6 + dst + udp,
     f"layers/tcpip_test.go:{line_of('layers/tcpip_test.go', 'func TestIPv6UDPChecksumWithIPv6DstOpts')}",
     ["IPv6", "IPv6ExtensionSkipper", "UDP", "Payload"],
     {"decoded": ["IPv6", "IPv6Destination", "UDP"], "err": None, "truncated": False, "l4_csum": 0,
      "l4_csum_zeroed": 0x4D21},
     "layers/tcpip_test.go:17,95-137 (Wireshark-confirmed 0x4d21; DstOpts with one PadN(4) option)",
     first="IPv6")

# IPv6 destination options (ip6_test.go): IPv6Destination has DecodeFromBytes but no CanDecode /
# NextLayerType (ip6.go:633-667), so it is not a DecodingLayer; a DLP reaches it through
# IPv6ExtensionSkipper (CanDecode LayerClassIPv6Extension, layertypes.go:193-198)
p = go_bytes_at("layers/ip6_test.go", "var testPacketIPv6Destination0")
src = f"layers/ip6_test.go:{line_of('layers/ip6_test.go', 'var testPacketIPv6Destination0')}"
case("ipv6_destination0", p, src, ["IPv6", "IPv6ExtensionSkipper", "Payload"],
     {"decoded": ["IPv6", "IPv6Destination"], "err": None, "truncated": False,
      "ipv6": {"contents": [0, 40], "payload": [40, 48]}},
     "layers/ip6_test.go:244-300 (checkLayers [IPv6 IPv6Destination]; IPv6 Length 8, NextHeader "
     "60, HopLimit 64; the destination header's Contents = bytes 40..48, NextHeader NoNextHeader, "
     "empty Payload); DLP: the skipper consumes the header (ip6.go:443-461), next = Payload "
     "(enums.go IPProtocolNoNextHeader), and the empty payload ends the loop "
     "(layers_decoder.go:71-73)", first="IPv6")
case("ipv6_destination0_unregistered", p, src, ["IPv6", "Payload"],
     {"decoded": ["IPv6"], "err": "No decoder for layer type IPv6Destination", "stop": 49,
      "truncated": False},
     "derived: without IPv6ExtensionSkipper the loop stops at LayerTypeIPv6Destination "
     "(parser.go:308-314)", first="IPv6")

# 15. ICMPv4 and LLC decoders
p = go_bytes_at("layers/vxlan_test.go", "var testPacketVXLAN")
src = f"layers/vxlan_test.go:{line_of('layers/vxlan_test.go', 'var testPacketVXLAN')}"
case("vxlan_icmp_full", p, src, ["Ethernet", "IPv4", "UDP", "VXLAN", "ICMPv4", "Payload"],
     {"decoded": ["Ethernet", "IPv4", "UDP", "VXLAN", "Ethernet", "IPv4", "ICMPv4", "Payload"],
      "err": None, "truncated": False,
      "vxlan": {"contents": [42, 50], "VNI": 255, "ValidIDFlag": True},
      "icmpv4": {"contents": [84, 92], "payload": [92, len(p)], "Type": 8, "Code": 0},
      "inner_ipv4_contents": [64, 84]},
     "layers/vxlan_test.go:53-80 (checkLayers [Ethernet IPv4 UDP VXLAN Ethernet IPv4 ICMPv4 "
     "Payload], VNI 255, I flag); the inner IPv4 stays in the reused ip4 object (A11)")
p = go_bytes_at("layers/decode_test.go", "var testICMP = ")
src = f"layers/decode_test.go:{line_of('layers/decode_test.go', 'var testICMP = ')}"
case("icmp4_unreachable", p, src, ["Ethernet", "IPv4", "ICMPv4", "TCP", "UDP", "Payload"],
     {"decoded": ["Ethernet", "IPv4", "ICMPv4", "Payload"], "err": None, "truncated": False,
      "ip4_csum": 0xD7A7,
      "icmpv4": {"contents": [34, 42], "payload": [42, 70], "Type": 3, "Code": 13,
                 "Checksum": 0x946E, "Id": 0, "Seq": 0}},
     "layers/decode_test.go:1094-1100 (checkLayers [Ethernet IPv4 ICMPv4 Payload]; "
     "testSerialization re-creates the bytes, pinning the IPv4 checksum 0xd7a7); icmp4.go:220-231 "
     "fields")
case("icmp4_truncated", p[:14 + 20 + 5], src, ["Ethernet", "IPv4", "ICMPv4", "Payload"],
     {"decoded": ["Ethernet", "IPv4"], "err": "ICMP layer less then 8 bytes for ICMPv4 packet",
      "truncated": True},
     "derived: ip4.go:228-230 (Length 56 > 25 captured: Truncated), icmp4.go:221-223 (< 8 bytes: "
     "SetTruncated + error)")
p = go_bytes_at("layers/decode_test.go", "testSTPpacket := ")
src = f"layers/decode_test.go:{line_of('layers/decode_test.go', 'testSTPpacket := ')}"
case("stp_llc", p, src, ["Ethernet", "LLC", "Payload"],
     {"decoded": ["Ethernet", "LLC"], "err": "No decoder for layer type STP", "stop": 121,
      "truncated": False,
      "llc": {"contents": [14, 17], "payload": [17, 52], "DSAP": 0x42, "SSAP": 0x42, "Control": 3}},
     "layers/decode_test.go:1376-1380 (checkLayers [Ethernet LLC STP]); ethernet.go:50-57 trims the "
     "payload to the 802.3 length 38; llc.go:40-50 one-byte control; STP is not registered in "
     "this DLP (parser.go:308-314)")
case("stp_llc_ignore", p, src, ["Ethernet", "LLC", "Payload"],
     {"decoded": ["Ethernet", "LLC"], "err": None, "stop": 121, "truncated": False},
     "as stp_llc with IgnoreUnsupported (parser.go:310-312)", ignore_unsupported=True)
p = go_bytes_at("layers/decode_test.go", "func TestDecodeNortelDiscovery")
src = f"layers/decode_test.go:{line_of('layers/decode_test.go', 'func TestDecodeNortelDiscovery')}"
case("nortel_llc_snap", p, src, ["Ethernet", "LLC", "Payload"],
     {"decoded": ["Ethernet", "LLC"], "err": "No decoder for layer type SNAP", "stop": 23,
      "truncated": False,
      "llc": {"contents": [14, 17], "payload": [17, 33], "DSAP": 0xAA, "SSAP": 0xAA, "Control": 3}},
     "layers/decode_test.go:970-974 (checkLayers [Ethernet LLC SNAP NortelDiscovery]); the DLP "
     "has no SNAP decoder, so it stops there (parser.go:308-314)")

# 14. pcap fixtures
for fn in ("test_ethernet.pcap", "test_dns.pcap"):
    shutil.copyfile(os.path.join(REF, "pcap", fn), os.path.join(OUT, fn))

meta = {
    "generated_by": "tests/golden/make_golden.py",
    "reference": "google/gopacket (read as text)",
    "pcaps": {
        "test_ethernet.pcap": {"num": 10, "caplens": [74, 74, 66, 138, 66, 89, 66, 421, 66, 66],
                               "expected_layers_contain": ["Ethernet", "IPv4", "TCP"],
                               "pinned_by": "pcap/pcap_test.go:64-71,111-115"},
        "test_dns.pcap": {"num": 10, "expected_layers_contain": ["Ethernet", "IPv4", "UDP", "DNS"],
                          "pinned_by": "pcap/pcap_test.go:72-80,111-115"},
    },
    "udp6_jumbogram_checksum_kat": {
        "src": "20010db8000000000000000000000001", "dst": "20010db8000000000000000000000002",
        "udp_header": "3039270f00000000", "payload_byte": 0xFE, "payload_len": 65536,
        "want": 0xCDA8,
        "pinned_by": "layers/tcpip_test.go:18,139-185 (computeChecksum over UDP header with "
                     "Length 0 + 65536 x 0xfe, IPv6 pseudo-header, length >> 16 term)"},
    "cases": cases,
}
with open(os.path.join(OUT, "golden.json"), "w") as f:
    json.dump(meta, f, indent=1)
print(f"{len(cases)} cases -> {OUT}/golden.json")
