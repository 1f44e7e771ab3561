"""One packet per decode-error site of the reference (the 31 GPD_E_* codes of include/gpd.h), each
with the error arguments its `return fmt.Errorf(...)` formats, stated by hand from the cited
reference lines, plus stacks deeper than the core record's 12 layers.

These are test vectors, not reference fixtures: the reference's tests assert only a few of these
texts.  tests/test_error_sites.py pins every case against the C oracle (CPU); the GPU tests then
check the kernel's detail records (gpd.h gpd_detail) and the error texts rebuilt from them.
"""
from __future__ import annotations

import struct

MAC = bytes.fromhex("001122334455") + bytes.fromhex("66778899aabb")


def eth(ethertype: int, payload: bytes) -> bytes:
    return MAC + struct.pack(">H", ethertype) + payload


def ip4(payload: bytes, proto: int = 6, ihl: int = 5, length=None, opts: bytes = b"",
        flags_frag: int = 0) -> bytes:
    hdr = bytearray(20) + bytearray(opts)
    hdr[0] = 0x40 | ihl
    total = len(hdr) + len(payload) if length is None else length
    struct.pack_into(">HHHBB", hdr, 2, total, 0x1234, flags_frag, 64, proto)
    hdr[12:16] = bytes([10, 0, 0, 1])
    hdr[16:20] = bytes([10, 0, 0, 2])
    return bytes(hdr) + payload


def ip6(payload: bytes, nh: int = 6, length=None) -> bytes:
    hdr = bytearray(40)
    hdr[0] = 0x60
    struct.pack_into(">HBB", hdr, 4, len(payload) if length is None else length, nh, 64)
    hdr[8:24] = bytes(range(16))
    hdr[24:40] = bytes(range(16, 32))
    return bytes(hdr) + payload


def tcp(payload: bytes = b"", doff: int = 5, opts: bytes = b"", sport=40000, dport=8080) -> bytes:
    hdr = bytearray(20) + bytearray(opts)
    struct.pack_into(">HHIIBB", hdr, 0, sport, dport, 1, 2, doff << 4, 0x18)
    return bytes(hdr) + payload


def udp(payload: bytes = b"", length=None, sport=40000, dport=8080) -> bytes:
    return struct.pack(">HHHH", sport, dport, 8 + len(payload) if length is None else length, 0) + payload


# (name, packet, code, arg0, arg1): the reference site each case reaches (paths relative to
# google/gopacket) and its format arguments.
CASES = [
    ("eth_too_small", b"\x00" * 13, 1, 0, 0),                                  # ethernet.go:42-43
    ("dot1q_2_bytes", eth(0x8100, b"\x00\x01"), 2, 2, 0),                      # dot1q.go:30-32 len(data)
    ("ip4_10_bytes", eth(0x0800, b"\x45" + b"\x00" * 9), 3, 10, 0),            # ip4.go:189-191 len(data)
    ("ip4_length_10", eth(0x0800, ip4(tcp(), length=10)), 4, 10, 0),          # ip4.go:220-221 ip.Length
    ("ip4_ihl_4", eth(0x0800, ip4(tcp(), ihl=4, length=40)), 5, 4, 0),         # ip4.go:222-223 ip.IHL
    ("ip4_ihl_15_len_40", eth(0x0800, ip4(tcp(), ihl=15, length=40)), 6, 15, 40),  # :224-225 IHL, Length
    ("ip4_hdr_trunc", eth(0x0800, ip4(tcp(), ihl=15, length=100)), 7, 0, 0),   # ip4.go:231-232
    ("ip4_opt_lt2", eth(0x0800, ip4(tcp(), ihl=6, opts=b"\x01\x01\x01\x07")), 8, 1, 0),   # :257-259 len
    ("ip4_opt_exceeds", eth(0x0800, ip4(tcp(), ihl=6, opts=b"\x07\x08\x00\x00")), 9, 7, 8),  # :262-264
    ("ip4_opt_le2", eth(0x0800, ip4(tcp(), ihl=6, opts=b"\x07\x02\x00\x00")), 10, 7, 2),   # :266-267
    ("ip4_opt_le2_type_130", eth(0x0800, ip4(tcp(), ihl=6, opts=b"\x82\x01\x00\x00")), 10, 130, 1),
    ("ip6_30_bytes", eth(0x86DD, b"\x60" + b"\x00" * 29), 11, 30, 0),          # ip6.go:222-224 len
    ("ip6ext_1_byte", eth(0x86DD, ip6(b"\x06", nh=60)), 12, 1, 0),             # ip6.go:419-421 len
    ("ip6ext_lt_spec", eth(0x86DD, ip6(b"\x06\x01" + b"\x00" * 6, nh=60)), 13, 8, 16),  # :426-427
    ("ip6_hbh_pad1_at_end", eth(0x86DD, ip6(b"\x3b\x00" + b"\x00" * 6, nh=0)), 14, 0, 0),  # :328-330
    ("ip6_hbh_tlv_trunc", eth(0x86DD, ip6(b"\x3b\x00\x05\x0a" + b"\x00" * 4, nh=0)), 15, 0, 0),  # :340-342
    ("ip6_jumbo_len_2", eth(0x86DD, ip6(b"\x3b\x00\xc2\x02\x00\x00\x01\x00", nh=0, length=0)), 16, 0, 0),
    ("ip6_jumbo_small", eth(0x86DD, ip6(b"\x3b\x00\xc2\x04\x00\x00\xff\xff", nh=0, length=0)), 17, 0, 0),
    ("ip6_jumbo_and_len", eth(0x86DD, ip6(b"\x3b\x00\xc2\x04\x00\x01\x00\x00", nh=0, length=8)), 18, 0, 0),
    ("ip6_len0_no_jumbo", eth(0x86DD, ip6(b"\x3b\x00\x01\x04\x00\x00\x00\x00", nh=0, length=0)), 19, 0, 0),
    ("ip6_len0_tcp", eth(0x86DD, ip6(tcp(), nh=6, length=0)), 20, 6, 0),      # ip6.go:266-267 %v
    ("ip6_len0_udp", eth(0x86DD, ip6(udp(), nh=17, length=0)), 20, 17, 0),
    ("ip6_len0_unknown", eth(0x86DD, ip6(b"\x00" * 8, nh=253, length=0)), 20, 253, 0),
    ("tcp_10_bytes", eth(0x0800, ip4(b"\x00" * 10)), 21, 10, 0),              # tcp.go:230-232 len
    ("tcp_doff_4", eth(0x0800, ip4(tcp(doff=4))), 22, 4, 0),                   # tcp.go:260-261
    ("tcp_doff_gt_len", eth(0x0800, ip4(tcp(doff=15))), 23, 0, 0),             # tcp.go:264-268
    ("tcp_opt_lt2_rem", eth(0x0800, ip4(tcp(doff=6, opts=b"\x01\x01\x01\x02"))), 24, 1, 0),  # :286-288
    ("tcp_opt_len_1", eth(0x0800, ip4(tcp(doff=6, opts=b"\x02\x01\x00\x00"))), 25, 1, 0),   # :291-292
    ("tcp_opt_exceeds", eth(0x0800, ip4(tcp(doff=6, opts=b"\x02\x08\x00\x00"))), 26, 8, 4),  # :293-295
    ("udp_5_bytes", eth(0x0800, ip4(b"\x00" * 5, proto=17)), 27, 5, 0),        # udp.go:31-33 len
    ("udp_length_5", eth(0x0800, ip4(udp(b"\x00" * 8, length=5), proto=17)), 28, 5, 0),  # :52-53 Length
    ("vxlan_5_bytes", eth(0x0800, ip4(udp(b"\x08" + b"\x00" * 4, dport=4789), proto=17)), 29, 0, 0),
    ("icmp4_5_bytes", eth(0x0800, ip4(b"\x08" + b"\x00" * 4, proto=1)), 30, 0, 0),  # icmp4.go:221-223
    ("llc_2_bytes", MAC + struct.pack(">H", 2) + b"\xaa\xaa", 31, 0, 0),       # llc.go:32-33
    ("llc_3_bytes_i_format", MAC + struct.pack(">H", 3) + b"\x42\x42\x00", 31, 0, 0),  # llc.go:42-43
    # inner-stack errors after a VXLAN pass (the second pass's objects)
    ("vxlan_inner_ip4_length_10",
     eth(0x0800, ip4(udp(b"\x08\x00\x00\x00\x00\x00\xff\x00" + eth(0x0800, ip4(tcp(), length=10)), dport=4789),
                     proto=17)), 4, 10, 0),
    ("vxlan_inner_tcp_opt_exceeds",
     eth(0x0800, ip4(udp(b"\x08\x00\x00\x00\x00\x00\xff\x00" +
                         eth(0x0800, ip4(tcp(doff=6, opts=b"\x02\x08\x00\x00"))), dport=4789), proto=17)), 26, 8, 4),
]


def deep_stack(tags: int, inner: bytes = None) -> bytes:
    """Ethernet + `tags` 802.1Q tags + IPv4/UDP: len(decoded) = tags + 4 (Payload included)."""
    inner = ip4(udp(b"\x00" * 8), proto=17) if inner is None else inner
    body = b""
    for k in range(tags):
        body += struct.pack(">HH", k + 1, 0x8100 if k + 1 < tags else 0x0800)
    return MAC + struct.pack(">H", 0x8100) + body + inner


# (name, packet, n_layers): stacks past the core record's 12 layers (ext / detail carry them)
DEEP = [
    ("tags_9", deep_stack(9), 13),
    ("tags_12", deep_stack(12), 16),
    ("tags_20", deep_stack(20), 24),
    ("tags_27", deep_stack(27), 31),
    ("tags_28_saturated", deep_stack(28), 32),
    ("tags_40_saturated", deep_stack(40), 44),
    ("tags_14_tcp_doff_4", deep_stack(14, ip4(tcp(doff=4))), 16),  # deep AND a decode error
]


def packets() -> list:
    return [p for _, p, *_ in CASES] + [p for _, p, _ in DEEP]
