"""TEST INFRASTRUCTURE ONLY: pure-Python restatement of the reference's TPACKET_V3 read loop.

Only tests/ may use this.  It follows (paths relative to google/gopacket):
  afpacket/afpacket.go:300-330  ZeroCopyReadPacketData (the empty-block retry at :313-316,
                                CaptureInfo at :318-326), running loop (headerNextNeeded set)
  afpacket/afpacket.go:445-453  getTPacketHeader, TPacketVersion3 case (block k at k*blockSize)
  afpacket/afpacket.go:457-483  pollForFirstPacket (stop where the kernel owns the block)
  afpacket/header.go:74-82      insertVlanHeader (OptAddVLANHeader)
  afpacket/header.go:144-195    initV3Wrapper and the v3wrapper methods
over ring memory laid out as linux/if_packet.h defines it.  The reference itself needs a
Go toolchain and a live socket; it is not runnable here, so this
restatement is pinned by the kernel's struct layouts and tested against real rings the
kernel filled on the loopback device where the test host allows AF_PACKET sockets.
"""
from __future__ import annotations

import struct

TP_STATUS_USER, TP_STATUS_VLAN_VALID = 1, 16


def _align(x, a=16):
    return (x + a - 1) & ~(a - 1)


def read_loop(ring: bytes, block_size: int, num_blocks: int, first_block: int = 0,
              max_blocks: int | None = None, add_vlan_header: bool = False):
    """Every packet ZeroCopyReadPacketData returns before it would poll: a list of dicts
    (data, caplen, length, ts_ns, ifindex, vlan) and the number of blocks consumed."""
    out = []
    nblk = 0
    limit = num_blocks if max_blocks is None else min(max_blocks, num_blocks)
    while nblk < limit:
        k = (first_block + nblk) % num_blocks
        base = k * block_size
        status, num_pkts, first = struct.unpack_from("<III", ring, base + 8)
        if not status & TP_STATUS_USER:
            break  # pollForFirstPacket would block here
        pos, used = first, 0

        def hdr(p):
            nxt, sec, nsec, snap, ln, st = struct.unpack_from("<IIIIII", ring, base + p)
            mac, _net = struct.unpack_from("<HH", ring, base + p + 24)
            tci = struct.unpack_from("<I", ring, base + p + 32)[0]
            ifi = struct.unpack_from("<i", ring, base + p + 48 + 4)[0]
            return nxt, sec, nsec, snap, ln, st, mac, tci, ifi

        h = hdr(pos)
        emit = True
        if h[4] == 0:  # getLength() == 0: retry -> next()
            used += 1
            if used >= num_pkts:
                emit = False
            else:
                pos += h[0] if h[0] else _align(h[3] + h[6])
                h = hdr(pos)
        while emit:
            nxt, sec, nsec, snap, ln, st, mac, tci, ifi = h
            data = bytes(ring[base + pos + mac:base + pos + mac + snap])
            if add_vlan_header and tci != 0:
                data = data[:12] + bytes([0x81, 0, (tci >> 8) & 0xFF, tci & 0xFF]) + data[12:]
            out.append({"data": data, "caplen": len(data), "length": ln,
                        "ts_ns": sec * 10**9 + nsec, "ifindex": ifi,
                        "vlan": (tci & 0xFFF) if st & TP_STATUS_VLAN_VALID else -1,
                        "offset": base + pos + mac, "snaplen": snap})
            used += 1
            if used >= num_pkts:
                break
            pos += nxt if nxt else _align(snap + mac)
            h = hdr(pos)
        nblk += 1
    return out, nblk
