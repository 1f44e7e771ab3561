"""TEST INFRASTRUCTURE ONLY — the CPU oracle of the pcap ingest.

Only tests/ (and bench.py's cpu_baseline leg) may import this module; the product path is the
native walker in gopacket_amd/csrc/gpd_pcap.cpp behind include/gpd_pcap.h.

A plain sequential restatement of pcapgo's reader (paths relative to google/gopacket):
the header checks of readHeader (pcapgo/read.go:78-117: the four magics, version 2.4, gzip
transparency), then ReadPacketData (read.go:120-137) + readPacketHeader (read.go:165-177) in
a loop until the first error, with the reference's error texts.  `walk()` returns what the
loop saw: every record (data offset, caplen, wire length, timestamp in Unix ns) and how it
ended.  Pinned by the pcapgo/read_test.go vectors and pcap/*.pcap files (tests/golden).
"""
from __future__ import annotations

import gzip
import struct
from dataclasses import dataclass

import numpy as np

from gopacket_amd.batch import PAD, PacketBatch

MAGIC_MICRO = 0xA1B2C3D4
MAGIC_NANO = 0xA1B23C4D
MAGIC_MICRO_BE = 0xD4C3B2A1
MAGIC_NANO_BE = 0x4D3CB2A1
VERSION_MAJOR, VERSION_MINOR = 2, 4   # pcapgo/write.go:32-34
LINKTYPE_ETHERNET = 1


class PcapError(Exception):
    pass


@dataclass
class Pcap:
    batch: PacketBatch
    ts_sec: np.ndarray     # uint32[n]
    ts_nsec: np.ndarray    # uint32[n]
    length: np.ndarray     # uint32[n] original (wire) length
    linktype: int
    snaplen: int


STOP_LIMIT, STOP_EOF, STOP_SHORT_HDR, STOP_SNAPLEN, STOP_ORIGLEN, STOP_SHORT_DATA = range(6)


def header(buf: bytes):
    """readHeader, pcapgo/read.go:78-117 -> (byte order, nano factor, snaplen, linktype)."""
    if len(buf) < 2:
        raise PcapError("EOF")                 # bufio Peek(2) (read.go:80-83)
    if len(buf) < 24:
        raise PcapError("unexpected EOF")      # io.ReadFull(24) (read.go:91-95)
    magic = struct.unpack("<I", buf[:4])[0]
    if magic == MAGIC_NANO:
        bo, nano = "<", 1
    elif magic == MAGIC_NANO_BE:
        bo, nano = ">", 1
    elif magic == MAGIC_MICRO:
        bo, nano = "<", 1000
    elif magic == MAGIC_MICRO_BE:
        bo, nano = ">", 1000
    else:
        raise PcapError(f"Unknown magic {magic:x}")
    vmaj, vmin = struct.unpack(bo + "HH", buf[4:8])
    if vmaj != VERSION_MAJOR:
        raise PcapError(f"Unknown major version {vmaj}")
    if vmin != VERSION_MINOR:
        raise PcapError(f"Unknown minor version {vmin}")
    snaplen, linktype = struct.unpack(bo + "II", buf[16:24])
    return bo, nano, snaplen, linktype


def walk(buf: bytes, pos: int = 24, max_n: int = 1 << 62):
    """ReadPacketData in a loop from `pos` (read.go:120-137,165-177).  Returns
    (records, stop, next_pos, error text or None); records = [(data offset, caplen, wirelen,
    ts_ns)]."""
    bo, nano, snaplen, _ = header(buf)
    hdr = struct.Struct(bo + "IIII")
    recs = []
    o = pos
    while True:
        if len(recs) == max_n:
            return recs, STOP_LIMIT, o, None
        avail = len(buf) - o
        if avail == 0:
            return recs, STOP_EOF, o, None
        if avail < 16:
            return recs, STOP_SHORT_HDR, o, "unexpected EOF"
        sec, frac, incl, orig = hdr.unpack_from(buf, o)
        if incl > snaplen:
            return recs, STOP_SNAPLEN, o, f"capture length exceeds snap length: {incl} > {snaplen}"
        if incl > orig:
            return recs, STOP_ORIGLEN, o, \
                f"capture length exceeds original packet length: {incl} > {orig}"
        if avail - 16 < incl:
            return recs, STOP_SHORT_DATA, o, "EOF" if avail == 16 else "unexpected EOF"
        recs.append((o + 16, incl, orig, sec * 1_000_000_000 + ((frac * nano) & 0xFFFFFFFF)))
        o += 16 + incl


def parse_pcap(buf: bytes, align: int = 16) -> Pcap:
    if buf[:2] == b"\x1f\x8b":
        buf = gzip.decompress(buf)
    if len(buf) < 24:
        raise PcapError("Not enough data for read")
    magic = struct.unpack("<I", buf[:4])[0]
    if magic == MAGIC_NANO:
        bo, nano = "<", 1
    elif magic == MAGIC_NANO_BE:
        bo, nano = ">", 1
    elif magic == MAGIC_MICRO:
        bo, nano = "<", 1000
    elif magic == MAGIC_MICRO_BE:
        bo, nano = ">", 1000
    else:
        raise PcapError(f"Unknown magic {magic:x}")
    vmaj, vmin = struct.unpack(bo + "HH", buf[4:8])
    if vmaj != VERSION_MAJOR:
        raise PcapError(f"Unknown major version {vmaj}")
    if vmin != VERSION_MINOR:
        raise PcapError(f"Unknown minor version {vmin}")
    snaplen, linktype = struct.unpack(bo + "II", buf[16:24])
    # pass 1: walk records (sequential), collect (data offset, incl, orig, ts)
    recs = []
    o = 24
    hdr = struct.Struct(bo + "IIII")
    while o + 16 <= len(buf):
        ts, tfrac, incl, orig = hdr.unpack_from(buf, o)
        if incl > snaplen:
            raise PcapError(f"capture length exceeds snap length: {incl} > {snaplen}")
        if incl > orig:
            raise PcapError(f"capture length exceeds original packet length: {incl} > {orig}")
        if o + 16 + incl > len(buf):
            break  # io.ReadFull short read: stream ends
        recs.append((o + 16, incl, orig, ts, (tfrac * nano) & 0xFFFFFFFF))
        o += 16 + incl
    n = len(recs)
    src = np.fromiter((r[0] for r in recs), np.int64, n)
    lens = np.fromiter((r[1] for r in recs), np.int64, n)
    slot = (lens + align - 1) // align * align
    offs = np.zeros(n, np.int64)
    if n > 1:
        np.cumsum(slot[:-1], out=offs[1:])
    total = int(offs[-1] + lens[-1]) if n else 0
    data = np.zeros(total + PAD, np.uint8)
    raw = np.frombuffer(buf, np.uint8)
    for s, l, d in zip(src, lens, offs):
        data[d:d + l] = raw[s:s + l]
    batch = PacketBatch(data, total, offs.astype(np.uint32), lens.astype(np.uint32))
    return Pcap(batch, np.fromiter((r[3] for r in recs), np.uint32, n),
                np.fromiter((r[4] for r in recs), np.uint32, n),
                np.fromiter((r[2] for r in recs), np.uint32, n), linktype, snaplen)


def read_pcap(path: str, align: int = 16) -> Pcap:
    with open(path, "rb") as f:
        return parse_pcap(f.read(), align)


def write_pcap(batch: PacketBatch, linktype: int = LINKTYPE_ETHERNET, snaplen: int = 262144,
               ts_sec=None, ts_usec=None) -> bytes:
    """A little-endian microsecond pcap stream (pcapgo/write.go:74-120 layout)."""
    out = [struct.pack("<IHHiIII", MAGIC_MICRO, VERSION_MAJOR, VERSION_MINOR, 0, 0, snaplen, linktype)]
    for i in range(batch.n):
        p = batch.packet(i)
        s = int(ts_sec[i]) if ts_sec is not None else i // 1000000
        u = int(ts_usec[i]) if ts_usec is not None else i % 1000000
        out.append(struct.pack("<IIII", s, u, len(p), len(p)))
        out.append(p)
    return b"".join(out)
