"""pcap ingest -> PacketBatch.

Restates pcapgo's reader (pcapgo/read.go:65-177): the four magics
(microsecond/nanosecond, little/big endian), version 2.4 only, gzip-transparent,
per-record checks `capture length exceeds snap length` and `capture length
exceeds original packet length` with the same error text.  The record walk is
sequential by nature (each 16-byte header gives the next offset); the result is
one 16-byte-aligned PacketBatch plus per-packet timestamps and wire lengths.
"""
from __future__ import annotations

import gzip
import struct
from dataclasses import dataclass

import numpy as np

from .batch import PAD, PacketBatch

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
