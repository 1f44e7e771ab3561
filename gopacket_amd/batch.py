"""Packet batches: one byte buffer + offset/caplen arrays (the gpd_batch layout).

The reference decodes one `[]byte` per call (parser.go:302); a batch holds many
of them back to back.  Packet starts are 16-byte aligned by default and the
buffer is padded past its end (include/gpd.h needs it readable to round_up(len,16);
PAD adds slack), so the kernel's 16-byte loads never read outside the allocation.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Iterable, Optional

import numpy as np

PAD = 64  # bytes of slack after the last packet (>= 16 + alignment)


@dataclass
class PacketBatch:
    data: np.ndarray      # uint8, len >= data_len + PAD
    data_len: int
    offset: np.ndarray    # uint32[n]
    caplen: np.ndarray    # uint32[n]

    @property
    def n(self) -> int:
        return int(self.offset.shape[0])

    def packet(self, i: int) -> bytes:
        o, l = int(self.offset[i]), int(self.caplen[i])
        return self.data[o:o + l].tobytes()

    @classmethod
    def from_packets(cls, packets: Iterable[bytes], align: int = 16) -> "PacketBatch":
        pkts = [bytes(p) for p in packets]
        n = len(pkts)
        lens = np.fromiter((len(p) for p in pkts), dtype=np.int64, count=n)
        if align > 1:
            slot = (lens + align - 1) // align * align
        else:
            slot = lens
        offs = np.zeros(n, dtype=np.int64)
        if n > 1:
            np.cumsum(slot[:-1], out=offs[1:])
        total = int(offs[-1] + lens[-1]) if n else 0
        if total >= 2 ** 32 - 16:
            raise ValueError("batch larger than the 32-bit offset range; split it")
        buf = np.zeros(total + PAD, dtype=np.uint8)
        for p, o in zip(pkts, offs):
            buf[o:o + len(p)] = np.frombuffer(p, dtype=np.uint8)
        return cls(buf, total, offs.astype(np.uint32), lens.astype(np.uint32))

    @classmethod
    def from_arrays(cls, data: np.ndarray, offset: np.ndarray, caplen: np.ndarray,
                    data_len: Optional[int] = None) -> "PacketBatch":
        data = np.ascontiguousarray(data, dtype=np.uint8)
        dl = int(data.shape[0]) if data_len is None else int(data_len)
        if data.shape[0] < dl + PAD:
            data = np.concatenate([data[:dl], np.zeros(dl + PAD - dl, dtype=np.uint8)])
        return cls(data, dl, np.ascontiguousarray(offset, dtype=np.uint32),
                   np.ascontiguousarray(caplen, dtype=np.uint32))

    def slice(self, lo: int, hi: int) -> "PacketBatch":
        """Packets [lo, hi) as their own batch (rebased copy), e.g. a shard for one GPU."""
        if hi <= lo:
            return PacketBatch(np.zeros(PAD, np.uint8), 0, np.zeros(0, np.uint32), np.zeros(0, np.uint32))
        off = self.offset[lo:hi].astype(np.int64)
        ln = self.caplen[lo:hi].astype(np.int64)
        start = int(off.min()) & ~15
        end = int((off + ln).max())
        data = np.zeros(end - start + PAD, dtype=np.uint8)
        data[:end - start] = self.data[start:end]
        return PacketBatch(data, end - start, (off - start).astype(np.uint32), ln.astype(np.uint32))
