"""AF_PACKET TPACKET_V3 ring ingest (include/gpd_afpacket.h), the reference's afpacket.TPacket
read loop for whole blocks.

The reference hands out one packet per ZeroCopyReadPacketData call and releases a block when
it moves past it (afpacket/afpacket.go:282-330, header.go:137-195).  `TPv3Ring.Walk` returns,
in one native call, every packet of every block the kernel has handed to user space, as
offsets into the ring (its bytes are the batch buffer: nothing is repacked), and
`DecodingLayerParser.DecodeTPv3` decodes them on the GPU.  Opening the socket and mapping the
ring (afpacket.NewTPacket) stays with the caller; any mapped ring memory works (a mmap object,
a numpy array).
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from typing import Optional

import numpy as np

from ._lib import check, lib
from .batch import PacketBatch


class GpdTPv3Ring(C.Structure):
    _fields_ = [("base", C.c_void_p), ("block_size", C.c_uint32), ("num_blocks", C.c_uint32)]


class GpdTPv3Pkts(C.Structure):
    _fields_ = [("offset", C.c_void_p), ("caplen", C.c_void_p), ("wire_len", C.c_void_p),
                ("ts_ns", C.c_void_p), ("ifindex", C.c_void_p), ("vlan", C.c_void_p),
                ("vlan_tci", C.c_void_p)]


@dataclass
class CaptureInfo:
    """Per-packet CaptureInfo arrays of a walk (afpacket.go:318-326)."""
    offset: np.ndarray    # u64, frame start in the ring
    caplen: np.ndarray    # u32, tp_snaplen
    length: np.ndarray    # u32, tp_len
    ts_ns: np.ndarray     # u64
    ifindex: np.ndarray   # i32
    vlan: np.ndarray      # i32, AncillaryVLAN or -1
    vlan_tci: np.ndarray  # u32, as stored

    @staticmethod
    def alloc(n: int) -> "CaptureInfo":
        return CaptureInfo(np.zeros(n, np.uint64), np.zeros(n, np.uint32), np.zeros(n, np.uint32),
                           np.zeros(n, np.uint64), np.zeros(n, np.int32), np.zeros(n, np.int32),
                           np.zeros(n, np.uint32))

    def c(self) -> GpdTPv3Pkts:
        return GpdTPv3Pkts(*(a.ctypes.data for a in (self.offset, self.caplen, self.length,
                                                     self.ts_ns, self.ifindex, self.vlan,
                                                     self.vlan_tci)))

    def head(self, n: int) -> "CaptureInfo":
        return CaptureInfo(*(a[:n] for a in (self.offset, self.caplen, self.length, self.ts_ns,
                                             self.ifindex, self.vlan, self.vlan_tci)))


class TPv3Ring:
    """A mapped TPACKET_V3 ring: `mem` is any writable buffer of num_blocks * block_size
    bytes (mmap of the socket, or a numpy array).  `offset` is the reader's block index,
    like TPacket.offset (afpacket.go:445-453)."""

    def __init__(self, mem, block_size: int, num_blocks: int):
        self.mem = mem
        self.arr = np.frombuffer(mem, np.uint8)
        if self.arr.nbytes < block_size * num_blocks:
            raise ValueError("ring memory smaller than num_blocks * block_size")
        self._keep = (C.c_char * self.arr.nbytes).from_buffer(mem) if not isinstance(mem, np.ndarray) \
            else None
        base = C.addressof(self._keep) if self._keep is not None else self.arr.ctypes.data
        self.c = GpdTPv3Ring(base, block_size, num_blocks)
        self.block_size, self.num_blocks = block_size, num_blocks
        self.offset = 0

    def Walk(self, max_n: int = 1 << 20, max_blocks: Optional[int] = None, nthreads: int = 0):
        """(CaptureInfo of every packet in the user-owned blocks from self.offset on, blocks)."""
        ci = CaptureInfo.alloc(max_n)
        n, nb = C.c_uint64(), C.c_uint32()
        check(lib.gpd_tpv3_walk(C.byref(self.c), self.offset % self.num_blocks,
                                self.num_blocks if max_blocks is None else int(max_blocks),
                                int(max_n), C.byref(ci.c()), C.byref(n), C.byref(nb), int(nthreads)),
              "gpd_tpv3_walk")
        return ci.head(n.value), nb.value

    def Release(self, blocks: int) -> None:
        """Hand `blocks` blocks from self.offset on back to the kernel and advance."""
        check(lib.gpd_tpv3_release(C.byref(self.c), self.offset % self.num_blocks, int(blocks)),
              "gpd_tpv3_release")
        self.offset = (self.offset + int(blocks)) % self.num_blocks

    def batch(self, ci: CaptureInfo) -> PacketBatch:
        """The walked packets as a PacketBatch over the ring bytes (offsets into the ring)."""
        return PacketBatch(self.arr, int(self.arr.nbytes), ci.offset.astype(np.uint32), ci.caplen.copy())
