"""pcap ingest: a capture in memory -> a PacketBatch over its own bytes.

The reference reads a capture record by record with pcapgo.Reader.ReadPacketData
(pcapgo/read.go:120-177), copying each record out.  Here the whole capture is indexed in one
native call (include/gpd_pcap.h gpd_pcap_index: a parallel, speculative-and-stitched record
walk whose result equals the sequential loop's), and the offsets it returns point into the
capture buffer itself: the capture IS the batch buffer, so nothing is repacked and the raw
capture bytes are what go to HBM.  gzip captures are inflated first, as pcapgo does
transparently (read.go:79-86).  Errors keep pcapgo's texts; the records before the one the
reference rejects are returned with the error, as a ReadPacketData loop would have seen them.
"""
from __future__ import annotations

import ctypes as C
import gzip
import struct
from dataclasses import dataclass
from typing import Optional

import numpy as np

from ._lib import GPD_ERR_PCAP, GpdError, GpdPcapInfo, check, lib
from .batch import PAD, PacketBatch

MAGIC_MICRO = 0xA1B2C3D4   # pcapgo/write.go:32
MAGIC_NANO = 0xA1B23C4D    # pcapgo/read.go:47
VERSION_MAJOR, VERSION_MINOR = 2, 4   # pcapgo/write.go:33-34
LINKTYPE_ETHERNET = 1
STOP_LIMIT, STOP_EOF, STOP_SHORT_HDR, STOP_SNAPLEN, STOP_ORIGLEN, STOP_SHORT_DATA = range(6)


class PcapError(Exception):
    pass


@dataclass
class Pcap:
    batch: PacketBatch        # data = the capture bytes (+ PAD), offsets into it
    ts_ns: np.ndarray         # uint64[n] CaptureInfo.Timestamp as Unix ns
    length: np.ndarray        # uint32[n] CaptureInfo.Length (wire length)
    linktype: int
    snaplen: int
    nano: bool                # Resolution(): nanosecond timestamps
    stop: int                 # STOP_* : how the ReadPacketData loop ended
    next_pos: int             # byte position of the next (or the rejected) record header
    err: Optional[str]        # the reference's error text, None for a clean EOF / limit


def capture_array(buf) -> np.ndarray:
    """Capture bytes as a uint8 array with PAD bytes of slack (the batch contract), inflating
    gzip (pcapgo/read.go:79-86)."""
    b = bytes(buf) if not isinstance(buf, np.ndarray) else buf
    if len(b) >= 2 and b[0] == 0x1F and b[1] == 0x8B:
        b = gzip.decompress(bytes(b))
    n = len(b)
    a = np.zeros(n + PAD, np.uint8)
    a[:n] = np.frombuffer(b, np.uint8) if not isinstance(b, np.ndarray) else b[:n]
    return a


def header(cap: np.ndarray, n: Optional[int] = None) -> GpdPcapInfo:
    """pcapgo.NewReader's header parse (read.go:78-117)."""
    info = GpdPcapInfo()
    n = cap.shape[0] - PAD if n is None else n
    rc = lib.gpd_pcap_header(cap.ctypes.data, n, C.byref(info))
    if rc != 0:
        raise PcapError(lib.gpd_last_error_string().decode())
    return info


def index(cap: np.ndarray, max_n: Optional[int] = None, nthreads: int = 0,
          data_len: Optional[int] = None, pos: int = 24, info: Optional[GpdPcapInfo] = None) -> Pcap:
    """Index every record of a capture array (capture_array()) — the ReadPacketData loop —
    from record header position `pos` (24: the first record).  `info`: the capture's parsed
    file header, for a window of a capture (cap = a view from some record on; offsets are
    relative to the view)."""
    dl = cap.shape[0] - PAD if data_len is None else int(data_len)
    info = header(cap, dl) if info is None else info
    cap_n = (dl - pos) // 16 + 1 if max_n is None else int(max_n)
    off = np.empty(cap_n, np.uint32)
    ln = np.empty(cap_n, np.uint32)
    wl = np.empty(cap_n, np.uint32)
    ts = np.empty(cap_n, np.uint64)
    n = C.c_uint64()
    nxt = C.c_uint64()
    stop = C.c_int()
    rc = lib.gpd_pcap_index(cap.ctypes.data, dl, C.byref(info), int(pos), cap_n, off.ctypes.data,
                            ln.ctypes.data, wl.ctypes.data, ts.ctypes.data, C.byref(n),
                            C.byref(nxt), C.byref(stop), int(nthreads))
    err = None
    if rc == GPD_ERR_PCAP:
        err = lib.gpd_last_error_string().decode()
    elif rc != 0:
        check(rc, "gpd_pcap_index")
    k = n.value  # views: the untouched tail of the arrays was never paged in
    batch = PacketBatch(cap, dl, off[:k], ln[:k])
    return Pcap(batch, ts[:k], wl[:k], info.linktype, info.snaplen, bool(info.nano),
                stop.value, nxt.value, err)


def locate(cap: np.ndarray, targets, pos: int = 24, data_len: Optional[int] = None,
           nthreads: int = 0, info: Optional[GpdPcapInfo] = None):
    """gpd_pcap_locate: header positions of records `targets` (ascending record numbers of the
    ReadPacketData walk from `pos`) with one parallel counting pass and no per-record arrays.
    Returns (positions uint64[len(targets)], records in the walk, STOP_* of its end)."""
    dl = cap.shape[0] - PAD if data_len is None else int(data_len)
    info = header(cap, dl) if info is None else info
    t = np.ascontiguousarray(np.asarray(targets, dtype=np.uint64))
    out = np.zeros(len(t), np.uint64)
    n, stop = C.c_uint64(), C.c_int()
    check(lib.gpd_pcap_locate(cap.ctypes.data, dl, C.byref(info), int(pos), t.ctypes.data, len(t),
                              out.ctypes.data, C.byref(n), C.byref(stop), int(nthreads)),
          "gpd_pcap_locate")
    return out, n.value, stop.value


def shard_bounds(n_records: int, world: int):
    """Record ranges [g*N/G, (g+1)*N/G) of the G shards of an N-record capture."""
    return [(n_records * g // world, n_records * (g + 1) // world) for g in range(world)]


def last_walk_stats():
    """(segments walked in parallel, speculations met, segments re-walked) of the last index."""
    t, m, r = C.c_int(), C.c_int(), C.c_int()
    lib.gpd_pcap_last_stats(C.byref(t), C.byref(m), C.byref(r))
    return t.value, m.value, r.value


def read_pcap(path: str, nthreads: int = 0) -> Pcap:
    with open(path, "rb") as f:
        return index(capture_array(f.read()), nthreads=nthreads)


def parse_pcap(buf, nthreads: int = 0) -> Pcap:
    return index(capture_array(buf), nthreads=nthreads)


def write_pcap(batch: PacketBatch, linktype: int = LINKTYPE_ETHERNET, snaplen: int = 262144,
               ts_sec=None, ts_usec=None) -> bytes:
    """A little-endian microsecond capture (the layout of pcapgo.Writer, pcapgo/write.go:74-120)."""
    out = [struct.pack("<IHHiIII", MAGIC_MICRO, VERSION_MAJOR, VERSION_MINOR, 0, 0, snaplen, linktype)]
    for i in range(batch.n):
        p = batch.packet(i)
        s = int(ts_sec[i]) if ts_sec is not None else i // 1000000
        u = int(ts_usec[i]) if ts_usec is not None else i % 1000000
        out.append(struct.pack("<IIII", s, u, len(p), len(p)))
        out.append(p)
    return b"".join(out)


def synth_capture(batch: PacketBatch, snaplen: int = 262144) -> np.ndarray:
    """The pcap stream of a batch, built with numpy (large synthetic captures for the bench):
    record i = 16-byte LE header {i // 10^6, i % 10^6, caplen, caplen} + the packet bytes."""
    n = batch.n
    ln = batch.caplen.astype(np.int64)
    rec = 16 + ln
    start = np.zeros(n, np.int64)
    if n > 1:
        np.cumsum(rec[:-1], out=start[1:])
    start += 24
    total = 24 + int(rec.sum())
    cap = np.zeros(total + PAD, np.uint8)
    cap[:24] = np.frombuffer(struct.pack("<IHHiIII", MAGIC_MICRO, VERSION_MAJOR, VERSION_MINOR, 0, 0,
                                         snaplen, LINKTYPE_ETHERNET), np.uint8)
    hdr = np.empty((n, 4), np.uint32)
    idx = np.arange(n, dtype=np.uint64)
    hdr[:, 0] = (idx // 1000000).astype(np.uint32)
    hdr[:, 1] = (idx % 1000000).astype(np.uint32)
    hdr[:, 2] = batch.caplen
    hdr[:, 3] = batch.caplen
    hb = hdr.view(np.uint8).reshape(n, 16)
    pos = start[:, None] + np.arange(16)[None, :]
    cap[pos.ravel()] = hb.ravel()
    # packet bytes: gather every packet's bytes with one fancy index per length class
    src_off = batch.offset.astype(np.int64)
    for L in np.unique(ln):
        sel_all = np.nonzero(ln == L)[0]
        step = max(1, (1 << 24) // max(int(L), 1))  # bound the index arrays to ~16M entries
        for c in range(0, sel_all.size if L else 0, step):
            sel = sel_all[c:c + step]
            s = src_off[sel][:, None] + np.arange(L)[None, :]
            d = (start[sel] + 16)[:, None] + np.arange(L)[None, :]
            cap[d.ravel()] = batch.data[s.ravel()]
    return cap
