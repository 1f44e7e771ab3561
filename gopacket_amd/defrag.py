"""IPv4 fragment hand-off: ip4defrag's per-packet pre-steps for a whole decoded batch, on the GPU.

The reference's application calls IPv4Defragmenter.DefragIPv4(&ip4) for every decoded IPv4
layer (ip4defrag/defrag.go:76-135).  That call returns the layer unchanged unless it is a
fragment (dontDefrag, :162-172), rejects hand-crafted fragments (securityChecks, :175-198), and
otherwise files the layer under ipv4{NetworkFlow(), Id} (:331-342) for the stateful insert.
`IPv4Fragments` runs the first two steps and builds the key for every packet of an
HBM-resident batch the parser just decoded (gpd_ip4_fragments, include/gpd_defrag.h) and
returns, in packet order, exactly the packets the defragmenter still has to see.
"""
from __future__ import annotations

import ctypes as C
from typing import Optional

import numpy as np

from ._lib import check, lib
from .parser import DecodingLayerParser, DeviceBatch, DeviceResult, _torch

# verdicts (gpd_defrag.h GPD_FRAG_*)
FRAG_INSERT, FRAG_TOO_SMALL, FRAG_OFFSET, FRAG_OVERRUN, FRAG_WHOLE = 0, 1, 2, 3, 4

FRAG_DTYPE = np.dtype([("packet", "<u4"), ("net_off", "<u4"), ("src", "u1", (4,)), ("dst", "u1", (4,)),
                       ("id", "<u2"), ("frag_offset", "<u2"), ("length", "<u2"), ("flags", "u1"),
                       ("ihl", "u1"), ("payload_len", "<u4"), ("verdict", "u1"), ("reserved", "u1", (3,))])
assert FRAG_DTYPE.itemsize == 32

# securityChecks' error texts (defrag.go:180-194), by verdict
FRAG_ERRORS = {
    FRAG_TOO_SMALL: "defrag: fragment too small (handcrafted? {} < {})",
    FRAG_OFFSET: "defrag: fragment offset too big (handcrafted? {} > {})",
    FRAG_OVERRUN: "defrag: fragment will overrun (handcrafted? {} > {})",
}


def frag_error(rec) -> Optional[str]:
    """The error DefragIPv4 returns for a handed-over record (None for FRAG_INSERT/WHOLE)."""
    v = int(rec["verdict"])
    if v == FRAG_TOO_SMALL:
        return FRAG_ERRORS[v].format((int(rec["length"]) - int(rec["ihl"]) * 4) & 0xFFFF, 8)
    if v == FRAG_OFFSET:
        return FRAG_ERRORS[v].format(int(rec["frag_offset"]), 8183)
    if v == FRAG_OVERRUN:
        return FRAG_ERRORS[v].format((int(rec["frag_offset"]) * 8 + int(rec["length"])) & 0xFFFF, 65535)
    return None


def IPv4Fragments(parser: DecodingLayerParser, dbatch: DeviceBatch, dres: DeviceResult,
                  max_out: Optional[int] = None, stream=None, out=None):
    """The fragment hand-off of a batch `parser` decoded into `dres` (hdr_off required).
    Returns (uint8 device tensor of count x 32-byte records, count); synchronises `stream`.
    `out` (a uint8 device tensor of at least max_out * 32 bytes) is reused when given."""
    torch = _torch()
    if dres.hdr_off is None:
        raise ValueError("IPv4Fragments needs a DeviceResult with hdr_off")
    m = dbatch.n if max_out is None else int(max_out)
    if out is None:
        out = torch.empty(max(m, 1) * FRAG_DTYPE.itemsize, dtype=torch.uint8,
                          device=torch.device("cuda", parser.device))
    elif out.numel() < m * FRAG_DTYPE.itemsize:
        raise ValueError("IPv4Fragments: `out` holds fewer than max_out records")
    s = stream if stream is not None else torch.cuda.current_stream(parser.device)
    cnt = C.c_uint64()
    b, r = dbatch.c_batch(), dres.c_result()
    check(lib.gpd_ip4_fragments(parser.ctx().h, C.byref(b), C.byref(r), C.c_void_p(out.data_ptr()), m,
                                C.byref(cnt), C.c_void_p(s.cuda_stream)), "gpd_ip4_fragments")
    return out, int(cnt.value)


def fragments_to_host(out, count: int, allow_partial: bool = False) -> np.ndarray:
    """FRAG_DTYPE[count] copy of IPv4Fragments' records.  When the batch had more fragments
    than `out` holds (IPv4Fragments' max_out), raises unless allow_partial: a defragmenter fed
    only the first records would report holes or never complete the datagrams."""
    k = min(count, out.numel() // FRAG_DTYPE.itemsize)
    if k < count and not allow_partial:
        raise ValueError(f"fragments_to_host: {count} fragments, `out` holds {k}; "
                         f"call IPv4Fragments with a larger max_out")
    return out[:k * FRAG_DTYPE.itemsize].cpu().numpy().view(FRAG_DTYPE).copy()
