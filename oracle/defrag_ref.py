"""TEST INFRASTRUCTURE ONLY: CPU restatement of ip4defrag's per-packet pre-steps (the F4
fragment hand-off oracle).

Only tests/ may use this; the product path (gpd_ip4_fragments, include/gpd_defrag.h) never does.

For every packet whose DecodeLayers left an IPv4 layer in `decoded`, the application calls
IPv4Defragmenter.DefragIPv4(&ip4) (ip4defrag/defrag.go:76-135) with the parser's IPv4 object as
the call leaves it (the oracle's ext record, obj[2]): its last successful DecodeFromBytes, or a
later IPv4 call that failed after assigning the header fields and Contents = data
(ip4.go:195-210; e.g. IPv4-in-IPv4 with a broken inner header, tests/golden/errpath.json).
DefragIPv4WithTimestamp:
  * returns the layer unchanged when dontDefrag holds (defrag.go:88-91,162-172):
    Flags & DontFragment, or neither MoreFragments nor a FragOffset;
  * else runs securityChecks (:93-96,175-198) on fragSize = Length - IHL*4 (uint16), FragOffset
    and fragOffset + Length — the last sum is of two uint16 values in Go, so it wraps and
    `> IPv4MaximumSize (65535)` never holds;
  * else keys the layer by ipv4{NetworkFlow(), Id} (:102-103,331-342) and inserts it.
The hand-off lists, in packet order, every packet that passes the first step, with the key, the
fields the insert and build read, and the security verdict (GPD_FRAG_* codes).

The IPv4 fields come from the header bytes as ip4.go:193-206 reads them; Length is the field,
or len(data) when it is 0 (ip4.go:214-218), which is Contents + Payload after that decode.
Pinned by the reference's own fragments (ip4defrag/defrag_test.go testPing1Frag1..4 /
testPing2Frag1..4 through tests/golden/defrag_vectors.json) and the IPv4 structs of
TestDefragTooSmall / TestDefragFragmentOffset / TestDefragMaxSize / TestNotFrag, rebuilt as
frames.  (Packets whose IPv4 header starts past byte 65534, which the device pass reports as
GPD_FRAG_WHOLE records, are not restated: no test frame is that long.)
"""
from __future__ import annotations

import numpy as np

FRAG_INSERT, FRAG_TOO_SMALL, FRAG_OFFSET, FRAG_OVERRUN, FRAG_WHOLE = 0, 1, 2, 3, 4
OBJ_IPV4 = 2

FRAG_DTYPE = np.dtype([("packet", "<u4"), ("net_off", "<u4"), ("src", "u1", (4,)), ("dst", "u1", (4,)),
                       ("id", "<u2"), ("frag_offset", "<u2"), ("length", "<u2"), ("flags", "u1"),
                       ("ihl", "u1"), ("payload_len", "<u4"), ("verdict", "u1"), ("reserved", "u1", (3,))])
assert FRAG_DTYPE.itemsize == 32


def dont_defrag(flags: int, frag_offset: int) -> bool:
    """defrag.go:162-172."""
    if flags & 2:  # IPv4DontFragment
        return True
    return (flags & 1) == 0 and frag_offset == 0


def security_verdict(length: int, ihl: int, frag_offset: int) -> int:
    """defrag.go:175-198 (uint16 arithmetic as in Go)."""
    frag_size = (length - ihl * 4) & 0xFFFF
    if frag_size < 8:  # IPv4MinimumFragmentSize
        return FRAG_TOO_SMALL
    if frag_offset > 8183:  # IPv4MaximumFragmentOffset
        return FRAG_OFFSET
    if ((frag_offset * 8 + length) & 0xFFFF) > 65535:  # IPv4MaximumSize: a uint16 sum never exceeds it
        return FRAG_OVERRUN
    return FRAG_INSERT


def ip4_fragments(batch, res) -> np.ndarray:
    """FRAG_DTYPE records for an oracle BatchResult decoded with ext records."""
    if res.ext is None:
        raise ValueError("the fragment oracle reads the IPv4 object from ext records")
    out = []
    valid = (res.ext["obj_valid"].astype(np.uint32) >> OBJ_IPV4) & 1
    for i in np.nonzero(valid)[0]:
        o = res.ext["obj"][i, OBJ_IPV4]
        p = batch.packet(int(i))
        h = p[int(o["contents_off"]):]
        ff = (h[6] << 8) | h[7]
        flags, fo = ff >> 13, ff & 0x1FFF
        if dont_defrag(flags, fo):
            continue
        raw_len = (h[2] << 8) | h[3]
        length = raw_len if raw_len else int(o["contents_len"]) + int(o["payload_len"])
        ihl = h[0] & 0x0F
        r = np.zeros((), FRAG_DTYPE)
        r["packet"] = i
        r["net_off"] = o["contents_off"]
        r["src"] = np.frombuffer(bytes(h[12:16]), np.uint8)
        r["dst"] = np.frombuffer(bytes(h[16:20]), np.uint8)
        r["id"] = (h[4] << 8) | h[5]
        r["frag_offset"] = fo
        r["length"] = length
        r["flags"] = flags
        r["ihl"] = ihl
        r["payload_len"] = o["payload_len"]
        r["verdict"] = security_verdict(length, ihl, fo)
        out.append(r)
    return np.array(out, FRAG_DTYPE) if out else np.zeros(0, FRAG_DTYPE)
