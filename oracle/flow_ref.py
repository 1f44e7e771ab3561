"""TEST INFRASTRUCTURE ONLY: CPU restatement of tcpassembly's connection keying (the F3 oracle).

Only tests/ and bench.py's cpu_baseline leg may use this; the product path never does.

The reference keys a packet by key{netFlow, tcp.TransportFlow()} (tcpassembly/assembly.go:289,
543; reassembly/tcpassembly.go:389,644) and finds or creates its connection in a Go map
(getConnection, assembly.go:495-511).  A gopacket.Flow is compared field by field: the
EndpointType, both lengths and the raw endpoint bytes zero-padded to 16 (flows.go:140-146,
NewFlow :214-224).  So grouping a batch by that key is a group-by over the tuple
(net type, src[16], dst[16], transport type, src port bytes, dst port bytes), with
NetworkFlow/TransportFlow read from the layer objects as DecodeLayers leaves them
(ip4.go:63-65, ip6.go:49-51, tcp.go:331-333, udp.go:123-125).  Parity for this row is pinned by
that restatement only: the reference's tests hold no golden flow tables.
"""
from __future__ import annotations

import numpy as np


def flow_keys(batch, res):
    """(keyed mask, key bytes u8[n, 40]) from an oracle/device BatchResult with hdr_off."""
    n = batch.n
    st = res.status.astype(np.uint32)
    nt = (st >> 20) & 15
    tt = (st >> 24) & 15
    no = res.hdr_off.astype(np.uint32) & 0xFFFF
    to = res.hdr_off.astype(np.uint32) >> 16
    keyed = (nt != 0) & (tt != 0) & (no != 0xFFFF) & (to != 0xFFFF)
    keys = np.zeros((n, 40), np.uint8)
    for i in np.nonzero(keyed)[0]:
        p = batch.packet(int(i))
        a = 4 if nt[i] == 1 else 16
        s0 = int(no[i]) + (12 if nt[i] == 1 else 8)
        keys[i, 0:a] = np.frombuffer(p[s0:s0 + a], np.uint8)
        keys[i, 16:16 + a] = np.frombuffer(p[s0 + a:s0 + 2 * a], np.uint8)
        t0 = int(to[i])
        keys[i, 32:36] = np.frombuffer(p[t0:t0 + 4], np.uint8)
        keys[i, 36] = nt[i]
        keys[i, 37] = tt[i]
        keys[i, 38] = a
    return keyed, keys


def group(batch, res, index_base: int = 0):
    """The connection map after inserting the batch: dict key-bytes -> {first, last, packets,
    bytes}, and each packet's key (None when it has no network + transport pair)."""
    keyed, keys = flow_keys(batch, res)
    flows = {}
    per_packet = [None] * batch.n
    for i in np.nonzero(keyed)[0]:
        k = keys[i].tobytes()
        seq = index_base + int(i)
        f = flows.get(k)
        if f is None:
            flows[k] = f = {"first": seq, "last": seq, "packets": 0, "bytes": 0}
        f["first"] = min(f["first"], seq)
        f["last"] = max(f["last"], seq)
        f["packets"] += 1
        f["bytes"] += int(batch.caplen[i])
        per_packet[i] = k
    return flows, per_packet


def record_key(rec) -> bytes:
    """Key bytes of an exported gpd_flow_rec in flow_keys' layout."""
    k = np.zeros(40, np.uint8)
    k[0:16] = rec["src"]
    k[16:32] = rec["dst"]
    k[32:34] = rec["sport"]
    k[34:36] = rec["dport"]
    k[36] = rec["net_type"]
    k[37] = rec["tp_type"]
    k[38] = rec["addr_len"]
    return k.tobytes()
