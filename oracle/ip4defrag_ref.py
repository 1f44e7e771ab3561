"""TEST INFRASTRUCTURE ONLY: ip4defrag's IPv4Defragmenter restated over the GPU fragment
hand-off's records.  Only tests/ use it, as the checker that the hand-off (gpd_ip4_fragments,
the product) gives a defragmenter everything it needs: ip4defrag's stateful reassembly is OUT
OF SCOPE for the engine, so this lives beside the oracles, not in the package.

The reference reassembles IPv4 datagrams in ip4defrag/defrag.go: `DefragIPv4WithTimestamp`
(:86-135) filters with dontDefrag (:162-172), rejects with securityChecks (:175-198), files
the layer under ipv4{NetworkFlow(), Id} (:331-342) and inserts it into that key's fragment
list (`fragmentList.insert` :216-273, `build` :278-328).  The batch decode hands over exactly
the packets that pass the filter, with the key and the verdict already computed
(gpd_ip4_fragments, include/gpd_defrag.h, `defrag.IPv4Fragments`); this class is the
stateful rest, restated step for step — the per-key list is sequential and order-dependent
(BSD-right insertion), so it stays on the host, fed in packet order:

    out, n = IPv4Fragments(parser, dbatch, dres)
    d = IPv4Defragmenter()
    for rec in fragments_to_host(out, n):
        whole, err = d.DefragIPv4WithTimestamp(rec, batch.packet(int(rec["packet"])), ts)

Quirks of the reference are kept: a fragment whose offset is below the list's highest end but
above every stored offset is counted without being stored (:222-249); `build` advances an
overlapping fragment's offset by its own start (:298); counters are uint16.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Optional, Tuple

from gopacket_amd.defrag import FRAG_INSERT, FRAG_WHOLE, frag_error

IPv4MinimumFragmentSize = 8
IPv4MaximumSize = 65535
IPv4MaximumFragmentOffset = 8183
IPv4MaximumFragmentListLen = 8192

IPV4_MORE_FRAGMENTS = 1


@dataclass
class Fragment:
    """The fields of one handed-over IPv4 layer that insert() and build() read."""
    frag_offset: int  # units of 8 bytes
    length: int
    flags: int
    ihl: int
    ident: int
    src: bytes
    dst: bytes
    payload: bytes


@dataclass
class Reassembled:
    """The IPv4 layer build() returns (defrag.go:309-326): Length = the list's highest end,
    Flags and FragOffset 0, Payload = the datagram's bytes; the other header fields are the
    completing fragment's."""
    length: int
    ident: int
    ihl: int
    src: bytes
    dst: bytes
    payload: bytes
    flags: int = 0
    frag_offset: int = 0


@dataclass
class FragmentList:
    """defrag.go:204-210."""
    frags: List[Fragment] = field(default_factory=list)
    highest: int = 0
    current: int = 0
    final_received: bool = False
    last_seen: float = 0.0

    def insert(self, f: Fragment, t: float) -> Tuple[Optional[Reassembled], Optional[str]]:
        """defrag.go:216-273."""
        frag_offset = (f.frag_offset * 8) & 0xFFFF
        if frag_offset >= self.highest:
            self.frags.append(f)
        else:
            for k, e in enumerate(self.frags):
                if f.frag_offset == e.frag_offset:
                    return None, None  # a duplicate: ignored (:225-240)
                if f.frag_offset < e.frag_offset:
                    self.frags.insert(k, f)
                    break
        self.last_seen = t
        frag_length = (f.length - 20) & 0xFFFF
        if self.highest < ((frag_offset + frag_length) & 0xFFFF):
            self.highest = (frag_offset + frag_length) & 0xFFFF
        self.current = (self.current + frag_length) & 0xFFFF
        if f.flags & IPV4_MORE_FRAGMENTS == 0:
            self.final_received = True
        if self.final_received and self.highest == self.current:
            return self.build(f)
        return None, None

    def build(self, f: Fragment) -> Tuple[Optional[Reassembled], Optional[str]]:
        """defrag.go:278-328."""
        final = bytearray()
        current_offset = 0
        for e in self.frags:
            off8 = (e.frag_offset * 8) & 0xFFFF
            if off8 == current_offset:
                final += e.payload
                current_offset = (current_offset + e.length - 20) & 0xFFFF
            elif off8 < current_offset:
                start_at = (current_offset - off8) & 0xFFFF
                if start_at > ((e.length - 20) & 0xFFFF):
                    return None, "defrag: building - invalid fragment"
                final += e.payload[start_at:]
                current_offset = (current_offset + off8) & 0xFFFF  # (sic, :298)
            else:
                return None, "defrag: building - hole found"
        return Reassembled(length=self.highest, ident=f.ident, ihl=f.ihl, src=f.src, dst=f.dst,
                           payload=bytes(final)), None


class IPv4Defragmenter:
    """defrag.go:344-358: the fragment lists of all running datagrams, keyed ipv4{Flow, Id}."""

    def __init__(self):
        self.ip_flows = {}

    def DefragIPv4WithTimestamp(self, rec, packet: bytes, t: float):
        """One handed-over packet (a gpd_ip4_frag record and its packet bytes): returns
        (layer, error) as DefragIPv4WithTimestamp returns them — ("unchanged", None) for a layer
        that needs no reassembly, (None, None) for a fragment filed, (Reassembled, None) when
        it completes its datagram, (None, text) on an error."""
        v = int(rec["verdict"])
        if v == FRAG_WHOLE:
            return "unchanged", None
        if v != FRAG_INSERT:
            return None, frag_error(rec)
        net, ihl = int(rec["net_off"]), int(rec["ihl"])
        p0 = net + 4 * ihl
        f = Fragment(frag_offset=int(rec["frag_offset"]), length=int(rec["length"]), flags=int(rec["flags"]),
                     ihl=ihl, ident=int(rec["id"]), src=bytes(rec["src"]), dst=bytes(rec["dst"]),
                     payload=bytes(packet[p0:p0 + int(rec["payload_len"])]))
        key = (f.src, f.dst, f.ident)
        fl = self.ip_flows.get(key)
        if fl is None:
            fl = self.ip_flows[key] = FragmentList()
        out, err = fl.insert(f, t)
        if out is None and len(fl.frags) + 1 > IPv4MaximumFragmentListLen:
            self.ip_flows.pop(key, None)
            return None, ("defrag: Fragment List hits its maximumsize(%d), without success. "
                          "Flushing the list" % IPv4MaximumFragmentListLen)
        if out is not None:
            self.ip_flows.pop(key, None)
            return out, None
        return None, err

    def DiscardOlderThan(self, t: float) -> int:
        """defrag.go:140-151."""
        old = [k for k, v in self.ip_flows.items() if v.last_seen < t]
        for k in old:
            del self.ip_flows[k]
        return len(old)


def NewIPv4Defragmenter() -> IPv4Defragmenter:
    return IPv4Defragmenter()
