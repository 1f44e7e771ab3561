"""Per-packet result words (include/gpd.h) and their reading as gopacket values.

BatchResult answers, per packet index, what the reference's caller reads after
`err := parser.DecodeLayers(data, &decoded)` (parser.go:302-316): the decoded
slice, the error value (exact text), parser.Truncated, the flows' FastHash
(flows.go:167-174), the IPv4 header checksum (ip4.go:158-179) and
TCP.ComputeChecksum() (tcp.go:193-195).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import numpy as np

from .errors import DecodeError, UnsupportedLayerType
from .layers import CODE_TO_LAYERTYPE

OBJ_NAMES = ("Ethernet", "Dot1Q", "IPv4", "IPv6", "IPv6ExtensionSkipper", "TCP", "UDP", "VXLAN",
             "Payload", "Fragment", "ICMPv4", "LLC")

LAYER_REC_DTYPE = np.dtype([("contents_off", "<u4"), ("contents_len", "<u4"),
                            ("payload_off", "<u4"), ("payload_len", "<u4")])
# gpd_record (gpd.h): the AoS form of status, csum, layers, net_hash, tp_hash (32 B)
RECORD_DTYPE = np.dtype([("status", "<u4"), ("csum", "<u4"), ("layers", "<u8"), ("net_hash", "<u8"),
                         ("tp_hash", "<u8")])
assert RECORD_DTYPE.itemsize == 32

EXT_DTYPE = np.dtype([("layer_codes", "<u8", (2,)), ("err_arg0", "<u4"), ("err_arg1", "<u4"),
                      ("obj_valid", "<u2"), ("err_obj", "u1"), ("err_wrote", "u1"), ("err_off", "<u4"),
                      ("obj", LAYER_REC_DTYPE, (12,))])
assert EXT_DTYPE.itemsize == 224
# gpd_detail (gpd.h): the first 24 bytes of the ext record, written for decode errors and
# stacks deeper than the core word's 12 layers only
DETAIL_DTYPE = np.dtype([("layer_codes", "<u8", (2,)), ("err_arg0", "<u4"), ("err_arg1", "<u4")])
assert DETAIL_DTYPE.itemsize == 24

ST_OK, ST_UNSUPPORTED, ST_DECODE_ERROR = 0, 1, 2


def st_class(s):
    return s & 3


def st_truncated(s):
    return (s >> 2) & 1


def st_nlayers(s):
    return (s >> 4) & 31


def st_errcode(s):
    return (s >> 9) & 63


# ---- Endpoint / Flow (flows.go, layers/endpoints.go:20-35) ----------------------------------
EndpointIPv4, EndpointIPv6, EndpointTCPPort, EndpointUDPPort = 1, 2, 4, 5
EndpointMAC, EndpointSCTPPort, EndpointRUDPPort, EndpointUDPLitePort, EndpointPPP = 3, 6, 7, 8, 9
MaxEndpointSize = 16  # flows.go:27
# The names the layers package registers (layers/endpoints.go:20-36); EndpointType.String()
# (flows.go:126-131) prints a registered type's name, else its number.
ENDPOINT_TYPE_NAMES = {1: "IPv4", 2: "IPv6", 3: "MAC", 4: "TCP", 5: "UDP", 6: "SCTP", 7: "RUDP",
                       8: "UDPLite", 9: "PPP"}


def EndpointTypeString(typ: int) -> str:
    """EndpointType.String() (flows.go:126-131)."""
    return ENDPOINT_TYPE_NAMES.get(int(typ), str(int(typ)))


_FNV_BASIS, _FNV_PRIME, _M64 = 14695981039346656037, 1099511628211, (1 << 64) - 1


def _fnv(raw: bytes) -> int:
    """fnvHash (flows.go:60-67).  Host arithmetic for ONE caller-built key: the reference's
    FastHash is a CPU function of a few bytes, and a device launch per key (tens of µs) would
    make hashing keys in a loop far slower than it; many keys go to the GPU via FastHashes, and
    decoded packets' hashes come from the decode kernel."""
    h = _FNV_BASIS
    for b in raw:
        h = ((h ^ b) * _FNV_PRIME) & _M64
    return h


def _go_ip_string(b: bytes) -> str:
    """net.IP(b).String() (Go net/ip.go): dotted quad for 4-byte and IPv4-mapped 16-byte
    addresses, RFC 5952 hex groups with the first longest run (>1 group) of zeros as '::',
    '?'+hex for any other length, '<nil>' for none."""
    if len(b) == 0:
        return "<nil>"
    if len(b) == 4 or (len(b) == 16 and b[:10] == bytes(10) and b[10:12] == b"\xff\xff"):
        return ".".join(str(x) for x in b[-4:])
    if len(b) != 16:
        return "?" + b.hex()
    e0 = e1 = -1
    i = 0
    while i < 16:
        j = i
        while j < 16 and b[j] == 0 and b[j + 1] == 0:
            j += 2
        if j > i and j - i > e1 - e0:
            e0, e1, i = i, j, j
        i += 2
    if e1 - e0 <= 2:
        e0 = e1 = -1
    out, i = "", 0
    while i < 16:
        if i == e0:
            out += "::"
            i = e1
            if i >= 16:
                break
        elif i > 0:
            out += ":"
        out += format((b[i] << 8) | b[i + 1], "x")
        i += 2
    return out


def _device_fast_hash(typs, srcs, dsts=None, device: Optional[int] = None) -> np.ndarray:
    """FastHash of n endpoints (dsts None) or flows on the GPU (gpd_fast_hash, flows.go:60-83,
    167-174): the raw bytes zero-padded to 16 as gopacket keeps them."""
    import torch
    from ._lib import check, lib
    if not torch.cuda.is_available():
        raise RuntimeError("FastHash of a caller-built Endpoint/Flow runs on the GPU (gpd_fast_hash); no GPU")
    n = len(typs)
    dev = torch.cuda.current_device() if device is None else int(device)

    def pack(raws):
        a = np.zeros((max(n, 1), 16), np.uint8)
        ln = np.zeros(max(n, 1), np.uint8)
        for i, r in enumerate(raws):
            a[i, :len(r)] = np.frombuffer(r, np.uint8)
            ln[i] = len(r)
        return torch.from_numpy(a).to(dev), torch.from_numpy(ln).to(dev)
    t = torch.from_numpy(np.asarray(typs, np.int64).reshape(-1)).to(dev)
    s, sl = pack(srcs)
    d, dl = pack(dsts) if dsts is not None else (None, None)
    out = torch.empty(max(n, 1), dtype=torch.int64, device=dev)
    stream = torch.cuda.current_stream(dev)
    check(lib.gpd_fast_hash(dev, n, t.data_ptr(), s.data_ptr(), sl.data_ptr(),
                            d.data_ptr() if d is not None else None, dl.data_ptr() if dl is not None else None,
                            out.data_ptr(), stream.cuda_stream), "gpd_fast_hash")
    stream.synchronize()
    return out.cpu().numpy().view(np.uint64)[:n]


def FastHashes(objs, device: Optional[int] = None) -> np.ndarray:
    """FastHash of many Endpoints or many Flows in one device launch (uint64[n])."""
    objs = list(objs)
    if not objs:
        return np.zeros(0, np.uint64)
    if all(isinstance(o, Flow) for o in objs):
        return _device_fast_hash([o.typ for o in objs], [o.src for o in objs], [o.dst for o in objs], device)
    if all(isinstance(o, Endpoint) for o in objs):
        return _device_fast_hash([o.typ for o in objs], [o.raw for o in objs], None, device)
    raise TypeError("FastHashes: all Endpoints or all Flows")


class Endpoint:
    """flows.go:24-110: an endpoint type and its raw bytes (a view of the packet's)."""

    def __init__(self, typ: int, raw: bytes):
        self.typ, self.raw = int(typ), bytes(raw)

    def EndpointType(self) -> int:
        return self.typ

    def Raw(self) -> bytes:
        return self.raw

    def LessThan(self, b: "Endpoint") -> bool:  # flows.go:53-55
        return self.typ < b.typ or (self.typ == b.typ and self.raw < b.raw)

    def FastHash(self) -> int:  # flows.go:78-83 (one key on the host; FastHashes on the GPU)
        return ((_fnv(self.raw) ^ (self.typ & _M64)) * _FNV_PRIME) & _M64

    def String(self) -> str:  # layers/endpoints.go:20-36 formatters, else flows.go:133-138
        t, b = self.typ, self.raw
        if t in (EndpointIPv4, EndpointIPv6):
            return _go_ip_string(b)
        if t == EndpointMAC:  # net.HardwareAddr.String
            return ":".join(format(x, "02x") for x in b)
        if t in (EndpointTCPPort, EndpointUDPPort, EndpointSCTPPort, EndpointUDPLitePort):
            return str(int.from_bytes(b[:2], "big"))  # binary.BigEndian.Uint16
        if t == EndpointRUDPPort:
            return str(b[0])
        if t == EndpointPPP:
            return "point"
        # fmt.Sprintf("%v:%v", a.typ, a.raw): raw is the whole [MaxEndpointSize]byte array
        arr = b + bytes(MaxEndpointSize - len(b))
        return f"{EndpointTypeString(t)}:[{' '.join(str(x) for x in arr)}]"

    __str__ = String

    def __eq__(self, o):
        return isinstance(o, Endpoint) and (self.typ, self.raw) == (o.typ, o.raw)

    def __hash__(self):
        return hash((self.typ, self.raw))


class Flow:
    """flows.go:112-224: the two endpoints of one layer, in packet order.  A Flow from a
    decoded batch (BatchResult.NetworkFlow / TransportFlow) carries the FastHash the kernel
    computed for it; FastHash is symmetric (flows.go:159-174), so Reverse() keeps it."""

    def __init__(self, typ: int, src: bytes, dst: bytes, fast_hash: Optional[int] = None):
        self.typ, self.src, self.dst, self._hash = int(typ), bytes(src), bytes(dst), fast_hash

    def EndpointType(self) -> int:
        return self.typ

    def Src(self) -> Endpoint:
        return Endpoint(self.typ, self.src)

    def Dst(self) -> Endpoint:
        return Endpoint(self.typ, self.dst)

    def Endpoints(self):
        return self.Src(), self.Dst()

    def Reverse(self) -> "Flow":
        return Flow(self.typ, self.dst, self.src, self._hash)

    def FastHash(self) -> int:  # flows.go:167-174
        if self._hash is None:  # a caller-built flow: host FNV (FastHashes batches on the GPU)
            h = (_fnv(self.src) + _fnv(self.dst)) & _M64
            self._hash = ((h ^ (self.typ & _M64)) * _FNV_PRIME) & _M64
        return self._hash

    def String(self) -> str:  # flows.go:207-212
        return f"{self.Src()}->{self.Dst()}"

    __str__ = String

    def __eq__(self, o):
        return isinstance(o, Flow) and (self.typ, self.src, self.dst) == (o.typ, o.src, o.dst)

    def __hash__(self):
        return hash((self.typ, self.src, self.dst))


def NewEndpoint(typ: int, raw: bytes) -> Endpoint:
    """flows.go:89-97 (a raw longer than MaxEndpointSize panics there: ValueError here)."""
    if len(raw) > MaxEndpointSize:
        raise ValueError("raw byte length greater than MaxEndpointSize")
    return Endpoint(typ, raw)


def NewFlow(typ: int, src: bytes, dst: bytes) -> Flow:
    """flows.go:214-224."""
    if len(src) > MaxEndpointSize or len(dst) > MaxEndpointSize:
        raise ValueError("flow raw byte length greater than MaxEndpointSize")
    return Flow(typ, src, dst)


def FlowFromEndpoints(src: Endpoint, dst: Endpoint):
    """flows.go:151-157: (Flow, None), or (an empty Flow, the error) for mismatched types."""
    if src.typ != dst.typ:
        return Flow(0, b"", b""), ValueError(
            f"Mismatched endpoint types: {EndpointTypeString(src.typ)}->{EndpointTypeString(dst.typ)}")
    return Flow(src.typ, src.raw, dst.raw), None


@dataclass
class BatchResult:
    status: np.ndarray            # uint32[n]
    layers: np.ndarray            # uint64[n]
    net_hash: Optional[np.ndarray] = None
    tp_hash: Optional[np.ndarray] = None
    csum: Optional[np.ndarray] = None
    ext: Optional[np.ndarray] = None  # EXT_DTYPE[n]
    hdr_off: Optional[np.ndarray] = None  # uint32[n], gpd.h header offsets word
    detail: Optional[np.ndarray] = None  # DETAIL_DTYPE[n]: valid where has_detail(i)

    def __len__(self):
        return int(self.status.shape[0])

    # --- the DecodeLayers outputs -------------------------------------------------
    def has_detail(self, i: int) -> bool:
        """Whether the kernel wrote packet i's detail record (gpd.h gpd_detail): a decode
        error, or more layers than the core word holds."""
        s = int(self.status[i])
        return st_class(s) == ST_DECODE_ERROR or st_nlayers(s) > 12 or bool((s >> 3) & 1)

    def decoded(self, i: int) -> list:
        """The `decoded` slice (LayerType values), layers_decoder.go:69."""
        s = int(self.status[i])
        n = st_nlayers(s)
        words = None
        if self.ext is not None:
            words = self.ext["layer_codes"][i]
        elif n > 12 and self.detail is not None:
            words = self.detail["layer_codes"][i]
        if words is not None:
            n = min(n, 32)
            return [CODE_TO_LAYERTYPE[(int(words[k // 16]) >> (4 * (k % 16))) & 15] for k in range(n)]
        w = int(self.layers[i])
        if n > 12:
            raise ValueError(f"packet {i}: {n} layers exceed the core record; decode with detail or ext")
        return [CODE_TO_LAYERTYPE[(w >> (16 + 4 * k)) & 15] for k in range(n)]

    def stop_type(self, i: int) -> int:
        """LayerType the loop stopped at for want of a decoder (0 = none)."""
        return int(self.layers[i]) & 0xFFFF

    def err(self, i: int):
        """The error DecodeLayers returned: None, UnsupportedLayerType or DecodeError."""
        s = int(self.status[i])
        c = st_class(s)
        if c == ST_OK:
            return None
        if c == ST_UNSUPPORTED:
            return UnsupportedLayerType(self.stop_type(i))
        a0 = a1 = 0
        if self.ext is not None:
            a0, a1 = int(self.ext["err_arg0"][i]), int(self.ext["err_arg1"][i])
        elif self.detail is not None:
            a0, a1 = int(self.detail["err_arg0"][i]), int(self.detail["err_arg1"][i])
        return DecodeError(st_errcode(s), a0, a1)

    def truncated(self, i: int) -> bool:
        return bool(st_truncated(int(self.status[i])))

    def network_flow_hash(self, i: int) -> Optional[int]:
        s = int(self.status[i])
        return int(self.net_hash[i]) if (s >> 16) & 1 else None

    def transport_flow_hash(self, i: int) -> Optional[int]:
        s = int(self.status[i])
        return int(self.tp_hash[i]) if (s >> 17) & 1 else None

    def ip4_checksum(self, i: int) -> Optional[int]:
        s = int(self.status[i])
        return int(self.csum[i]) & 0xFFFF if (s >> 18) & 1 else None

    def l4_checksum(self, i: int) -> Optional[int]:
        s = int(self.status[i])
        return int(self.csum[i]) >> 16 if (s >> 19) & 1 else None

    def network_offset(self, i: int) -> Optional[int]:
        """Offset of the layer NetworkFlow() reads (the last IPv4/IPv6), or None."""
        h = int(self.hdr_off[i]) & 0xFFFF
        return None if h == 0xFFFF else h

    def transport_offset(self, i: int) -> Optional[int]:
        """Offset of the layer TransportFlow() reads (the last TCP/UDP), or None."""
        h = int(self.hdr_off[i]) >> 16
        return None if h == 0xFFFF else h

    def NetworkFlow(self, i: int, batch) -> Optional[Flow]:
        """ip4/ip6.NetworkFlow() (ip4.go:63-65, ip6.go:49-51) of packet i as the call leaves the
        object: its addresses read from the packet bytes at the header offset (zero copy from
        `batch`, the PacketBatch decoded), its FastHash the kernel's.  None without one."""
        s = int(self.status[i])
        ept, off = (s >> 20) & 15, self.network_offset(i)
        if ept == 0 or off is None:
            return None
        p = batch.packet(i)
        a, n = (12, 4) if ept == EndpointIPv4 else (8, 16)
        return Flow(ept, p[off + a:off + a + n], p[off + a + n:off + a + 2 * n], self.network_flow_hash(i))

    def TransportFlow(self, i: int, batch) -> Optional[Flow]:
        """tcp/udp.TransportFlow() (tcp.go:331-333, udp.go:123-125): the ports, as above."""
        s = int(self.status[i])
        ept, off = (s >> 24) & 15, self.transport_offset(i)
        if ept == 0 or off is None:
            return None
        p = batch.packet(i)
        return Flow(ept, p[off:off + 2], p[off + 2:off + 4], self.transport_flow_hash(i))

    def layer(self, i: int, name: str):
        """(contents, payload) byte ranges of a layer object after the call, or None."""
        if self.ext is None:
            raise ValueError("layer records need ext=True")
        k = OBJ_NAMES.index(name)
        if not (int(self.ext["obj_valid"][i]) >> k) & 1:
            return None
        r = self.ext["obj"][i][k]
        c0, p0 = int(r["contents_off"]), int(r["payload_off"])
        return (c0, c0 + int(r["contents_len"])), (p0, p0 + int(r["payload_len"]))


def empty_result(n: int, ext: bool = False, detail: bool = False) -> BatchResult:
    return BatchResult(np.zeros(n, np.uint32), np.zeros(n, np.uint64), np.zeros(n, np.uint64),
                       np.zeros(n, np.uint64), np.zeros(n, np.uint32),
                       np.zeros(n, EXT_DTYPE) if ext else None, np.zeros(n, np.uint32),
                       np.zeros(n, DETAIL_DTYPE) if detail else None)
