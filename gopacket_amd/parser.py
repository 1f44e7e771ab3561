"""DecodingLayerParser — the reference's parser surface over the MI355X engine.

Mirrors gopacket's API (parser.go:182-350) with batch entry points added:

    eth, ip4, tcp, payload = Ethernet(), IPv4(), TCP(), Payload()
    parser = NewDecodingLayerParser(LayerTypeEthernet, eth, ip4, tcp, payload)
    parser.IgnoreUnsupported = True
    res = parser.DecodeBatch(batch)          # one kernel launch for the whole batch
    res.decoded(i), res.err(i), res.truncated(i), res.network_flow_hash(i) ...
    err = parser.DecodeLayers(data, decoded) # single packet, same call shape as Go

The decoder objects only select which DecodingLayers are registered (their
CanDecode sets); decoding runs in the HIP kernel through the C-ABI
(include/gpd.h).  A parser snapshots the dispatch tables (layers.TABLES) when
its device context is created; call reload_tables() after Register*().
"""
from __future__ import annotations

import ctypes as C
from typing import Optional

import numpy as np

from . import layers as L
from ._lib import GPD_ERR_PCAP, GpdBatch, GpdConfig, GpdResult, check, lib
from .batch import PAD, PacketBatch
from .errors import UnsupportedLayerType
from .results import DETAIL_DTYPE, EXT_DTYPE, RECORD_DTYPE, BatchResult

DEC_ETHERNET, DEC_DOT1Q, DEC_IPV4, DEC_IPV6, DEC_IPV6_EXT = 1, 2, 4, 8, 16
DEC_TCP, DEC_UDP, DEC_VXLAN, DEC_PAYLOAD, DEC_FRAGMENT = 32, 64, 128, 256, 512
DEC_ICMPV4, DEC_LLC = 1024, 2048
OPT_IGNORE_UNSUPPORTED, OPT_IGNORE_PANIC = 1, 2
OPT_NO_CHECKSUMS, OPT_NO_FLOW_HASH = 256, 512


class DecodingLayer:
    """A registrable decoder (parser.go:29-46); `bit` selects it in the kernel."""
    bit = 0
    can_decode: tuple = ()

    def CanDecode(self):
        return self.can_decode


class Ethernet(DecodingLayer):      # layers/ethernet.go:106-108
    bit, can_decode = DEC_ETHERNET, (L.LayerTypeEthernet,)


class Dot1Q(DecodingLayer):         # layers/dot1q.go:43-45
    bit, can_decode = DEC_DOT1Q, (L.LayerTypeDot1Q,)


class IPv4(DecodingLayer):          # layers/ip4.go:277-279
    bit, can_decode = DEC_IPV4, (L.LayerTypeIPv4,)


class IPv6(DecodingLayer):          # layers/ip6.go:281-283
    bit, can_decode = DEC_IPV6, (L.LayerTypeIPv6,)


class IPv6ExtensionSkipper(DecodingLayer):  # layers/ip6.go:454-456
    bit, can_decode = DEC_IPV6_EXT, L.LayerClassIPv6Extension


class TCP(DecodingLayer):           # layers/tcp.go:304-306
    bit, can_decode = DEC_TCP, (L.LayerTypeTCP,)


class UDP(DecodingLayer):           # layers/udp.go:98-100
    bit, can_decode = DEC_UDP, (L.LayerTypeUDP,)


class VXLAN(DecodingLayer):         # layers/vxlan.go:43-45
    bit, can_decode = DEC_VXLAN, (L.LayerTypeVXLAN,)


class Payload(DecodingLayer):       # base.go:54
    bit, can_decode = DEC_PAYLOAD, (L.LayerTypePayload,)


class Fragment(DecodingLayer):      # base.go:111
    bit, can_decode = DEC_FRAGMENT, (L.LayerTypeFragment,)


class ICMPv4(DecodingLayer):        # layers/icmp4.go:256-258
    bit, can_decode = DEC_ICMPV4, (L.LayerTypeICMPv4,)


class LLC(DecodingLayer):           # layers/llc.go:55-57
    bit, can_decode = DEC_LLC, (L.LayerTypeLLC,)


DECODER_BY_NAME = {c.__name__: c for c in (Ethernet, Dot1Q, IPv4, IPv6, IPv6ExtensionSkipper, TCP,
                                            UDP, VXLAN, Payload, Fragment, ICMPv4, LLC)}


# ---- DecodingLayerContainer (parser.go:54-177) ------------------------------------------------
class DecodingLayerContainer:
    """parser.go:56-67: Put / Decoder / LayersDecoder.  Put returns the container (the reference's
    value-receiver convention).  The engine registers decoder *kinds*: `engine_mask()` is the set
    of kinds the container holds for every type of their CanDecode set."""

    def Put(self, d) -> "DecodingLayerContainer":
        raise NotImplementedError

    def Decoder(self, typ: int):
        raise NotImplementedError

    def LayersDecoder(self, first: int, df=None, device: int = 0) -> "DecodingLayerFunc":
        """layers_decoder.go:11-101: a DecodingLayerFunc over this container's decoders."""
        return DecodingLayerFunc(self, first, df, device)

    def held(self):
        """Every decoder the container holds (the three containers below enumerate theirs; a
        user container is probed at the LayerTypes this engine's decoders take)."""
        for cls in DECODER_BY_NAME.values():
            for t in cls.can_decode:
                d, ok = self.Decoder(t)
                if ok:
                    yield t, d

    def engine_mask(self) -> int:
        """The decoder kinds to register; a held decoder this engine cannot run (a user-defined
        DecodingLayer, or one of ours under a LayerType outside its CanDecode) is refused with
        the TypeError NewDecodingLayerParser raises for it, instead of being dropped silently
        (its packets would stop with UnsupportedLayerType later)."""
        for t, d in self.held():
            if not isinstance(d, DecodingLayer) or not d.bit or t not in d.can_decode:
                raise TypeError(f"{d!r} (held for LayerType {t}) is not a DecodingLayer this engine implements")
        m = 0
        for cls in DECODER_BY_NAME.values():
            held = [isinstance(self.Decoder(t)[0], cls) for t in cls.can_decode]
            if all(held):
                m |= cls.bit
            elif any(held):  # (e.g. IPv6ExtensionSkipper for some of 46..49 only)
                raise ValueError(f"{cls.__name__} is held for only part of its CanDecode set "
                                 f"{cls.can_decode}: the engine registers decoder kinds whole")
        return m


class DecodingLayerSparse(DecodingLayerContainer):
    """parser.go:69-108: a slice indexed by LayerType."""

    def __init__(self, layers=None):
        self.dl = list(layers or [])

    def Put(self, d):
        for t in d.CanDecode():
            if t >= len(self.dl):
                self.dl.extend([None] * (t + 1 - len(self.dl)))
            self.dl[t] = d
        return self

    def Decoder(self, typ):
        if 0 <= typ < len(self.dl) and self.dl[typ] is not None:
            return self.dl[typ], True
        return None, False

    def held(self):
        return ((t, d) for t, d in enumerate(self.dl) if d is not None)


class DecodingLayerArray(DecodingLayerContainer):
    """parser.go:110-146: (type, decoder) pairs searched linearly; a Put of a type already held
    replaces its decoder in place."""

    def __init__(self):
        self.dl = []

    def Put(self, d):
        for t in d.CanDecode():
            for e in self.dl:
                if e[0] == t:
                    e[1] = d
                    break
            else:
                self.dl.append([t, d])
        return self

    def Decoder(self, typ):
        for t, d in self.dl:
            if t == typ:
                return d, True
        return None, False

    def held(self):
        return ((t, d) for t, d in self.dl)


class DecodingLayerMap(DecodingLayerContainer):
    """parser.go:148-169: a map by LayerType (NewDecodingLayerParser's default)."""

    def __init__(self):
        self.dl = {}

    def Put(self, d):
        for t in d.CanDecode():
            self.dl[t] = d
        return self

    def Decoder(self, typ):
        d = self.dl.get(typ)
        return d, d is not None

    def held(self):
        return iter(list(self.dl.items()))


class DecodingLayerFunc:
    """parser.go:52 / layers_decoder.go:11-101: fn(data, decoded) -> (LayerType, error) for one
    packet, decoded on the GPU with the container's decoders: (first, None) leaving `decoded`
    untouched when no decoder takes `first`; (0, err) on a decode error; (typ, None) when no
    decoder takes typ; (0, None) on success.  A Truncated packet calls df.SetTruncated()."""

    def __init__(self, dlc: DecodingLayerContainer, first: int, df, device: int):
        self.first, self.df = int(first), df
        self.has_first = dlc.Decoder(self.first)[1]
        self.p = DecodingLayerParser(self.first, device=device)
        self.p._mask = dlc.engine_mask()

    def __call__(self, data: bytes, decoded: list):
        if not self.has_first:
            return self.first, None
        res = self.p.DecodeBatch(PacketBatch.from_packets([data]), detail=True)
        decoded[:] = res.decoded(0)
        if res.truncated(0) and self.df is not None:
            self.df.SetTruncated()
        st = int(res.status[0]) & 3
        if st == 2:
            return L.LayerTypeZero, res.err(0)
        if st == 1:
            return res.stop_type(0), None
        return L.LayerTypeZero, None


def decoder_mask(decoders) -> int:
    m = 0
    for d in decoders:
        if isinstance(d, str):
            d = DECODER_BY_NAME[d]
        if isinstance(d, type):
            d = d()
        if not isinstance(d, DecodingLayer):
            raise TypeError(f"{d!r} is not a DecodingLayer this engine implements")
        m |= d.bit
    return m


def _torch():
    import torch
    if not torch.cuda.is_available():
        raise RuntimeError("gopacket_amd: no GPU visible to torch; the decode path runs only on HIP")
    return torch


class _Ctx:
    """One gpd_ctx on a device: its decoder set and options change in place (ABI 8), as the
    reference parser's do; only a new device or first layer makes a new context."""

    def __init__(self, device: int, first: int, mask: int, options: int, tables: L.DispatchTables):
        self.tables = tables.copy()
        cfg = self._cfg(first, mask, options)
        h = C.c_void_p()
        check(lib.gpd_ctx_create(device, C.byref(cfg), C.byref(h)), "gpd_ctx_create")
        self.h = h
        self.device, self.first, self.mask, self.options = device, first, mask, options

    def _cfg(self, first, mask, options):
        t = self.tables
        return GpdConfig(first, mask, options, 0, t.ethertype.ctypes.data, t.ipproto.ctypes.data,
                         t.tcp_port.ctypes.data, t.udp_port.ctypes.data)

    def reload(self, tables: L.DispatchTables):
        self.tables = tables.copy()
        cfg = self._cfg(self.first, self.mask, self.options)
        check(lib.gpd_ctx_reload_tables(self.h, C.byref(cfg)), "gpd_ctx_reload_tables")

    def set_options(self, options: int):
        if options != self.options:
            check(lib.gpd_ctx_set_options(self.h, options), "gpd_ctx_set_options")
            self.options = options

    def add_decoders(self, mask: int):
        if mask | self.mask != self.mask:
            check(lib.gpd_ctx_add_decoders(self.h, mask), "gpd_ctx_add_decoders")
            self.mask |= mask

    def set_decoders(self, mask: int):
        if mask == self.mask:
            return
        if mask & ~self.mask == mask ^ self.mask:  # only added: AddDecodingLayer
            self.add_decoders(mask)
            return
        check(lib.gpd_ctx_set_decoders(self.h, mask), "gpd_ctx_set_decoders")
        self.mask = mask

    def __del__(self):
        h = getattr(self, "h", None)
        if h is not None and h.value:
            lib.gpd_ctx_destroy(h)
            self.h = None


class DeviceBatch:
    """A PacketBatch resident in HBM (torch tensors on `device`)."""

    def __init__(self, batch: PacketBatch, device: int = 0):
        torch = _torch()
        dev = torch.device("cuda", device)
        self.n = batch.n
        self.data_len = batch.data_len
        self.data = torch.from_numpy(batch.data).to(dev)
        # offset[] and caplen[] share one allocation, caplen[] right after offset[]: the two
        # descriptor streams are read in lock-step, and their relative placement in HBM moves
        # the 4 KiB kernels by 4-5 % (DESIGN §5a "Tile order and descriptor placement");
        # adjacent halves of one allocation measured fast at every address tried.  caplen[]
        # starts on a 64-B boundary (no gap when n is a multiple of 16).
        n, pad = self.n, (-self.n) % 16
        host = np.zeros(2 * n + pad, dtype=np.int32)
        host[:n] = batch.offset.view(np.int32)
        host[n + pad:] = batch.caplen.view(np.int32)
        desc = torch.from_numpy(host).to(dev)
        self.offset, self.caplen = desc[:n], desc[n + pad:]
        self.device = device

    def c_batch(self) -> GpdBatch:
        return GpdBatch(self.data.data_ptr(), self.data_len, self.offset.data_ptr(),
                        self.caplen.data_ptr(), self.n)


class DeviceResult:
    """Results in HBM — the SoA arrays, or (records=True) one 32-B gpd_record per packet;
    .to_host() gives a BatchResult either way.  detail=True adds the gpd_detail array (the
    error arguments and deep stacks, written by the generic decoder only: the fast path stays
    on)."""

    def __init__(self, n: int, device: int = 0, ext: bool = False, hdr_off: bool = True,
                 records: bool = False, detail: bool = False):
        torch = _torch()
        dev = torch.device("cuda", device)
        self.n = n
        self.records = None
        if records:
            self.records = torch.empty(n * RECORD_DTYPE.itemsize, dtype=torch.uint8, device=dev)
            self.status = self.layers = self.net_hash = self.tp_hash = self.csum = None
        else:
            self.status = torch.empty(n, dtype=torch.int32, device=dev)
            self.layers = torch.empty(n, dtype=torch.int64, device=dev)
            self.net_hash = torch.empty(n, dtype=torch.int64, device=dev)
            self.tp_hash = torch.empty(n, dtype=torch.int64, device=dev)
            self.csum = torch.empty(n, dtype=torch.int32, device=dev)
        self.ext = torch.empty(n * EXT_DTYPE.itemsize, dtype=torch.uint8, device=dev) if ext else None
        self.hdr_off = torch.empty(n, dtype=torch.int32, device=dev) if hdr_off else None
        # (the kernel writes a packet's detail only where its status asks for one; to_host copies
        # back just those rows)
        self.detail = torch.empty(n * DETAIL_DTYPE.itemsize, dtype=torch.uint8, device=dev) if detail else None

    def c_result(self) -> GpdResult:
        p = lambda t: t.data_ptr() if t is not None else None
        return GpdResult(p(self.status), p(self.layers), p(self.net_hash), p(self.tp_hash),
                         p(self.csum), p(self.ext), p(self.hdr_off), p(self.records), p(self.detail))

    def to_host(self) -> BatchResult:
        u = lambda t, dt: t.cpu().numpy().view(dt)
        ext = self.ext.cpu().numpy().view(EXT_DTYPE) if self.ext is not None else None
        hoff = u(self.hdr_off, np.uint32) if self.hdr_off is not None else None
        if self.records is not None:
            r = self.records.cpu().numpy().view(RECORD_DTYPE)
            res = BatchResult(r["status"].copy(), r["layers"].copy(), r["net_hash"].copy(),
                              r["tp_hash"].copy(), r["csum"].copy(), ext, hoff, None)
        else:
            res = BatchResult(u(self.status, np.uint32), u(self.layers, np.uint64),
                              u(self.net_hash, np.uint64), u(self.tp_hash, np.uint64),
                              u(self.csum, np.uint32), ext, hoff, None)
        if self.detail is not None:
            res.detail = self._detail_rows(res.status)
        return res

    def _detail_rows(self, status: np.ndarray) -> np.ndarray:
        """The detail records of the packets that have one (decode errors, > 12 layers; gpd.h
        gpd_detail), gathered on the device so the copy back is 24 B per such packet, not per
        packet; every other entry is zero."""
        torch = _torch()
        st = status.astype(np.uint32)
        rows = np.nonzero(((st & 3) == 2) | (((st >> 4) & 31) > 12) | (((st >> 3) & 1) == 1))[0]
        det = np.zeros(self.n, DETAIL_DTYPE)
        if len(rows):
            d = self.detail.view(self.n, DETAIL_DTYPE.itemsize)
            idx = torch.from_numpy(rows.astype(np.int64)).to(d.device)
            det[rows] = d.index_select(0, idx).cpu().numpy().view(DETAIL_DTYPE).reshape(-1)
        return det


class DecodingLayerParser:
    """parser.go:182-195 (DecodingLayerParser) + :336-350 (options)."""

    def __init__(self, first: int, *decoders, device: int = 0):
        self.first = int(first)
        self._mask = decoder_mask(decoders)
        self.IgnoreUnsupported = False
        self.IgnorePanic = False
        self.ComputeChecksums = True   # engine knob: the fused ComputeChecksum / ip4 checksum
        self.ComputeFlowHashes = True  # engine knob: the fused FastHash
        self.Truncated = False
        self.device = device
        self._ctx: Optional[_Ctx] = None
        self._tables = L.TABLES.copy()
        self._dlc: DecodingLayerContainer = DecodingLayerMap()  # parser.go:226 (the default)
        for d in decoders:
            d = DECODER_BY_NAME[d]() if isinstance(d, str) else (d() if isinstance(d, type) else d)
            self._dlc = self._dlc.Put(d)

    # --- registration (parser.go:197-241) ---------------------------------------
    def AddDecodingLayer(self, d) -> None:
        """parser.go:197-202 (the container's Put); applied to an existing context in place
        (gpd_ctx_add_decoders)."""
        d = DECODER_BY_NAME[d]() if isinstance(d, str) else (d() if isinstance(d, type) else d)
        self._mask |= decoder_mask([d])
        self._dlc = self._dlc.Put(d)

    def SetDecodingLayerContainer(self, dlc: DecodingLayerContainer) -> None:
        """parser.go:236-242: the container's decoders replace the registered set
        (gpd_ctx_set_decoders on an existing context: device and tables kept)."""
        mask = dlc.engine_mask()  # a container this engine cannot run is refused, parser unchanged
        self._dlc, self._mask = dlc, mask

    def SetTruncated(self) -> None:
        """parser.go:204-209 (DecodeFeedback)."""
        self.Truncated = True

    @property
    def decoders(self) -> int:
        return self._mask

    def reload_tables(self) -> None:
        """Re-snapshot layers.TABLES (after RegisterTCPPortLayerType etc.)."""
        self._tables = L.TABLES.copy()
        if self._ctx is not None:
            self._ctx.reload(self._tables)

    @property
    def options(self) -> int:
        o = OPT_IGNORE_UNSUPPORTED if self.IgnoreUnsupported else 0
        o |= OPT_IGNORE_PANIC if self.IgnorePanic else 0
        o |= 0 if self.ComputeChecksums else OPT_NO_CHECKSUMS
        o |= 0 if self.ComputeFlowHashes else OPT_NO_FLOW_HASH
        o |= getattr(self, "_diag_options", 0)
        return o

    def ctx(self) -> _Ctx:
        """The device context, created once per (device, first layer); options and added
        decoders apply in place (gpd_ctx_set_options / gpd_ctx_add_decoders), so the table
        snapshot, tuning and staging survive them as the reference parser's state does."""
        c = self._ctx
        if c is None or (c.device, c.first) != (self.device, self.first):
            self._ctx = c = _Ctx(self.device, self.first, self._mask, self.options, self._tables)
            c.tuned = None
        else:
            c.set_decoders(self._mask)
            c.set_options(self.options)
        if self._ctx.tuned != self.Tuning:
            self._apply_tuning()
        return self._ctx

    # Engine tuning (gpd_ctx_set_tuning): staging choices that never change a result.
    # Keys: window_bytes (0 auto / 4096 / 8192), shift and reg_prefix (-1 auto / 0 / 1),
    # waves_per_simd (0 auto / 2 / 3 / 4), header_once (-1 auto / 0 / 1 windows / 2 rounds),
    # device_walk (-1 auto / 0 / 1), grid_rounds (0 auto / 1..8) and split (-1 auto / 0 / 1).
    Tuning: Optional[dict] = None

    def _apply_tuning(self):
        from ._lib import GpdTuning
        t = dict(window_bytes=0, shift=-1, reg_prefix=-1, waves_per_simd=0, header_once=-1,
                 device_walk=-1, grid_rounds=0, split=-1)
        t.update(self.Tuning or {})
        g = GpdTuning(int(t["window_bytes"]), int(t["shift"]), int(t["reg_prefix"]),
                      int(t["waves_per_simd"]), int(t["header_once"]), int(t["device_walk"]),
                      int(t["grid_rounds"]), int(t["split"]))
        check(lib.gpd_ctx_set_tuning(self._ctx.h, C.byref(g)), "gpd_ctx_set_tuning")
        self._ctx.tuned = dict(self.Tuning) if self.Tuning else None

    # --- decoding -----------------------------------------------------------------
    def decode_device(self, dbatch: DeviceBatch, dres: DeviceResult, stream=None) -> None:
        """Asynchronous decode of an HBM-resident batch on `stream` (torch stream or None =
        torch's current stream)."""
        torch = _torch()
        if stream is None:
            stream = torch.cuda.current_stream(self.device)
        b, r = dbatch.c_batch(), dres.c_result()
        check(lib.gpd_decode(self.ctx().h, C.byref(b), C.byref(r), C.c_void_p(stream.cuda_stream)),
              "gpd_decode")

    def DecodeBatch(self, batch: PacketBatch, ext: bool = False, detail: bool = True,
                    records: bool = False) -> BatchResult:
        """Decode every packet of a host batch on the GPU (H2D, kernel, D2H).  With detail (the
        default) res.err(i) carries the reference's exact text and res.decoded(i) any depth; the
        batch keeps the fast path, and only the failing / deep packets' 24-B records come back
        (a device gather: no extra transfer for a clean batch).  ext adds the layer records
        (generic path); records selects the gpd_record result form on the device (the form the
        loader / decoder split kernel writes for small frames)."""
        torch = _torch()
        db = DeviceBatch(batch, self.device)
        dr = DeviceResult(batch.n, self.device, ext, detail=detail, records=records)
        self.decode_device(db, dr)
        torch.cuda.synchronize(self.device)
        return dr.to_host()

    def DecodeBatchHost(self, batch: PacketBatch, ext: bool = False,
                        out: Optional[BatchResult] = None, detail: bool = False) -> BatchResult:
        """Host-memory path through gpd_decode_host (pinned, chunked, double-buffered).
        `out` reuses a result of the same size (no allocation per call; its detail array, if
        any, is filled)."""
        n = batch.n
        res = out if out is not None else BatchResult(
            np.zeros(n, np.uint32), np.zeros(n, np.uint64), np.zeros(n, np.uint64),
            np.zeros(n, np.uint64), np.zeros(n, np.uint32), np.zeros(n, EXT_DTYPE) if ext else None,
            np.zeros(n, np.uint32), np.zeros(n, DETAIL_DTYPE) if detail else None)
        b = GpdBatch(batch.data.ctypes.data, batch.data_len, batch.offset.ctypes.data,
                     batch.caplen.ctypes.data, n)
        r = _c_result(res)
        check(lib.gpd_decode_host(self.ctx().h, C.byref(b), C.byref(r)), "gpd_decode_host")
        return res

    def DecodePcap(self, cap: np.ndarray, max_n: Optional[int] = None, nthreads: int = 0,
                   data_len: Optional[int] = None, out: Optional[BatchResult] = None,
                   detail: bool = False):
        """A whole in-memory capture (pcap.capture_array) through gpd_decode_pcap: records
        indexed natively, their raw bytes chunked host -> device, decoded, results back.
        Returns (BatchResult of the decoded records, number of records, error text or None —
        the ReadPacketData loop's stop, pcapgo/read.go:120-137).  `out` (a BatchResult with
        hdr_off, at least max_n entries) is reused when given."""
        dl = cap.shape[0] - PAD if data_len is None else int(data_len)
        m = (dl - 24) // 16 + 1 if max_n is None else int(max_n)
        if out is not None:
            if len(out.status) < m or out.hdr_off is None:
                raise ValueError("DecodePcap: out must hold max_n entries, with hdr_off")
            res = out
        else:
            res = BatchResult(np.zeros(m, np.uint32), np.zeros(m, np.uint64), np.zeros(m, np.uint64),
                              np.zeros(m, np.uint64), np.zeros(m, np.uint32), None,
                              np.zeros(m, np.uint32), np.zeros(m, DETAIL_DTYPE) if detail else None)
        r = _c_result(res)
        n, nxt, stop = C.c_uint64(), C.c_uint64(), C.c_int()
        rc = lib.gpd_decode_pcap(self.ctx().h, cap.ctypes.data, dl, m, C.byref(r), C.byref(n),
                                 C.byref(nxt), C.byref(stop), int(nthreads))
        err = None
        if rc == GPD_ERR_PCAP:
            err = lib.gpd_last_error_string().decode()
        elif rc != 0:
            check(rc, "gpd_decode_pcap")
        k = n.value
        return _head(res, k), k, err

    def DecodePcapAt(self, cap: np.ndarray, info, pos: int, max_n: int, out: BatchResult,
                     nthreads: int = 0, data_len: Optional[int] = None):
        """The ReadPacketData loop continued from record header `pos` (gpd_decode_pcap_at): the
        next max_n records decoded into `out` (a BatchResult with hdr_off and at least max_n
        entries, reused across calls).  Returns (records decoded, next record position, STOP_*,
        error text or None)."""
        dl = cap.shape[0] - PAD if data_len is None else int(data_len)
        if len(out.status) < max_n or out.hdr_off is None:
            raise ValueError("DecodePcapAt: out must hold max_n entries, with hdr_off")
        r = _c_result(out)
        n, nxt, stop = C.c_uint64(), C.c_uint64(), C.c_int()
        rc = lib.gpd_decode_pcap_at(self.ctx().h, cap.ctypes.data, dl, C.byref(info), int(pos),
                                    int(max_n), C.byref(r), C.byref(n), C.byref(nxt), C.byref(stop),
                                    int(nthreads))
        err = None
        if rc == GPD_ERR_PCAP:
            err = lib.gpd_last_error_string().decode()
        elif rc != 0:
            check(rc, "gpd_decode_pcap_at")
        return n.value, nxt.value, stop.value, err

    def DecodeTPv3(self, ring, max_n: int = 1 << 20, max_blocks: Optional[int] = None,
                   add_vlan_header: bool = False, nthreads: int = 0, out=None, ci=None,
                   detail: bool = False):
        """Every packet of the user-owned blocks of a TPACKET_V3 ring (afpacket.TPv3Ring) from
        ring.offset on, decoded on the GPU where it lies (gpd_decode_tpv3).  The blocks are not
        released.  Returns (BatchResult, CaptureInfo, blocks walked).  `out` (a BatchResult with
        hdr_off) and `ci` (a CaptureInfo), both of at least max_n entries, are reused when given
        — a capture loop keeps them across calls instead of touching fresh pages each time.
        detail adds the gpd_detail records (exact error texts, deep stacks) to a new `out`."""
        from .afpacket import CaptureInfo
        if ci is None:
            ci = CaptureInfo.alloc(max_n)
        res = out if out is not None else BatchResult(
            np.zeros(max_n, np.uint32), np.zeros(max_n, np.uint64), np.zeros(max_n, np.uint64),
            np.zeros(max_n, np.uint64), np.zeros(max_n, np.uint32), None, np.zeros(max_n, np.uint32),
            np.zeros(max_n, DETAIL_DTYPE) if detail else None)
        if len(res.status) < max_n or res.hdr_off is None or len(ci.offset) < max_n:
            raise ValueError("DecodeTPv3: out / ci must hold max_n entries (out with hdr_off)")
        r = _c_result(res)
        n, nb = C.c_uint64(), C.c_uint32()
        check(lib.gpd_decode_tpv3(self.ctx().h, C.byref(ring.c), ring.offset % ring.num_blocks,
                                  ring.num_blocks if max_blocks is None else int(max_blocks),
                                  int(bool(add_vlan_header)), int(max_n), C.byref(r),
                                  C.byref(ci.c()), C.byref(n), C.byref(nb), int(nthreads)),
              "gpd_decode_tpv3")
        k = n.value
        return _head(res, k), ci.head(k), nb.value

    def DecodeLayers(self, data: bytes, decoded: list):
        """parser.go:302-316 for one packet: fills `decoded`, sets self.Truncated, returns the
        error value (None on success)."""
        self.Truncated = False
        if not any(c.bit & self._mask and self.first in c.can_decode for c in DECODER_BY_NAME.values()):
            # layers_decoder.go:12-16: no decoder for `first` returns before `decoded` is
            # truncated, so the caller's slice keeps its previous contents
            return None if self.IgnoreUnsupported else UnsupportedLayerType(self.first)
        res = self.DecodeBatch(PacketBatch.from_packets([data]), detail=True)
        decoded[:] = res.decoded(0)
        self.Truncated = res.truncated(0)
        return res.err(0)


def _c_result(res: BatchResult) -> GpdResult:
    """The C-ABI result struct over a host BatchResult's arrays (SoA; absent arrays NULL)."""
    p = lambda a: a.ctypes.data if a is not None else None
    return GpdResult(p(res.status), p(res.layers), p(res.net_hash), p(res.tp_hash), p(res.csum),
                     p(res.ext), p(res.hdr_off), None, p(res.detail))


def _head(res: BatchResult, k: int) -> BatchResult:
    h = lambda a: a[:k] if a is not None else None
    return BatchResult(h(res.status), h(res.layers), h(res.net_hash), h(res.tp_hash), h(res.csum),
                       h(res.ext), h(res.hdr_off), h(res.detail))


def NewDecodingLayerParser(first: int, *decoders, device: int = 0) -> DecodingLayerParser:
    """parser.go:222-233."""
    return DecodingLayerParser(first, *decoders, device=device)
