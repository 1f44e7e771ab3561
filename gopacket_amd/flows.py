"""Flow table: tcpassembly's connection map for a whole decoded batch, on the GPU.

Mirrors the reference's StreamPool (tcpassembly/assembly.go:305-343): the pool maps
key{NetworkFlow(), TransportFlow()} (assembly.go:289,543) to a connection, creating one for
a new key (getConnection, assembly.go:495-511).  Here `FlowTable.Insert` does that lookup
for every packet of an HBM-resident batch the parser just decoded, in one launch
(gpd_flow_insert, include/gpd_flow.h), and returns each packet's flow record index.  The
records keep the key (raw endpoint bytes and EndpointTypes, as gopacket.Flow holds them,
flows.go:140-146) and per-flow counters.  Flows are directional, as Flow map keys are.
"""
from __future__ import annotations

import ctypes as C
from typing import Optional

import numpy as np

from ._lib import check, lib
from .parser import DeviceBatch, DeviceResult, DecodingLayerParser, _torch

FLOW_REC_DTYPE = np.dtype([("fp", "<u8"), ("src", "u1", (16,)), ("dst", "u1", (16,)),
                           ("sport", "u1", (2,)), ("dport", "u1", (2,)), ("net_type", "u1"),
                           ("tp_type", "u1"), ("addr_len", "u1"), ("reserved", "u1"),
                           ("first", "<u8"), ("packets", "<u8"), ("bytes", "<u8"), ("last", "<u8")])
assert FLOW_REC_DTYPE.itemsize == 80

FLOW_NONE, FLOW_FULL, FLOW_COLLISION = 0xFFFFFFFF, 0xFFFFFFFE, 0x80000000


class FlowStats(C.Structure):
    _fields_ = [("flows", C.c_uint64), ("packets", C.c_uint64), ("no_key", C.c_uint64),
                ("full", C.c_uint64), ("collisions", C.c_uint64), ("capacity", C.c_uint64)]

    def as_dict(self) -> dict:
        return {f: int(getattr(self, f)) for f, _ in self._fields_}


class FlowTable:
    """A GPU flow table of at least `capacity` records on the parser's device."""

    def __init__(self, parser: DecodingLayerParser, capacity: int):
        self.parser = parser
        h = C.c_void_p()
        check(lib.gpd_flow_create(parser.ctx().h, int(capacity), C.byref(h)), "gpd_flow_create")
        self.h = h

    def __del__(self):
        if getattr(self, "h", None):
            lib.gpd_flow_destroy(self.h)
            self.h = None

    def Reset(self, stream=None) -> None:
        check(lib.gpd_flow_reset(self.h, self._stream(stream)), "gpd_flow_reset")

    def _stream(self, stream):
        torch = _torch()
        s = stream if stream is not None else torch.cuda.current_stream(self.parser.device)
        return C.c_void_p(s.cuda_stream)

    def Insert(self, dbatch: DeviceBatch, dres: DeviceResult, flow_id=None, index_base: int = 0,
               stream=None):
        """getConnection for every packet of a decoded device batch (asynchronous).  Returns
        the int32 device tensor of flow record indices (GPD_FLOW_* values as uint32)."""
        torch = _torch()
        if dres.hdr_off is None:
            raise ValueError("FlowTable.Insert needs a DeviceResult with hdr_off")
        if flow_id is None:
            flow_id = torch.empty(dbatch.n, dtype=torch.int32, device=dres.status.device)
        b, r = dbatch.c_batch(), dres.c_result()
        check(lib.gpd_flow_insert(self.h, C.byref(b), C.byref(r), C.c_void_p(flow_id.data_ptr()),
                                  int(index_base), self._stream(stream)), "gpd_flow_insert")
        return flow_id

    def Stats(self, stream=None) -> dict:
        st = FlowStats()
        check(lib.gpd_flow_stats_get(self.h, C.byref(st), self._stream(stream)), "gpd_flow_stats_get")
        return st.as_dict()

    def Export(self, max_flows: Optional[int] = None, stream=None):
        """(records FLOW_REC_DTYPE[m] ordered by first packet, their record indices)."""
        m = self.Stats(stream)["flows"] if max_flows is None else int(max_flows)
        recs = np.zeros(m, FLOW_REC_DTYPE)
        idx = np.zeros(m, np.uint32)
        n = C.c_uint64()
        check(lib.gpd_flow_export(self.h, recs.ctypes.data, idx.ctypes.data, m, C.byref(n),
                                  self._stream(stream)), "gpd_flow_export")
        return recs[:n.value], idx[:n.value]


def NewFlowTable(parser: DecodingLayerParser, capacity: int) -> FlowTable:
    return FlowTable(parser, capacity)
