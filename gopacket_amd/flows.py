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
            flow_id = torch.empty(dbatch.n, dtype=torch.int32, device=dres.hdr_off.device)
        b, r = dbatch.c_batch(), dres.c_result()
        check(lib.gpd_flow_insert(self.h, C.byref(b), C.byref(r), C.c_void_p(flow_id.data_ptr()),
                                  int(index_base), self._stream(stream)), "gpd_flow_insert")
        return flow_id

    def _test_fingerprint_bits(self, bits: int) -> None:
        """Testing hook (gpd_flow_test_fingerprint_bits): narrow every key fingerprint to
        `bits` bits so that distinct keys collide; call on an empty table."""
        check(lib.gpd_flow_test_fingerprint_bits(self.h, int(bits)), "gpd_flow_test_fingerprint_bits")

    def _test_counter_bits(self, bits: int) -> None:
        """Testing hook (gpd_flow_test_counter_bits): split the packed counter word at `bits`
        so that its fields carry and wrap within a test; call on an empty table."""
        check(lib.gpd_flow_test_counter_bits(self.h, int(bits)), "gpd_flow_test_counter_bits")

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


# ---------------------------------------------------------------- flow-affine sharding
FLOW_KEY_DTYPE = np.dtype([("key", "<u4", (10,)), ("caplen", "<u4"), ("owner", "<u4"),
                           ("seq", "<u8"), ("fp", "<u8")])
assert FLOW_KEY_DTYPE.itemsize == 64
KEY_WORDS = 8  # a key record as int64 words: the unit the exchange moves


def exchange_keys(keys, counts, group=None):
    """The all-to-all of key records: `keys` is an int64 tensor [m, 8] grouped
    by owner rank, `counts` the records per owner (host ints).  Returns (received records
    [r, 8], records received from each rank).  On a `gloo` group the records travel through
    host memory; on `nccl` (RCCL over xGMI) they stay in HBM."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    assert len(counts) == world
    host = dist.get_backend(group) == "gloo"
    dev = keys.device
    send_counts = torch.tensor([int(c) for c in counts], dtype=torch.int64)
    recv_counts = torch.empty(world, dtype=torch.int64)
    if host:
        dist.all_to_all_single(recv_counts, send_counts, group=group)
    else:
        rc = recv_counts.to(dev)
        dist.all_to_all_single(rc, send_counts.to(dev), group=group)
        recv_counts = rc.cpu()
    rcv = [int(c) for c in recv_counts]
    src = keys.cpu() if host else keys
    out = torch.empty((sum(rcv), KEY_WORDS), dtype=torch.int64, device=src.device)
    dist.all_to_all_single(out, src.contiguous(), output_split_sizes=rcv,
                           input_split_sizes=[int(c) for c in counts], group=group)
    return (out.to(dev) if host else out), rcv


def return_ids(ids, recv_counts, send_counts, group=None):
    """The reverse all-to-all: each rank's flow ids for the records it received go back to the
    senders, in the order they were sent."""
    import torch
    import torch.distributed as dist
    host = dist.get_backend(group) == "gloo"
    dev = ids.device
    src = ids.cpu() if host else ids
    out = torch.empty(sum(int(c) for c in send_counts), dtype=ids.dtype, device=src.device)
    dist.all_to_all_single(out, src.contiguous(), output_split_sizes=[int(c) for c in send_counts],
                           input_split_sizes=[int(c) for c in recv_counts], group=group)
    return out.to(dev) if host else out


class ShardedFlowTable:
    """The flow table sharded over the ranks of a torch.distributed group, one table per GPU.

    The reference fans packets out to workers by flow hash (doc.go:216-228,
    `flow.FastHash() % numWorkers`); here every rank decodes its own packets, turns the keyed
    ones into 64-byte key records grouped by owning rank (gpd_flow_keys), exchanges them with
    one all-to-all (RCCL over xGMI on `nccl`), and inserts what it received into its table
    (gpd_flow_insert_keys).  Each flow, both directions of a conversation included, lives on
    exactly one rank.  Insert returns each local packet's (owner rank, flow record index on
    that rank); Export lists this rank's flows."""

    def __init__(self, parser: DecodingLayerParser, capacity: int, group=None):
        import torch.distributed as dist
        self.table = FlowTable(parser, capacity)
        self.group = group
        self.single = not (dist.is_available() and dist.is_initialized())  # one rank, no exchange
        self.world = 1 if self.single else dist.get_world_size(group)
        self.rank = 0 if self.single else dist.get_rank(group)
        self.last_ms = {}  # host-clock phases of the last Insert (synchronised), for diagnostics

    def Insert(self, dbatch: DeviceBatch, dres: DeviceResult, index_base: int = 0, stream=None):
        """Partition, exchange, insert (synchronous).  Returns int32 device tensors (owner rank
        per packet, -1 without a key; flow record index on the owner, GPD_FLOW_* as uint32)."""
        import time
        torch = _torch()
        t = self.table
        if dres.hdr_off is None:
            raise ValueError("ShardedFlowTable.Insert needs a DeviceResult with hdr_off")
        dev = dres.hdr_off.device
        t0 = time.perf_counter()
        keys = torch.empty((max(dbatch.n, 1), KEY_WORDS), dtype=torch.int64, device=dev)
        counts = (C.c_uint64 * self.world)()
        b, r = dbatch.c_batch(), dres.c_result()
        check(lib.gpd_flow_keys(t.h, C.byref(b), C.byref(r), self.world, int(index_base),
                                C.c_void_p(keys.data_ptr()), counts, t._stream(stream)), "gpd_flow_keys")
        send = [int(c) for c in counts]
        m = sum(send)
        t1 = time.perf_counter()
        if self.single:
            recv, rcv = keys[:m], send
        else:
            recv, rcv = exchange_keys(keys[:m], send, self.group)
            # the collective completes on torch's current stream; a caller's own stream must
            # wait for it before the insert reads the received records
            self._after_collective(stream, dev)
        t2 = time.perf_counter()
        ids = torch.empty(max(recv.shape[0], 1), dtype=torch.int32, device=dev)
        check(lib.gpd_flow_insert_keys(t.h, C.c_void_p(recv.data_ptr()), int(recv.shape[0]),
                                       C.c_void_p(ids.data_ptr()), t._stream(stream)),
              "gpd_flow_insert_keys")
        if stream is not None:
            stream.synchronize()
        torch.cuda.synchronize(dev)
        t3 = time.perf_counter()
        if self.single:
            back = ids[:m]
        else:
            back = return_ids(ids[:recv.shape[0]], rcv, send, self.group)
            self._after_collective(stream, dev)
        owner = torch.empty(dbatch.n, dtype=torch.int32, device=dev)
        flow_id = torch.empty(dbatch.n, dtype=torch.int32, device=dev)
        check(lib.gpd_flow_key_ids(t.h, C.c_void_p(keys.data_ptr()), m, C.c_void_p(back.data_ptr()),
                                   int(index_base), dbatch.n, C.c_void_p(owner.data_ptr()),
                                   C.c_void_p(flow_id.data_ptr()), t._stream(stream)), "gpd_flow_key_ids")
        torch.cuda.synchronize(dev)
        t4 = time.perf_counter()
        self.last_ms = {"keys": (t1 - t0) * 1e3, "exchange": (t2 - t1) * 1e3,
                        "insert": (t3 - t2) * 1e3, "return": (t4 - t3) * 1e3}
        return owner, flow_id

    @staticmethod
    def _after_collective(stream, dev):
        if stream is not None:
            torch = _torch()
            cur = torch.cuda.current_stream(dev)
            if stream != cur:
                stream.wait_stream(cur)

    def Stats(self, stream=None) -> dict:
        return self.table.Stats(stream)

    def Export(self, max_flows: Optional[int] = None, stream=None):
        return self.table.Export(max_flows, stream)


def flow_owner(net_hash, tp_hash, nparts: int):
    """The owner rank gpd_flow_keys assigns (include/gpd_flow.h), for host-side checks."""
    h = (np.asarray(net_hash, np.uint64) ^ np.asarray(tp_hash, np.uint64)) >> np.uint64(32)
    return ((h * np.uint64(nparts)) >> np.uint64(32)).astype(np.uint32)
