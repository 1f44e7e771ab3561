"""TEST INFRASTRUCTURE: ctypes binding of the CPU oracle (oracle/libgpd_oracle.so).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_LIB = os.path.join(ROOT, "oracle", "libgpd_oracle.so")

import sys  # noqa: E402

if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

from gopacket_amd.layers import TABLES, DispatchTables  # noqa: E402
from gopacket_amd.results import EXT_DTYPE, BatchResult  # noqa: E402


class _Tables(C.Structure):
    _fields_ = [("ethertype", C.c_void_p), ("ipproto", C.c_void_p), ("tcp_port", C.c_void_p),
                ("udp_port", C.c_void_p)]


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(ORACLE_LIB):
            from gopacket_amd.build import build_oracle
            build_oracle()
        L = C.CDLL(ORACLE_LIB)
        L.gpo_decode_batch.restype = None
        L.gpo_decode_batch.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint32,
                                       C.c_uint32, C.c_uint32, C.POINTER(_Tables), C.c_void_p,
                                       C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                       C.c_void_p, C.c_int]
        L.gpo_ip4_header_checksum.restype = C.c_uint16
        L.gpo_ip4_header_checksum.argtypes = [C.c_char_p, C.c_uint32]
        L.gpo_tcpip_checksum.restype = C.c_uint16
        L.gpo_tcpip_checksum.argtypes = [C.c_char_p, C.c_uint32, C.c_uint32]
        L.gpo_pseudo_v4.restype = C.c_uint32
        L.gpo_pseudo_v4.argtypes = [C.c_char_p, C.c_char_p]
        L.gpo_pseudo_v6.restype = C.c_uint32
        L.gpo_pseudo_v6.argtypes = [C.c_char_p, C.c_char_p]
        L.gpo_fnv_hash.restype = C.c_uint64
        L.gpo_fnv_hash.argtypes = [C.c_char_p, C.c_uint32]
        L.gpo_flow_fasthash.restype = C.c_uint64
        L.gpo_flow_fasthash.argtypes = [C.c_uint32, C.c_char_p, C.c_uint32, C.c_char_p, C.c_uint32]
        L.gpo_endpoint_fasthash.restype = C.c_uint64
        L.gpo_endpoint_fasthash.argtypes = [C.c_uint32, C.c_char_p, C.c_uint32]
        _lib = L
    return _lib


def decode(batch, first: int = 17, decoders: int = 0x3FF, options: int = 0,
           tables: DispatchTables | None = None, ext: bool = True, nthreads: int = 1,
           out: BatchResult | None = None) -> BatchResult:
    """Oracle decode of a PacketBatch; same output words as the device path.  `out` (a
    BatchResult of batch.n entries with hdr_off, ext as requested) is reused when given."""
    t = tables or TABLES
    tabs = _Tables(t.ethertype.ctypes.data, t.ipproto.ctypes.data, t.tcp_port.ctypes.data,
                   t.udp_port.ctypes.data)
    n = batch.n
    res = out if out is not None else BatchResult(
        np.zeros(n, np.uint32), np.zeros(n, np.uint64), np.zeros(n, np.uint64),
        np.zeros(n, np.uint64), np.zeros(n, np.uint32),
        np.zeros(n, EXT_DTYPE) if ext else None, np.zeros(n, np.uint32))
    lib().gpo_decode_batch(batch.data.ctypes.data, batch.offset.ctypes.data, batch.caplen.ctypes.data,
                           n, first, decoders, options, C.byref(tabs), res.status.ctypes.data,
                           res.layers.ctypes.data, res.net_hash.ctypes.data, res.tp_hash.ctypes.data,
                           res.csum.ctypes.data, res.hdr_off.ctypes.data,
                           res.ext.ctypes.data if ext else None, nthreads)
    return res
