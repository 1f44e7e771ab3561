"""ctypes binding of the in-tree libgpd.so (the C-ABI in include/gpd.h).

The product path has no CPU fallback: if the HIP library is missing this module
raises at import, and every decode goes through gpd_decode / gpd_decode_host.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# The product library.  bench.py's stream-only ablations (--ablate nodecode / nowait) set
# GPD_DIAGNOSTIC_LIBRARY=1 to load libgpd_diag.so instead: the same sources built with
# -DGPD_DIAG, whose runtime accepts the two ablation option bits that libgpd.so refuses.
LIB_PATH = os.path.join(_HERE, "libgpd.so")
DIAG_LIB_PATH = os.path.join(_HERE, "libgpd_diag.so")
if os.environ.get("GPD_DIAGNOSTIC_LIBRARY") == "1":
    LIB_PATH = DIAG_LIB_PATH

GPD_ABI_VERSION = 10
GPD_OK = 0
GPD_ERR_INVALID = -1


class GpdConfig(C.Structure):
    _fields_ = [("first_layer", C.c_uint32), ("decoders", C.c_uint32), ("options", C.c_uint32),
                ("reserved", C.c_uint32), ("ethertype", C.c_void_p), ("ipproto", C.c_void_p),
                ("tcp_port", C.c_void_p), ("udp_port", C.c_void_p)]


class GpdBatch(C.Structure):
    _fields_ = [("data", C.c_void_p), ("data_len", C.c_uint64), ("offset", C.c_void_p),
                ("caplen", C.c_void_p), ("n", C.c_uint64)]


class GpdResult(C.Structure):
    _fields_ = [("status", C.c_void_p), ("layers", C.c_void_p), ("net_hash", C.c_void_p),
                ("tp_hash", C.c_void_p), ("csum", C.c_void_p), ("ext", C.c_void_p),
                ("hdr_off", C.c_void_p), ("records", C.c_void_p), ("detail", C.c_void_p)]


class GpdTuning(C.Structure):
    _fields_ = [("window_bytes", C.c_uint32), ("shift", C.c_int32), ("reg_prefix", C.c_int32),
                ("waves_per_simd", C.c_int32), ("header_once", C.c_int32),
                ("device_walk", C.c_int32), ("grid_rounds", C.c_int32), ("split", C.c_int32)]


class GpdPcapInfo(C.Structure):
    _fields_ = [("magic", C.c_uint32), ("big_endian", C.c_uint32), ("nano", C.c_uint32),
                ("version_major", C.c_uint32), ("version_minor", C.c_uint32),
                ("snaplen", C.c_uint32), ("linktype", C.c_uint32), ("reserved", C.c_uint32)]


EXPORTS = {
    # name: (restype, argtypes)
    "gpd_abi_version": (C.c_int, []),
    "gpd_default_tables": (None, [C.c_void_p] * 4),
    "gpd_ctx_create": (C.c_int, [C.c_int, C.POINTER(GpdConfig), C.POINTER(C.c_void_p)]),
    "gpd_ctx_reload_tables": (C.c_int, [C.c_void_p, C.POINTER(GpdConfig)]),
    "gpd_ctx_set_options": (C.c_int, [C.c_void_p, C.c_uint32]),
    "gpd_ctx_add_decoders": (C.c_int, [C.c_void_p, C.c_uint32]),
    "gpd_ctx_set_decoders": (C.c_int, [C.c_void_p, C.c_uint32]),
    "gpd_ctx_destroy": (C.c_int, [C.c_void_p]),
    "gpd_decode": (C.c_int, [C.c_void_p, C.POINTER(GpdBatch), C.POINTER(GpdResult), C.c_void_p]),
    "gpd_decode_host": (C.c_int, [C.c_void_p, C.POINTER(GpdBatch), C.POINTER(GpdResult)]),
    "gpd_sync": (C.c_int, [C.c_void_p, C.c_void_p]),
    "gpd_ctx_set_timing": (C.c_int, [C.c_void_p, C.c_int]),
    "gpd_last_kernel_ms": (C.c_float, [C.c_void_p]),
    "gpd_ctx_set_tuning": (C.c_int, [C.c_void_p, C.c_void_p]),
    "gpd_last_launch_split": (C.c_int, [C.c_void_p, C.POINTER(C.c_uint64), C.POINTER(C.c_float),
                                        C.POINTER(C.c_float)]),
    "gpd_last_error_string": (C.c_char_p, []),
    # include/gpd_pcap.h
    "gpd_pcap_header": (C.c_int, [C.c_void_p, C.c_uint64, C.POINTER(GpdPcapInfo)]),
    "gpd_pcap_index": (C.c_int, [C.c_void_p, C.c_uint64, C.POINTER(GpdPcapInfo), C.c_uint64,
                                 C.c_uint64, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                 C.POINTER(C.c_uint64), C.POINTER(C.c_uint64),
                                 C.POINTER(C.c_int), C.c_int]),
    "gpd_decode_pcap": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint64,
                                  C.POINTER(GpdResult), C.POINTER(C.c_uint64),
                                  C.POINTER(C.c_uint64), C.POINTER(C.c_int), C.c_int]),
    "gpd_decode_pcap_at": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint64, C.POINTER(GpdPcapInfo),
                                     C.c_uint64, C.c_uint64, C.POINTER(GpdResult),
                                     C.POINTER(C.c_uint64), C.POINTER(C.c_uint64),
                                     C.POINTER(C.c_int), C.c_int]),
    "gpd_pcap_locate": (C.c_int, [C.c_void_p, C.c_uint64, C.POINTER(GpdPcapInfo), C.c_uint64,
                                  C.c_void_p, C.c_uint64, C.c_void_p, C.POINTER(C.c_uint64),
                                  C.POINTER(C.c_int), C.c_int]),
    "gpd_pcap_last_stats": (None, [C.POINTER(C.c_int)] * 3),
    "gpd_decode_pcap_last_times": (None, [C.c_void_p]),
    "gpd_decode_pcap_last_walk_counts": (None, [C.c_void_p]),
    "gpd_decode_pcap_last_walk_miss": (None, [C.c_void_p]),
    "gpd_host_register": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint64]),
    "gpd_host_unregister": (C.c_int, [C.c_void_p, C.c_void_p]),
    "gpd_host_bind_local": (C.c_int, [C.c_int, C.c_void_p, C.c_uint64, C.POINTER(C.c_int)]),
    # include/gpd_flow.h
    "gpd_flow_create": (C.c_int, [C.c_void_p, C.c_uint64, C.POINTER(C.c_void_p)]),
    "gpd_flow_reset": (C.c_int, [C.c_void_p, C.c_void_p]),
    "gpd_flow_insert": (C.c_int, [C.c_void_p, C.POINTER(GpdBatch), C.POINTER(GpdResult), C.c_void_p,
                                  C.c_uint64, C.c_void_p]),
    "gpd_flow_stats_get": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p]),
    "gpd_flow_export": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64,
                                  C.POINTER(C.c_uint64), C.c_void_p]),
    "gpd_flow_destroy": (C.c_int, [C.c_void_p]),
    "gpd_fast_hash": (C.c_int, [C.c_int, C.c_uint64, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                C.c_void_p, C.c_void_p, C.c_void_p]),
    "gpd_flow_test_fingerprint_bits": (C.c_int, [C.c_void_p, C.c_uint32]),
    "gpd_flow_test_counter_bits": (C.c_int, [C.c_void_p, C.c_uint32]),
    "gpd_flow_keys": (C.c_int, [C.c_void_p, C.POINTER(GpdBatch), C.POINTER(GpdResult), C.c_uint32,
                                C.c_uint64, C.c_void_p, C.c_void_p, C.c_void_p]),
    "gpd_flow_insert_keys": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p]),
    "gpd_flow_key_ids": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint64,
                                   C.c_uint64, C.c_void_p, C.c_void_p, C.c_void_p]),
    # include/gpd_afpacket.h
    "gpd_tpv3_walk": (C.c_int, [C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint64, C.c_void_p,
                                C.POINTER(C.c_uint64), C.POINTER(C.c_uint32), C.c_int]),
    "gpd_tpv3_release": (C.c_int, [C.c_void_p, C.c_uint32, C.c_uint32]),
    "gpd_decode_tpv3": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32, C.c_int,
                                  C.c_uint64, C.POINTER(GpdResult), C.c_void_p,
                                  C.POINTER(C.c_uint64), C.POINTER(C.c_uint32), C.c_int]),
    "gpd_decode_tpv3_last_path": (C.c_int, []),
    # include/gpd_defrag.h
    "gpd_ip4_fragments": (C.c_int, [C.c_void_p, C.POINTER(GpdBatch), C.POINTER(GpdResult), C.c_void_p,
                                    C.c_uint64, C.POINTER(C.c_uint64), C.c_void_p]),
}

GPD_ERR_PCAP = -5


class GpdError(RuntimeError):
    pass


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"gopacket_amd: native library {LIB_PATH} is missing — build it with "
            "`python -m gopacket_amd.build` (hipcc, gfx950); there is no CPU fallback")
    # One HIP runtime per process.  PyTorch ships its own libamdhip64 / libhsa-runtime64 and
    # its extension modules NEED them under a different name than libgpd.so does
    # (libamdhip64.so vs .so.7), so loading libgpd.so first would bring up a second runtime,
    # which finds no device once torch's has opened it.  Loading torch first makes libgpd.so
    # bind to torch's (same SONAME).  Without torch (a C or Go host) libgpd.so uses /opt/rocm's.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = C.CDLL(LIB_PATH)
    for name, (res, args) in EXPORTS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.gpd_abi_version() != GPD_ABI_VERSION:
        raise ImportError(f"gopacket_amd: {os.path.basename(LIB_PATH)} ABI version mismatch")
    return lib


lib = _load()


def check(rc: int, what: str) -> None:
    if rc != GPD_OK:
        msg = lib.gpd_last_error_string()
        raise GpdError(f"{what}: rc={rc}: {msg.decode() if msg else ''}")
