"""Streaming-structure sweep with libgpd_probe.so (diagnostic): the attainable probe of a
config's traffic shape at several workgroups per CU, with LDS capping the resident waves as
the decode kernel's LDS does, and with each round copied to LDS first.
    python tools/probe_sweep.py [imix|udp64]"""
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
lib = C.CDLL(os.path.join(ROOT, "gopacket_amd", "libgpd_probe.so"))
lib.gpd_probe_stream_ex.argtypes = [C.c_int, C.c_uint32, C.c_uint32, C.c_int, C.c_float, C.c_uint32,
                                    C.c_uint32, C.c_int, C.POINTER(C.c_float)]
SHAPES = {"imix": (1 << 16, 23190), "udp64": (1 << 18, 4608), "vxlan": (1 << 17, 8704)}
for name in sys.argv[1:] or ["imix", "udp64"]:
    nt, rb = SHAPES[name]
    for wpc in (2, 3, 4, 8):
        for lds in (0, 50 * 1024):
            for commit in (0, 1):
                ms = C.c_float(0)
                rc = lib.gpd_probe_stream_ex(0, nt, rb, 20, 100.0, wpc, lds, commit, C.byref(ms))
                gbps = nt * (rb + 2048) / (ms.value * 1e-3) / 1e9 if rc == 0 else 0
                print(json.dumps({"shape": name, "wpc": wpc, "lds_per_wg": lds, "commit": commit, "rc": rc,
                                  "ms": round(ms.value, 4), "GBps": round(gbps, 1)}), flush=True)
