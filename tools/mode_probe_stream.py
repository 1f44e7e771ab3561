"""Does a pure stream (libgpd_probe.so gpd_probe_stream2: config 2's read bytes per tile, the
record stores, no decode) show the same placement modes as the decode launch?  Each trial holds
another 1 GiB torch allocation first so the probe's own buffers land elsewhere.

    python tools/mode_probe_stream.py [trials]
"""
import ctypes as C
import json
import os
import sys


def main():
    import torch
    trials = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    lib = C.CDLL(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                              "gopacket_amd", "libgpd_probe.so"))
    lib.gpd_probe_stream2.argtypes = [C.c_int, C.c_uint32, C.c_uint32, C.c_int, C.c_float, C.c_int,
                                      C.POINTER(C.c_float)]
    ntiles, per_tile = (1 << 24) // 64, 4096 + 512
    hold = []
    for t in range(trials):
        hold.append(torch.empty(1 << 30 if t % 2 else 3 << 29, dtype=torch.uint8, device="cuda:0"))
        out = {"trial": t}
        for form, name in ((0, "records"), (2, "read_only")):
            ms = C.c_float(0.0)
            rc = lib.gpd_probe_stream2(0, ntiles, per_tile, 20, 150.0, form, C.byref(ms))
            out[name] = round(ms.value, 4) if rc == 0 else f"rc={rc}"
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
