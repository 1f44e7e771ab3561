"""Diagnostic: does libgpd.so find the GPU when torch is NOT loaded first (the Go/cgo case)?"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
if len(sys.argv) > 1 and sys.argv[1] == "torch":
    import torch
    print("torch sees", torch.cuda.device_count(), "devices")
hip = C.CDLL("libamdhip64.so.7")
n = C.c_int(-1)
rc = hip.hipGetDeviceCount(C.byref(n))
hip.hipGetErrorString.restype = C.c_char_p
print("hipGetDeviceCount rc", rc, hip.hipGetErrorString(rc).decode(), "n", n.value)
with open("/proc/self/maps") as f:
    print(sorted({l.split()[-1] for l in f if "amdhip" in l or "hsa-runtime" in l}))
for k in sorted(os.environ):
    if any(t in k for t in ("HIP", "ROCR", "HSA", "GPU", "CUDA", "LD_")):
        print(k, "=", os.environ[k])
