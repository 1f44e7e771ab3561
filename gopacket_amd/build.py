"""Build the in-tree native libraries.

  gopacket_amd/libgpd.so       product: HIP kernels (gfx950) + C-ABI runtime (include/gpd.h)
  gopacket_amd/libgpd_diag.so  diagnostics only (--diag): the same with -DGPD_DIAG (bench --ablate)
  oracle/libgpd_oracle.so      test infrastructure: CPU restatement (oracle/)
  tests/c/abi_host             test driver: a plain C host on the C-ABI (no Python/torch)
  gopacket_amd/libgpd_synth.so workload generator for the bench (config 5 captures); not product
  gopacket_amd/libgpd_probe.so attainable-bandwidth probe bench.py prints beside each roofline; not product

Both are built with plain compiler invocations (hipcc / gcc); no cmake.  The .so
files are git-ignored and travel to the GPU box with the repository snapshot.
"""
from __future__ import annotations

import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "gopacket_amd")
CSRC = os.path.join(PKG, "csrc")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("GPD_OFFLOAD_ARCH", "gfx950")

LIB = os.path.join(PKG, "libgpd.so")
DIAG_LIB = os.path.join(PKG, "libgpd_diag.so")
ORACLE_LIB = os.path.join(ROOT, "oracle", "libgpd_oracle.so")

SOURCES = [os.path.join(CSRC, "gpd_kernels.hip"), os.path.join(CSRC, "gpd_runtime.cpp"),
           os.path.join(CSRC, "gpd_pcap.cpp"), os.path.join(CSRC, "gpd_flow.hip"),
           os.path.join(CSRC, "gpd_pcapwalk.hip"), os.path.join(CSRC, "gpd_tpv3walk.hip"),
           os.path.join(CSRC, "gpd_afpacket.cpp")]
HEADERS = [os.path.join(CSRC, "gpd_internal.h"), os.path.join(ROOT, "include", "gpd.h"),
           os.path.join(ROOT, "include", "gpd_pcap.h"), os.path.join(ROOT, "include", "gpd_flow.h"),
           os.path.join(ROOT, "include", "gpd_afpacket.h"), os.path.join(ROOT, "include", "gpd_defrag.h")]


def _stale(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def build_lib(force: bool = False, verbose: bool = False, diag: bool = False) -> str:
    """libgpd.so, or with diag=True libgpd_diag.so: the same sources with -DGPD_DIAG, whose
    runtime also takes bench.py's stream-only ablation bits (never loaded by the product)."""
    out = DIAG_LIB if diag else LIB
    if force or _stale(out, SOURCES + HEADERS):
        extra = os.environ.get("GPD_EXTRA_CFLAGS", "").split()  # A/B builds (tools/)
        if diag:
            extra.append("-DGPD_DIAG")
        # one hipcc per source in parallel (the kernels' TU dominates), then one link
        objdir = os.path.join(ROOT, "build", "diag" if diag else "lib")
        os.makedirs(objdir, exist_ok=True)
        base = [HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-Wall",
                "-Wno-unused-function", "-pthread", "-I", os.path.join(ROOT, "include"), *extra]
        objs = [os.path.join(objdir, os.path.basename(src) + ".o") for src in SOURCES]
        cmds = [base + ["-c", src, "-o", obj] for src, obj in zip(SOURCES, objs)]
        if verbose:
            for c in cmds:
                print(" ".join(c), flush=True)
        with ThreadPoolExecutor(max_workers=min(len(cmds), os.cpu_count() or 1)) as ex:
            for r in list(ex.map(lambda c: subprocess.run(c), cmds)):
                if r.returncode != 0:
                    raise subprocess.CalledProcessError(r.returncode, r.args)
        subprocess.run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-pthread", *objs,
                        "-o", out + ".tmp"], check=True)
        os.replace(out + ".tmp", out)
    return out


def build_oracle(force: bool = False) -> str:
    src = [os.path.join(ROOT, "oracle", "gpd_oracle.c"), os.path.join(ROOT, "oracle", "gpd_oracle.h"),
           os.path.join(ROOT, "include", "gpd.h")]
    if force or _stale(ORACLE_LIB, src):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "-B" if force else "all"],
                       check=True)
    return ORACLE_LIB


ABI_HOST = os.path.join(ROOT, "tests", "c", "abi_host")
SYNTH_LIB = os.path.join(PKG, "libgpd_synth.so")


def build_synth(force: bool = False) -> str:
    """gopacket_amd/libgpd_synth.so: the native twin of synth.make_udp64 (plain C, gcc)."""
    src = os.path.join(CSRC, "synth", "gpd_synth.c")
    if force or _stale(SYNTH_LIB, [src]):
        subprocess.run(["gcc", "-O2", "-std=c11", "-Wall", "-fPIC", "-shared", "-pthread", src,
                        "-o", SYNTH_LIB + ".tmp"], check=True)
        os.replace(SYNTH_LIB + ".tmp", SYNTH_LIB)
    return SYNTH_LIB


PROBE_LIB = os.path.join(PKG, "libgpd_probe.so")


def build_probe(force: bool = False) -> str:
    """gopacket_amd/libgpd_probe.so: the streaming probe of bench.py's `roofline.attainable`."""
    src = os.path.join(CSRC, "gpd_probe.hip")
    if force or _stale(PROBE_LIB, [src]):
        subprocess.run([HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared", "-Wall",
                        src, "-o", PROBE_LIB + ".tmp"], check=True)
        os.replace(PROBE_LIB + ".tmp", PROBE_LIB)
    return PROBE_LIB


def build_abi_host(force: bool = False) -> str:
    """tests/c/abi_host: links libgpd.so (rpath to the in-tree copy) and the oracle."""
    src = os.path.join(ROOT, "tests", "c", "abi_host.c")
    deps = [src, LIB, ORACLE_LIB, os.path.join(ROOT, "include", "gpd.h")]
    if force or _stale(ABI_HOST, deps):
        subprocess.run(["gcc", "-O2", "-std=c11", "-Wall", "-D__HIP_PLATFORM_AMD__",
                        "-I/opt/rocm/include", src, "-o", ABI_HOST,
                        "-L" + PKG, "-lgpd", "-L" + os.path.dirname(ORACLE_LIB), "-lgpd_oracle",
                        "-L/opt/rocm/lib", "-lamdhip64",
                        "-Wl,-rpath,$ORIGIN/../../gopacket_amd:$ORIGIN/../../oracle:/opt/rocm/lib"],
                       check=True)
    return ABI_HOST


if __name__ == "__main__":
    force = "--force" in sys.argv
    print(build_lib(force=force, verbose=True))
    if "--diag" in sys.argv:
        print(build_lib(force=force, verbose=True, diag=True))
    print(build_oracle(force=force))
    print(build_abi_host(force=force))
    print(build_synth(force=force))
    print(build_probe(force=force))
