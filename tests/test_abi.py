"""The C-ABI library loads and exports every symbol include/gpd.h declares (CPU only).

No compute calls: this runs without a GPU.
"""
import ctypes as C
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import ROOT, gpu_available

HEADERS = [os.path.join(ROOT, "include", h) for h in ("gpd.h", "gpd_pcap.h", "gpd_flow.h", "gpd_afpacket.h",
                                                             "gpd_defrag.h")]


def declared_functions():
    src = "".join(open(h).read() for h in HEADERS)
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(gpd_[a-z0-9_]+)\s*\(", src)) -
                  {n for n in re.findall(r"#define\s+(gpd_\w+)", src)})


def test_header_declares_the_boundary():
    fns = declared_functions()
    for f in ("gpd_ctx_create", "gpd_decode", "gpd_decode_host", "gpd_sync", "gpd_ctx_destroy",
              "gpd_last_error_string", "gpd_ctx_reload_tables", "gpd_default_tables",
              "gpd_ctx_set_options", "gpd_ctx_add_decoders",
              "gpd_pcap_header", "gpd_pcap_index", "gpd_decode_pcap", "gpd_host_register", "gpd_host_bind_local",
              "gpd_flow_create", "gpd_flow_insert", "gpd_flow_export", "gpd_flow_stats_get",
              "gpd_ip4_fragments"):
        assert f in fns


def test_library_exports_every_declared_symbol():
    from gopacket_amd import _lib
    lib = C.CDLL(_lib.LIB_PATH)
    missing = [f for f in declared_functions() if not hasattr(lib, f)]
    assert not missing, missing
    assert lib.gpd_abi_version() == 10


def test_python_binding_covers_the_header():
    from gopacket_amd import _lib
    assert set(declared_functions()) == set(_lib.EXPORTS)


def test_default_tables_match_reference_restatement():
    from gopacket_amd import _lib
    from gopacket_amd.layers import DispatchTables
    eth = np.zeros(65536, np.uint16); pro = np.zeros(256, np.uint16)
    tcp = np.zeros(65536, np.uint16); udp = np.zeros(65536, np.uint16)
    _lib.lib.gpd_default_tables(eth.ctypes.data, pro.ctypes.data, tcp.ctypes.data, udp.ctypes.data)
    t = DispatchTables()
    assert np.array_equal(eth, t.ethertype) and np.array_equal(pro, t.ipproto)
    assert np.array_equal(tcp, t.tcp_port) and np.array_equal(udp, t.udp_port)


def test_struct_layouts_match_c(tmp_path):
    """sizeof/offsetof of the ABI structs as gcc sees them == the ctypes/numpy mirrors."""
    from gopacket_amd import _lib
    from gopacket_amd.results import EXT_DTYPE, RECORD_DTYPE
    prog = tmp_path / "sz.c"
    prog.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "gpd_pcap.h"\n#include "gpd_flow.h"\n'
                    'int main(void){'
                    'printf("%zu %zu %zu %zu %zu %zu %zu %zu %zu %zu %zu %zu %zu %zu\\n", sizeof(gpd_config), sizeof(gpd_batch),'
                    ' sizeof(gpd_result), sizeof(gpd_ext_rec), offsetof(gpd_ext_rec, obj),'
                    ' sizeof(gpd_layer_rec), sizeof(gpd_pcap_info), sizeof(gpd_flow_rec),'
                    ' offsetof(gpd_flow_rec, net_type), offsetof(gpd_flow_rec, first), sizeof(gpd_flow_stats),'
                    ' sizeof(gpd_record), offsetof(gpd_record, layers), sizeof(gpd_tuning));'
                    ' return 0;}\n')
    exe = tmp_path / "sz"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), str(prog), "-o", str(exe)], check=True)
    out = list(map(int, subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()))
    from gopacket_amd.flows import FLOW_REC_DTYPE, FlowStats
    assert out == [C.sizeof(_lib.GpdConfig), C.sizeof(_lib.GpdBatch), C.sizeof(_lib.GpdResult),
                   EXT_DTYPE.itemsize, EXT_DTYPE.fields["obj"][1], 16, C.sizeof(_lib.GpdPcapInfo),
                   FLOW_REC_DTYPE.itemsize, FLOW_REC_DTYPE.fields["net_type"][1],
                   FLOW_REC_DTYPE.fields["first"][1], C.sizeof(FlowStats),
                   RECORD_DTYPE.itemsize, RECORD_DTYPE.fields["layers"][1], C.sizeof(_lib.GpdTuning)]


@pytest.mark.skipif(gpu_available(), reason="checks the no-device error path")
def test_ctx_create_fails_loudly_without_device():
    from gopacket_amd import _lib
    h = C.c_void_p()
    rc = _lib.lib.gpd_ctx_create(0, None, C.byref(h))
    assert rc != 0 and h.value is None
    assert b"device" in _lib.lib.gpd_last_error_string()


@pytest.mark.gpu
def test_c_host_program_on_the_abi(tmp_path):
    """tests/c/abi_host: a plain C program (no Python, no torch in its process — the cgo case)
    decodes through gpd_decode on its own hipMalloc'ed buffers and stream and through
    gpd_decode_host and gpd_decode_pcap (the same packets as a capture file); all must equal the
    oracle bit for bit, and the device results must build a consistent flow table.  Then (ABI 8)
    a second context registers UDP 8472 as VXLAN, reloads its tables, adds the VXLAN decoder in
    place and flips IgnoreUnsupported both ways, each step host and device against the oracle on
    the same mutated tables; and it decodes an all-empty batch."""
    import golden_cases as G
    from gopacket_amd import synth
    from gopacket_amd.batch import PacketBatch
    exe = os.path.join(ROOT, "tests", "c", "abi_host")
    assert os.path.exists(exe), "build tests/c/abi_host first (__graft_entry__.build())"
    pkts = [G.case_bytes(c) for c in G.load()["cases"]]
    pkts += [p[:k] for p in pkts[:8] for k in range(0, len(p), 3)]
    mixed = synth.make_mixed(3000)
    pkts += [mixed.packet(i) for i in range(mixed.n)]
    import test_defrag as TD  # the ip4defrag fixtures and fragment fuzz frames
    pkts += list(TD._frames().values()) + [f for _, f in TD.struct_frames()] + TD.fuzz_frames(600, 5)
    import error_sites as ES
    import errpath_cases as EC
    import oracle_ref as O
    from gopacket_amd.layers import ip_protocol_name
    pkts += [bytes.fromhex(c["hex"]) for c in EC.load()]
    pkts += ES.packets()
    # VXLAN on UDP port 8472 (not a default port): the reconfiguration step registers it
    vx = synth.make_vxlan(96)
    for i in range(vx.n):
        p = bytearray(vx.packet(i))
        p[36:38] = (8472).to_bytes(2, "big")
        pkts.append(bytes(p))
    names = tmp_path / "ipproto_names.txt"
    names.write_text("".join(ip_protocol_name(p) + "\n" for p in range(256)))
    for decoders, options in ((0xFFF, 0), (0x3FF, 1), (0x1 | 0x4 | 0x400 | 0x20 | 0x40 | 0x100, 0)):
        b = PacketBatch.from_packets(pkts)
        f = tmp_path / f"batch_{decoders:x}_{options}.bin"
        with open(f, "wb") as fh:
            fh.write(np.array([b.data_len, b.n], np.uint64).tobytes())
            fh.write(np.array([decoders, options], np.uint32).tobytes())
            fh.write(b.data[:b.data_len].tobytes())
            fh.write(b.offset.astype(np.uint32).tobytes())
            fh.write(b.caplen.astype(np.uint32).tobytes())
        errs = tmp_path / f"errors_{decoders:x}_{options}.txt"
        r = subprocess.run([exe, str(f), str(errs), str(names), "8472"], capture_output=True, text=True,
                           timeout=90)
        assert r.returncode == 0, r.stdout + r.stderr
        words = r.stdout.split()
        assert words[:3] == ["abi_host", "ok", str(b.n)], r.stdout
        assert int(words[3]) > 100, r.stdout  # the mixed traffic holds many TCP/UDP flows
        assert int(words[4]) > 100, r.stdout  # ip4defrag's fragments and the fuzz frames
        if decoders & 0x80:  # the in-place reconfiguration reached VXLAN on the registered port
            assert int(words[5]) >= 96, r.stdout
        # the C host's error texts (from status + gpd_detail) == the oracle's, packet by packet
        ref = O.decode(b, 17, decoders, options, ext=True, nthreads=8)
        want = {i: str(ref.err(i)) for i in range(b.n) if (int(ref.status[i]) & 3) == 2}
        got = {}
        for line in errs.read_text().splitlines():
            i, text = line.split("\t", 1)
            got[int(i)] = text
        assert got == want
        if decoders == 0xFFF:  # every decoder registered: every error site of gpd.h is reached
            assert {int(ref.status[i]) >> 9 & 63 for i in want} == set(range(1, 32))


def test_integration_build_command_names_every_source():
    """INTEGRATION.md §1's single hipcc command must name every file build.py compiles."""
    import re
    from gopacket_amd.build import SOURCES
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    cmd = re.search(r"```sh\nhipcc .*?```", text, re.S).group(0)
    for src in SOURCES:
        assert os.path.relpath(src, ROOT) in cmd, src


def test_probe_library_exports_its_entry_points():
    """bench.py's `roofline.attainable` comes from libgpd_probe.so (a diagnostic beside the
    product library, not part of include/): it builds for gfx950 and exports both probes."""
    import ctypes as C
    from gopacket_amd import build
    lib = C.CDLL(build.build_probe())
    for sym in ("gpd_probe_stream", "gpd_probe_stream2", "gpd_probe_stream_ex"):
        assert hasattr(lib, sym), sym


@pytest.mark.skipif(not os.path.exists("/opt/rocm/bin/hipcc"), reason="needs hipcc")
def test_fast_kernels_do_not_spill():
    """Every instance of the fast kernels (rs_kernel, ro_kernel, sp_kernel) fits its waves-per-SIMD register
    bound without scratch spills: a spill puts global-memory traffic into the streaming loop
    (a one-line change to the decode once cost 15-85 spilled VGPRs and 10-20 % of IMIX/VXLAN)."""
    import tempfile
    src = os.path.join(ROOT, "gopacket_amd", "csrc", "gpd_kernels.hip")
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "k.s")
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-I",
                        os.path.join(ROOT, "include"), "-S", "--cuda-device-only", src, "-o", out],
                       check=True, capture_output=True, timeout=600)
        txt = open(out).read()
    seen = 0
    for b in txt.split("  - .agpr_count:")[1:]:
        name = re.search(r"\.name:\s+(\S+)", b).group(1)
        if "rs_kernel" not in name and "ro_kernel" not in name and "sp_kernel" not in name:
            continue
        seen += 1
        spill = int(re.search(r"\.vgpr_spill_count:\s+(\d+)", b).group(1))
        assert spill == 0, f"{name}: {spill} VGPRs spilled"
    assert seen >= 20


def test_shipped_library_has_no_diagnostic_kernels():
    """the shipped libgpd.so instantiates every fast kernel without the skeleton
    diagnostic (rs_kernel's last template argument, DIAG, false), the config-2 4 KiB kernel
    included; only libgpd_diag.so (-DGPD_DIAG, bench --ablate) carries DIAG=true kernels."""
    lib = os.path.join(ROOT, "gopacket_amd", "libgpd.so")
    out = subprocess.run(["nm", "-C", lib], check=True, capture_output=True, text=True).stdout
    inst = set(re.findall(r"rs_kernel<([^>]*)>", out))
    assert len(inst) >= 20, inst
    diag = [a for a in inst if a.split(",")[-1].strip() == "true"]
    assert not diag, diag
    assert any(a.replace(" ", "").startswith("4096,true,true,4,") for a in inst)
