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

HEADERS = [os.path.join(ROOT, "include", h) for h in ("gpd.h", "gpd_pcap.h")]


def declared_functions():
    src = "".join(open(h).read() for h in HEADERS)
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(gpd_[a-z0-9_]+)\s*\(", src)) -
                  {n for n in re.findall(r"#define\s+(gpd_\w+)", src)})


def test_header_declares_the_boundary():
    fns = declared_functions()
    for f in ("gpd_ctx_create", "gpd_decode", "gpd_decode_host", "gpd_sync", "gpd_ctx_destroy",
              "gpd_last_error_string", "gpd_ctx_reload_tables", "gpd_default_tables",
              "gpd_pcap_header", "gpd_pcap_index", "gpd_decode_pcap", "gpd_host_register"):
        assert f in fns


def test_library_exports_every_declared_symbol():
    from gopacket_amd import _lib
    lib = C.CDLL(_lib.LIB_PATH)
    missing = [f for f in declared_functions() if not hasattr(lib, f)]
    assert not missing, missing
    assert lib.gpd_abi_version() == 2


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
    from gopacket_amd.results import EXT_DTYPE
    prog = tmp_path / "sz.c"
    prog.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "gpd_pcap.h"\nint main(void){'
                    'printf("%zu %zu %zu %zu %zu %zu %zu\\n", sizeof(gpd_config), sizeof(gpd_batch),'
                    ' sizeof(gpd_result), sizeof(gpd_ext_rec), offsetof(gpd_ext_rec, obj),'
                    ' sizeof(gpd_layer_rec), sizeof(gpd_pcap_info)); return 0;}\n')
    exe = tmp_path / "sz"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), str(prog), "-o", str(exe)], check=True)
    out = list(map(int, subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()))
    assert out == [C.sizeof(_lib.GpdConfig), C.sizeof(_lib.GpdBatch), C.sizeof(_lib.GpdResult),
                   EXT_DTYPE.itemsize, EXT_DTYPE.fields["obj"][1], 16, C.sizeof(_lib.GpdPcapInfo)]


@pytest.mark.skipif(gpu_available(), reason="checks the no-device error path")
def test_ctx_create_fails_loudly_without_device():
    from gopacket_amd import _lib
    h = C.c_void_p()
    rc = _lib.lib.gpd_ctx_create(0, None, C.byref(h))
    assert rc != 0 and h.value is None
    assert b"device" in _lib.lib.gpd_last_error_string()
