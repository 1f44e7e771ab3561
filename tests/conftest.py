import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path through the C-ABI)")


@pytest.fixture(scope="session", autouse=True)
def _built_libs():
    """Build libgpd.so (hipcc, gfx950) and the oracle if their sources are newer."""
    from gopacket_amd.build import build_abi_host, build_lib, build_oracle, build_synth
    build_oracle()
    build_synth()
    if os.path.exists("/opt/rocm/bin/hipcc"):
        build_lib()
        build_abi_host()
    yield


def gpu_available() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False
