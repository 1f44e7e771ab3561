"""gopacket_amd — MI355X-native batched DecodingLayerParser / Flow engine.

The product path is libgpd.so (HIP kernels for gfx950 behind the C-ABI in
include/gpd.h); this package is the host-side mirror of gopacket's parser API
(parser.py), its dispatch tables (layers.py), batch layout (batch.py), result
reading (results.py), input formats (pcap.py, afpacket.py, synth.py), the flow table
(flows.py) and the IPv4 fragment hand-off to ip4defrag (defrag.py).  (The stateful
reassembly over that hand-off is restated only as a test checker, oracle/ip4defrag_ref.py:
ip4defrag itself is out of scope.)
"""
from . import layers
from .layers import *  # noqa: F401,F403  LayerType constants, Register*PortLayerType
from .batch import PacketBatch
from .errors import DecodeError, UnsupportedLayerType
from .results import (BatchResult, Endpoint, FastHashes, Flow, FlowFromEndpoints, MaxEndpointSize,
                      NewEndpoint, NewFlow)

__all__ = ["layers", "PacketBatch", "BatchResult", "DecodeError", "UnsupportedLayerType",
           "Endpoint", "Flow", "NewEndpoint", "NewFlow", "FlowFromEndpoints", "FastHashes",
           "MaxEndpointSize", "parser"]


def __getattr__(name):
    # the parser pulls in libgpd.so; import it lazily so that pure-host helpers
    # (pcap, synth, layers) work in environments that only build.
    if name == "parser":
        import importlib
        return importlib.import_module(".parser", __name__)
    raise AttributeError(name)
