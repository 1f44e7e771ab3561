"""Boundary and robustness cases of the C-ABI on the GPU: batch-size refusals, packets that
reach the end of the buffer, and the fast path's IPv4-fragment decode in every flag/offset
combination (inner VXLAN fragments, Fragment unregistered, IgnoreUnsupported).
"""
import ctypes as C

import numpy as np
import pytest

import error_sites as ES
from gopacket_amd import layers as L
from gopacket_amd import synth
from gopacket_amd.batch import PacketBatch
from test_parity_gpu import ALL, _parser, run_both

pytestmark = pytest.mark.gpu

FRAGMENT = 0x200  # GPD_DEC_FRAGMENT


def test_batch_count_bound_is_refused():
    """gpd_decode / gpd_decode_host refuse n > 2^32 - 256 (packet and tile indices stay 32-bit
    in the kernels) before reading any descriptor."""
    import torch
    from gopacket_amd._lib import GPD_ERR_INVALID, GpdBatch, GpdResult, lib
    p = _parser()
    h = p.ctx().h
    buf = torch.zeros(64, dtype=torch.uint8, device="cuda")
    d = buf.data_ptr()
    for n in (1 << 32, 0xFFFFFF01, 1 << 40):
        b = GpdBatch(d, 16, d, d, n)
        r = GpdResult(d, d, None, None, None, None, None, None, None)
        assert lib.gpd_decode(h, C.byref(b), C.byref(r), None) == GPD_ERR_INVALID
        assert b"max 2^32 - 256" in lib.gpd_last_error_string()
        hb = (C.c_uint8 * 64)()
        b = GpdBatch(C.addressof(hb), 16, C.addressof(hb), C.addressof(hb), n)
        r = GpdResult(C.addressof(hb), C.addressof(hb), None, None, None, None, None, None, None)
        assert lib.gpd_decode_host(h, C.byref(b), C.byref(r)) == GPD_ERR_INVALID
        assert b"max 2^32 - 256" in lib.gpd_last_error_string()


def test_fallback_packets_ending_at_the_buffer_end():
    """Packets the fast kernel leaves to its fallback list (IPv4 options, cut headers) placed
    last, ending exactly at a 16-aligned data_len: the list's staging loads stay inside
    round_up(data_len, 16) (gpd.h gpd_batch), and the results are the oracle's.  Each tail
    length 1..48 past the last 16-B boundary is tried."""
    bulk = synth.make_udp64(512)
    base = [bulk.packet(i) for i in range(bulk.n)]
    tails = [ES.eth(0x0800, ES.ip4(ES.tcp(b"\x00" * 3), ihl=6, opts=b"\x01\x01\x01\x00")),
             ES.eth(0x0800, ES.ip4(ES.tcp(doff=15))), ES.eth(0x86DD, ES.ip6(b"\x3b\x00" + b"\x00" * 6, nh=0))]
    hit = 0
    for t in tails:
        for cut in range(0, 48):
            pk = base + [t[:max(14, len(t) - cut)]]
            b = PacketBatch.from_packets(pk)  # data_len = the last packet's end
            hit += b.data_len % 16 == 0
            run_both(b, L.LayerTypeEthernet, ALL, 0, ext=False)
    assert hit >= 6  # some batches end exactly on a 16-byte boundary


def _fragments():
    """IPv4 fragments in every flag / offset combination, bare, tagged and inside VXLAN."""
    out = []
    flags = [0x2000, 0x4000, 0x6000, 0x0001, 0x0010, 0x2010, 0x1FFF, 0x3FFF, 0x5FFF, 0x4010, 0x0000]
    vx = b"\x08\x00\x00\x00\x00\x00\xff\x00"
    for ff in flags:
        for l4, proto in ((ES.udp(b"\x00" * 16), 17), (ES.tcp(b"\x00" * 12), 6), (b"\x08" + b"\x00" * 15, 1)):
            ip = ES.ip4(l4, proto=proto, flags_frag=ff)
            out.append(ES.eth(0x0800, ip))
            out.append(ES.MAC + b"\x81\x00\x00\x05\x08\x00" + ip)  # one 802.1Q tag
            inner = ES.eth(0x0800, ip)
            out.append(ES.eth(0x0800, ES.ip4(ES.udp(vx + inner, dport=4789), proto=17)))  # inner fragment
            out.append(ES.eth(0x0800, ES.ip4(ES.udp(vx + inner, dport=4789), proto=17, flags_frag=ff)))  # outer
            out.append(ES.eth(0x0800, ip[:24]))  # a fragment cut short (empty / partial payload)
    return out


@pytest.mark.parametrize("mask", [ALL, 0x3FF, ALL & ~FRAGMENT, 0x3FF & ~FRAGMENT])
@pytest.mark.parametrize("options", [0, 1])
def test_fragment_decode_fast_path(mask, options):
    """The fast kernel's [.., IPv4, Fragment] decode (the LUT's Fragment entry, or the stop type 3
    when Fragment is unregistered) against the oracle: nonzero offsets, DF/MF combinations,
    fragments inside VXLAN's second pass, with and without IgnoreUnsupported; mixed among 64-B
    UDP traffic so the fast path (not only the fallback list) decodes them."""
    bulk = synth.make_udp64(2048)
    pk = [bulk.packet(i) for i in range(bulk.n)]
    fr = _fragments()
    for k, f in enumerate(fr):
        pk.insert(7 * k + 3, f)
    b = PacketBatch.from_packets(pk)
    run_both(b, L.LayerTypeEthernet, mask, options, ext=True)
    # the 64-B window shift and the 8 KiB windows both see the fragments as well
    for tuning in ({"shift": 1}, {"window_bytes": 8192, "shift": 0}):
        run_both(b, L.LayerTypeEthernet, mask, options, ext=False, tuning=tuning)


def test_fast_path_leaves_no_fragment_to_the_fallback():
    """IPv4 fragments decode on the fast path: in a batch of fragment frames only the cut or
    failing ones reach the fallback list (gpd_last_launch_split), with the results exact."""
    from gopacket_amd import parser as P
    from gopacket_amd._lib import check, lib
    fr = [f for f in _fragments() if len(f) >= 60]
    b = PacketBatch.from_packets(fr * 8)
    p = _parser()
    db, dr = P.DeviceBatch(b, 0), P.DeviceResult(b.n, 0)
    h = p.ctx().h
    check(lib.gpd_ctx_set_timing(h, 1), "timing")
    p.decode_device(db, dr)
    fb, f, l_ = C.c_uint64(), C.c_float(), C.c_float()
    check(lib.gpd_last_launch_split(h, C.byref(fb), C.byref(f), C.byref(l_)), "split")
    lib.gpd_ctx_set_timing(h, 0)
    import oracle_ref as O
    ref = O.decode(b, L.LayerTypeEthernet, ALL, 0, ext=False)
    res = dr.to_host()
    for k in ("status", "layers", "net_hash", "tp_hash", "csum", "hdr_off"):
        assert np.array_equal(getattr(res, k), getattr(ref, k)), k
    # only the cut / odd frames may fall back: every whole fragment is a fast-path decode
    whole = sum(1 for i in range(b.n) if (int(ref.status[i]) & 3) == 0)
    assert fb.value <= b.n - whole


def test_host_bind_local_places_pages_on_the_gpu_node():
    """gpd_host_bind_local: a fresh buffer bound before its first write has its pages on the
    GPU's NUMA node (sysfs numa_node of its PCI function); -1 / no-op where none is named."""
    import mmap

    import torch
    from gopacket_amd._lib import lib
    torch.cuda.init()
    n = 64 << 20
    mm = mmap.mmap(-1, n)
    a = np.frombuffer(mm, np.uint8)
    node = C.c_int(-2)
    assert lib.gpd_host_bind_local(0, a.ctypes.data, n, C.byref(node)) == 0, lib.gpd_last_error_string()
    a[::4096] = 1  # first touch
    if node.value < 0:
        pytest.skip("the platform names no NUMA node for the GPU")
    pages = {}
    lo, hi = a.ctypes.data, a.ctypes.data + n
    with open("/proc/self/numa_maps") as f:
        for line in f:
            if lo - 4096 <= int(line.split()[0], 16) < hi:
                for tok in line.split()[1:]:
                    if tok[0] == "N" and "=" in tok:
                        k, v = tok.split("=")
                        pages[int(k[1:])] = pages.get(int(k[1:]), 0) + int(v)
    assert pages, "buffer not found in numa_maps"
    assert pages.get(node.value, 0) >= 0.9 * sum(pages.values()), (node.value, pages)
    del a
    mm.close()


def test_round_kernel_tile_longer_than_its_round_field():
    """ro_kernel keeps a header's round of the tile's byte run in 16 bits.  A
    64-packet tile of 9-MiB frames back to back spans 576 MiB = 73,728 rounds of 8 KiB, so the
    later lanes' header rounds pass 0xFFFF: such a tile goes to the fallback list whole.  IMIX
    frames (their IPv4 Length bounds the decode) sit at the start of each 9-MiB slot; both the
    forced round kernel and the automatic choice equal the oracle."""
    imix = synth.make_imix(64, seed=0x5EED0641)
    slot = 9 << 20
    n = imix.n
    data = np.zeros(n * slot + 64, np.uint8)
    off = np.arange(n, dtype=np.uint64) * slot
    for i in range(n):
        p = np.frombuffer(imix.packet(i), np.uint8)
        data[off[i]:off[i] + len(p)] = p
    b = PacketBatch.from_arrays(data, off.astype(np.uint32), np.full(n, slot, np.uint32), n * slot)
    assert (b.data_len >> 13) > 0xFFFF
    for tuning in (dict(header_once=2), None):
        run_both(b, L.LayerTypeEthernet, ALL, 0, ext=False, tuning=tuning)
