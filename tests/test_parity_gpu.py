"""Device parity: the HIP path (through the C-ABI) vs the CPU oracle, bit-exact.

Every output word is compared: status, layers, both FastHashes, both checksums
and (with ext) the decoded list, error arguments and every layer object's
contents/payload ranges.  Cases: the reference's golden vectors, the synthetic
BASELINE configurations, exhaustive truncations and seeded byte mutations of the
golden packets, odd batch layouts (unaligned / shuffled offsets, packets larger
than an LDS window, empty packets) and mutated dispatch tables.
"""
import os

import numpy as np
import pytest

import golden_cases as G
import oracle_ref as O
from gopacket_amd import layers as L
from gopacket_amd import synth
from gopacket_amd.batch import PacketBatch

pytestmark = pytest.mark.gpu

ALL = 0xFFF  # every decoder, ICMPv4 and LLC included (gpd.h GPD_DEC_ALL)


def _parser(first=L.LayerTypeEthernet, mask=ALL, options=0, tables=None):
    from gopacket_amd import parser as P
    p = P.DecodingLayerParser(first)
    p._mask = mask
    p.IgnoreUnsupported = bool(options & 1)
    p.ComputeChecksums = not (options & 256)
    p.ComputeFlowHashes = not (options & 512)
    if tables is not None:
        p._tables = tables.copy()
    return p


def assert_same(dev, ref, batch=None, ext=True):
    for f in ("status", "layers", "net_hash", "tp_hash", "csum", "hdr_off"):
        a, b = getattr(dev, f), getattr(ref, f)
        if a is None or b is None:
            continue
        bad = np.nonzero(a != b)[0]
        if len(bad):
            i = int(bad[0])
            pk = batch.packet(i).hex() if batch is not None else "?"
            raise AssertionError(
                f"{f} differs at {len(bad)} packets; first i={i}: dev={int(a[i]):#x} ref={int(b[i]):#x} "
                f"dev_decoded={dev.decoded(i) if f != 'layers' else '-'} ref_decoded={ref.decoded(i)} "
                f"pkt={pk[:200]}")
    if ext:
        a = dev.ext.view(np.uint8).reshape(len(dev), -1)
        b = ref.ext.view(np.uint8).reshape(len(ref), -1)
        bad = np.nonzero(np.any(a != b, axis=1))[0]
        if len(bad):
            i = int(bad[0])
            raise AssertionError(f"ext differs at {len(bad)} packets; first i={i}: dev={dev.ext[i]} "
                                 f"ref={ref.ext[i]}")
    if getattr(dev, "detail", None) is not None and ref.ext is not None:
        assert_detail(dev, ref)


def detail_rows(st):
    """Packets whose gpd_detail record the kernel writes: decode errors, > 12 layers."""
    st = st.astype(np.uint32)
    return np.nonzero(((st & 3) == 2) | (((st >> 4) & 31) > 12) | (((st >> 3) & 1) == 1))[0]


def assert_detail(dev, ref, texts=True):
    """dev.detail (written by the generic decoder, fast path or not) == the oracle's ext prefix for
    every packet that has one; and the error values / decoded lists rebuilt from the core words +
    detail alone equal the oracle's."""
    rows = detail_rows(ref.status)
    a = dev.detail.view(np.uint8).reshape(len(dev), -1)[rows]
    b = ref.ext.view(np.uint8).reshape(len(ref), -1)[rows, :24]
    bad = np.nonzero(np.any(a != b, axis=1))[0]
    if len(bad):
        i = int(rows[bad[0]])
        raise AssertionError(f"detail differs at {len(bad)} packets; first i={i}: dev={dev.detail[i]} "
                             f"ref={ref.ext[i]['layer_codes']} {ref.ext[i]['err_arg0']} {ref.ext[i]['err_arg1']}")
    if texts:
        ext, dev.ext = dev.ext, None  # (the core words + detail only)
        try:
            for i in rows[:4096]:
                i = int(i)
                assert str(dev.err(i)) == str(ref.err(i)), (i, str(dev.err(i)), str(ref.err(i)))
                assert dev.decoded(i) == ref.decoded(i), i
        finally:
            dev.ext = ext


def run_both(batch, first=L.LayerTypeEthernet, mask=ALL, options=0, tables=None, ext=True,
             tuning=None):
    """Device vs oracle.  With ext=True both kernels are checked: the ext records force the
    generic decoder, so the same batch is decoded again without them, which takes the fast
    kernel + fallback list whenever it is eligible (gpd_kernels.hip fast_eligible)."""
    ref = O.decode(batch, first, mask, options, tables=tables, ext=ext, nthreads=8)
    out = None
    for e in ((True, False) if ext else (False,)):
        p = _parser(first, mask, options, tables)
        p.Tuning = tuning
        dev = p.DecodeBatch(batch, ext=e)
        assert_same(dev, ref, batch, e)
        out = out or dev
        if not e:  # the gpd_record form too: small frames then take the split kernel (round 6)
            assert_same(p.DecodeBatch(batch, records=True), ref, batch, False)
    return out  # the ext result when ext records were asked for


def test_error_sites_detail_and_texts():
    """One packet per reference error site (tests/error_sites.py, pinned on the oracle by
    tests/test_error_sites.py) and > 12-layer stacks, mixed into fast-path traffic: without ext
    (fast kernel, each failing packet decoded by its wave's fallback list) and with ext (generic
    kernel), the detail records and the texts rebuilt from them equal the oracle's.  The same
    batch through gpd_decode_host fills detail as well."""
    import error_sites as ES
    bulk = synth.make_udp64(4096)
    pk = [bulk.packet(i) for i in range(bulk.n)]
    sites = ES.packets()
    for k, p in enumerate(sites):  # spread among the fast-path packets
        pk.insert(37 * k + 5, p)
    b = PacketBatch.from_packets(pk)
    for opts in (0, 1):
        dev = run_both(b, L.LayerTypeEthernet, ALL, opts)
        ref = O.decode(b, L.LayerTypeEthernet, ALL, opts, ext=True, nthreads=8)
        rows = detail_rows(ref.status)
        assert len(rows) == len(sites)
        assert {int(ref.status[i]) >> 9 & 63 for i in rows} >= set(range(1, 32))
        host = _parser(options=opts).DecodeBatchHost(b, detail=True)
        assert_same(host, ref, b, ext=False)


def test_error_sites_detail_round_kernel():
    """The error sites and deep stacks among IMIX frames, through the round kernel
    (header_once 2: its waves' fallback rounds write the detail records) and the windowed
    kernels: detail and the texts rebuilt from it equal the oracle's."""
    import error_sites as ES
    bulk = synth.make_imix(4096, seed=0x5EED0631)
    pk = [bulk.packet(i) for i in range(bulk.n)]
    for k, p in enumerate(ES.packets()):
        pk.insert(29 * k + 3, p)
    b = PacketBatch.from_packets(pk)
    ref = O.decode(b, L.LayerTypeEthernet, ALL, 0, ext=True, nthreads=8)
    for ho in (2, 1, 0):
        p = _parser()
        p.Tuning = dict(header_once=ho)
        dev = p.DecodeBatch(b, ext=False)
        assert dev.detail is not None
        assert_same(dev, ref, b, ext=False)
        assert_detail(dev, ref)


META = G.load()
CASES = META["cases"]


@pytest.mark.parametrize("c", CASES, ids=[c["name"] for c in CASES])
def test_golden_case_on_device(c):
    first, mask, opts = G.case_config(c)
    dev = run_both(G.single_batch(c), first, mask, opts)
    G.check(c, dev)


def _golden_packets():
    return [G.case_bytes(c) for c in CASES]


@pytest.mark.parametrize("first", [L.LayerTypeEthernet, L.LayerTypeIPv4, L.LayerTypeIPv6,
                                   L.LayerTypeTCP, L.LayerTypeDot1Q, 999])
@pytest.mark.parametrize("mask", [ALL, 0x3FF, 0x1 | 0x4 | 0x20 | 0x100, 0x1 | 0x2 | 0x4 | 0x40 | 0x80,
                                  0x1 | 0x8 | 0x10 | 0x40 | 0x200,
                                  0x1 | 0x4 | 0x400 | 0x20 | 0x40 | 0x100,  # benchmark.go:216-218
                                  0x1 | 0x800 | 0x100])
def test_golden_batch_configs(first, mask):
    run_both(PacketBatch.from_packets(_golden_packets()), first, mask, 0)
    run_both(PacketBatch.from_packets(_golden_packets()), first, mask, 1)


def _mutations(seed=7, per_packet=400):
    rng = np.random.default_rng(seed)
    out = []
    for p in _golden_packets():
        p = p[:2048]
        # every truncation
        out += [p[:k] for k in range(len(p) + 1)]
        # byte flips and header-field fuzz in the first 128 bytes
        a = np.frombuffer(p, np.uint8)
        for _ in range(per_packet):
            b = a.copy()
            k = rng.integers(1, 6)
            pos = rng.integers(0, min(len(b), 128), size=k)
            b[pos] = rng.integers(0, 256, size=k, dtype=np.uint8)
            out.append(b.tobytes()[: rng.integers(len(b) // 2, len(b) + 1)])
    return out


@pytest.mark.parametrize("options", [0, 1])
def test_fuzz_truncations_and_mutations(options):
    pk = _mutations()
    b = PacketBatch.from_packets(pk)
    run_both(b, L.LayerTypeEthernet, ALL, options)
    run_both(b, L.LayerTypeEthernet, 0x3FF, options)
    run_both(b, L.LayerTypeIPv4, 0x4 | 0x20 | 0x40 | 0x100, options)


def test_fuzz_random_headers():
    """Random bytes behind valid-looking Ethernet/IPv4/IPv6 prefixes: exercises option walks,
    HBH/jumbogram paths and every error site."""
    rng = np.random.default_rng(11)
    pkts = []
    for k in range(20000):
        n = int(rng.integers(0, 200))
        body = rng.integers(0, 256, size=n, dtype=np.uint8).tobytes()
        kind = k % 6
        if kind == 0:
            pkts.append(b"\x00" * 12 + b"\x08\x00" + bytes([0x40 | rng.integers(0, 16)]) + body)
        elif kind == 1:
            pkts.append(b"\x00" * 12 + b"\x86\xdd" + b"\x60\x00\x00\x00" + body[:2] + b"\x00" + body)
        elif kind == 2:
            pkts.append(b"\x00" * 12 + b"\x81\x00" + body)
        elif kind == 3:
            pkts.append(b"\x00" * 12 + b"\x88\xa8" + b"\x00\x01\x81\x00" + body)
        elif kind == 4:
            pkts.append(b"\x00" * 12 + bytes([rng.integers(0, 8), rng.integers(0, 256)]) + body)
        else:
            pkts.append(body)
    run_both(PacketBatch.from_packets(pkts), L.LayerTypeEthernet, ALL, 0)


@pytest.mark.parametrize("maker", [synth.make_udp64, synth.make_imix, synth.make_vxlan, synth.make_mixed,
                                   synth.make_tcp64])
def test_synthetic_configs(maker):
    b = maker(1 << 15)
    run_both(b, ext=True)
    run_both(b, ext=False)


@pytest.mark.parametrize("rpfx", [0, 1])
def test_register_prefix_both_ways(rpfx):
    """8 KiB windows sum their chunks for long transport segments either from LDS after the
    decode (window_prefix) or from the registers as they are committed (predicted per wave).
    Force each (gpd_ctx_set_tuning) on long-frame and mixed batches."""
    t = dict(window_bytes=8192, reg_prefix=rpfx)
    for maker in (synth.make_imix, synth.make_mixed, synth.make_vxlan):
        run_both(maker(1 << 13), ext=False, tuning=t)
    run_both(PacketBatch.from_packets(_mutations(seed=23, per_packet=40)), ext=False, tuning=t)
    run_both(PacketBatch.from_packets(_golden_packets() * 4, align=1), ext=False, tuning=t)


@pytest.mark.parametrize("shift,split", [(0, 0), (1, 0), (-1, 1)], ids=["plain", "shifted", "split"])
def test_window_shift_both_ways(shift, split):
    """The register-staged kernel copies windows into LDS either as they lie or shifted so that
    network headers land 16-byte aligned (chosen per batch by mean frame size); the loader /
    decoder split kernel (4 KiB windows, round 6) lands them as they lie by LDS-DMA.  Force each
    (gpd_ctx_set_tuning) on batches of every layout: aligned, packed unaligned, shuffled,
    pcap-like (offsets = 8 mod 16), tagged, VXLAN, mutated and truncated frames."""
    t = dict(shift=shift, split=split)
    pk = _golden_packets()
    run_both(PacketBatch.from_packets(pk), ext=False, tuning=t)
    run_both(PacketBatch.from_packets(pk * 3, align=1), ext=False, tuning=t)
    for k in (2, 8, 13):  # every start alignment class the planner's shift sees
        b = PacketBatch.from_packets([b"\x00" * k + p for p in pk[:40]] * 2, align=16)
        b = PacketBatch(b.data, b.data_len, (b.offset + k).astype(np.uint32), (b.caplen - k).astype(np.uint32))
        run_both(b, ext=False, tuning=t)
    mut = PacketBatch.from_packets(_mutations(seed=19, per_packet=40))
    run_both(mut, ext=False, tuning=t)
    for maker in (synth.make_udp64, synth.make_imix, synth.make_vxlan, synth.make_mixed):
        run_both(maker(1 << 13), ext=False, tuning=t)
    from gopacket_amd import pcap as NP
    cap = NP.synth_capture(synth.make_udp64(1 << 12))
    run_both(NP.index(cap).batch, ext=False, tuning=t)


@pytest.mark.parametrize("window,split", [(4096, 0), (4096, 1), (8192, -1)])
def test_window_sizes_both_ways(window, split):
    """Both LDS window sizes (4 KiB by the register loop and by the split kernel) on every
    synthetic mix and the mutated golden packets."""
    t = dict(window_bytes=window, split=split)
    for maker in (synth.make_udp64, synth.make_imix, synth.make_vxlan, synth.make_mixed):
        run_both(maker(1 << 12), ext=False, tuning=t)
    run_both(PacketBatch.from_packets(_mutations(seed=29, per_packet=20)), ext=False, tuning=t)


@pytest.mark.parametrize("lo,hi", [(44, 76), (48, 80), (60, 68)], ids=["mean60", "mean64", "mean64_narrow"])
def test_split_kernel_window_plans(lo, hi):
    """The split kernel plans each tile's window from its first packet's offset alone (always
    4 KiB, capped at the batch end) when the batch averages >= 63 bytes per packet, else from the
    first offset and the last packet's end.  Packed frames of random length around 64 bytes: tiles
    shorter than 4 KiB (over-read window), longer (packets past the window take the fallback
    list) and the batch's last, partial tile, on both sides of the threshold."""
    rng = np.random.default_rng(lo * 1000 + hi)
    base = synth.make_udp64(3000)
    pk = []
    for i in range(base.n):
        p = base.packet(i)
        k = int(rng.integers(lo, hi + 1))
        pk.append(p[:k] if k <= len(p) else p + bytes(k - len(p)))
    b = PacketBatch.from_packets(pk, align=1)
    assert (b.data_len >= 63 * b.n) == (lo + hi >= 2 * 63)
    run_both(b, ext=False, tuning=dict(window_bytes=4096, split=1))


@pytest.mark.parametrize("extra", [{}, {"reg_prefix": 0}, {"shift": 1}, {"waves_per_simd": 2}],
                         ids=["default", "lds_prefix", "shifted", "two_waves"])
@pytest.mark.parametrize("ho", [0, 1, 2])
def test_header_once_both_ways(ho, extra):
    """8 KiB windows decode a tile either once per window (the lanes each window holds) or
    once per tile from the headers seg_pass staged in registers as the windows passed, with
    the transport segment summed in its window (header_once 1), or once per tile over 8 KiB
    rounds of the tile's contiguous run (header_once 2, ro_kernel: segments summed across
    rounds).  Force each, over layouts whose tiles span one window or several, TCP options
    (mutations), VXLAN (which the header-once decode leaves to the generic decoder) and
    unaligned / pcap-like offsets (odd segment starts)."""
    t = dict(window_bytes=8192, header_once=ho, **extra)
    pk = _golden_packets()
    run_both(PacketBatch.from_packets(pk), ext=False, tuning=t)
    run_both(PacketBatch.from_packets(pk * 3, align=1), ext=False, tuning=t)
    run_both(PacketBatch.from_packets(_mutations(seed=31, per_packet=40)), ext=False, tuning=t)
    for maker in (synth.make_imix, synth.make_mixed, synth.make_traffic_mix, synth.make_vxlan,
                  synth.make_udp64):
        run_both(maker(1 << 13), ext=False, tuning=t)
    from gopacket_amd import pcap as NP
    cap = NP.synth_capture(synth.make_imix(1 << 12))
    run_both(NP.index(cap).batch, ext=False, tuning=t)


@pytest.mark.parametrize("ho", [1, 2])
def test_header_once_tile_shapes(ho):
    """The header-once kernels over batch shapes that stress their tiles and windows / rounds:
    1..200 packets (fewer tiles than waves, a partial last tile), tiles in reverse and shuffled
    order, frames larger than a window between small ones, and a long IMIX batch."""
    t = dict(window_bytes=8192, header_once=ho)
    base = synth.make_imix(1 << 12, seed=0x5EED0401)
    pk = [base.packet(i) for i in range(base.n)]
    for m in (1, 63, 64, 65, 130, 200):
        run_both(PacketBatch.from_packets(pk[:m]), ext=False, tuning=t)
    b = PacketBatch.from_packets(pk)
    for order in (np.arange(b.n)[::-1].copy(), np.random.default_rng(4).permutation(b.n),
                  np.concatenate([np.arange(64 * k, 64 * k + 64)[::-1] for k in range(b.n // 64)])):
        run_both(PacketBatch(b.data, b.data_len, b.offset[order].copy(), b.caplen[order].copy()),
                 ext=False, tuning=t)
    big = [G.case_bytes(c) for c in CASES if c["name"] == "ipv6_jumbogram_dlp"][0]
    mixed = []
    for i, p in enumerate(pk[:1500]):
        mixed.append(p)
        if i % 97 == 5:
            mixed.append(big + big[:3000])
    run_both(PacketBatch.from_packets(mixed), ext=False, tuning=t)
    run_both(synth.make_imix(1 << 17, seed=0x5EED0402), ext=False, tuning=t)


def _ip4_option_frames(n, seed):
    """Long TCP and UDP frames whose IPv4 headers carry 1..10 option words: valid walks (NOP,
    EOL + padding, Router Alert, record-route-like TLVs) and each ip4.go:240-273 error (length
    byte 0 / 1 / 2, a TLV past the header, a type byte alone at the end), some with IHL*4 beyond
    Length or the capture, checksums sometimes right."""
    rng = np.random.default_rng(seed)
    base = synth.make_imix(n, seed=seed)
    out = []
    for i in range(n):
        p = bytearray(base.packet(i))
        eth = 18 if p[12:14] == b"\x81\x00" else 14
        if len(p) < eth + 40:
            out.append(bytes(p))
            continue
        k = int(rng.integers(1, 11))
        opts = bytearray()
        while len(opts) < 4 * k:
            r = rng.random()
            room = 4 * k - len(opts)
            if r < 0.3:
                opts.append(1)
            elif r < 0.4:
                opts += b"\x00" + bytes(room - 1)
            elif r < 0.75 and room >= 3:
                ln = int(rng.integers(3, room + 1))
                opts += bytes([int(rng.integers(2, 255)), ln]) + bytes(rng.integers(0, 256, ln - 2, dtype=np.uint8))
            else:  # an error
                e = int(rng.integers(0, 4))
                if e == 0 and room >= 2:
                    opts += bytes([7, int(rng.integers(0, 3))])
                elif e == 1 and room >= 2:
                    opts += bytes([7, room + int(rng.integers(1, 9))])
                else:
                    opts += bytes([int(rng.integers(2, 255))])
        opts = opts[:4 * k]
        hdr = p[eth:eth + 20]
        hdr[0] = 0x40 | (5 + k)
        total = int.from_bytes(hdr[2:4], "big") + 4 * k
        if rng.random() < 0.1:
            total = 20 + int(rng.integers(0, 4 * k))
        hdr[2:4] = (total & 0xFFFF).to_bytes(2, "big")
        q = p[:eth] + hdr + opts + p[eth + 20:]
        if rng.random() < 0.05:
            q = q[:eth + 20 + int(rng.integers(0, 4 * k))]
        out.append(bytes(q))
    return out


@pytest.mark.parametrize("ho", [0, 1, 2])
def test_ip4_options_both_ways(ho):
    """IPv4 options on long frames: the header-once kernel walks them in seg_pass (ip4_options)
    and decodes the packets in its straight-line pass; the per-window kernel leaves them to the
    generic decoder.  Both against the oracle, valid and erroneous options alike."""
    t = dict(window_bytes=8192, header_once=ho)
    run_both(PacketBatch.from_packets(_ip4_option_frames(1 << 12, 0x5EED0501)), ext=False, tuning=t)
    pk = _ip4_option_frames(1 << 11, 0x5EED0502)
    run_both(PacketBatch.from_packets(pk, align=1), ext=False, tuning=t)


@pytest.mark.parametrize("waves", [2, 3])
def test_round_kernel_long_segments(waves):
    """ro_kernel (header_once 2) sums a transport segment across any number of 8 KiB rounds:
    TCP and UDP frames of 1 B .. 64 KiB between IMIX frames (segments ending on, before and
    after round and chunk boundaries), at 16-byte and odd offsets (the segment summed in the
    other byte order), with right and wrong checksums, against the oracle — the jumbo frames on
    the fast path here, where the windowed kernels hand them to the generic decoder."""
    import error_sites as ES
    rng = np.random.default_rng(0x5EED0601)
    base = synth.make_imix(1 << 11, seed=0x5EED0602)
    pk = [base.packet(i) for i in range(base.n)]
    sizes = [0, 1, 15, 16, 17, 1000, 8100, 8175, 8176, 8177, 8192, 8193, 9000, 16370, 16384, 30001,
             65400]
    k = 0
    for sz in sizes:
        for proto in (6, 17):
            body = bytes(rng.integers(0, 256, sz, dtype=np.uint8))
            l4 = ES.tcp(body) if proto == 6 else ES.udp(body)
            if len(l4) + 20 > 65535:
                l4 = l4[:65535 - 20]
            p = ES.eth(0x0800, ES.ip4(l4, proto=proto))
            pk.insert(31 * k + 7, p)
            k += 1
    t = dict(header_once=2, waves_per_simd=waves)
    for align in (16, 1):
        run_both(PacketBatch.from_packets(pk, align=align), ext=False, tuning=t)


@pytest.mark.parametrize("align", [16, 4, 1])
def test_round_kernel_short_segments_in_long_frames(align):
    """ro_kernel: IMIX frames padded with trailing bytes to 129 B .. 9 KB (the IP length keeps
    the segment short, so it can end in the round before the one the frame's 128 header bytes
    reach: summed from the carried bytes and prefix words), among unpadded frames, against the
    oracle.  The r04 device-walk capture test found such a frame summed from a wrong prefix."""
    rng = np.random.default_rng(0x5EED0611 + align)
    base = synth.make_imix(1 << 13, seed=0x5EED0612)
    pk = [base.packet(i) for i in range(base.n)]
    for i in rng.choice(len(pk), size=len(pk) // 8, replace=False):
        want = int(rng.choice([129, 200, 1600, 8200, 9000]))
        if len(pk[i]) < want:
            pk[i] = pk[i] + bytes(rng.integers(0, 256, want - len(pk[i]), dtype=np.uint8))
    for ho in (2, 1):
        run_both(PacketBatch.from_packets(pk, align=align), ext=False, tuning=dict(header_once=ho))


def _vxlan_frames(rng):
    """VXLAN frames in every outer shape fast_decode's first pass accepts or refuses, over inner
    frames the round kernel's tile decode takes (Ethernet [Dot1Q] IPv4/IPv6 TCP/UDP) or leaves
    to the generic decoder (no transport, inner IPv6 under outer IPv4, nested VXLAN, errors)."""
    import struct

    import error_sites as ES

    def body(n):
        return bytes(rng.integers(0, 256, n, dtype=np.uint8))

    def vx(inner, outer="v4", tags=0, frag=0, udp_len=None, ip_len=None, pad=0, sport=40001, dport=4789):
        u = ES.udp(b"\x08\x00\x00\x00\x00\x12\x34\x00" + inner, sport=sport, dport=dport, length=udp_len)
        if outer == "v4":
            l3, et = ES.ip4(u, proto=17, length=ip_len, flags_frag=frag), 0x0800
        else:
            l3, et = ES.ip6(u, nh=17, length=ip_len), 0x86DD
        for _ in range(tags):
            l3, et = struct.pack(">HH", 100, et) + l3, 0x8100
        return ES.eth(et, l3) + bytes(pad)

    inner = [ES.eth(0x0800, ES.ip4(ES.tcp(body(int(rng.integers(0, 300)))))),
             ES.eth(0x0800, ES.ip4(ES.udp(body(40)), proto=17)),
             ES.eth(0x86DD, ES.ip6(ES.tcp(body(24)))),
             ES.eth(0x86DD, ES.ip6(ES.udp(body(9)), nh=17)),
             ES.eth(0x8100, struct.pack(">HH", 7, 0x0800) + ES.ip4(ES.tcp(body(30)))),
             ES.eth(0x0800, ES.ip4(ES.tcp(body(20), doff=7, opts=b"\x02\x04\x05\xb4\x01\x01\x01\x00"))),
             ES.eth(0x0800, ES.ip4(ES.tcp(body(5), doff=4))),               # inner decode error
             ES.eth(0x0800, ES.ip4(body(8), proto=1)),                      # ICMPv4: no transport
             ES.eth(0x0806, body(28)),                                      # ARP: unsupported
             ES.eth(0x0800, ES.ip4(ES.tcp(body(8)), ihl=6, opts=b"\x01\x01\x01\x00")),
             ES.eth(0x0800, ES.ip4(ES.tcp(body(3000)))),                     # a long inner segment
             ES.eth(0x0800, ES.ip4(ES.tcp(body(60)))[:50])]                   # inner frame cut
    inner.append(vx(inner[0])[:])  # nested VXLAN
    out = []
    for inn in inner:
        out += [vx(inn), vx(inn, outer="v6"), vx(inn, tags=1), vx(inn, tags=2), vx(inn, pad=30),
                vx(inn, ip_len=20 + 8 + 8 + len(inn) + 40), vx(inn, frag=0x2000), vx(inn, udp_len=0),
                vx(inn, udp_len=5), vx(inn, udp_len=8 + 8 + len(inn) + 10), vx(inn, sport=4789, dport=80),
                vx(inn)[:14 + 20 + 8 + 8 + 20], vx(inn, outer="v6", tags=1, pad=3)]
    out.append(vx(b""))   # VXLAN header only
    out.append(vx(b"\x00" * 7))
    return out


@pytest.mark.parametrize("align", [16, 1])
def test_vxlan_frame_shapes_in_every_kernel(align):
    """Every outer and inner VXLAN shape above, among IMIX frames and config 4's VXLAN frames,
    through the round kernel (which hands VXLAN frames to its wave's generic decoder), the
    windowed header-once kernel (which decodes them per window) and the per-window kernels,
    equals the oracle."""
    rng = np.random.default_rng(0x5EED0621 + align)
    base = synth.make_imix(1 << 12, seed=0x5EED0622)
    vxb = synth.make_vxlan(1 << 11, seed=0x5EED0623)
    pk = [base.packet(i) for i in range(base.n)] + [vxb.packet(i) for i in range(vxb.n)]
    pk += _vxlan_frames(rng) * 3
    order = rng.permutation(len(pk))
    b = PacketBatch.from_packets([pk[i] for i in order], align=align)
    for ho in (2, 1, 0):
        run_both(b, ext=False, tuning=dict(header_once=ho))
    run_both(b, ext=False, tuning=dict(header_once=2, waves_per_simd=2))
    run_both(b, mask=0x3FF, options=1, ext=False, tuning=dict(header_once=2))


@pytest.mark.parametrize("geom", [dict(waves_per_simd=2, grid_rounds=1), dict(waves_per_simd=3, grid_rounds=2),
                                  dict(waves_per_simd=4, grid_rounds=8), dict(grid_rounds=1), dict(split=1),
                                  dict(split=1, grid_rounds=3), dict(split=0), dict(split=0, grid_rounds=1)],
                         ids=["w2r1", "w3r2", "w4r8", "r1", "split", "split_r3", "nosplit", "nosplit_r1"])
def test_launch_geometry_never_changes_results(geom):
    """gpd_tuning.waves_per_simd (now enforced: an LDS reservation of 1/W of the CU per
    workgroup), grid_rounds and split (ABI 10) change only how many waves stream and how many
    tiles each takes, through every fast kernel (4 KiB windows shifted, 8 KiB AL / plain /
    header-once windows, rounds, the loader / decoder split over an LDS ring) with fallback
    lists, against the oracle; with more tiles than one round of waves and with fewer, and 4 KiB
    windows too small for a tile's bytes (the split kernel lists the uncovered packets)."""
    mixed = synth.make_mixed(6000)
    golden = PacketBatch.from_packets(_golden_packets() * 7)
    cases = [(synth.make_udp64(40000), {}), (synth.make_vxlan(20000), {}), (synth.make_imix(12000), {}),
             (mixed, {}), (mixed, dict(window_bytes=8192, header_once=1)), (mixed, dict(window_bytes=4096)),
             (golden, dict(window_bytes=4096)), (synth.make_udp64(3000), {}), (synth.make_udp64(70), {})]
    for b, t in cases:
        run_both(b, ext=False, tuning=dict(t, **geom))


def test_layouts_unaligned_shuffled_large_empty():
    pk = _golden_packets() + [b"", b"\x01", b"\x00" * 13]
    big = [G.case_bytes(c) for c in CASES if c["name"] == "ipv6_jumbogram_dlp"][0]
    pk += [big, big[:20000], big + big[:5000]]
    pk = pk * 5
    # unaligned packed layout
    b = PacketBatch.from_packets(pk, align=1)
    run_both(b)
    # shuffled (non-monotonic) offsets over the same buffer
    perm = np.random.default_rng(3).permutation(b.n)
    b2 = PacketBatch(b.data, b.data_len, b.offset[perm].copy(), b.caplen[perm].copy())
    run_both(b2)
    # n not a multiple of 64, single packet
    run_both(PacketBatch.from_packets(pk[:65]))
    run_both(PacketBatch.from_packets(pk[:1]))


def test_mutated_dispatch_tables():
    t = L.DispatchTables()
    t.udp_port[9999] = L.LayerTypeVXLAN       # RegisterUDPPortLayerType(9999, VXLAN)
    t.tcp_port[80] = L.LayerTypeIPv4          # a deliberately odd registration
    t.ethertype[0x0800] = L.LayerTypeIPv6     # EthernetTypeMetadata override
    t.ipproto[6] = L.LayerTypeUDP
    pk = _golden_packets() + [synth.make_vxlan(64).packet(k) for k in range(64)]
    run_both(PacketBatch.from_packets(pk), tables=t)


def test_reconfigure_in_place_keeps_tables_and_context():
    """ABI 8 through the Python parser (parser.go:182-202, layers/ports.go:126-128): register a
    UDP port as VXLAN and reload the tables, add the VXLAN decoder, then flip IgnoreUnsupported
    both ways.  The context is the same gpd_ctx throughout (no re-creation that would drop the
    reloaded tables), and every step equals the oracle on the mutated tables, on the fast path
    (ext=False) and the generic one."""
    from gopacket_amd import parser as P
    saved = L.TABLES.copy()
    try:
        pk = _golden_packets()
        vx = synth.make_vxlan(128)
        for i in range(vx.n):
            q = bytearray(vx.packet(i))
            q[36:38] = (8472).to_bytes(2, "big")
            pk.append(bytes(q))
        b = PacketBatch.from_packets(pk)
        p = P.NewDecodingLayerParser(L.LayerTypeEthernet, P.Ethernet(), P.Dot1Q(), P.IPv4(), P.IPv6(),
                                     P.TCP(), P.UDP(), P.Payload())
        p.DecodeBatch(b)  # the context exists before anything changes
        h = p.ctx().h.value
        L.RegisterUDPPortLayerType(8472, L.LayerTypeVXLAN)
        p.reload_tables()
        p.AddDecodingLayer(P.VXLAN())
        for ign in (True, False, True):
            p.IgnoreUnsupported = ign
            ref = O.decode(b, L.LayerTypeEthernet, p.decoders, p.options, tables=L.TABLES, ext=True,
                           nthreads=8)
            assert any(L.LayerTypeVXLAN in ref.decoded(i) for i in range(len(pk) - 8, len(pk)))
            for e in (False, True):
                dev = p.DecodeBatch(b, ext=e)
                assert_same(dev, ref, b, e)
            assert_same(p.DecodeBatchHost(b, detail=True), ref, b, ext=False)
            assert p.ctx().h.value == h, "the context was re-created"
    finally:
        L.TABLES.udp_port[:] = saved.udp_port


def test_option_bits_outside_the_header_are_refused():
    """include/gpd.h: the reference has two options (parser.go:336-350), the engine two more;
    every other bit — the runtime's launch flags (24-29) and the ablation bits 30 (no DMA wait)
    and 31 (no decode), which only the diagnostic library takes — is GPD_ERR_INVALID from
    gpd_ctx_set_options and gpd_ctx_create, and a refused bit leaves the context's options as
    they were (its next decode equals the oracle)."""
    import ctypes as C
    from gopacket_amd import parser as P
    from gopacket_amd._lib import GPD_ERR_INVALID, GpdConfig, lib
    assert os.path.basename(P.lib._name) == "libgpd.so"
    p = _parser()
    b = PacketBatch.from_packets(_golden_packets())
    p.DecodeBatch(b)
    h = p.ctx().h
    known = P.OPT_IGNORE_UNSUPPORTED | P.OPT_IGNORE_PANIC | P.OPT_NO_CHECKSUMS | P.OPT_NO_FLOW_HASH
    for bit in range(32):
        if (1 << bit) & known:
            continue
        assert lib.gpd_ctx_set_options(h, p.options | (1 << bit)) == GPD_ERR_INVALID, bit
        cfg = GpdConfig(L.LayerTypeEthernet, p.decoders, 1 << bit, 0, None, None, None, None)
        out = C.c_void_p()
        assert lib.gpd_ctx_create(0, C.byref(cfg), C.byref(out)) == GPD_ERR_INVALID, bit
        assert not out.value
    ref = O.decode(b, L.LayerTypeEthernet, p.decoders, p.options, ext=False)
    assert_same(p.DecodeBatch(b), ref, b, False)


def test_set_decoding_layer_container_in_place():
    """SetDecodingLayerContainer (parser.go:236-242) replaces the registered decoders — fewer
    here, then more — on the same gpd_ctx (gpd_ctx_set_decoders), and each set equals the oracle
    with that mask; a DecodingLayerFunc (layers_decoder.go:11-101) from a Sparse container
    returns the reference's (LayerType, error) pairs; DecodeLayers with no decoder for `first`
    leaves the caller's decoded list as it was (layers_decoder.go:12-16)."""
    from gopacket_amd import parser as P
    pk = _golden_packets()
    b = PacketBatch.from_packets(pk)
    p = P.NewDecodingLayerParser(L.LayerTypeEthernet, *[P.DECODER_BY_NAME[k]() for k in P.DECODER_BY_NAME])
    p.DecodeBatch(b)
    h = p.ctx().h.value
    small = P.DecodingLayerSparse()
    for d in (P.Ethernet(), P.IPv4(), P.UDP(), P.Payload()):
        small = small.Put(d)
    arr = P.DecodingLayerArray()
    for d in (P.Ethernet(), P.Dot1Q(), P.IPv6(), P.TCP(), P.VXLAN(), P.IPv4(), P.UDP()):
        arr = arr.Put(d)
    for dlc in (small, arr):
        p.SetDecodingLayerContainer(dlc)
        ref = O.decode(b, L.LayerTypeEthernet, p.decoders, 0, ext=True, nthreads=8)
        for e in (False, True):
            assert_same(p.DecodeBatch(b, ext=e), ref, b, e)
        assert p.ctx().h.value == h, "the context was re-created"
    fn = small.LayersDecoder(L.LayerTypeEthernet, p)
    ref = O.decode(b, L.LayerTypeEthernet, small.engine_mask(), 0, ext=True, nthreads=8)
    for i in range(0, len(pk), 3):
        decoded = []
        p.Truncated = False
        typ, err = fn(pk[i], decoded)
        st = int(ref.status[i]) & 3
        assert decoded == ref.decoded(i), i
        assert typ == (ref.stop_type(i) if st == 1 else 0), i
        assert str(err) == str(ref.err(i) if st == 2 else None), i
        assert p.Truncated == ref.truncated(i), i
    q = P.NewDecodingLayerParser(L.LayerTypeIPv4, P.Ethernet(), P.TCP())  # nothing takes IPv4
    decoded = [L.LayerTypeEthernet, L.LayerTypeTCP]
    err = q.DecodeLayers(pk[0], decoded)
    assert decoded == [L.LayerTypeEthernet, L.LayerTypeTCP]
    assert str(err) == str(P.UnsupportedLayerType(L.LayerTypeIPv4))


def test_flows_from_results():
    """NetworkFlow() / TransportFlow() rebuilt from the result words and the packet bytes
    (gopacket_amd.results.Flow): testSimpleTCPPacket's endpoints as decode_test.go:404-405,430-431
    asserts them ("172.17.81.73" -> "173.222.254.225", "50679" -> "80"); over the mixed batch
    (IPv4, IPv6, VXLAN inner flows) each Flow's endpoints are the bytes at the oracle's header
    offsets, its FastHash the oracle's, and Reverse() keeps it (doc.go:216-219)."""
    from gopacket_amd import parser as P
    from gopacket_amd.results import EndpointIPv4, EndpointTCPPort
    c = next(c for c in CASES if c["name"] == "simple_tcp_full")
    b = G.single_batch(c)
    first, mask, opts = G.case_config(c)
    res = _parser(first, mask, opts).DecodeBatch(b)
    nf, tf = res.NetworkFlow(0, b), res.TransportFlow(0, b)
    assert nf.EndpointType() == EndpointIPv4 and tf.EndpointType() == EndpointTCPPort
    assert (str(nf.Src()), str(nf.Dst())) == ("172.17.81.73", "173.222.254.225")
    assert (str(tf.Src()), str(tf.Dst())) == ("50679", "80")
    assert nf.String() == "172.17.81.73->173.222.254.225"
    mb = synth.make_mixed(3000)
    p = P.NewDecodingLayerParser(L.LayerTypeEthernet, *[P.DECODER_BY_NAME[k]() for k in P.DECODER_BY_NAME])
    dev = p.DecodeBatch(mb)
    ref = O.decode(mb, L.LayerTypeEthernet, p.decoders, 0, ext=False, nthreads=8)
    seen = set()
    for i in range(mb.n):
        pk = mb.packet(i)
        for f, h, off in ((dev.NetworkFlow(i, mb), ref.network_flow_hash(i), ref.network_offset(i)),
                          (dev.TransportFlow(i, mb), ref.transport_flow_hash(i), ref.transport_offset(i))):
            if h is None:
                assert f is None or off is not None
                continue
            assert f is not None and f.FastHash() == h and f.Reverse().FastHash() == h
            seen.add(f.EndpointType())
            if f.EndpointType() in (1, 2):
                a, n = (12, 4) if f.EndpointType() == 1 else (8, 16)
                assert f.src == pk[off + a:off + a + n] and f.dst == pk[off + a + n:off + a + 2 * n]
            else:
                assert f.src == pk[off:off + 2] and f.dst == pk[off + 2:off + 4]
    assert seen >= {1, 4, 5}


def test_fast_hash_of_built_flows_and_endpoints():
    """gpd_fast_hash (ABI 9): Flow.FastHash / Endpoint.FastHash of caller-built keys on the device
    (flows.go:60-83,167-174) against the oracle's FNV — raw lengths 0..16, EndpointTypes in and
    beyond 32 bits (RegisterEndpointType numbers, negative int64), a flow and its Reverse(); and
    NewFlow() copies of the mixed batch's decoded flows hash to what the decode kernel computed."""
    from gopacket_amd import parser as P
    from gopacket_amd.results import FastHashes, NewEndpoint, NewFlow
    ol = O.lib()
    M = (1 << 64) - 1

    def ofnv(b):
        return int(ol.gpo_fnv_hash(bytes(b), len(b)))

    rng = np.random.default_rng(9)
    typs = [1, 2, 4, 5, 1000, 77777, (1 << 40) + 3, -5, 0]
    flows, eps, want_f, want_e = [], [], [], []
    for k in range(600):
        t = typs[k % len(typs)]
        a = rng.integers(0, 256, int(rng.integers(0, 17)), dtype=np.uint8).tobytes()
        b = rng.integers(0, 256, int(rng.integers(0, 17)), dtype=np.uint8).tobytes()
        flows.append(NewFlow(t, a, b))
        eps.append(NewEndpoint(t, a))
        want_f.append((((ofnv(a) + ofnv(b)) & M) ^ (t & M)) * 1099511628211 & M)
        want_e.append(((ofnv(a) ^ (t & M)) * 1099511628211) & M)
        if 0 <= t < (1 << 32):
            assert want_f[-1] == ol.gpo_flow_fasthash(t, a, len(a), b, len(b))
            assert want_e[-1] == ol.gpo_endpoint_fasthash(t, a, len(a))
    assert [int(x) for x in FastHashes(flows)] == want_f
    assert [int(x) for x in FastHashes([f.Reverse() for f in flows])] == want_f
    assert [int(x) for x in FastHashes(eps)] == want_e
    assert flows[3].FastHash() == want_f[3] and eps[5].FastHash() == want_e[5]
    mb = synth.make_mixed(2000)
    p = P.NewDecodingLayerParser(L.LayerTypeEthernet, *[P.DECODER_BY_NAME[k]() for k in P.DECODER_BY_NAME])
    dev = p.DecodeBatch(mb)
    got, built = [], []
    for i in range(mb.n):
        for f in (dev.NetworkFlow(i, mb), dev.TransportFlow(i, mb)):
            if f is not None:
                got.append(f.FastHash())
                built.append(NewFlow(f.EndpointType(), f.src, f.dst))
    assert len(built) > 2000 and [int(x) for x in FastHashes(built)] == got


def test_all_empty_batch():
    """A batch whose every packet is empty (CapLen 0, data_len 0): Ethernet's "too small" error
    for each, on the device and host paths."""
    b = PacketBatch.from_packets([b""] * 37)
    assert b.data_len == 0
    ref = run_both(b)
    assert all(str(ref.err(i)) == "Ethernet packet too small" for i in range(b.n))
    host = _parser().DecodeBatchHost(b, detail=True)
    assert_same(host, O.decode(b, L.LayerTypeEthernet, ALL, 0, ext=True), b, ext=False)


def test_options_no_checksums_no_hashes():
    b = synth.make_mixed(3000)
    for opt in (256, 512, 768, 769):
        run_both(b, options=opt)


def test_host_path_matches_device_path():
    """gpd_decode_host in both staging modes: span (a back-to-back batch travels as one
    window of the caller's buffer) and repack (shuffled / overlapping / gappy layouts), with
    and without the buffer registered, against the device path."""
    from gopacket_amd import parser as P
    from gopacket_amd._lib import check, lib
    b = synth.make_mixed(5000)
    p = P.DecodingLayerParser(L.LayerTypeEthernet)
    p._mask = ALL
    dev = p.DecodeBatch(b, ext=True)
    host = p.DecodeBatchHost(b, ext=True)
    assert_same(host, dev, b)
    check(lib.gpd_host_register(p.ctx().h, b.data.ctypes.data, b.data.nbytes), "gpd_host_register")
    try:
        assert_same(p.DecodeBatchHost(b, ext=True), dev, b)
    finally:
        lib.gpd_host_unregister(p.ctx().h, b.data.ctypes.data)
    rng = np.random.default_rng(2)
    perm = rng.permutation(b.n)
    shuffled = PacketBatch(b.data, b.data_len, b.offset[perm].copy(), b.caplen[perm].copy())
    assert_same(p.DecodeBatchHost(shuffled, ext=True), p.DecodeBatch(shuffled, ext=True), shuffled)
    sparse = PacketBatch(b.data, b.data_len, b.offset[::7].copy(), b.caplen[::7].copy())  # gaps
    assert_same(p.DecodeBatchHost(sparse, ext=False), p.DecodeBatch(sparse, ext=False), sparse, ext=False)


def test_host_path_with_registered_descriptors():
    """Span chunks whose offset and caplen arrays are registered too travel without a host pass:
    the descriptors by DMA as they are, the window read through a base pointer moved back by the
    chunk's start.  Several 2^20-packet chunks (chunk starts far from 0), a batch starting past
    byte 0, and the tail chunk, against the device path."""
    from gopacket_amd import parser as P
    from gopacket_amd._lib import check, lib
    u = synth.make_udp64((1 << 21) + 12345)
    m = synth.make_mixed(3000)
    p = P.DecodingLayerParser(L.LayerTypeEthernet)
    p._mask = ALL
    h = p.ctx().h
    for b in (u, PacketBatch(m.data, m.data_len, m.offset[40:].copy(), m.caplen[40:].copy())):
        want = p.DecodeBatch(b, ext=False)
        arrs = [b.data, b.offset, b.caplen]
        for a in arrs:
            check(lib.gpd_host_register(h, a.ctypes.data, a.nbytes), "register")
        try:
            assert_same(p.DecodeBatchHost(b, ext=False), want, b, ext=False)
        finally:
            for a in arrs:
                lib.gpd_host_unregister(h, a.ctypes.data)


def test_decode_layers_single_packet_api():
    from gopacket_amd import parser as P
    c = [c for c in CASES if c["name"] == "simple_tcp_dlp4"][0]
    p = P.NewDecodingLayerParser(L.LayerTypeEthernet, P.Ethernet(), P.IPv4(), P.TCP(), P.Payload())
    decoded = []
    err = p.DecodeLayers(G.case_bytes(c), decoded)
    assert err is None and decoded == [17, 20, 44, 2] and not p.Truncated
    c = [c for c in CASES if c["name"] == "udp_truncated"][0]
    p2 = P.NewDecodingLayerParser(L.LayerTypeEthernet, P.Ethernet(), P.Dot1Q(), P.IPv4(), P.UDP(),
                                  P.Payload())
    err = p2.DecodeLayers(G.case_bytes(c), decoded)
    assert err is None and p2.Truncated and decoded == [17, 15, 20, 45, 2]


def _oracle_threads() -> int:
    """The cores this process may use (affinity, capped by a cgroup v2 quota)."""
    import os
    n = len(os.sched_getaffinity(0))
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            n = min(n, max(1, -(-int(q) // int(per))))
    except (OSError, ValueError):
        pass
    return max(1, min(n, 64))


BENCH_MASK = 0x3FF  # the decoder set bench.py times (bench.py: Ethernet .. Fragment, no ICMPv4 / LLC)


def _full_size_exact(b):
    """Every packet of a full-size batch, all five result words and hdr_off, in the gpd_record
    (AoS) form and in the SoA form, against the multi-threaded oracle — with the decoder set the
    bench times `value` on (BENCH_MASK) and with every decoder.  Returns the last SoA result for
    the property checks."""
    import torch
    from gopacket_amd import parser as P
    db = P.DeviceBatch(b, 0)
    res = None
    for mask in (BENCH_MASK, ALL):
        ref = O.decode(b, L.LayerTypeEthernet, mask, 0, ext=False, nthreads=_oracle_threads())
        p = _parser(mask=mask)
        for records in (True, False):
            dr = P.DeviceResult(b.n, 0, hdr_off=True, records=records)
            p.decode_device(db, dr)
            torch.cuda.synchronize()
            res = dr.to_host()
            del dr
            assert_same(res, ref, b, ext=False)
        del ref
    del db
    torch.cuda.empty_cache()
    return res


def test_full_size_config2_exact():
    """BASELINE config 2 at full size (2^24 x 64 B Eth/IPv4/UDP): every packet bit-exact against
    the oracle in both result forms, plus the size-independent properties."""
    n = 1 << 24
    b = synth.make_udp64(n)
    res = _full_size_exact(b)
    assert np.all(res.status & 3 == 0)
    assert np.all(((res.status >> 4) & 31) == 4)
    bad = (np.arange(n) % 64) == 63
    stored = (b.data[24:n * 64:64].astype(np.uint32) << 8) | b.data[25:n * 64:64]
    assert np.array_equal((res.csum & 0xFFFF) == stored, ~bad)
    assert np.all(res.csum >> 16 == 0)


def test_full_size_tcp64_exact():
    """The north star's literal target at the bench's size (2^24 x 64 B Eth/IPv4/TCP): every
    packet bit-exact in both result forms; TCP ComputeChecksum 0 exactly on the valid ones."""
    n = 1 << 24
    b = synth.make_tcp64(n)
    res = _full_size_exact(b)
    _full_size_common(b, res, [17, 20, 44, 2], 14, n)


def _full_size_common(b, res, want_decoded, ip_off, n):
    """Properties every packet of a full-size synthetic config shares."""
    assert np.all(res.status & 3 == 0), "every packet decodes cleanly"
    assert np.all(((res.status >> 4) & 31) == len(want_decoded))
    assert np.all(res.layers == res.layers[0]), "one decoded stack for all"
    assert res.decoded(0) == want_decoded
    bad = (np.arange(n) % 64) == 63  # synth: 1 in 64 carries a corrupted TCP checksum
    assert np.array_equal((res.csum >> 16) != 0, bad), "TCP ComputeChecksum is 0 exactly when valid"
    off = b.offset.astype(np.int64) + ip_off + 10
    stored = (b.data[off].astype(np.uint32) << 8) | b.data[off + 1]
    assert np.array_equal(res.csum & 0xFFFF, stored), "IPv4 header checksum equals the stored one"


def test_full_size_config3_imix_exact():
    """BASELINE config 3 at full size (2^22 IMIX 64/576/1500 Eth/Dot1Q/IPv4/TCP): every window
    class, multi-window tiles and the wave-cooperative transport checksum at their real mix;
    every packet bit-exact in both result forms."""
    n = 1 << 22
    b = synth.make_imix(n)
    res = _full_size_exact(b)
    _full_size_common(b, res, [17, 15, 20, 44, 2], 18, n)
    # (the transport FastHash is symmetric in the two ports, so port pairs share values)
    assert len(np.unique(res.net_hash)) > n // 2 and len(np.unique(res.tp_hash)) > n // 64


def test_full_size_config4_vxlan_exact():
    """BASELINE config 4 at full size (2^23 x 128 B VXLAN): the two-pass stack
    [Eth, IPv4, UDP, VXLAN, Eth, IPv4, TCP, Payload] on every packet, inner flow keys (A11);
    every packet bit-exact in both result forms."""
    n = 1 << 23
    b = synth.make_vxlan(n)
    res = _full_size_exact(b)
    _full_size_common(b, res, [17, 20, 45, 116, 17, 20, 44, 2], 64, n)
    # the flow keys are the inner 5-tuple: the inner addresses and ports of packet 0
    ref0 = O.decode(PacketBatch.from_packets([b.packet(0)[50:]]), ext=False)
    assert int(res.net_hash[0]) == int(ref0.net_hash[0]) and int(res.tp_hash[0]) == int(ref0.tp_hash[0])


@pytest.mark.parametrize("mask", [ALL, 0x3FF])
def test_traffic_mix_both_kernels(mask):
    """The traffic mix (ICMPv4 echo, 802.3/LLC, IPv6/TCP, VXLAN, TCP/UDP, and the generic
    decoder's share: IPv4 options, IPv6 hop-by-hop, cut TCP headers; its IPv4 fragments decode on
    the fast path) with every
    decoder registered and without ICMPv4/LLC (they then stop as unsupported)."""
    run_both(synth.make_traffic_mix(1 << 15), mask=mask, ext=True)
    run_both(synth.make_traffic_mix(1 << 15, seed=9), mask=mask, options=1, ext=False)


def test_fallback_split_counts_the_generic_share():
    """gpd_last_launch_split: the fast decode takes ICMPv4, IPv6/TCP and VXLAN itself, and
    (and IPv4 fragments) itself, and leaves exactly the IPv4-options, hop-by-hop, LLC/STP and
    cut-TCP frames to the generic decoder (each wave's fallback list, decoded at the end of that
    wave) — with header-once off.  With header-once on (the mix's long frames choose it), a
    wave's few VXLAN frames fall back too, and the results stay exact."""
    import ctypes as C
    from gopacket_amd import parser as P
    from gopacket_amd._lib import check, lib
    n = 1 << 16
    b = synth.make_traffic_mix(n)
    wsum = sum(w for _, _, w in synth.MIX_CLASSES)
    want = sum(n * w // wsum for name, _, w in synth.MIX_CLASSES if name in synth.MIX_FALLBACK)
    n_vx = sum(n * w // wsum for name, _, w in synth.MIX_CLASSES if name == "vxlan")
    ref = O.decode(b, L.LayerTypeEthernet, ALL, 0, ext=False, nthreads=8)
    for ho in (0, -1):
        p = P.DecodingLayerParser(L.LayerTypeEthernet)
        p._mask = ALL
        p.Tuning = {"header_once": ho}
        db, dr = P.DeviceBatch(b, 0), P.DeviceResult(n, 0)
        h = p.ctx().h
        check(lib.gpd_ctx_set_timing(h, 1), "timing")
        p.decode_device(db, dr)
        fb, f, l = C.c_uint64(), C.c_float(), C.c_float()
        check(lib.gpd_last_launch_split(h, C.byref(fb), C.byref(f), C.byref(l)), "split")
        if ho == 0:
            assert fb.value == want
        else:
            assert want < fb.value <= want + n_vx
        assert f.value > 0 and l.value >= 0  # (the lists are decoded inside the fast kernel)
        res = dr.to_host()
        for k in ("status", "layers", "net_hash", "tp_hash", "csum", "hdr_off"):
            assert np.array_equal(getattr(res, k), getattr(ref, k)), k
        lib.gpd_ctx_set_timing(h, 0)


def test_host_path_recovers_after_a_failed_call():
    """gpd_decode_host fails on a packet no staging slot holds (> 256 MB) after earlier chunks
    were already in flight; the next call on the same context must start from idle slots and
    decode its own batch exactly (no stale chunk drained into its results)."""
    from gopacket_amd import parser as P
    from gopacket_amd._lib import GpdError
    small = synth.make_udp64(3 * (1 << 20) // 2)  # two chunks in flight before the big one
    big = (257 << 20)
    data = np.zeros(small.data_len + big + 64, np.uint8)
    data[:small.data_len] = small.data[:small.data_len]
    off = np.concatenate([small.offset, [small.data_len]]).astype(np.uint32)
    cap = np.concatenate([small.caplen, [big]]).astype(np.uint32)
    bad = PacketBatch(data, small.data_len + big, off, cap)
    p = P.DecodingLayerParser(L.LayerTypeEthernet)
    p._mask = ALL
    with pytest.raises(GpdError, match="larger than"):
        p.DecodeBatchHost(bad)
    del data, bad
    nxt = synth.make_mixed(5000, seed=0x77)
    ref = O.decode(nxt, L.LayerTypeEthernet, ALL, 0, ext=False, nthreads=8)
    assert_same(p.DecodeBatchHost(nxt), ref, nxt, ext=False)


def test_host_path_chunks_with_everything_registered():
    """The bench's PCIe-inclusive path over several chunks: batch, descriptors and result arrays
    all registered, so every chunk's H2D and its results' D2H (on the slot's second stream) are
    DMA straight from / into the caller's arrays while the next chunks travel — three 2^20-packet
    chunks and a tail, against the device path."""
    from gopacket_amd import parser as P
    from gopacket_amd._lib import check, lib
    from gopacket_amd.results import BatchResult
    b = synth.make_udp64((3 << 20) + 4321)
    p = P.DecodingLayerParser(L.LayerTypeEthernet)
    p._mask = ALL
    want = p.DecodeBatch(b, ext=False)
    z = lambda dt: np.zeros(b.n, dt)
    out = BatchResult(z(np.uint32), z(np.uint64), z(np.uint64), z(np.uint64), z(np.uint32), None,
                      z(np.uint32))
    arrs = [b.data, b.offset, b.caplen, out.status, out.layers, out.net_hash, out.tp_hash, out.csum,
            out.hdr_off]
    h = p.ctx().h
    for a in arrs:
        check(lib.gpd_host_register(h, a.ctypes.data, a.nbytes), "register")
    try:
        for _ in range(2):  # (the second call reuses the slots and their events)
            assert_same(p.DecodeBatchHost(b, out=out), want, b, ext=False)
    finally:
        for a in arrs:
            lib.gpd_host_unregister(h, a.ctypes.data)


def test_host_paths_into_registered_result_arrays():
    """Result arrays registered with gpd_host_register receive the results by DMA (no staging
    copy): gpd_decode_host and gpd_decode_pcap_at must give the same words either way."""
    from gopacket_amd import parser as P
    from gopacket_amd import pcap as NP
    from gopacket_amd._lib import check, lib
    from gopacket_amd.results import BatchResult
    b = synth.make_mixed(9000)
    p = P.DecodingLayerParser(L.LayerTypeEthernet)
    p._mask = ALL
    ref = p.DecodeBatchHost(b)
    z = lambda dt: np.zeros(b.n, dt)
    out = BatchResult(z(np.uint32), z(np.uint64), z(np.uint64), z(np.uint64), z(np.uint32), None,
                      z(np.uint32))
    arrs = [out.status, out.layers, out.net_hash, out.tp_hash, out.csum, out.hdr_off]
    h = p.ctx().h
    for a in arrs:
        check(lib.gpd_host_register(h, a.ctypes.data, a.nbytes), "register")
    try:
        assert_same(p.DecodeBatchHost(b, out=out), ref, b, ext=False)
        cap = NP.synth_capture(synth.make_udp64(3 << 18))  # 3 parts of 2^18 records
        info = NP.header(cap)
        want = p.DecodeBatch(NP.index(cap).batch)
        m = 3 << 18
        big = BatchResult(np.zeros(m, np.uint32), np.zeros(m, np.uint64), np.zeros(m, np.uint64),
                          np.zeros(m, np.uint64), np.zeros(m, np.uint32), None, np.zeros(m, np.uint32))
        for a in (big.status, big.layers, big.net_hash, big.tp_hash, big.csum, big.hdr_off):
            check(lib.gpd_host_register(h, a.ctypes.data, a.nbytes), "register")
            arrs.append(a)
        k, nxt, stop, err = p.DecodePcapAt(cap, info, 24, m, big)
        assert k == m and err is None and stop == NP.STOP_LIMIT
        assert_same(big, want, None, ext=False)
    finally:
        for a in arrs:
            lib.gpd_host_unregister(h, a.ctypes.data)


def test_record_form_equals_soa():
    """gpd_result.records (one 32-B gpd_record per packet) carries exactly the five SoA words,
    through the fast kernel, its fallback list and the generic decoder (ext records), with
    hdr_off beside it; a result naming both forms is refused."""
    import ctypes as C
    import torch
    from gopacket_amd import parser as P
    from gopacket_amd._lib import GPD_ERR_INVALID, GpdResult, lib
    batches = [PacketBatch.from_packets(_golden_packets() * 3),
               PacketBatch.from_packets(_mutations(seed=37, per_packet=40)),
               synth.make_udp64(1 << 13), synth.make_imix(1 << 13), synth.make_vxlan(1 << 12),
               synth.make_traffic_mix(1 << 13)]
    for b in batches:
        p = _parser()
        db = P.DeviceBatch(b, 0)
        for ext in (False, True):
            soa = P.DeviceResult(b.n, 0, ext=ext, hdr_off=True)
            aos = P.DeviceResult(b.n, 0, ext=ext, hdr_off=True, records=True)
            p.decode_device(db, soa)
            p.decode_device(db, aos)
            torch.cuda.synchronize()
            x, y = soa.to_host(), aos.to_host()
            for f in ("status", "layers", "net_hash", "tp_hash", "csum", "hdr_off"):
                assert np.array_equal(getattr(x, f), getattr(y, f)), (f, ext)
            if ext:
                assert np.array_equal(x.ext, y.ext)
    soa, aos = P.DeviceResult(4, 0), P.DeviceResult(4, 0, records=True)
    r = soa.c_result()
    r.records = aos.records.data_ptr()
    db = P.DeviceBatch(synth.make_udp64(4), 0)
    rc = lib.gpd_decode(_parser().ctx().h, C.byref(db.c_batch()), C.byref(r), None)
    assert rc == GPD_ERR_INVALID


@pytest.mark.parametrize("ho", [0, 1, 2])
def test_long_frame_mutations_both_ways(ho):
    """Long frames (a header-once batch: 8 KiB windows, tiles spanning several) with their
    headers fuzzed — EtherType and tags, IPv4 version/IHL/length/flags/protocol, TCP data
    offset and option bytes (the Timestamps shortcut's pattern among them), UDP length — and
    cut at random lengths, mixed among intact IMIX frames, against the oracle with
    header-once forced off, per window and per round."""
    rng = np.random.default_rng(41 + ho)
    base = synth.make_imix(1 << 12)
    n = base.n
    data = base.data.copy()
    offs, lens = base.offset.astype(np.int64), base.caplen.astype(np.int64).copy()
    hot = (12, 13, 14, 15, 16, 17, 18, 19, 20, 21, 24, 25, 27, 28, 31, 50, 51, 58, 59, 60, 61, 62, 63, 64, 65)
    for i in rng.choice(n, size=n // 2, replace=False):
        o = int(offs[i])
        for _ in range(int(rng.integers(1, 4))):
            k = int(rng.choice(hot)) if rng.random() < 0.8 else int(rng.integers(0, min(128, lens[i])))
            if k < lens[i]:
                data[o + k] = rng.integers(0, 256)
        if rng.random() < 0.2:
            lens[i] = int(rng.integers(0, lens[i] + 1))
        if rng.random() < 0.1 and lens[i] >= 70:  # NOP NOP Timestamps on a 32-B TCP header
            data[o + 18 + 20 + 12] = 0x80
            data[o + 58:o + 62] = (1, 1, 8, 10)
    b = PacketBatch(data, base.data_len, base.offset.copy(), lens.astype(np.uint32))
    t = dict(window_bytes=8192, header_once=ho)
    run_both(b, ext=False, tuning=t)
    run_both(b, L.LayerTypeEthernet, 0x3FF, ext=False, tuning=t)


@pytest.mark.parametrize("ho", [0, 1, 2])
def test_llc_frames_in_every_kernel(ho):
    """802.3 length framing among long frames: Length below, at and above the captured payload,
    0..4 bytes of LLC, SNAP / STP / other SAP pairs, one- and two-byte control fields
    (ethernet.go:53-58, llc.go:31-69) — the header-once tile decode takes these frames itself
    (gpd_kernels.hip fast_decode<HO>, the et0 < 0x0600 exit), the windowed kernels leave them to
    the generic decoder; with LLC registered and not, against the oracle."""
    rng = np.random.default_rng(77 + ho)
    base = synth.make_imix(1 << 12)
    n = base.n
    data = base.data.copy()
    offs, lens = base.offset.astype(np.int64), base.caplen.astype(np.int64).copy()
    saps = ((0xAA, 0xAA), (0x42, 0x42), (0xAB, 0xAA), (0x43, 0x43), (0xF0, 0xF0), (0x06, 0x07))
    for i in rng.choice(n, size=n // 3, replace=False):
        o = int(offs[i])
        pl = int(lens[i]) - 14
        r = rng.random()
        if r < 0.3:
            ln = pl  # Length = the payload
        elif r < 0.5:
            ln = int(rng.integers(0, 5))  # 0..4 bytes of LLC
        elif r < 0.75:
            ln = int(rng.integers(0, max(pl, 1)))  # Ethernet padding trimmed
        else:
            ln = int(rng.integers(pl, 0x600))  # longer than captured: truncated
        ln = min(ln, 0x5FF)
        data[o + 12:o + 14] = (ln >> 8, ln & 0xFF)
        d, sp = saps[int(rng.integers(0, len(saps)))]
        data[o + 14:o + 17] = (d, sp, int(rng.choice([0x03, 0x00, 0x01, 0xF3, 0x02, 0x05])))
        if rng.random() < 0.15:
            lens[i] = int(rng.integers(12, min(lens[i], 40) + 1))  # cut inside the LLC header
    b = PacketBatch(data, base.data_len, base.offset.copy(), lens.astype(np.uint32))
    t = dict(window_bytes=8192, header_once=ho)
    run_both(b, ext=False, tuning=t)
    run_both(b, L.LayerTypeEthernet, 0x3FF, ext=False, tuning=t)
