"""Deterministic synthetic packet batches for the BASELINE.json configurations.

  config 2  make_udp64(n)   64 B Eth/IPv4/UDP, seed 0x5EED0002
  config 3  make_imix(n)    IMIX 64/576/1500 (7:4:1) Eth/Dot1Q/IPv4/TCP, seed 0x5EED0003
  config 4  make_vxlan(n)   128 B Eth/IPv4/UDP:4789/VXLAN/Eth/IPv4/TCP, seed 0x5EED0004
  (north star) make_tcp64(n) 64 B Eth/IPv4/TCP, seed 0x5EED0008

Random fields come from a vectorised splitmix64 stream; ports avoid every key of
the reference's port tables (layers/ports.go:62-122) so the transport's next layer
is Payload.  Checksums are valid except for 1 packet in 64, whose checksum is
corrupted on purpose (IPv4 header for config 2, TCP for configs 3 and 4).
"""
from __future__ import annotations

import numpy as np

from .batch import PAD, PacketBatch
from .layers import TABLES

_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)
_GOLD = np.uint64(0x9E3779B97F4A7C15)


def splitmix64(seed: int, n: int, stream: int = 0, base: int = 0) -> np.ndarray:
    """Outputs base+1 .. base+n of splitmix64 stream `stream` (state seed + stream*2^40)."""
    with np.errstate(over="ignore"):
        idx = np.arange(base + 1, base + n + 1, dtype=np.uint64) + \
            np.uint64((stream << 40) & 0xFFFFFFFFFFFFFFFF)
        z = np.uint64(seed & 0xFFFFFFFFFFFFFFFF) + idx * _GOLD
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
        return z ^ (z >> np.uint64(31))


def _free_ports(table: np.ndarray) -> np.ndarray:
    p = np.arange(1024, 65536, dtype=np.int64)
    return p[table[p] == 0]


def _pick(values: np.ndarray, r: np.ndarray) -> np.ndarray:
    return values[(r % np.uint64(len(values))).astype(np.int64)]


def _be16(a: np.ndarray, col: int, v: np.ndarray) -> None:
    a[:, col] = (v >> 8) & 0xFF
    a[:, col + 1] = v & 0xFF


def _be32(a: np.ndarray, col: int, v: np.ndarray) -> None:
    v = v.astype(np.uint64)
    for k in range(4):
        a[:, col + k] = ((v >> np.uint64(24 - 8 * k)) & np.uint64(0xFF)).astype(np.uint8)


def _sum16(a: np.ndarray) -> np.ndarray:
    """Sum of big-endian 16-bit words of each row (odd length: last byte << 8)."""
    a = a.astype(np.uint64)
    if a.shape[1] % 2:
        a = np.concatenate([a, np.zeros((a.shape[0], 1), np.uint64)], axis=1)
    return ((a[:, 0::2] << np.uint64(8)) | a[:, 1::2]).sum(axis=1)


def _fold_not(s: np.ndarray) -> np.ndarray:
    s = s.astype(np.uint64)
    s = s & np.uint64(0xFFFFFFFF)  # the reference accumulates in uint32
    while np.any(s > 0xFFFF):
        s = np.where(s > 0xFFFF, (s >> np.uint64(16)) + (s & np.uint64(0xFFFF)), s)
    return (~s.astype(np.uint16)).astype(np.uint16)


def _ip4_header(a: np.ndarray, c: int, length: np.ndarray, ident: np.ndarray, ttl: np.ndarray,
                proto: int, src: np.ndarray, dst: np.ndarray) -> None:
    a[:, c] = 0x45
    a[:, c + 1] = 0
    _be16(a, c + 2, length)
    _be16(a, c + 4, ident)
    a[:, c + 6] = 0x40  # DF
    a[:, c + 7] = 0
    a[:, c + 8] = ttl
    a[:, c + 9] = proto
    a[:, c + 10:c + 12] = 0
    _be32(a, c + 12, src)
    _be32(a, c + 16, dst)
    cs = _fold_not(_sum16(a[:, c:c + 20]))
    _be16(a, c + 10, cs)


def _l4_checksum(a: np.ndarray, ip: int, l4: int, seg_len: int, proto: int, col: int) -> None:
    """Valid TCP/UDP checksum (tcpip.go:26-88) for rows whose segment is a[:, l4:l4+seg_len]."""
    a[:, l4 + col:l4 + col + 2] = 0
    s = _sum16(a[:, ip + 12:ip + 20]) + np.uint64(proto) + np.uint64(seg_len & 0xFFFF) + \
        np.uint64(seg_len >> 16) + _sum16(a[:, l4:l4 + seg_len])
    _be16(a, l4 + col, _fold_not(s))


def _corrupt(a: np.ndarray, rows: np.ndarray, col: int) -> None:
    a[rows, col] ^= 0x5A


def _rand_bytes(seed: int, stream: int, n: int, width: int, base: int = 0) -> np.ndarray:
    """(n, width) random bytes from splitmix64 stream `stream` (rows base .. base+n)."""
    w = (width + 7) // 8
    return splitmix64(seed, n * w, stream, base * w).view(np.uint8).reshape(n, w * 8)[:, :width]


def _udp64_rows(a: np.ndarray, seed: int, base: int, free: np.ndarray) -> None:
    n = a.shape[0]
    r = [splitmix64(seed, n, k, base) for k in range(4)]
    a[:, 0:12] = _rand_bytes(seed, 100, n, 12, base) & 0xFE  # unicast MACs
    _be16(a, 12, np.full(n, 0x0800))
    src = (r[1] & np.uint64(0xFFFFFFFF)).astype(np.uint64)
    dst = (r[1] >> np.uint64(32)).astype(np.uint64)
    ident = (r[2] & np.uint64(0xFFFF)).astype(np.int64)
    ttl = ((r[2] >> np.uint64(16)) & np.uint64(0xFF)).astype(np.uint8) | 1
    _ip4_header(a, 14, np.full(n, 50), ident, ttl, 17, src, dst)
    _be16(a, 34, _pick(free, r[3]))
    _be16(a, 36, _pick(free, r[3] >> np.uint64(32)))
    _be16(a, 38, np.full(n, 30))
    a[:, 42:64] = _rand_bytes(seed, 101, n, 22, base)
    _l4_checksum(a, 14, 34, 30, 17, 6)
    bad = np.nonzero(((np.arange(n) + base) % 64) == 63)[0]
    _corrupt(a, bad, 24)  # IPv4 header checksum byte


def host_threads() -> int:
    """Threads for host-side generation: the cores this process may use (affinity, capped by a
    cgroup v2 quota, at most 16), shared by the node's ranks (LOCAL_WORLD_SIZE)."""
    import os
    try:
        nt = len(os.sched_getaffinity(0))
    except AttributeError:
        nt = os.cpu_count() or 1
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            nt = min(nt, max(1, -(-int(q) // int(per))))
    except (OSError, ValueError):
        pass
    return max(1, min(16, nt) // max(1, int(os.environ.get("LOCAL_WORLD_SIZE", "1"))))


def _parallel(jobs) -> None:
    """Run independent chunk jobs on a thread pool: numpy's kernels release the GIL, and every
    chunk's bytes depend only on (seed, stream, packet index), so the result is the same bytes
    whatever the order."""
    from concurrent.futures import ThreadPoolExecutor
    nt = max(1, min(host_threads(), len(jobs)))
    if nt == 1:
        for j in jobs:
            j()
        return
    with ThreadPoolExecutor(nt) as ex:
        for f in [ex.submit(j) for j in jobs]:
            f.result()


def _fixed_rows(n: int, size: int, fill, chunk: int) -> PacketBatch:
    """n frames of `size` bytes back to back; fill(rows, base) writes rows base .. base+len."""
    data = np.zeros(n * size + PAD, dtype=np.uint8)
    rows = data[: n * size].reshape(n, size)

    def job(c0):
        def run():
            a = np.zeros((min(chunk, n - c0), size), dtype=np.uint8)
            fill(a, c0)
            rows[c0:c0 + a.shape[0]] = a
        return run
    _parallel([job(c0) for c0 in range(0, n, chunk)])
    return PacketBatch(data, n * size, (np.arange(n, dtype=np.uint64) * size).astype(np.uint32),
                       np.full(n, size, dtype=np.uint32))


def make_udp64(n: int, seed: int = 0x5EED0002, chunk: int = 1 << 18) -> PacketBatch:
    """Config 2: 64 B Eth/IPv4/UDP (IHL 5, Length 50, UDP Length 30)."""
    free = _free_ports(TABLES.udp_port)
    return _fixed_rows(n, 64, lambda a, base: _udp64_rows(a, seed, base, free), chunk)


_native = None


def _native_lib():
    """gopacket_amd/libgpd_synth.so (csrc/synth/gpd_synth.c): make_udp64's bytes, natively."""
    global _native
    if _native is None:
        import ctypes as C
        import os
        path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libgpd_synth.so")
        if not os.path.exists(path):
            from .build import build_synth
            build_synth()
        L = C.CDLL(path)
        L.gpds_udp64.restype = None
        L.gpds_udp64.argtypes = [C.c_void_p, C.c_uint64, C.c_uint64, C.c_uint64, C.c_void_p,
                                 C.c_uint32, C.c_int, C.c_int]
        _native = L
    return _native


def udp64_native(dst: np.ndarray, lo: int, hi: int, seed: int = 0x5EED0002, records: bool = False,
                 nthreads: int = 16) -> None:
    """Packets [lo, hi) of make_udp64(seed) into dst (a uint8 array or a view of one): 64 B back
    to back, or as pcap records (16-B header {i // 10^6, i % 10^6, 64, 64} + 64 B, the framing
    of pcap.synth_capture) when `records`."""
    need = (hi - lo) * (80 if records else 64)
    if dst.dtype != np.uint8 or dst.size < need or not dst.flags.c_contiguous:
        raise ValueError("udp64_native: dst must be a contiguous uint8 array of the records' size")
    free = _free_ports(TABLES.udp_port).astype(np.uint16)
    _native_lib().gpds_udp64(dst.ctypes.data, lo, hi, seed & 0xFFFFFFFFFFFFFFFF, free.ctypes.data,
                             len(free), int(bool(records)), int(nthreads))


IMIX_SIZES = (64, 576, 1500)
IMIX_WEIGHTS = (7, 4, 1)


def _tcp_frames(n: int, size: int, r: list, opts: np.ndarray, vlan: bool, free: np.ndarray,
                bad: np.ndarray, seed: int, stream: int, base: int = 0) -> np.ndarray:
    """n Eth(/Dot1Q)/IPv4/TCP frames of `size` bytes; rows in `opts` carry NOP,NOP,TS."""
    a = np.zeros((n, size), dtype=np.uint8)
    a[:, 0:12] = _rand_bytes(seed, stream, n, 12, base) & 0xFE
    c = 12
    if vlan:
        _be16(a, 12, np.full(n, 0x8100))
        _be16(a, 14, (r[5] & np.uint64(0x0FFF)).astype(np.int64))
        c = 16
    _be16(a, c, np.full(n, 0x0800))
    ip = c + 2
    l4 = ip + 20
    seg = size - l4
    src = (r[1] & np.uint64(0xFFFFFFFF)).astype(np.uint64)
    dst = (r[1] >> np.uint64(32)).astype(np.uint64)
    ident = (r[2] & np.uint64(0xFFFF)).astype(np.int64)
    ttl = ((r[2] >> np.uint64(16)) & np.uint64(0xFF)).astype(np.uint8) | 1
    _ip4_header(a, ip, np.full(n, size - ip), ident, ttl, 6, src, dst)
    _be16(a, l4, _pick(free, r[3]))
    _be16(a, l4 + 2, _pick(free, r[3] >> np.uint64(32)))
    _be32(a, l4 + 4, r[4] & np.uint64(0xFFFFFFFF))
    _be32(a, l4 + 8, r[4] >> np.uint64(32))
    a[:, l4 + 12] = 0x50
    a[:, l4 + 13] = 0x10 | (((r[2] >> np.uint64(24)) & np.uint64(1)).astype(np.uint8) << 3)  # ACK(+PSH)
    _be16(a, l4 + 14, ((r[2] >> np.uint64(32)) & np.uint64(0xFFFF)).astype(np.int64))
    if seg > 20:
        body = _rand_bytes(seed, stream + 1, n, seg - 20, base)
        a[:, l4 + 20:] = body
    if len(opts):
        a[opts, l4 + 12] = 0x80
        a[opts, l4 + 20] = 1
        a[opts, l4 + 21] = 1
        a[opts, l4 + 22] = 8
        a[opts, l4 + 23] = 10
    _l4_checksum(a, ip, l4, seg, 6, 16)
    _corrupt(a, bad, l4 + 16)
    return a


def make_imix(n: int, seed: int = 0x5EED0003, vlan: bool = True, align: int = 16,
              chunk: int = 16384) -> PacketBatch:
    """Config 3: IMIX 64/576/1500 B (7:4:1), Eth/Dot1Q/IPv4/TCP, seeded shuffle.

    3 in 10 of the 576/1500 B packets (1/8 of all) carry NOP,NOP,Timestamp options
    (doff 8); a 64 B frame has no room for them.  Packet starts are `align`-aligned.
    """
    wsum = sum(IMIX_WEIGHTS)
    cls = np.repeat(np.arange(3), [n * w // wsum for w in IMIX_WEIGHTS])
    cls = np.concatenate([cls, np.zeros(n - len(cls), dtype=cls.dtype)])
    perm = np.argsort(splitmix64(seed, n, 99), kind="stable")
    cls = cls[perm]
    sizes = np.array(IMIX_SIZES, dtype=np.int64)[cls]
    slot = (sizes + align - 1) // align * align
    offs = np.zeros(n, dtype=np.int64)
    if n > 1:
        np.cumsum(slot[:-1], out=offs[1:])
    total = int(offs[-1] + sizes[-1]) if n else 0
    data = np.zeros(total + PAD, dtype=np.uint8)
    free = _free_ports(TABLES.tcp_port)
    gidx = np.arange(n)
    bad_all = (gidx % 64) == 63
    ropt = splitmix64(seed, n, 98)
    opt_all = (cls > 0) & ((ropt % np.uint64(10)) < np.uint64(3))
    def job(k, size, rows, c0):
        def run():
            m = len(rows)
            r = [splitmix64(seed + c0, m, 16 * k + j) for j in range(6)]
            opts = np.nonzero(opt_all[rows])[0]
            bad = np.nonzero(bad_all[rows])[0]
            frames = _tcp_frames(m, size, r, opts, vlan, free, bad, seed + c0, 200 + 2 * k)
            idx = offs[rows][:, None] + np.arange(size)[None, :]
            data[idx.reshape(-1)] = frames.reshape(-1)
        return run
    jobs = []
    for k, size in enumerate(IMIX_SIZES):
        rows_all = np.nonzero(cls == k)[0]
        jobs += [job(k, size, rows_all[c0:c0 + chunk], c0) for c0 in range(0, len(rows_all), chunk)]
    _parallel(jobs)
    return PacketBatch(data, total, offs.astype(np.uint32), sizes.astype(np.uint32))


def _vxlan_rows(a: np.ndarray, seed: int, base: int, free_u: np.ndarray, free_t: np.ndarray) -> None:
    n = a.shape[0]
    r = [splitmix64(seed, n, k, base) for k in range(10)]
    a[:, 0:12] = _rand_bytes(seed, 100, n, 12, base) & 0xFE
    _be16(a, 12, np.full(n, 0x0800))
    _ip4_header(a, 14, np.full(n, 114), (r[1] & np.uint64(0xFFFF)).astype(np.int64),
                np.full(n, 64, np.uint8), 17, (r[2] & np.uint64(0xFFFFFFFF)),
                (r[2] >> np.uint64(32)))
    _be16(a, 34, _pick(free_u, r[3]))
    _be16(a, 36, np.full(n, 4789))
    _be16(a, 38, np.full(n, 94))
    a[:, 42] = 0x08  # VXLAN I flag
    _be32(a, 46, (r[4] & np.uint64(0xFFFFFF)) << np.uint64(8))
    a[:, 50:62] = _rand_bytes(seed, 101, n, 12, base) & 0xFE
    _be16(a, 62, np.full(n, 0x0800))
    ttl = ((r[6] >> np.uint64(16)) & np.uint64(0xFF)).astype(np.uint8) | 1
    _ip4_header(a, 64, np.full(n, 64), (r[6] & np.uint64(0xFFFF)).astype(np.int64), ttl, 6,
                (r[7] & np.uint64(0xFFFFFFFF)), (r[7] >> np.uint64(32)))
    _be16(a, 84, _pick(free_t, r[8]))
    _be16(a, 86, _pick(free_t, r[8] >> np.uint64(32)))
    _be32(a, 88, r[9] & np.uint64(0xFFFFFFFF))
    _be32(a, 92, r[9] >> np.uint64(32))
    a[:, 96] = 0x50
    a[:, 97] = 0x18
    _be16(a, 98, np.full(n, 0x2000))
    a[:, 104:128] = _rand_bytes(seed, 102, n, 24, base)
    _l4_checksum(a, 64, 84, 44, 6, 16)
    # outer UDP checksum 0 ("not computed"), as VXLAN encapsulators commonly send
    bad = np.nonzero(((np.arange(n) + base) % 64) == 63)[0]
    _corrupt(a, bad, 84 + 16)


def make_vxlan(n: int, seed: int = 0x5EED0004, chunk: int = 1 << 17) -> PacketBatch:
    """Config 4: 128 B Eth/IPv4/UDP(4789)/VXLAN/Eth/IPv4/TCP (104 B of headers + 24 B payload)."""
    free_u, free_t = _free_ports(TABLES.udp_port), _free_ports(TABLES.tcp_port)
    return _fixed_rows(n, 128, lambda a, base: _vxlan_rows(a, seed, base, free_u, free_t), chunk)


def make_tcp64(n: int, seed: int = 0x5EED0008, chunk: int = 1 << 18) -> PacketBatch:
    """The north star's literal target: 64 B Eth/IPv4/TCP frames (IHL 5, a 20-B TCP header with
    ACK(+PSH), 10 payload bytes), seed 0x5EED0008; valid checksums except the TCP checksum of 1
    packet in 64.  Not one of BASELINE.json's configs: config 2 is the same size over UDP."""
    free = _free_ports(TABLES.tcp_port)

    def fill(a, base):
        m = a.shape[0]
        r = [splitmix64(seed, m, j, base) for j in range(6)]
        bad = np.nonzero(((np.arange(m) + base) % 64) == 63)[0]
        a[:] = _tcp_frames(m, 64, r, np.zeros(0, np.int64), False, free, bad, seed, 400, base)
    return _fixed_rows(n, 64, fill, chunk)


# ---- a traffic mix with the rarer stacks and the generic decoder's share -------------------
# (class, frame bytes, weight in 100): what the fast kernel decodes itself, then what it leaves
# to the generic decoder (IPv4 options, fragments, IPv6 hop-by-hop, a TCP header cut short)
MIX_CLASSES = (("tcp64", 64, 30), ("tcp576", 576, 15), ("tcp1500", 1500, 8), ("udp64", 64, 20),
               ("vxlan", 128, 5), ("icmp4", 98, 5), ("tcp6", 86, 5), ("stp", 60, 1),
               ("ip4opt", 68, 4), ("frag", 64, 3), ("ip6hbh", 90, 2), ("tcpcut", 64, 2))
MIX_FALLBACK = ("stp", "ip4opt", "ip6hbh", "tcpcut")  # (IPv4 fragments: the fast path, r03)


def _mix_class(name: str, m: int, seed: int, free_t, free_u) -> np.ndarray:
    """m frames of one traffic-mix class (rows of the class's frame size)."""
    r = [splitmix64(seed, m, k) for k in range(8)]
    if name.startswith("tcp") and name != "tcp6" and name != "tcpcut":
        return _tcp_frames(m, int(name[3:]), r, np.zeros(0, np.int64), False, free_t,
                           np.nonzero((np.arange(m) % 64) == 63)[0], seed, 300)
    if name == "tcpcut":  # a 64-B TCP frame captured to 50 B: the header is cut (tcp.go:264-265)
        return _tcp_frames(m, 64, r, np.zeros(0, np.int64), False, free_t, np.zeros(0, np.int64),
                           seed, 302)
    if name in ("udp64", "frag", "ip4opt"):
        a = np.zeros((m, 64), np.uint8)
        _udp64_rows(a, seed, 0, free_u)
        if name == "frag":  # More Fragments set: next layer Fragment (ip4.go:281-286)
            a[:, 20] = 0x20
            a[:, 24:26] = 0
            _be16(a, 24, _fold_not(_sum16(a[:, 14:34])))
            return a
        if name == "ip4opt":  # IHL 6: Router Alert (RFC 2113), options walk (ip4.go:240-273)
            b = np.zeros((m, 68), np.uint8)
            b[:, :34] = a[:, :34]
            b[:, 34:38] = np.array([0x94, 0x04, 0, 0], np.uint8)
            b[:, 38:] = a[:, 34:]
            b[:, 14] = 0x46
            _be16(b, 16, np.full(m, 54))
            b[:, 24:26] = 0
            _be16(b, 24, _fold_not(_sum16(b[:, 14:38])))
            return b
        return a
    if name == "vxlan":
        return make_vxlan(m, seed).data[:m * 128].reshape(m, 128)
    if name == "icmp4":  # echo request with 56 bytes of data (icmp4.go:220-231)
        a = np.zeros((m, 98), np.uint8)
        a[:, 0:12] = _rand_bytes(seed, 110, m, 12) & 0xFE
        _be16(a, 12, np.full(m, 0x0800))
        _ip4_header(a, 14, np.full(m, 84), (r[1] & np.uint64(0xFFFF)).astype(np.int64),
                    np.full(m, 64, np.uint8), 1, r[2] & np.uint64(0xFFFFFFFF), r[2] >> np.uint64(32))
        a[:, 34] = 8
        _be16(a, 38, (r[3] & np.uint64(0xFFFF)).astype(np.int64))
        _be16(a, 40, ((r[3] >> np.uint64(16)) & np.uint64(0xFFFF)).astype(np.int64))
        a[:, 42:98] = _rand_bytes(seed, 111, m, 56)
        _be16(a, 36, _fold_not(_sum16(a[:, 34:98])))
        return a
    if name in ("tcp6", "ip6hbh"):
        size = 86 if name == "tcp6" else 90
        a = np.zeros((m, size), np.uint8)
        a[:, 0:12] = _rand_bytes(seed, 112, m, 12) & 0xFE
        _be16(a, 12, np.full(m, 0x86DD))
        a[:, 14] = 0x60
        a[:, 21] = 64
        a[:, 22:54] = _rand_bytes(seed, 113, m, 32)
        if name == "tcp6":  # IPv6 / TCP, 12 bytes of payload
            _be16(a, 18, np.full(m, 32))
            a[:, 20] = 6
            _be16(a, 54, _pick(free_t, r[4]))
            _be16(a, 56, _pick(free_t, r[4] >> np.uint64(32)))
            a[:, 66] = 0x50
            a[:, 67] = 0x18
            _be16(a, 68, np.full(m, 0x2000))
            a[:, 74:86] = _rand_bytes(seed, 114, m, 12)
            a[:, 70:72] = 0
            s = _sum16(a[:, 22:54]) + np.uint64(6) + np.uint64(32) + _sum16(a[:, 54:86])
            _be16(a, 70, _fold_not(s))
            return a
        # IPv6 / hop-by-hop (Router Alert for MLD) / ICMPv6: HBH parsed inside IPv6 (ip6.go:509-526)
        _be16(a, 18, np.full(m, 36))
        a[:, 20] = 0
        a[:, 54:62] = np.array([58, 0, 5, 2, 0, 0, 1, 0], np.uint8)
        a[:, 62] = 143
        a[:, 66:90] = _rand_bytes(seed, 115, m, 24)
        return a
    if name == "stp":  # 802.3 length 38, LLC 42/42/03, a spanning-tree BPDU (llc.go:31-69)
        a = np.zeros((m, 60), np.uint8)
        a[:, 0:6] = np.array([0x01, 0x80, 0xC2, 0, 0, 0], np.uint8)
        a[:, 6:12] = _rand_bytes(seed, 116, m, 6) & 0xFE
        _be16(a, 12, np.full(m, 38))
        a[:, 14:17] = np.array([0x42, 0x42, 0x03], np.uint8)
        a[:, 17:52] = _rand_bytes(seed, 117, m, 35)
        return a
    raise ValueError(name)


def make_traffic_mix(n: int, seed: int = 0x5EED0007, align: int = 16) -> PacketBatch:
    """A seeded mix of MIX_CLASSES by weight, shuffled: TCP 64/576/1500, UDP 64, VXLAN, ICMPv4
    echo, IPv6/TCP and IPv4 fragments that the fast kernel decodes, plus 802.3/LLC frames, IPv4
    options, IPv6 hop-by-hop and cut TCP headers (MIX_FALLBACK, 9 %) that it leaves to the
    generic decoder.  Checksums are valid except 1 in 64 TCP frames."""
    wsum = sum(w for _, _, w in MIX_CLASSES)
    counts = [n * w // wsum for _, _, w in MIX_CLASSES]
    counts[0] += n - sum(counts)
    cls = np.repeat(np.arange(len(MIX_CLASSES)), counts)
    cls = cls[np.argsort(splitmix64(seed, n, 97), kind="stable")]
    sizes = np.array([sz for _, sz, _ in MIX_CLASSES], np.int64)[cls]
    slot = (sizes + align - 1) // align * align
    offs = np.zeros(n, np.int64)
    if n > 1:
        np.cumsum(slot[:-1], out=offs[1:])
    total = int(offs[-1] + sizes[-1]) if n else 0
    data = np.zeros(total + PAD, np.uint8)
    free_t, free_u = _free_ports(TABLES.tcp_port), _free_ports(TABLES.udp_port)
    caplen = sizes.copy()
    for k, (name, size, _) in enumerate(MIX_CLASSES):
        rows = np.nonzero(cls == k)[0]
        if not len(rows):
            continue
        frames = _mix_class(name, len(rows), seed + 1000 * (k + 1), free_t, free_u)
        idx = offs[rows][:, None] + np.arange(size)[None, :]
        data[idx.reshape(-1)] = frames.reshape(-1)
        if name == "tcpcut":
            caplen[rows] = 50
    return PacketBatch(data, total, offs.astype(np.uint32), caplen.astype(np.uint32))


def make_mixed(n: int, seed: int = 0x5EED0005) -> PacketBatch:
    """A mixed batch (the three configurations interleaved) for parity tests."""
    parts = [make_udp64(n // 3 + 1, seed), make_imix(n // 3 + 1, seed + 1), make_vxlan(n // 3 + 1, seed + 2)]
    pkts = []
    for k in range(n):
        b = parts[k % 3]
        pkts.append(b.packet(k // 3))
    return PacketBatch.from_packets(pkts)


# ---- TPACKET_V3 rings (linux/if_packet.h layouts) for the AF_PACKET ingest -------------
TPV3_BLOCK_DESC = 48      # sizeof(struct tpacket_block_desc)
TPV3_HDR = 48             # sizeof(struct tpacket3_hdr)
TPV3_HDRLEN = 48 + 20     # TPACKET_ALIGN(sizeof(tpacket3_hdr)) + sizeof(struct sockaddr_ll)
TP_STATUS_USER, TP_STATUS_VLAN_VALID = 1, 16


def _align16(x: int) -> int:
    return (x + 15) & ~15


def make_tpv3_ring(packets, block_size: int = 1 << 16, num_blocks: int = 8, first_block: int = 0,
                   vlan=None, next_offset_zero_every: int = 3, ifindex: int = 7, seed: int = 0x5EED0006,
                   empty_blocks=(), kernel_blocks=(), wire_extra: int = 0):
    """A TPACKET_V3 ring as the kernel fills it (net/packet/af_packet.c layout): packets are
    placed block by block from `first_block` on (wrapping); each frame sits at the kernel's
    tp_mac (TPACKET_ALIGN(TPACKET3_HDRLEN + 16) - 14 for Ethernet); every
    `next_offset_zero_every`-th packet leaves tp_next_offset 0 (the reader then steps by
    tpAlign(snaplen + mac), afpacket/header.go:181-195).  `vlan`: per-packet (tci, valid) or
    None.  Walk positions (0 = first_block) in `empty_blocks` are handed over with no
    packets; those in `kernel_blocks`, and every block after the packets ran out, stay owned
    by the kernel.
    Returns (ring u8[num_blocks * block_size], blocks_used in ring order)."""
    ring = np.zeros(num_blocks * block_size, np.uint8)
    rng = np.random.default_rng(seed)
    mac = _align16(TPV3_HDRLEN + 16) - 14
    empty, kernel = set(empty_blocks), set(kernel_blocks)  # walk positions (0 = first_block)
    k, used = 0, []
    blk_i = 0
    while k < len(packets) or any(e >= blk_i for e in empty):
        if blk_i >= num_blocks:
            raise ValueError("packets do not fit the ring")
        b = (first_block + blk_i) % num_blocks
        base = b * block_size
        pos = _align16(TPV3_BLOCK_DESC)
        first, n_in, prev = pos, 0, None
        if blk_i not in empty:
            while k < len(packets):
                p = packets[k]
                need = _align16(mac + len(p))
                if pos + need > block_size:
                    break
                h = base + pos
                sec, nsec = 1_700_000_000 + k, int(rng.integers(0, 10**9))
                tci, valid = vlan[k] if vlan is not None else (0, False)
                hdr = np.zeros(TPV3_HDR, np.uint8)
                hdr[4:8] = np.frombuffer(np.uint32(sec).tobytes(), np.uint8)
                hdr[8:12] = np.frombuffer(np.uint32(nsec).tobytes(), np.uint8)
                hdr[12:16] = np.frombuffer(np.uint32(len(p)).tobytes(), np.uint8)
                hdr[16:20] = np.frombuffer(np.uint32(len(p) + wire_extra).tobytes(), np.uint8)
                st = TP_STATUS_USER | (TP_STATUS_VLAN_VALID if valid else 0)
                hdr[20:24] = np.frombuffer(np.uint32(st).tobytes(), np.uint8)
                hdr[24:26] = np.frombuffer(np.uint16(mac).tobytes(), np.uint8)
                hdr[26:28] = np.frombuffer(np.uint16(mac + 14).tobytes(), np.uint8)
                hdr[32:36] = np.frombuffer(np.uint32(tci).tobytes(), np.uint8)
                ring[h:h + TPV3_HDR] = hdr
                ring[h + 48 + 4:h + 48 + 8] = np.frombuffer(np.int32(ifindex).tobytes(), np.uint8)
                ring[h + mac:h + mac + len(p)] = np.frombuffer(p, np.uint8)
                if prev is not None:  # the previous packet's tp_next_offset
                    nxt = 0 if (k - 1) % next_offset_zero_every == 0 else pos - prev
                    ring[base + prev:base + prev + 4] = np.frombuffer(np.uint32(nxt).tobytes(), np.uint8)
                prev = pos
                pos += need
                n_in += 1
                k += 1
        bd = np.zeros(TPV3_BLOCK_DESC, np.uint8)
        bd[0:4] = np.frombuffer(np.uint32(3).tobytes(), np.uint8)  # TPACKET_V3
        own = blk_i not in kernel
        bd[8:12] = np.frombuffer(np.uint32(TP_STATUS_USER if own else 0).tobytes(), np.uint8)
        bd[12:16] = np.frombuffer(np.uint32(n_in).tobytes(), np.uint8)
        bd[16:20] = np.frombuffer(np.uint32(first).tobytes(), np.uint8)
        bd[20:24] = np.frombuffer(np.uint32(pos).tobytes(), np.uint8)
        bd[24:32] = np.frombuffer(np.uint64(blk_i + 1).tobytes(), np.uint8)
        ring[base:base + TPV3_BLOCK_DESC] = bd
        used.append(b)
        blk_i += 1
    return ring, used
