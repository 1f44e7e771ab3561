#!/usr/bin/env python3
"""Benchmark: device-resident batched DecodingLayerParser decode + checksums + flow hashes.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config udp64|tcp64|imix|vxlan|pcap64|replay]

One step = one pass of the fused decode over one resident batch (default: BASELINE.json
configs[1], 2^24 synthetic 64 B Eth/IPv4/UDP packets per GPU).  `--gpus N` with N > 1 starts
N ranks (one per GPU) through torch.distributed.run as a child process, before anything
touches a GPU; under a launcher WORLD_SIZE must equal --gpus.  Every rank decodes its own shard
by packet index (no data-path collective: packets are independent units); the barriers and
the max-over-ranks timing use RCCL.

`--config replay` is BASELINE config 5: ONE seeded pcap capture of 10^9 x 64 B records in host
memory (shared by the node's ranks), cut by packet index into shards [g*N/G, (g+1)*N/G) with
gpd_pcap_locate; each rank decodes its shard device-resident (the metric) and streamed from
host memory in 2^24-record calls of gpd_decode_pcap_at (PCIe-inclusive, reported beside it).

Rank 0 prints one JSON line with `value` in Mpackets/s (whole job), a `roofline` object for
the decode kernel (algorithmic HBM bytes per launch — packet bytes and descriptors read,
result records written — over the mean launch time measured with HIP events on the launch
stream) and a `cpu_baseline` object (the C restatement of gopacket's DLP in oracle/ on
BASELINE.md's config-1 workload, one thread and all of this host's cores).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
DESC_BYTES = 8         # u32 offset + u32 caplen per packet

CONFIGS = {
    "udp64": ("config2: 2^24 x 64 B Eth/IPv4/UDP, fixed-format header extract + IPv4 header "
              "checksum (+UDP checksum, flow hashes), synthetic seed 0x5EED0002", 1 << 24),
    "imix": ("config3: 2^22 IMIX 64/576/1500 B (7:4:1) Eth/Dot1Q/IPv4/TCP, TCP checksum + "
             "5-tuple flow hashes, synthetic seed 0x5EED0003", 1 << 22),
    "vxlan": ("config4: 2^23 x 128 B Eth/IPv4/UDP/VXLAN/Eth/IPv4/TCP, inner flow keys, "
              "synthetic seed 0x5EED0004", 1 << 23),
    "mixed": ("traffic mix (not a BASELINE config): 2^22 frames of TCP 64/576/1500, UDP 64, VXLAN, "
              "ICMPv4 echo, IPv6/TCP (fast kernel) and 802.3/LLC/STP, IPv4 options, fragments, "
              "IPv6 hop-by-hop, cut TCP headers (12 %, generic decoder); every decoder registered, "
              "synthetic seed 0x5EED0007", 1 << 22),
    "tcp64": ("north-star target (not a BASELINE config): 2^24 x 64 B Eth/IPv4/TCP, IPv4 header "
              "checksum + TCP pseudo-header checksum + 5-tuple flow hashes, synthetic seed 0x5EED0008",
              1 << 24),
    "pcap64": ("config5 (per GPU): a pcap capture of 2^24 x 64 B Eth/IPv4/UDP records decoded in "
               "place (the capture bytes are the batch buffer: 16-B record headers interleaved), "
               "records indexed by the native pcap walker; synthetic seed 0x5EED0002", 1 << 24),
}


def make_batch(config: str, n: int, rank: int):
    from gopacket_amd import synth
    seed_off = rank * 0x1000
    if config == "udp64":
        return synth.make_udp64(n, 0x5EED0002 + seed_off)
    if config == "imix":
        return synth.make_imix(n, 0x5EED0003 + seed_off)
    if config == "tcp64":
        return synth.make_tcp64(n, 0x5EED0008 + seed_off)
    if config == "mixed":
        return synth.make_traffic_mix(n, 0x5EED0007 + seed_off)
    if config == "pcap64":
        from gopacket_amd import pcap as NP
        return NP.synth_capture(synth.make_udp64(n, 0x5EED0002 + seed_off))
    return synth.make_vxlan(n, 0x5EED0004 + seed_off)


CONFIG1_DECODERS = ("Ethernet", "Dot1Q", "IPv4", "IPv6", "TCP", "UDP", "Payload")


def host_cores():
    """CPUs this process may run on (its affinity mask), and the machine's count beside it."""
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    quota = None
    try:  # a cgroup v2 CPU quota caps the usable cores below the affinity mask
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = round(int(q) / int(per), 2)
    except (OSError, ValueError):
        pass
    return aff, os.cpu_count() or 1, quota


def rank_threads(args) -> int:
    """Host threads for this rank's host work (capture generation, record walks): --threads,
    else the cores this process may use (affinity, capped by a cgroup quota) shared by the
    node's ranks (LOCAL_WORLD_SIZE), at least 1."""
    if args.threads:
        return args.threads
    aff, _, quota = host_cores()
    cores = min(aff, max(1, int(-(-quota // 1)))) if quota else aff
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", os.environ.get("WORLD_SIZE", "1")))
    return max(1, min(64, cores) // max(1, local_world))


def _time_oracle(batch, decoders, threads, budget_s, out):
    import oracle_ref as O
    O.decode(batch, decoders=decoders, ext=False, nthreads=threads, out=out)  # warm
    done, t0 = 0, time.perf_counter()
    while True:
        O.decode(batch, decoders=decoders, ext=False, nthreads=threads, out=out)
        done += batch.n
        el = time.perf_counter() - t0
        if el >= budget_s:
            return done / el / 1e6, done, el


def cpu_baseline(config_batch=None, budget_s: float = 5.0):
    """the C restatement of gopacket's DecodingLayerParser (oracle/, test
    infrastructure) with the reference benchmark's decoder set {Ethernet, Dot1Q, IPv4, IPv6,
    TCP, UDP, Payload} (pcap/gopacket_benchmark/benchmark.go:216-218), the IPv4 header
    checksum, TCP ComputeChecksum and both FastHashes per packet, over config 1:
    pcap/test_ethernet.pcap looped 10^6 times (10^7 decodes) — on one thread and on every core
    this process may use (one decoder per thread).  The same all-core work over a sample of
    the metric's own packets is reported beside it."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from gopacket_amd import parser as P
    from gopacket_amd import pcap as NP
    from gopacket_amd.batch import PacketBatch
    from gopacket_amd.results import BatchResult
    aff, machine, quota = host_cores()
    threads = min(aff, max(1, int(-(-quota // 1)))) if quota else aff  # the cores we may use
    dec = P.decoder_mask(CONFIG1_DECODERS)
    pc = NP.read_pcap(os.path.join(ROOT, "tests", "golden", "test_ethernet.pcap"))
    loops = 1000000
    b = PacketBatch(pc.batch.data, pc.batch.data_len, np.tile(pc.batch.offset, loops),
                    np.tile(pc.batch.caplen, loops))
    z = lambda dt: np.zeros(b.n, dt)
    out = BatchResult(z(np.uint32), z(np.uint64), z(np.uint64), z(np.uint64), z(np.uint32), None,
                      z(np.uint32))
    one, _, _ = _time_oracle(b, dec, 1, budget_s, out)
    allc, _, _ = _time_oracle(b, dec, threads, budget_s, out)
    res = {"value": round(allc, 3), "unit": "Mpackets/s", "cores": threads, "kind": "port",
           "sample": f"config 1: test_ethernet.pcap (10 Eth/IPv4/TCP packets) looped {loops}x = "
                     f"{b.n} decodes per pass, timed >= {budget_s:.0f} s per row; C restatement "
                     f"of gopacket DecodingLayerParser ({'/'.join(CONFIG1_DECODERS)}) + IPv4 header "
                     f"checksum + TCP ComputeChecksum + net/transport FastHash, one decoder per "
                     f"thread, {threads} threads (all cores this process may use: affinity "
                     f"{aff} CPUs, cgroup quota {quota} CPUs)",
           "single_core": {"value": round(one, 3), "unit": "Mpackets/s", "cores": 1},
           "host_cpus": machine, "cgroup_cpu_quota": quota,
           "implementation": "C restatement of gopacket DecodingLayerParser (oracle/gpd_oracle.c), "
                             "not gopacket itself (no Go toolchain on this box)"}
    if config_batch is not None:
        m = min(config_batch.n, 1 << 21)
        sb = PacketBatch(config_batch.data, config_batch.data_len, config_batch.offset[:m].copy(),
                         config_batch.caplen[:m].copy())
        zz = lambda dt: np.zeros(m, dt)
        o2 = BatchResult(zz(np.uint32), zz(np.uint64), zz(np.uint64), zz(np.uint64), zz(np.uint32),
                         None, zz(np.uint32))
        r2, _, _ = _time_oracle(sb, 0x3FF, threads, budget_s, o2)
        res["same_workload_all_cores"] = {"value": round(r2, 3), "unit": "Mpackets/s",
                                          "cores": threads, "packets": m,
                                          "decoders": "the GPU parser's set"}
    return res


def load_traffic(config: str):
    """HBM bytes per launch of the decode kernel from the newest committed rocprofv3 summary
    (profiles/rNN/<config>/summary.json, written by tools/prof_summary.py from separate
    FETCH_SIZE / WRITE_SIZE passes with the gfx950 x2 FETCH_SIZE correction)."""
    import glob
    paths = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", config, "summary.json")))
    if not paths:
        return None
    try:
        s = json.load(open(paths[-1]))
    except (OSError, ValueError):
        return None
    k = [v for n, v in s.get("kernels", {}).items() if "decode_kernel" in n or "rs_kernel" in n or "ro_kernel" in n or "sp_kernel" in n]
    return {"read": s.get("hbm_read_bytes_per_launch"), "write": s.get("hbm_write_bytes_per_launch"),
            "kernel_us": k[0]["avg_us"] if k else None,
            "source": os.path.relpath(paths[-1], ROOT)}


COMM_DEVICE = None  # where collective operands live: the rank's GPU (nccl) or "cpu" (gloo)


def dist_max(values, dist, device):
    """Max over ranks of a few floats (identity without torch.distributed)."""
    if not dist:
        return [float(v) for v in values]
    import torch
    t = torch.tensor([float(v) for v in values], dtype=torch.float64, device=COMM_DEVICE or device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return [float(v) for v in t.cpu()]


def summarize(workload, n, world, steps, warmup, elapsed, kern_ms, kern_ms_max, batch, n_err,
              interleaved=0):
    """The contract JSON object: `value` = packets all ranks decoded / max-over-ranks time.
    `interleaved`: bytes per packet the windows stream besides the packet (pcap record headers)."""
    total_pkts = n * world * steps
    value = total_pkts / elapsed / 1e6
    read_bytes = int(batch.caplen.astype(np.int64).sum()) + (DESC_BYTES + interleaved) * n
    write_bytes = 4 + 8 + 8 + 8 + 4  # status, layers, net_hash, tp_hash, csum per packet
    alg_bytes = read_bytes + write_bytes * n  # every byte the launch must move through HBM
    achieved = alg_bytes / (kern_ms * 1e-3) / 1e9
    return {
        "metric": "Mpackets/s device-resident Eth/IP/TCP decode+cksum+flow-hash; GB/s vs HBM peak",
        "value": round(value, 2),
        "unit": "Mpackets/s",
        "n_gpus": world,
        "steps": steps,
        "warmup": warmup,
        "ms_per_step": round(elapsed / steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic",
        "config": {"workload": workload, "packets_per_gpu": n, "parallelism": f"shard{world}",
                   "read_bytes_per_packet": round(read_bytes / n, 2),
                   "result_bytes_per_packet": write_bytes,
                   "decode_errors_in_batch": n_err},
        # achieved = algorithmic HBM bytes of one launch (packet bytes + descriptors read,
        # 32-B result records written) / the launch time on its stream.
        # read_frac is the north-star "HBM-read roofline" (reads only) beside it.
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None,
                     "kernel_ms": round(kern_ms, 4), "kernel_ms_max_rank": round(kern_ms_max, 4),
                     "algorithmic_bytes_per_launch": alg_bytes,
                     "algorithmic_read_bytes": read_bytes,
                     "algorithmic_write_bytes": write_bytes * n,
                     "read_frac": round(read_bytes / (kern_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)},
    }


def bench_record36(parser, dev_batch, n, local, stream, out, args, records=False, soa=False, hdr=None):
    """The same launch writing the 36-B record: the five SoA arrays (or, records=True, one
    gpd_record per packet) plus hdr_off (the NetworkFlow / TransportFlow header offsets the F3
    flow table reads).  Event-timed like the metric.  soa=True / records=True without hdr: the
    32-B record as the five SoA arrays / as gpd_records."""
    import torch
    from gopacket_amd import parser as P
    if hdr is None:
        hdr = not (records or soa)
    res = P.DeviceResult(n, local, ext=False, hdr_off=hdr, records=records)
    # the clocks drop while the host works between lines: settle again (as for the metric)
    settle(lambda: parser.decode_device(dev_batch, res, stream), min(args.settle_ms, 150.0), local)
    k = max(5, min(args.steps, 20))
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(k)]
    for a, b in ev:
        a.record(stream)
        parser.decode_device(dev_batch, res, stream)
        b.record(stream)
    torch.cuda.synchronize(local)
    ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    rb = out["roofline"]["algorithmic_read_bytes"]
    wb = 36 if hdr else 32
    alg = rb + wb * n
    del res
    return {"result_bytes_per_packet": wb, "kernel_ms": round(ms, 4),
            "Mpackets_per_s": round(n / ms / 1e3, 1),
            "frac": round(alg / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "read_frac": round(rb / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}


def attainable(n: int, read_bytes: int, local: int, achieved_gbps: float, soa: bool = False):
    """The streaming ceiling for this launch's traffic shape on this box (libgpd_probe.so): the
    same read bytes per 64-packet tile as one contiguous run and the same 32 B of results per
    packet in the same form as the launch (two 16-B record stores per lane, or the five SoA
    arrays), no decode, no packet boundaries, after its own clock settle.  `frac` of the decode is
    read against peak; `of_attainable` against this.  An SoA line carries the
    record-form probe beside it (`record_form_probe`).  None without the probe."""
    import ctypes as C
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "gopacket_amd", "libgpd_probe.so")
    if not os.path.exists(path):
        return None
    lib = C.CDLL(path)
    lib.gpd_probe_stream2.argtypes = [C.c_int, C.c_uint32, C.c_uint32, C.c_int, C.c_float, C.c_int,
                                      C.POINTER(C.c_float)]
    ntiles = (n + 63) // 64
    per_tile = -(-read_bytes // ntiles)

    def probe(form_soa):
        ms = C.c_float(0.0)
        rc = lib.gpd_probe_stream2(local, ntiles, per_tile, 20, 150.0, int(form_soa), C.byref(ms))
        if rc != 0 or ms.value <= 0:
            return None, rc
        return (ntiles * per_tile + ntiles * 2048) / (ms.value * 1e-3) / 1e9, ms.value

    gbps, ms = probe(soa)
    if gbps is None:
        return {"error": f"gpd_probe_stream2 rc={ms}"}
    out = {"GBps": round(gbps, 1), "frac_of_peak": round(gbps / HBM_PEAK_GBS, 4),
           "of_attainable": round(achieved_gbps / gbps, 4), "probe_ms": round(ms, 4),
           "read_bytes_per_tile": per_tile, "write_bytes_per_tile": 2048,
           "result_form": "SoA arrays" if soa else "gpd_record",
           "probe": "gpd_probe_stream2: contiguous 16-B-per-lane nt loads of each tile's read bytes + "
                    + ("the five SoA result arrays (u32, u64, u64, u64, u32) as nt stores"
                       if soa else "two 16-B nt record stores per lane")
                    + ", no decode (2 and 4 workgroups per CU, best)"}
    if soa:  # the record-form probe too, for comparison with earlier rounds' lines
        g2, ms2 = probe(False)
        if g2 is not None:
            out["record_form_probe"] = {"GBps": round(g2, 1), "probe_ms": round(ms2, 4),
                                        "of_attainable": round(achieved_gbps / g2, 4)}
    # the read-only leg: the same loads with no stores — the measured ceiling the north star's
    # "HBM-read roofline" target is judged against
    g3, ms3 = probe(2)
    if g3 is not None:
        rg = ntiles * per_tile / (ms3 * 1e-3) / 1e9
        ach_read = achieved_gbps * read_bytes / (read_bytes + n * 32)  # the launch's read share
        out["read_only"] = {"GBps": round(rg, 1), "frac_of_peak": round(rg / HBM_PEAK_GBS, 4),
                            "probe_ms": round(ms3, 4), "achieved_read_GBps": round(ach_read, 1),
                            "of_read_ceiling": round(ach_read / rg, 4),
                            "probe": "gpd_probe_stream2(soa=2): the same 16-B-per-lane nt loads, no stores"}
    return out


SIDE_CONFIGS = ("tcp64", "imix", "vxlan", "pcap64")  # timed beside the default line (N = 1)


def bench_side(config, parser, args, local, stream):
    """Another configuration on this GPU, timed the way the metric is: its own resident batch,
    clock settle, warmup, then event-timed launches on the launch stream (result form as
    records_form chooses for it).  Reported in the default line beside `value` so the driver's
    run carries configs 3, 4 and 5 (per GPU) and the north star's 64-B TCP target."""
    import torch
    from gopacket_amd import parser as P
    workload, n = CONFIGS[config]
    t0 = time.perf_counter()
    batch = make_batch(config, n, 0)
    interleaved = 0
    if config == "pcap64":  # the capture bytes are the batch buffer (16-B record headers between)
        from gopacket_amd import pcap as NP
        pc = NP.index(batch, nthreads=rank_threads(args))
        assert pc.err is None and pc.batch.n == n, (pc.err, pc.batch.n)
        batch, interleaved = pc.batch, 16
    t_gen = time.perf_counter() - t0
    aos = config not in ("imix", "mixed")
    db = P.DeviceBatch(batch, local)
    dr = P.DeviceResult(n, local, ext=False, hdr_off=False, records=aos)
    settled = settle(lambda: parser.decode_device(db, dr, stream), args.settle_ms, local)
    for _ in range(args.warmup):
        parser.decode_device(db, dr, stream)
    k = max(10, min(args.steps, 20))
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(k)]
    torch.cuda.synchronize(local)
    for a, b in ev:
        a.record(stream)
        parser.decode_device(db, dr, stream)
        b.record(stream)
    torch.cuda.synchronize(local)
    ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    st = (dr.records.view(torch.int32)[0::8] if aos else dr.status).cpu().numpy().view(np.uint32)
    read = int(batch.caplen.astype(np.int64).sum()) + (DESC_BYTES + interleaved) * n
    write = 32 * n
    out = {"workload": workload, "packets": n, "result_form": "gpd_record (AoS)" if aos else "SoA arrays",
           "kernel_ms": round(ms, 4), "launches": k, "Mpackets_per_s": round(n / ms / 1e3, 1),
           "achieved_GBps": round((read + write) / (ms * 1e-3) / 1e9, 1),
           "frac": round((read + write) / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
           "read_frac": round(read / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
           "algorithmic_read_bytes": read, "algorithmic_write_bytes": write,
           "decode_errors_in_batch": int(np.count_nonzero((st & 3) != 0)),
           "settle_ms": settled, "generate_s": round(t_gen, 2)}
    if not args.no_probe:
        out["attainable"] = attainable(n, read, local, out["achieved_GBps"], soa=not aos)
    tr = load_traffic(config)
    if tr and tr["read"] and tr["write"]:
        out["traffic"] = int(tr["read"]) + int(tr["write"])
        out["traffic_source"] = tr["source"]
        out["profiled_kernel_us"] = tr["kernel_us"]
    del db, dr, batch
    torch.cuda.empty_cache()
    return out


def bench_host(parser, batch, n, mode, steps, warmup):
    """PCIe-inclusive rate of the same batch from host memory: gpd_decode_host (host batch ->
    pinned staging or, mode "registered", the caller's pinned arrays -> H2D -> decode -> D2H ->
    host results), wall clock over `steps` calls."""
    res = parser.DecodeBatchHost(batch)
    regd = []
    from gopacket_amd._lib import check, lib
    if mode == "registered":  # a capture loop pins its batch and result arrays once
        for a in (batch.data, batch.offset, batch.caplen, res.status, res.layers, res.net_hash,
                  res.tp_hash, res.csum, res.hdr_off):
            check(lib.gpd_host_register(parser.ctx().h, a.ctypes.data, a.nbytes), "register")
            regd.append(a)
    try:
        for _ in range(warmup):
            parser.DecodeBatchHost(batch, out=res)
        t0 = time.perf_counter()
        for _ in range(steps):
            parser.DecodeBatchHost(batch, out=res)
        el = time.perf_counter() - t0
    finally:
        for a in regd:
            lib.gpd_host_unregister(parser.ctx().h, a.ctypes.data)
    return {"Mpackets_per_s": round(n * steps / el / 1e6, 2), "ms_per_step": round(el / steps * 1e3, 3),
            "steps": steps, "host_arrays": mode, "host_bytes_in": int(batch.data_len) + 8 * n,
            "GBps_in": round((batch.data_len + 8 * n) * steps / el / 1e9, 2),
            "decode_errors_in_batch": int(np.count_nonzero((res.status & 3) != 0)),
            "path": "host batch + result arrays pinned once (gpd_host_register) -> gpd_decode_host: "
                    "chunked H2D, decode, D2H into the registered arrays; wall clock"}


def bench_split(parser, dev_batch, dev_res, n, local, stream):
    """gpd_last_launch_split: how many packets the fast decode left to the generic decoder
    (options, fragments, hop-by-hop, errors ...; each wave decodes its own list at its end, in
    the same kernel) and the event-timed kernel time (mean of 5); list_kernel_ms is what the
    launch spent after that kernel (~0 since the lists moved into it)."""
    import ctypes as C

    import torch
    from gopacket_amd._lib import check, lib
    h = parser.ctx().h
    check(lib.gpd_ctx_set_timing(h, 1), "gpd_ctx_set_timing")
    fb, fast, lst = C.c_uint64(), C.c_float(), C.c_float()
    rows = []
    try:
        for _ in range(5):
            parser.decode_device(dev_batch, dev_res, stream)
            check(lib.gpd_last_launch_split(h, C.byref(fb), C.byref(fast), C.byref(lst)),
                  "gpd_last_launch_split")
            rows.append((fb.value, fast.value, lst.value))
    finally:
        lib.gpd_ctx_set_timing(h, 0)
    torch.cuda.synchronize(local)
    return {"packets": int(rows[-1][0]), "fraction": round(rows[-1][0] / n, 5),
            "fast_kernel_ms": round(float(np.mean([r[1] for r in rows])), 4),
            "list_kernel_ms": round(float(np.mean([r[2] for r in rows])), 4)}


def bench_flows(parser, dev_batch, n, args, stream, local):
    """F3 diagnostic: decode (with header offsets) then find-or-create every packet's flow
    record in an empty table (gpd_flow_insert: insert + key-verify launches), timed with HIP
    events on the launch stream around the insert alone."""
    import torch
    from gopacket_amd import flows as FL
    from gopacket_amd import parser as P
    res = P.DeviceResult(n, local, ext=False, hdr_off=True)
    parser.decode_device(dev_batch, res, stream)
    cap = 1 << max(10, (2 * n - 1).bit_length())  # load factor <= 1/2
    ft = FL.NewFlowTable(parser, cap)
    fid = torch.empty(n, dtype=torch.int32, device=f"cuda:{local}")
    steps = max(3, min(args.steps, 10))
    ins, rst = [], []
    for k in range(steps + 1):
        e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        e[0].record(stream)
        ft.Reset(stream)
        e[1].record(stream)
        ft.Insert(dev_batch, res, fid, 0, stream)
        e[2].record(stream)
        torch.cuda.synchronize(local)
        if k:  # the first round is warm-up
            rst.append(e[0].elapsed_time(e[1]))
            ins.append(e[1].elapsed_time(e[2]))
    st = ft.Stats(stream)
    # the same packets again into the filled table: every packet finds an existing flow
    ex = []
    for k in range(steps):
        e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ft.Reset(stream)
        ft.Insert(dev_batch, res, fid, 0, stream)
        e[0].record(stream)
        ft.Insert(dev_batch, res, fid, n, stream)
        e[1].record(stream)
        torch.cuda.synchronize(local)
        ex.append(e[0].elapsed_time(e[1]))
    ms = float(np.mean(ins))
    out = {"diag": "F3 flow table (not the metric)", "packets": n, "insert_ms": round(ms, 4),
           "insert_Mpackets_per_s": round(n / ms / 1e3, 1), "reset_ms": round(float(np.mean(rst)), 4),
           "capacity": st["capacity"], "flows": st["flows"], "keyed_packets": st["packets"],
           "collisions": st["collisions"], "full": st["full"],
           "existing_flows": {"insert_ms": round(float(np.mean(ex)), 4),
                              "insert_Mpackets_per_s": round(n / float(np.mean(ex)) / 1e3, 1)}}
    # bursts: the same packets, each repeated 16 times back to back (descriptors only, the
    # bytes are shared), so a wave's lanes fold 16-packet runs before their atomics
    rep = 16
    bb = P.DeviceBatch.__new__(P.DeviceBatch)
    bb.n, bb.data_len, bb.data, bb.device = n, dev_batch.data_len, dev_batch.data, local
    bb.offset = dev_batch.offset[: n // rep].repeat_interleave(rep).contiguous()
    bb.caplen = dev_batch.caplen[: n // rep].repeat_interleave(rep).contiguous()
    bres = P.DeviceResult(n, local, ext=False, hdr_off=True)
    parser.decode_device(bb, bres, stream)
    bins = []
    for k in range(steps + 1):
        e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ft.Reset(stream)
        e[0].record(stream)
        ft.Insert(bb, bres, fid, 0, stream)
        e[1].record(stream)
        torch.cuda.synchronize(local)
        if k:
            bins.append(e[0].elapsed_time(e[1]))
    bst = ft.Stats(stream)
    bms = float(np.mean(bins))
    out["bursts16"] = {"insert_ms": round(bms, 4), "insert_Mpackets_per_s": round(n / bms / 1e3, 1),
                       "flows": bst["flows"], "keyed_packets": bst["packets"],
                       "collisions": bst["collisions"]}
    # the flow-affine sharded table (one table per rank, key records exchanged all-to-all):
    # host clock per phase, synchronised; with one rank the exchange is skipped
    sft = FL.ShardedFlowTable(parser, cap)
    rank = int(os.environ.get("RANK", "0"))
    phases = []
    for k in range(steps + 1):
        sft.table.Reset(stream)
        torch.cuda.synchronize(local)
        sft.Insert(dev_batch, res, index_base=rank * n, stream=stream)
        if k:
            phases.append(sft.last_ms)
    ph = {key: round(float(np.mean([p[key] for p in phases])), 4) for key in phases[0]}
    tot = sum(ph.values())
    out["sharded"] = {"ranks": sft.world, "phase_ms": ph, "total_ms": round(tot, 4),
                      "Mpackets_per_s_per_rank": round(n / tot / 1e3, 1),
                      "flows_on_rank": sft.Stats(stream)["flows"]}
    return out


def bench_tpv3(parser, batch, args):
    """F2 diagnostic: the config's first packets laid out as the kernel fills a TPACKET_V3
    ring (1 MiB blocks, 256 of them), host-registered like a pinned socket ring, then
    gpd_decode_tpv3 (H2D of the blocks, the block walk and the decode on the device, D2H of
    the results and capture info) timed on the host clock, with the result and capture-info
    arrays reused across calls and registered once, as a capture loop keeps them.
    PCIe-inclusive; never the metric."""
    from gopacket_amd import afpacket as A
    from gopacket_amd import synth
    from gopacket_amd._lib import check, lib
    bs, nb = 1 << 20, 256
    per = bs // (((82 + int(batch.caplen.max())) + 15) // 16 * 16) - 1
    m = min(batch.n, per * nb)
    arr, used = synth.make_tpv3_ring([batch.packet(i) for i in range(m)], bs, nb)
    ring = A.TPv3Ring(arr, bs, nb)
    check(lib.gpd_host_register(parser.ctx().h, arr.ctypes.data, arr.nbytes), "gpd_host_register")
    try:
        from gopacket_amd.results import BatchResult
        out = BatchResult(np.zeros(m, np.uint32), np.zeros(m, np.uint64), np.zeros(m, np.uint64),
                          np.zeros(m, np.uint64), np.zeros(m, np.uint32), None, np.zeros(m, np.uint32))
        cinfo = A.CaptureInfo.alloc(m)
        pinned = [out.status, out.layers, out.net_hash, out.tp_hash, out.csum, out.hdr_off, cinfo.offset,
                  cinfo.caplen, cinfo.length, cinfo.ts_ns, cinfo.ifindex, cinfo.vlan, cinfo.vlan_tci]
        for x in pinned:
            check(lib.gpd_host_register(parser.ctx().h, x.ctypes.data, x.nbytes), "gpd_host_register")
        parser.DecodeTPv3(ring, max_n=m, out=out, ci=cinfo)  # warm (and first touch)
        reps, t0 = 0, time.perf_counter()
        while True:
            res, ci, nblk = parser.DecodeTPv3(ring, max_n=m, out=out, ci=cinfo)
            reps += 1
            el = time.perf_counter() - t0
            if el > 3 or reps >= 20:
                break
        path = lib.gpd_decode_tpv3_last_path()
        for x in pinned:
            lib.gpd_host_unregister(parser.ctx().h, x.ctypes.data)
    finally:
        lib.gpd_host_unregister(parser.ctx().h, arr.ctypes.data)
    assert len(res) == m and nblk == len(used)
    return {"diag": "F2 TPACKET_V3 ring walk + decode (PCIe-inclusive, not the metric)",
            "packets": m, "blocks": nblk, "block_size": bs, "ring_bytes": int(arr.nbytes),
            "ms_per_ring": round(el / reps * 1e3, 3), "Mpackets_per_s": round(m * reps / el / 1e6, 1),
            "GBps_ring_in": round(len(used) * bs * reps / el / 1e9, 2),
            "walk": "device" if path == 1 else "host"}


def replay_pcap(parser, cap, n, total, threads):
    """PCIe-inclusive rate: the capture in (registered) host memory replayed through
    gpd_decode_pcap — native index, raw capture bytes H2D, decode, results D2H — until `total`
    packets were decoded.  Diagnostic beside the device-resident value, never `value`."""
    from gopacket_amd._lib import check, lib
    check(lib.gpd_host_register(parser.ctx().h, cap.ctypes.data, cap.nbytes), "gpd_host_register")
    try:
        from gopacket_amd.results import BatchResult
        # room for the most records the bytes could hold (the walk stays parallel without a
        # bound); only the entries the records fill are ever touched
        from gopacket_amd.batch import PAD
        m = (cap.shape[0] - PAD - 24) // 16 + 1
        out = BatchResult(np.zeros(m, np.uint32), np.zeros(m, np.uint64), np.zeros(m, np.uint64),
                          np.zeros(m, np.uint64), np.zeros(m, np.uint32), None, np.zeros(m, np.uint32))
        parser.DecodePcap(cap, nthreads=threads, out=out)  # warm: slots, streams, pages
        done, t0, reps = 0, time.perf_counter(), 0
        while done < total:
            res, k, err = parser.DecodePcap(cap, nthreads=threads, out=out)
            assert err is None and k == n
            done += k
            reps += 1
        el = time.perf_counter() - t0
    finally:
        lib.gpd_host_unregister(parser.ctx().h, cap.ctypes.data)
    return {"packets": done, "replays": reps, "s": round(el, 3),
            "Mpackets_per_s": round(done / el / 1e6, 1),
            "GBps_capture_in": round(reps * (cap.nbytes - 64) / el / 1e9, 2),
            "path": "registered host capture -> native index -> raw bytes H2D -> decode -> D2H"}


# ---------------------------------------------------------------- config 5: sharded pcap replay
REPLAY_CHUNK = 1 << 24   # records per device index chunk and per gpd_decode_pcap_at call
REPLAY_SEED = 0x5EED0002


def host_placement(arr, local: int) -> dict:
    """Where a large host buffer's pages sit (diagnostic of the PCIe-inclusive leg): its NUMA
    nodes (pages per node, /proc/self/numa_maps), how much of it transparent huge pages back
    (AnonHugePages, /proc/self/smaps) and the GPU's own NUMA node (sysfs, by PCI bus id)."""
    out = {}
    lo = arr.ctypes.data
    hi = lo + arr.nbytes
    try:
        nodes = {}
        with open("/proc/self/numa_maps") as f:
            for line in f:
                a = int(line.split()[0], 16)
                if lo - (1 << 21) <= a < hi:
                    for tok in line.split()[1:]:
                        if tok[0] == "N" and "=" in tok:
                            k, v = tok.split("=")
                            nodes[k] = nodes.get(k, 0) + int(v)
        out["numa_pages"] = nodes
    except (OSError, ValueError):
        pass
    try:
        huge, rss, cur = 0, 0, None
        with open("/proc/self/smaps") as f:
            for line in f:
                head = line.split()[0]
                if "-" in head and not head.endswith(":"):
                    a, b = (int(x, 16) for x in head.split("-"))
                    cur = a < hi and b > lo
                elif cur and head == "AnonHugePages:":
                    huge += int(line.split()[1])
                elif cur and head == "Rss:":
                    rss += int(line.split()[1])
        out["rss_kB"], out["anon_huge_kB"] = rss, huge
    except (OSError, ValueError):
        pass
    try:
        import torch
        pr = torch.cuda.get_device_properties(local)
        bus = f"{getattr(pr, 'pci_domain_id', 0):04x}:{pr.pci_bus_id:02x}:{pr.pci_device_id:02x}.0"
        out["gpu_pci"] = bus
        with open(f"/sys/bus/pci/devices/{bus}/numa_node") as f:
            out["gpu_numa_node"] = int(f.read().strip())
    except Exception:  # noqa: BLE001 (diagnostic only)
        pass
    return out


def shm_fits(nbytes: int) -> bool:
    st = os.statvfs("/dev/shm")
    return st.f_bavail * st.f_frsize >= nbytes


def capture_memory(args, nbytes: int, world: int, rank: int, dist, bcast_device) -> str:
    """Where the capture lives: "private" (one rank, or --capture-memory private, or /dev/shm
    too small for the whole capture on this node) or "shared" (one /dev/shm mapping for the
    node's ranks).  Rank 0 decides for all (one broadcast), so the ranks agree."""
    if world == 1:
        return "private"
    mode = args.capture_memory
    if mode == "auto":
        mode = "shared" if shm_fits(nbytes) else "private"
    if dist:
        import torch
        t = torch.tensor([1 if mode == "shared" else 0], dtype=torch.int64, device=bcast_device)
        dist.broadcast(t, 0)
        mode = "shared" if int(t.item()) else "private"
    return mode


def host_buffer(nbytes: int, shared: bool, local: int, key: str, dist):
    """The capture's host memory: private (anonymous) or one shared mapping for all the node's
    ranks (a /dev/shm file created by local rank 0).  Huge pages are asked for; returns
    (uint8 array, mmap object, path or None)."""
    import mmap
    path = None
    if not shared:
        mm = mmap.mmap(-1, nbytes)
    else:
        path = os.path.join("/dev/shm", f"gpd_replay_{key}")
        if local == 0:
            with open(path, "wb") as f:
                f.truncate(nbytes)
        dist.barrier()
        fd = os.open(path, os.O_RDWR)
        mm = mmap.mmap(fd, nbytes)
        os.close(fd)
    try:
        mm.madvise(mmap.MADV_HUGEPAGE)
    except (AttributeError, OSError):
        pass
    return np.frombuffer(mm, np.uint8), mm, path


def bind_local(arr, local: int) -> dict:
    """Put a host buffer's pages on the GPU's NUMA node before they are written
    (gpd_host_bind_local): the PCIe-inclusive leg streams the capture from there, not across
    the socket link (r04: a capture first-touched by the generator's threads lay 44 % on the
    far node, and the calls that read it ran 1.1-1.7x longer)."""
    import ctypes as C
    from gopacket_amd._lib import lib
    node = C.c_int(-1)
    rc = lib.gpd_host_bind_local(local, arr.ctypes.data, arr.nbytes, C.byref(node))
    out = {"node": node.value, "rc": rc}
    if rc:
        out["error"] = lib.gpd_last_error_string().decode()
    return out


PCAP_FILE_HEADER = (0xA1B2C3D4, 2, 4, 0, 0, 262144, 1)  # pcapgo framing: LE, microseconds


class ReplayCapture:
    """This rank's view of config 5's ONE seeded capture (pcapgo framing, LE microseconds,
    snaplen 262144): records i = 0..n-1 are config 2's packets (synth.make_udp64(seed
    0x5EED0002) packet i), each behind its 16-B record header.

    shared: the whole capture in one /dev/shm mapping; the ranks write disjoint record ranges
      in parallel (setup, untimed), and rank 0 finds the shard cuts by walking the records
      (gpd_pcap_locate) and broadcasts them.
    private (/dev/shm too small for the node, e.g. 80 GB for 10^9 records): each rank builds
      only its own shard [g*N/G, (g+1)*N/G) — the file header followed by exactly those records,
      byte-identical to that stretch of the whole capture — in private memory.  The cut is
      then where the shard's bytes start (the records are fixed 80-B synthetic records, so
      record g*N/G of the whole capture sits at 24 + 80*(g*N/G)); the rank still walks its
      own records for the chunk boundaries, and `base` maps its positions to the whole
      capture's.
    `cap` is the rank's buffer, [start, end) its shard's records in it."""

    def __init__(self, args, n: int, world: int, rank: int, local: int, dist, threads: int,
                 bcast_device, gpu=None):
        import struct
        from gopacket_amd import pcap as NP
        from gopacket_amd import synth
        from gopacket_amd.batch import PAD
        self.n = n
        key = f"{REPLAY_SEED:x}_{n}_{os.environ.get('MASTER_PORT', '0')}"
        lo, hi = NP.shard_bounds(n, world)[rank]
        self.mode = capture_memory(args, 24 + 80 * n + PAD, world, rank, dist, bcast_device)
        hdr = np.frombuffer(struct.pack("<IHHiIII", *PCAP_FILE_HEADER), np.uint8)
        if self.mode == "private":
            m = hi - lo
            cap, mm, _ = host_buffer(24 + 80 * m + PAD, False, local, key, dist)
            self.bind = bind_local(cap, gpu) if args.numa_bind and gpu is not None else None
            cap[:24] = hdr
            synth.udp64_native(cap[24:24 + 80 * m], lo, hi, REPLAY_SEED, records=True, nthreads=threads)
            cap[24 + 80 * m:] = 0
            self.cap, self.mm = cap, mm
            self.start, self.end, self.base = 24, 24 + 80 * m, 80 * lo
            self.data_len = 24 + 80 * m
            if dist:
                dist.barrier()
            return
        cap, mm, path = host_buffer(24 + 80 * n + PAD, True, local, key, dist)
        # this rank's records on its GPU's node (each rank writes and streams only its own)
        self.bind = (bind_local(cap[24 + 80 * lo:24 + 80 * hi], gpu) if args.numa_bind and gpu is not None
                     else None)
        try:
            if rank == 0:
                cap[:24] = hdr
            synth.udp64_native(cap[24 + 80 * lo:24 + 80 * hi], lo, hi, REPLAY_SEED, records=True,
                               nthreads=threads)
            cap[24 + 80 * n:] = 0
            dist.barrier()
        finally:  # every rank has mapped the file: its name is no longer needed
            if path and local == 0 and os.path.exists(path):
                os.unlink(path)
        self.cap, self.mm, self.base, self.data_len = cap, mm, 0, 24 + 80 * n
        bounds = NP.shard_bounds(n, world)
        if rank == 0:
            pos, total, stop = NP.locate(cap, [b for b, _ in bounds] + [n], data_len=self.data_len,
                                         nthreads=threads)
            assert total == n and stop == NP.STOP_EOF, (total, stop)
        else:
            pos = np.zeros(world + 1, np.uint64)
        import torch
        pt = torch.from_numpy(pos.view(np.int64).copy()).to(bcast_device)
        dist.broadcast(pt, 0)
        pos = pt.cpu().numpy().view(np.uint64)
        self.start, self.end = int(pos[rank]), int(pos[rank + 1])


class _Res:
    """Result SoA views (torch tensors, possibly slices of larger ones) as a gpd_result, or
    (records) a byte view of 32-B gpd_records."""

    def __init__(self, status=None, layers=None, net_hash=None, tp_hash=None, csum=None, records=None):
        self.status, self.layers, self.net_hash, self.tp_hash, self.csum = (
            status, layers, net_hash, tp_hash, csum)
        self.records = records

    def c_result(self):
        from gopacket_amd._lib import GpdResult
        if self.records is not None:
            return GpdResult(None, None, None, None, None, None, None, self.records.data_ptr())
        return GpdResult(self.status.data_ptr(), self.layers.data_ptr(), self.net_hash.data_ptr(),
                         self.tp_hash.data_ptr(), self.csum.data_ptr(), None, None)

    def fields(self, lo, hi):
        """Host copies of the five result words of packets [lo, hi)."""
        from gopacket_amd.results import RECORD_DTYPE
        if self.records is not None:
            r = self.records[32 * lo:32 * hi].cpu().numpy().view(RECORD_DTYPE)
            return {f: r[f].copy() for f in ("status", "layers", "net_hash", "tp_hash", "csum")}
        dt = {"status": np.uint32, "layers": np.uint64, "net_hash": np.uint64, "tp_hash": np.uint64,
              "csum": np.uint32}
        return {f: getattr(self, f)[lo:hi].cpu().numpy().view(d) for f, d in dt.items()}


def settle(fn, ms, local):
    """Run fn() (a launch of the timed step) untimed for >= ms of wall clock before the warmup
    steps.  The GPU's clocks ramp up under sustained load over tens of milliseconds: measured on
    one MI355X, config 2 ran at 0.354 ms per launch after 5 warmup launches and at 0.318-0.324 ms
    after 300 or 1000 (same box, alternating runs), so a handful of warmup launches would time
    the ramp rather than the steady state.  Returns the settle time spent (ms)."""
    import torch
    if ms <= 0:
        return 0.0
    t0 = time.perf_counter()
    while (time.perf_counter() - t0) * 1e3 < ms:
        for _ in range(8):
            fn()
        torch.cuda.synchronize(local)
    return round((time.perf_counter() - t0) * 1e3, 1)


def records_form(args) -> bool:
    """The result form the line is timed with: one 32-B gpd_record per packet (AoS) for configs
    2, 4 and 5, whose specs name no layout; the SoA arrays for IMIX (config 3 names "SoA
    outputs") and the traffic mix."""
    if args.result_form != "auto":
        return args.result_form == "aos"
    return args.config not in ("imix", "mixed")


def bench_replay(args, world, rank, local, dist):
    """BASELINE config 5 on this rank: locate the shard, decode it device-resident (timed steps),
    then stream it from host memory through gpd_decode_pcap_at (PCIe-inclusive)."""
    import ctypes as C

    import torch
    from gopacket_amd import layers as L
    from gopacket_amd import parser as P
    from gopacket_amd import pcap as NP
    from gopacket_amd._lib import GpdBatch, check, lib
    from gopacket_amd.results import BatchResult
    n = args.packets or 10 ** 9
    threads = rank_threads(args)
    dev = torch.device("cuda", local)
    t0 = time.perf_counter()
    host_local = int(os.environ.get("LOCAL_RANK", local))  # the host roles (--same-device keeps them)
    rc = ReplayCapture(args, n, world, rank, host_local, dist, threads, COMM_DEVICE or dev, gpu=local)
    cap, mm = rc.cap, rc.mm
    t_gen = time.perf_counter() - t0
    dl = rc.data_len
    info = NP.header(cap, dl)
    t0 = time.perf_counter()
    start, end = rc.start, rc.end
    bounds = NP.shard_bounds(n, world)
    lo, hi = bounds[rank]
    m = hi - lo
    chunks = [(c, min(c + REPLAY_CHUNK, m)) for c in range(0, m, REPLAY_CHUNK)]
    cpos, cn, _ = NP.locate(cap, [a for a, _ in chunks] + [m], pos=start, data_len=end, nthreads=threads)
    assert cn == m and int(cpos[-1]) == end
    t_locate = time.perf_counter() - t0
    layers = [P.Ethernet(), P.Dot1Q(), P.IPv4(), P.IPv6(), P.IPv6ExtensionSkipper(), P.TCP(),
              P.UDP(), P.VXLAN(), P.Payload(), P.Fragment()]
    if args.decoders == "novxlan":
        layers = [d for d in layers if not isinstance(d, P.VXLAN)]
    parser = P.NewDecodingLayerParser(L.LayerTypeEthernet, *layers, device=local)
    h = parser.ctx().h
    # pin the shard's pages (the H2D of both legs reads them in place)
    reg_lo, reg_hi = start & ~4095, min(len(cap), (end + 4095) & ~4095)
    t0 = time.perf_counter()
    registered = lib.gpd_host_register(h, cap[reg_lo:].ctypes.data, reg_hi - reg_lo) == 0
    t_reg = time.perf_counter() - t0
    # device-resident leg: the shard's bytes in HBM, indexed chunk by chunk
    base0 = start & ~15
    t0 = time.perf_counter()
    d_bytes = torch.empty(end - base0 + 64, dtype=torch.uint8, device=dev)
    step_b = 1 << 30
    for a in range(base0, end, step_b):
        b = min(end, a + step_b)
        d_bytes[a - base0:b - base0].copy_(torch.from_numpy(cap[a:b]))
    torch.cuda.synchronize(local)
    t_h2d = time.perf_counter() - t0
    t0 = time.perf_counter()
    d_off = torch.empty(m, dtype=torch.int32, device=dev)
    d_len = torch.empty(m, dtype=torch.int32, device=dev)
    aos = records_form(args)
    if aos:
        res = _Res(records=torch.empty(32 * m, dtype=torch.uint8, device=dev))
    else:
        res = _Res(torch.empty(m, dtype=torch.int32, device=dev), torch.empty(m, dtype=torch.int64, device=dev),
                   torch.empty(m, dtype=torch.int64, device=dev), torch.empty(m, dtype=torch.int64, device=dev),
                   torch.empty(m, dtype=torch.int32, device=dev))
    launches, read_bytes = [], 0
    for k, (a, b) in enumerate(chunks):
        hdr = int(cpos[k])
        base = hdr & ~15
        cend = int(cpos[k + 1])
        pc = NP.index(cap[base:], max_n=b - a, nthreads=threads, data_len=cend - base, pos=hdr - base,
                      info=info)
        assert pc.batch.n == b - a and pc.err is None
        d_off[a:b].copy_(torch.from_numpy(pc.batch.offset.view(np.int32)))
        d_len[a:b].copy_(torch.from_numpy(pc.batch.caplen.view(np.int32)))
        read_bytes += int(pc.batch.caplen.astype(np.int64).sum()) + (8 + 16) * (b - a)
        sl = slice(a, b)
        part = (_Res(records=res.records[32 * a:32 * b]) if aos else
                _Res(res.status[sl], res.layers[sl], res.net_hash[sl], res.tp_hash[sl], res.csum[sl]))
        launches.append((GpdBatch(d_bytes.data_ptr() + (base - base0), cend - base,
                                  d_off[sl].data_ptr(), d_len[sl].data_ptr(), b - a), part.c_result()))
    torch.cuda.synchronize(local)
    t_index = time.perf_counter() - t0
    stream = torch.cuda.current_stream(local)
    sp = C.c_void_p(stream.cuda_stream)

    def step():
        for b, r in launches:
            check(lib.gpd_decode(h, C.byref(b), C.byref(r), sp), "gpd_decode")

    settled = settle(step, args.settle_ms, local)
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(local)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(args.steps)]
    if dist:
        dist.barrier()
    torch.cuda.synchronize(local)
    t0 = time.perf_counter()
    for k in range(args.steps):
        ev[k][0].record(stream)
        step()
        ev[k][1].record(stream)
    torch.cuda.synchronize(local)
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kern_ms = float(np.mean([x.elapsed_time(y) for x, y in ev]))
    st = (res.records.view(torch.int32)[0::8] if aos else res.status).cpu().numpy().view(np.uint32)
    n_err = int(np.count_nonzero((st & 3) != 0))
    # PCIe-inclusive leg: the shard streamed from host memory in 2^24-record calls
    call = args.pcie_call_records or REPLAY_CHUNK  # records per gpd_decode_pcap_at call
    z = lambda dt: np.zeros(call, dt)
    out = BatchResult(z(np.uint32), z(np.uint64), z(np.uint64), z(np.uint64), z(np.uint32), None,
                      z(np.uint32))
    # a capture loop keeps its result arrays: registered, the results land in them by DMA
    outs = [out.status, out.layers, out.net_hash, out.tp_hash, out.csum, out.hdr_off]
    for a in outs:
        check(lib.gpd_host_register(h, a.ctypes.data, a.nbytes), "gpd_host_register")
    parser.DecodePcapAt(cap, info, start, min(call, m), out, threads, data_len=end)  # warm
    if dist:
        dist.barrier()
    # where the time of the PCIe-inclusive leg goes: each call's wall time and its phases
    # (gpd_decode_pcap_last_times: walk, staging, waits for the slots' transfers + decode, drain)
    call_ms, phases, call_ph = [], np.zeros(6, np.float64), []
    wc, walk_counts = np.zeros(7, np.uint32), np.zeros(7, np.int64)
    wm, misses = np.zeros(2, np.uint64), []
    ph = np.zeros(6, np.float64)
    t0 = time.perf_counter()
    p, done, last = start, 0, 0
    while done < m:
        tc = time.perf_counter()
        k, p, stop, err = parser.DecodePcapAt(cap, info, p, min(call, m - done), out, threads,
                                              data_len=end)
        call_ms.append((time.perf_counter() - tc) * 1e3)
        lib.gpd_decode_pcap_last_times(ph.ctypes.data)
        lib.gpd_decode_pcap_last_walk_counts(wc.ctypes.data)
        if wc[1] or wc[6]:
            lib.gpd_decode_pcap_last_walk_miss(wm.ctypes.data)
            misses.append([int(wm[0]), int(wm[1])])
        phases += ph
        walk_counts += wc
        call_ph.append(ph.copy())
        assert err is None and k > 0, err
        done += k
        last = k
    if dist:
        dist.barrier()
    t_pcie = time.perf_counter() - t0
    cm = np.array(call_ms)
    pcie_diag = {"calls": len(call_ms), "call_ms_median": round(float(np.median(cm)), 3),
                 "call_ms_min": round(float(cm.min()), 3), "call_ms_max": round(float(cm.max()), 3),
                 "call_ms_first4": [round(float(x), 3) for x in cm[:4]],
                 "call_ms_by_quarter": [round(float(q.mean()), 3) for q in np.array_split(cm, 4) if len(q)],
                 "phases_ms_total": dict(zip(["total", "walk", "walk_wait", "stage", "sync", "drain"],
                                             [round(float(x), 1) for x in phases])),
                 "capture_placement": host_placement(cap, local), "numa_bind": rc.bind}
    pcie_diag["device_walk_chunks"] = dict(zip(
        ["walked", "to_host", "speculation_refuted", "record_rejected", "header_uncovered", "walk_short",
         "segments_rewalked_on_device"],
        [int(x) for x in walk_counts]))
    pcie_diag["device_walk_misses"] = misses[:16]  # [start, segment] capture positions
    names = ["total", "walk", "walk_wait", "stage", "sync", "drain"]
    pcie_diag["slowest_calls"] = [
        {"call": int(j), "ms": round(float(cm[j]), 2),
         **{k: round(float(v), 2) for k, v in zip(names, call_ph[j])}}
        for j in np.argsort(cm)[::-1][:6]]
    pcie_diag["phases_ms_by_quarter"] = [
        {k: round(float(v), 1) for k, v in zip(names, np.sum(q, axis=0))}
        for q in np.array_split(np.array(call_ph), 4) if len(q)]
    # the streamed results of the last call equal the resident ones for the same records
    tail = res.fields(m - last, m)
    same = all(np.array_equal(getattr(out, f)[:last], tail[f])
               for f in ("status", "layers", "net_hash", "tp_hash", "csum"))
    for a in outs:
        lib.gpd_host_unregister(h, a.ctypes.data)
    if registered:
        lib.gpd_host_unregister(h, cap[reg_lo:].ctypes.data)
    # per-rank figures to rank 0
    mine = [elapsed, kern_ms, t_pcie, float(read_bytes), float(m), float(n_err), float(same),
            t_gen, t_locate, t_reg, t_h2d, t_index, float(registered)]
    rows = [mine]
    if dist:
        t = torch.tensor(mine, dtype=torch.float64, device=COMM_DEVICE or dev)
        g = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(g, t)
        rows = [list(x.cpu().numpy()) for x in g]
    del d_bytes, d_off, d_len, res, launches
    if rank != 0:
        return None
    el_max = max(r[0] for r in rows)
    kmax = max(r[1] for r in rows)
    pcie_max = max(r[2] for r in rows)
    write_per = 4 + 8 + 8 + 8 + 4
    rb0, m0 = rows[0][3], rows[0][4]
    alg0 = rb0 + write_per * m0
    per_rank = [{"rank": i, "packets": int(r[4]), "kernel_ms_per_step": round(r[1], 4),
                 "frac": round((r[3] + write_per * r[4]) / (r[1] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                 "read_frac": round(r[3] / (r[1] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                 "pcie_inclusive_s": round(r[2], 3), "decode_errors": int(r[5]),
                 "streamed_equals_resident": bool(r[6]), "registered": bool(r[12])}
                for i, r in enumerate(rows)]
    achieved = alg0 / (rows[0][1] * 1e-3) / 1e9
    out = {
        "metric": "Mpackets/s device-resident Eth/IP/TCP decode+cksum+flow-hash; GB/s vs HBM peak",
        "value": round(n * args.steps / el_max / 1e6, 2), "unit": "Mpackets/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(el_max / args.steps * 1e3, 4),
        "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "u8",
        "data": "synthetic",
        "config": {"workload": f"config5: one pcap capture of {n} x 64 B Eth/IPv4/UDP records "
                               f"(config 2 packets, seed 0x{REPLAY_SEED:X}) in host memory, sharded "
                               f"by packet index over {world} GPU(s) (gpd_pcap_locate), each shard "
                               f"resident in HBM and decoded in place in 2^24-record launches",
                   "packets_total": n, "parallelism": f"shard{world}", "chunk_records": REPLAY_CHUNK,
                   "capture_bytes": 24 + 80 * n,
                   "capture_memory": {"private": "private (each rank builds its own shard's records)",
                                      "shared": "/dev/shm (shared)"}[rc.mode],
                   "host_threads_per_rank": threads,
                   "read_bytes_per_packet": round(rb0 / m0, 2), "result_bytes_per_packet": write_per,
                   "result_form": "gpd_record (AoS)" if aos else "SoA arrays", "settle_ms": settled,
                   "decode_errors": int(sum(r[5] for r in rows))},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None,
                     "kernel_ms": round(rows[0][1] / len(chunks), 4),
                     "kernel_ms_max_rank": round(kmax / len(chunks), 4),
                     "launches_per_step": len(chunks),
                     "algorithmic_bytes_per_launch": int(alg0 / len(chunks)),
                     "read_frac": round(rb0 / (rows[0][1] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                     "read_frac_per_rank": [x["read_frac"] for x in per_rank]},
        "pcie_inclusive": {"Mpackets_per_s": round(n / pcie_max / 1e6, 1), "s": round(pcie_max, 3),
                           "GBps_capture_in": round(dl / pcie_max / 1e9, 2),
                           "records_per_call": call,
                           "path": "registered capture -> gpd_decode_pcap_at per call "
                                   "(raw bytes H2D in 64 MiB chunks, records found in HBM by the "
                                   "device walk, decode, results D2H into registered result "
                                   "arrays)"},
        "per_rank": per_rank,
        "pcie_diag_rank0": pcie_diag,
        "setup_s": {"generate": round(rows[0][7], 2), "locate": round(rows[0][8], 2),
                    "register": round(rows[0][9], 2), "h2d": round(rows[0][10], 2),
                    "index": round(rows[0][11], 2)},
    }
    return out


def shard_check(args, world, rank, local, dist):
    """CPU, gloo (tests/test_replay.py): the replay's cut without a GPU — the capture built as
    bench_replay builds it, shard g located and indexed chunk by chunk, its records' header
    positions written to <dir>/rank<g>.npz."""
    from gopacket_amd import pcap as NP
    n = args.packets or 10 ** 9
    threads = rank_threads(args)
    host_local = int(os.environ.get("LOCAL_RANK", local))  # the host roles (--same-device keeps them)
    rc = ReplayCapture(args, n, world, rank, host_local, dist, threads, "cpu")
    cap, mm = rc.cap, rc.mm
    info = NP.header(cap, rc.data_len)
    bounds = NP.shard_bounds(n, world)
    start, end = rc.start, rc.end
    lo, hi = bounds[rank]
    m = hi - lo
    chunk = args.chunk or REPLAY_CHUNK
    chunks = [(c, min(c + chunk, m)) for c in range(0, m, chunk)]
    cpos, cn, _ = NP.locate(cap, [a for a, _ in chunks] + [m], pos=start, data_len=end, nthreads=threads)
    hdrs = []
    for k, (a, b) in enumerate(chunks):
        hdr = int(cpos[k])
        base = hdr & ~15
        pc = NP.index(cap[base:], max_n=b - a, nthreads=threads, data_len=int(cpos[k + 1]) - base,
                      pos=hdr - base, info=info)
        assert pc.batch.n == b - a and pc.err is None
        hdrs.append(pc.batch.offset.astype(np.uint64) + base - 16 + rc.base)  # whole-capture positions
    np.savez(os.path.join(args.shard_check, f"rank{rank}.npz"), hdr=np.concatenate(hdrs) if hdrs else
             np.zeros(0, np.uint64), lo=lo, hi=hi, start=start + rc.base, end=end + rc.base, world=world,
             cn=cn, mode=rc.mode, threads=threads)
    if dist:
        dist.barrier()


def launch_ranks(n: int, argv) -> int:
    """`--gpus N` without a launcher: N ranks through torch.distributed.run, started as a child
    process (this process has not touched a GPU; it only waits and passes the exit code on)."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__), *argv]
    return subprocess.run(cmd).returncode


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs (ranks) on this node; N > 1 starts N ranks through "
                    "torch.distributed.run unless already under a launcher (default: WORLD_SIZE or 1)")
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="udp64", choices=sorted(CONFIGS) + ["replay"])
    ap.add_argument("--packets", type=int, default=0, help="override packets per GPU (replay: "
                    "records in the whole capture, default 10^9)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--pcie-call-records", type=int, default=0,
                    help="config 5 PCIe-inclusive leg: records per gpd_decode_pcap_at call (default 2^24)")
    ap.add_argument("--no-numa-bind", dest="numa_bind", action="store_false",
                    help="config 5: leave the capture's pages where first touch puts them instead of "
                    "on the GPU's NUMA node (gpd_host_bind_local)")
    ap.add_argument("--no-side", action="store_true", help="skip the other configurations' "
                    "figures (tcp64, imix, vxlan, pcap64) the default udp64 line carries")
    ap.add_argument("--cpu-budget", type=float, default=10.0, help="seconds of CPU-baseline timing "
                    "(split over its rows)")
    ap.add_argument("--host", nargs="?", const="plain", default="", choices=("plain", "registered"),
                    help="diagnostic: PCIe-inclusive rate through gpd_decode_host (host arrays in, "
                    "host arrays out; 'registered': pinned once, as a capture loop would); never "
                    "the reported metric")
    ap.add_argument("--threads", type=int, default=0, help="host threads for the pcap walker "
                    "(0 = all cores)")
    ap.add_argument("--replay", type=int, default=0, help="pcap64: also replay the capture from "
                    "host memory through gpd_decode_pcap until this many packets were decoded "
                    "(PCIe-inclusive rate; a diagnostic beside the device-resident value)")
    ap.add_argument("--flows", action="store_true",
                    help="diagnostic: also time the F3 flow table (gpd_flow_insert) on the decoded "
                    "batch; printed as a separate line, never the reported metric")
    ap.add_argument("--tpv3", action="store_true",
                    help="diagnostic: walk + decode a TPACKET_V3 ring of the config's packets "
                    "(gpd_decode_tpv3, PCIe-inclusive); printed as a separate line")
    ap.add_argument("--decoders", default="all", choices=("all", "novxlan"),
                    help="registered decoders: all of the engine's set, or without VXLAN")
    ap.add_argument("--settle-ms", type=float, default=250.0,
                    help="untimed launches before the warmup steps, for at least this long (GPU "
                         "clock ramp; 0: none)")
    ap.add_argument("--result-form", default="auto", choices=("auto", "soa", "aos"),
                    help="result form timed: auto = gpd_record (AoS) except for imix/mixed (SoA, as "
                         "config 3 specifies)")
    ap.add_argument("--ablate", default="", help="diagnostics only: 'nocsum', 'nohash' or both "
                    "(comma separated); never used for the reported metric")
    ap.add_argument("--events", default="span", choices=["step", "span"],
                    help="timed loop: one HIP event pair on the launch stream around all K launches "
                         "(default; the per-launch time is their span / K, gaps included) or a "
                         "pair around every launch (A/B: each timing event costs the step ~5 us)")
    ap.add_argument("--tune", default="", help="A/B only: engine tuning, e.g. 'shift=0' or "
                    "'window_bytes=8192,reg_prefix=1' (gpd_ctx_set_tuning; never changes results)")
    ap.add_argument("--shard-check", default="", help="tests only (CPU, gloo): build the replay "
                    "capture, cut and index this rank's shard, write its record positions to DIR")
    ap.add_argument("--chunk", type=int, default=0, help="tests only: records per index chunk")
    ap.add_argument("--capture-memory", default="auto", choices=("auto", "shared", "private"),
                    help="replay with N > 1: the whole capture in one /dev/shm mapping (shared) or "
                         "each rank's shard in private memory (private); auto = shared when "
                         "/dev/shm has room for the whole capture")
    ap.add_argument("--dist-backend", default="nccl", choices=("nccl", "gloo"),
                    help="tests only: gloo rehearses the N-rank path without RCCL")
    ap.add_argument("--same-device", action="store_true",
                    help="tests only: every rank on cuda:0 (the N-rank path on a one-GPU box, gloo)")
    ap.add_argument("--no-probe", action="store_true", help="skip the attainable-bandwidth probe "
                    "(roofline.attainable)")
    ap.add_argument("--lean", action="store_true", help="only the timed launches (profiling runs: "
                    "no 36-B record line, no fallback split, no CPU baseline)")
    args = ap.parse_args()
    if "nodecode" in args.ablate or "nowait" in args.ablate:
        # the stream-only ablations exist only in the diagnostic library (libgpd_diag.so,
        # -DGPD_DIAG); the shipped libgpd.so refuses their option bits
        os.environ["GPD_DIAGNOSTIC_LIBRARY"] = "1"

    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and (args.gpus or 1) > 1:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    world = int(env_world or "1")
    if args.gpus is not None and args.gpus != world:
        raise SystemExit(f"bench: --gpus {args.gpus} but the launcher started WORLD_SIZE={world} ranks")
    rank = int(os.environ.get("RANK", "0"))
    local = 0 if args.same_device else int(os.environ.get("LOCAL_RANK", "0"))
    if args.same_device and args.dist_backend != "gloo":
        raise SystemExit("bench: --same-device needs --dist-backend gloo (RCCL wants a GPU per rank)")

    import torch
    dist = None
    if args.shard_check:  # CPU only
        if world > 1:
            import torch.distributed as dist
            dist.init_process_group("gloo")
        shard_check(args, world, rank, local, dist)
        if dist:
            dist.destroy_process_group()
        return
    global COMM_DEVICE
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        if args.dist_backend == "gloo":
            dist.init_process_group("gloo")
            COMM_DEVICE = "cpu"
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(local)

    if args.config == "replay":
        out = bench_replay(args, world, rank, local, dist)
        if rank == 0:
            print(json.dumps(out), flush=True)
        if dist:
            dist.destroy_process_group()
        return

    from gopacket_amd import layers as L
    from gopacket_amd import parser as P

    workload, n_default = CONFIGS[args.config]
    n = args.packets or n_default
    batch = make_batch(args.config, n, rank)
    pcap_info = None
    if args.config == "pcap64":  # index the capture: its bytes become the batch buffer
        from gopacket_amd import pcap as NP
        cap = batch
        t0 = time.perf_counter()
        pc = NP.index(cap, nthreads=rank_threads(args))
        t_index = time.perf_counter() - t0
        assert pc.err is None and pc.batch.n == n, (pc.err, pc.batch.n)
        batch = pc.batch
        pcap_info = {"capture_bytes": int(batch.data_len), "index_s": round(t_index, 4),
                     "index_Mrec_per_s": round(n / t_index / 1e6, 1),
                     "index_threads": NP.last_walk_stats()[0]}
    dev_batch = P.DeviceBatch(batch, local)
    aos = records_form(args)  # the 32-B record: gpd_record per packet, or the five SoA arrays
    dev_res = P.DeviceResult(n, local, ext=False, hdr_off=False, records=aos)
    layers = [P.Ethernet(), P.Dot1Q(), P.IPv4(), P.IPv6(), P.IPv6ExtensionSkipper(), P.TCP(),
              P.UDP(), P.VXLAN(), P.Payload(), P.Fragment()]
    if args.decoders == "novxlan":
        layers = [d for d in layers if not isinstance(d, P.VXLAN)]
    parser = P.NewDecodingLayerParser(L.LayerTypeEthernet, *layers, device=local)
    if args.config == "mixed":  # the reference benchmark's set and more: ICMPv4 and LLC too
        parser.AddDecodingLayer(P.ICMPv4())
        parser.AddDecodingLayer(P.LLC())
    stream = torch.cuda.current_stream(local)
    if args.tune:
        parser.Tuning = {k: int(v) for k, v in (kv.split("=") for kv in args.tune.split(","))}
    if "nocsum" in args.ablate:
        parser.ComputeChecksums = False
    if "nohash" in args.ablate:
        parser.ComputeFlowHashes = False
    if "nodecode" in args.ablate:
        parser._diag_options = 1 << 31  # kernel streams the windows and skips decoding (diag lib)
    if "nowait" in args.ablate:
        parser._diag_options = 1 << 30  # kernel skips the per-tile DMA wait (wrong results; diag lib)
    if "copy" in args.ablate:  # reference: device-to-device copy of the packet bytes
        src = dev_batch.data
        dst = torch.empty_like(src)
        for _ in range(3):
            dst.copy_(src)
        torch.cuda.synchronize(local)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(20):
            dst.copy_(src)
        e1.record(stream)
        torch.cuda.synchronize(local)
        ms = e0.elapsed_time(e1) / 20
        print(json.dumps({"diag": "torch copy", "bytes": src.numel(), "ms": ms,
                          "GBps_read_plus_write": 2 * src.numel() / ms / 1e6}), flush=True)
        return

    if args.host:  # PCIe-inclusive: repack into pinned slots, H2D, decode, D2H
        h = bench_host(parser, batch, n, args.host, max(1, min(args.steps, 5)), max(1, args.warmup // 2))
        if rank == 0:
            print(json.dumps({"metric": "DIAGNOSTIC (not the metric): PCIe-inclusive Mpackets/s "
                              "host batch -> gpd_decode_host -> host results",
                              "value": h["Mpackets_per_s"], "unit": "Mpackets/s",
                              "ms_per_step": h["ms_per_step"], "steps": h["steps"],
                              "config": {"workload": workload, "packets": n, "host_arrays": args.host,
                                         "host_bytes_in": h["host_bytes_in"],
                                         "decode_errors_in_batch": h["decode_errors_in_batch"]},
                              "GBps_in": h["GBps_in"]}), flush=True)
        return

    settled = settle(lambda: parser.decode_device(dev_batch, dev_res, stream), args.settle_ms, local)
    for _ in range(args.warmup):
        parser.decode_device(dev_batch, dev_res, stream)
    torch.cuda.synchronize(local)

    span = args.events == "span"  # one event pair around the K launches (per-launch pairs: --events step)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(1 if span else args.steps)]
    if dist:
        dist.barrier()
    torch.cuda.synchronize(local)
    t0 = time.perf_counter()
    if span:
        ev[0][0].record(stream)
    for k in range(args.steps):
        if not span:
            ev[k][0].record(stream)
        parser.decode_device(dev_batch, dev_res, stream)
        if not span:
            ev[k][1].record(stream)
    if span:
        ev[0][1].record(stream)
    torch.cuda.synchronize(local)
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in ev])) / (args.steps if span else 1)
    elapsed, kern_ms_max = dist_max([elapsed, kern_ms], dist, f"cuda:{local}")

    # correctness guard on what was measured (cheap: status classes only)
    st = (dev_res.records.view(torch.int32)[0::8] if aos else dev_res.status).cpu().numpy().view(np.uint32)
    n_err = int(np.count_nonzero((st & 3) != 0))
    out = summarize(workload, n, world, args.steps, args.warmup, elapsed, kern_ms, kern_ms_max,
                    batch, n_err, interleaved=16 if pcap_info else 0)
    out["config"]["result_form"] = "gpd_record (AoS)" if aos else "SoA arrays"
    out["config"]["settle_ms"] = settled
    out["roofline"]["kernel_ms_method"] = (
        "HIP events on the launch stream around the K timed launches, / K (gaps between launches "
        "included)" if span else "HIP events on the launch stream around each timed launch, mean")
    if not args.ablate and not args.lean:  # the 36-B record (hdr_off on, as the flow table uses)
        # the five SoA arrays + hdr_off (the decode -> flow table pipeline's form); gpd_records +
        # hdr_off beside it (gpd_flow_insert takes either; measured slower on this part)
        out["record36"] = bench_record36(parser, dev_batch, n, local, stream, out, args)
        out["record36"]["form"] = "SoA arrays + hdr_off"
        out["record36_aos"] = bench_record36(parser, dev_batch, n, local, stream, out, args, records=True, hdr=True)
        out["record36_aos"]["form"] = "gpd_record + hdr_off"
        if aos:  # the same launch writing the five SoA arrays
            out["record_soa"] = bench_record36(parser, dev_batch, n, local, stream, out, args, soa=True)
        else:
            out["record_aos"] = bench_record36(parser, dev_batch, n, local, stream, out, args, records=True)
        out["fallback"] = bench_split(parser, dev_batch, dev_res, n, local, stream)
        if world == 1 and batch is not None and not pcap_info:
            # the same batch from host memory (north star: the rate including pinned H2D/D2H)
            out["pcie_inclusive"] = bench_host(parser, batch, n, "registered", 3, 1)
    if not args.ablate and not args.lean and not args.no_probe:
        rf = out["roofline"]
        rf["attainable"] = attainable(n, rf["algorithmic_read_bytes"], local, rf["achieved"], soa=not aos)
    if pcap_info:
        out["pcap"] = pcap_info
        if args.replay:
            out["pcap"]["pcie_inclusive"] = replay_pcap(parser, cap, n, args.replay, rank_threads(args))
    tr = load_traffic(args.config) if n == n_default else None
    if tr and tr["read"] and tr["write"]:  # PMC bytes, same read+write scope as `achieved`
        out["roofline"]["traffic"] = int(tr["read"]) + int(tr["write"])
        out["roofline"]["traffic_read"] = int(tr["read"])
        out["roofline"]["traffic_write"] = int(tr["write"])
        out["roofline"]["traffic_source"] = tr["source"]
        out["roofline"]["profiled_kernel_us"] = tr["kernel_us"]
    if args.tune:
        out["tuning"] = parser.Tuning
    if args.ablate:
        out["ablation"] = args.ablate
        out["metric"] = "DIAGNOSTIC ablation (not the metric): " + out["metric"]
    if world == 1 and not args.ablate and not args.lean and not args.no_side and args.config == "udp64":
        # the other configurations, each timed on its own resident batch (BASELINE.json configs
        # 3, 4 and 5 per GPU, and the north star's 64-B Eth/IPv4/TCP)
        del dev_res
        for c in SIDE_CONFIGS:
            out[c] = bench_side(c, parser, args, local, stream)
    if rank == 0 and world == 1 and not args.no_cpu_baseline and not args.ablate and not args.lean:
        out["cpu_baseline"] = cpu_baseline(batch, args.cpu_budget / 3)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if args.tpv3 and rank == 0:
        print(json.dumps(bench_tpv3(parser, batch, args)), flush=True)
    if args.flows and rank == 0:
        print(json.dumps(bench_flows(parser, dev_batch, n, args, stream, local)), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
