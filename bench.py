#!/usr/bin/env python3
"""Benchmark: device-resident batched DecodingLayerParser decode + checksums + flow hashes.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config udp64|imix|vxlan]

One step = one launch of the fused decode kernel over one resident batch
(default: BASELINE.json configs[1], 2^24 synthetic 64 B Eth/IPv4/UDP packets per
GPU).  N > 1 runs under torch.distributed.run, one rank per GPU; every rank
decodes its own shard (weak scaling, no data-path collective — packets are
independent units); the barrier and the max-over-ranks timing use RCCL.

Rank 0 prints one JSON line with `value` in Mpackets/s (whole job), a
`roofline` object for the decode kernel (algorithmic HBM bytes per launch — packet
bytes and descriptors read, result records written — over the mean launch time measured with HIP events on the launch stream) and a
`cpu_baseline` object (the C restatement of gopacket's DLP in oracle/, timed on
this host's cores over a bounded sample of the same packets).
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
    if config == "pcap64":
        from gopacket_amd import pcap as NP
        return NP.synth_capture(synth.make_udp64(n, 0x5EED0002 + seed_off))
    return synth.make_vxlan(n, 0x5EED0004 + seed_off)


def cpu_baseline(batch, budget_s: float = 10.0, max_threads: int = 16):
    """The oracle (C restatement of the reference DLP, oracle/) over a bounded sample."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_ref as O
    from gopacket_amd.batch import PacketBatch
    threads = max(1, min(max_threads, os.cpu_count() or 1))
    m = min(batch.n, 1 << 21)
    sample = PacketBatch(batch.data, batch.data_len, batch.offset[:m].copy(), batch.caplen[:m].copy())
    O.decode(sample, ext=False, nthreads=threads)  # warm
    done, t0 = 0, time.perf_counter()
    while True:
        O.decode(sample, ext=False, nthreads=threads)
        done += m
        el = time.perf_counter() - t0
        if el >= budget_s or el > 30:
            break
    return {"value": round(done / el / 1e6, 3), "unit": "Mpackets/s", "cores": threads,
            "kind": "port",
            "sample": f"first {m} packets of the rank-0 batch, decoded {done // m}x in {el:.1f} s "
                      f"(C restatement of gopacket DecodingLayerParser + checksums + FastHash, "
                      f"{threads} threads)"}


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
    k = [v for n, v in s.get("kernels", {}).items() if "decode_kernel" in n or "rs_kernel" in n]
    return {"read": s.get("hbm_read_bytes_per_launch"), "write": s.get("hbm_write_bytes_per_launch"),
            "kernel_us": k[0]["avg_us"] if k else None,
            "source": os.path.relpath(paths[-1], ROOT)}


def dist_max(values, dist, device):
    """Max over ranks of a few floats (identity without torch.distributed)."""
    if not dist:
        return [float(v) for v in values]
    import torch
    t = torch.tensor([float(v) for v in values], dtype=torch.float64, device=device)
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
    gpd_decode_tpv3 (native block walk, H2D of the blocks, decode in place, D2H of the
    results) timed on the host clock.  PCIe-inclusive; never the metric."""
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
        parser.DecodeTPv3(ring, max_n=m, out=out, ci=cinfo)  # warm (and first touch)
        reps, t0 = 0, time.perf_counter()
        while True:
            res, ci, nblk = parser.DecodeTPv3(ring, max_n=m, out=out, ci=cinfo)
            reps += 1
            el = time.perf_counter() - t0
            if el > 3 or reps >= 20:
                break
    finally:
        lib.gpd_host_unregister(parser.ctx().h, arr.ctypes.data)
    assert len(res) == m and nblk == len(used)
    return {"diag": "F2 TPACKET_V3 ring walk + decode (PCIe-inclusive, not the metric)",
            "packets": m, "blocks": nblk, "block_size": bs, "ring_bytes": int(arr.nbytes),
            "ms_per_ring": round(el / reps * 1e3, 3), "Mpackets_per_s": round(m * reps / el / 1e6, 1),
            "GBps_ring_in": round(len(used) * bs * reps / el / 1e9, 2)}


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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="udp64", choices=sorted(CONFIGS))
    ap.add_argument("--packets", type=int, default=0, help="override packets per GPU")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=10.0)
    ap.add_argument("--host", action="store_true",
                    help="diagnostic: PCIe-inclusive rate through gpd_decode_host (host arrays in, "
                    "host arrays out); never the reported metric")
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
    ap.add_argument("--ablate", default="", help="diagnostics only: 'nocsum', 'nohash' or both "
                    "(comma separated); never used for the reported metric")
    args = ap.parse_args()

    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(local)

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
        pc = NP.index(cap, nthreads=args.threads)
        t_index = time.perf_counter() - t0
        assert pc.err is None and pc.batch.n == n, (pc.err, pc.batch.n)
        batch = pc.batch
        pcap_info = {"capture_bytes": int(batch.data_len), "index_s": round(t_index, 4),
                     "index_Mrec_per_s": round(n / t_index / 1e6, 1),
                     "index_threads": NP.last_walk_stats()[0]}
    dev_batch = P.DeviceBatch(batch, local)
    dev_res = P.DeviceResult(n, local, ext=False, hdr_off=False)  # the 32-B record
    parser = P.NewDecodingLayerParser(L.LayerTypeEthernet, P.Ethernet(), P.Dot1Q(), P.IPv4(),
                                      P.IPv6(), P.IPv6ExtensionSkipper(), P.TCP(), P.UDP(),
                                      P.VXLAN(), P.Payload(), P.Fragment(), device=local)
    stream = torch.cuda.current_stream(local)
    if "nocsum" in args.ablate:
        parser.ComputeChecksums = False
    if "nohash" in args.ablate:
        parser.ComputeFlowHashes = False
    if "nodecode" in args.ablate:
        parser._diag_options = 1 << 31  # kernel streams the windows and skips decoding
    if "nowait" in args.ablate:
        parser._diag_options = 1 << 30  # kernel skips the per-tile DMA wait (wrong results)
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
        res = parser.DecodeBatchHost(batch)
        for _ in range(max(1, args.warmup // 2)):
            parser.DecodeBatchHost(batch, out=res)
        steps = max(1, min(args.steps, 5))
        t0 = time.perf_counter()
        for _ in range(steps):
            parser.DecodeBatchHost(batch, out=res)
        el = time.perf_counter() - t0
        n_err = int(np.count_nonzero((res.status & 3) != 0))
        if rank == 0:
            print(json.dumps({"metric": "DIAGNOSTIC (not the metric): PCIe-inclusive Mpackets/s "
                              "host batch -> gpd_decode_host -> host results",
                              "value": round(n * steps / el / 1e6, 2), "unit": "Mpackets/s",
                              "ms_per_step": round(el / steps * 1e3, 3), "steps": steps,
                              "config": {"workload": workload, "packets": n,
                                         "host_bytes_in": int(batch.data_len) + 8 * n,
                                         "decode_errors_in_batch": n_err},
                              "GBps_in": round((batch.data_len + 8 * n) * steps / el / 1e9, 2)}),
                  flush=True)
        return

    for _ in range(args.warmup):
        parser.decode_device(dev_batch, dev_res, stream)
    torch.cuda.synchronize(local)

    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(args.steps)]
    if dist:
        dist.barrier()
    torch.cuda.synchronize(local)
    t0 = time.perf_counter()
    for k in range(args.steps):
        ev[k][0].record(stream)
        parser.decode_device(dev_batch, dev_res, stream)
        ev[k][1].record(stream)
    torch.cuda.synchronize(local)
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    elapsed, kern_ms_max = dist_max([elapsed, kern_ms], dist, f"cuda:{local}")

    # correctness guard on what was measured (cheap: status classes only)
    st = dev_res.status.cpu().numpy().view(np.uint32)
    n_err = int(np.count_nonzero((st & 3) != 0))
    out = summarize(workload, n, world, args.steps, args.warmup, elapsed, kern_ms, kern_ms_max,
                    batch, n_err, interleaved=16 if pcap_info else 0)
    if pcap_info:
        out["pcap"] = pcap_info
        if args.replay:
            out["pcap"]["pcie_inclusive"] = replay_pcap(parser, cap, n, args.replay, args.threads)
    tr = load_traffic(args.config) if n == n_default else None
    if tr and tr["read"] and tr["write"]:  # PMC bytes, same read+write scope as `achieved`
        out["roofline"]["traffic"] = int(tr["read"]) + int(tr["write"])
        out["roofline"]["traffic_read"] = int(tr["read"])
        out["roofline"]["traffic_write"] = int(tr["write"])
        out["roofline"]["traffic_source"] = tr["source"]
        out["roofline"]["profiled_kernel_us"] = tr["kernel_us"]
    if args.ablate:
        out["ablation"] = args.ablate
        out["metric"] = "DIAGNOSTIC ablation (not the metric): " + out["metric"]
    if rank == 0 and world == 1 and not args.no_cpu_baseline and not args.ablate:
        out["cpu_baseline"] = cpu_baseline(batch, args.cpu_budget)
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
