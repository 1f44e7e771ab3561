"""Multi-rank paths on CPU (gloo, world size 2): sharding, max-over-ranks timing, aggregate value.

bench.py shards the hot path by packet index with no data-path collective: every rank
builds and decodes its own shard (weak scaling), and torch.distributed is used only for
the start/stop barrier and the max-over-ranks time.  These tests run that logic with the
gloo backend; the per-shard decode is the oracle here (no GPU in this container).
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, n, out_dir):
    import bench
    import oracle_ref as O
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    try:
        batch = bench.make_batch("udp64", n, rank)
        res = O.decode(batch, ext=False, nthreads=1)
        # fake per-rank timings: the slowest rank must win
        elapsed, kern = (0.5 + rank) * 1e-3, 0.1 * (rank + 1)
        el_max, kern_max = bench.dist_max([elapsed, kern], dist, "cpu")
        out = bench.summarize("udp64-test", n, world, 3, 1, el_max, kern, kern_max, batch, 0)
        dist.barrier()
        np.savez(os.path.join(out_dir, f"rank{rank}.npz"), net_hash=res.net_hash,
                 status=res.status, data=batch.data[:batch.data_len], value=out["value"],
                 el_max=el_max, kern_max=kern_max)
    finally:
        dist.destroy_process_group()


@pytest.fixture(scope="module")
def two_ranks(tmp_path_factory):
    out = tmp_path_factory.mktemp("dist")
    n = 2048
    mp.spawn(_worker, args=(2, _free_port(), n, str(out)), nprocs=2, join=True)
    return n, [dict(np.load(out / f"rank{r}.npz")) for r in range(2)]


def test_max_over_ranks(two_ranks):
    n, r = two_ranks
    for x in r:
        assert float(x["el_max"]) == pytest.approx(1.5e-3)
        assert float(x["kern_max"]) == pytest.approx(0.2)


def test_aggregate_value_counts_every_rank(two_ranks):
    n, r = two_ranks
    # value = packets all ranks decoded / max-over-ranks wall time
    assert float(r[0]["value"]) == pytest.approx(n * 2 * 3 / 1.5e-3 / 1e6, rel=1e-3)


def test_shards_are_distinct_and_complete(two_ranks):
    n, r = two_ranks
    # each rank owns a different shard (its own seed), decoded completely and cleanly
    assert not np.array_equal(r[0]["data"], r[1]["data"])
    for x in r:
        assert x["status"].shape == (n,)
        assert np.all((x["status"] & 3) == 0)
        assert len(np.unique(x["net_hash"])) > n // 2


def test_shard_matches_single_rank_decode(two_ranks):
    """Rank 1's shard decoded alone equals the same packets decoded by one process."""
    import bench
    import oracle_ref as O
    n, r = two_ranks
    batch = bench.make_batch("udp64", n, 1)
    res = O.decode(batch, ext=False, nthreads=2)
    assert np.array_equal(res.net_hash, r[1]["net_hash"])
    assert np.array_equal(res.status, r[1]["status"])


# ---------------------------------------------------------------- flow-affine sharding (F3, §8(e))
def _key_records(batch, res, base, world):
    """Host-built key records (the layout gpd_flow_keys writes), grouped by owner rank."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import flow_ref as F
    from gopacket_amd import flows as FL
    keyed, keys = F.flow_keys(batch, res)
    owner = FL.flow_owner(res.net_hash, res.tp_hash, world)
    idx = np.nonzero(keyed)[0]
    idx = idx[np.argsort(owner[idx], kind="stable")]
    rec = np.zeros(len(idx), FL.FLOW_KEY_DTYPE)
    rec["key"] = keys[idx].view("<u4").reshape(-1, 10)
    rec["caplen"] = batch.caplen[idx]
    rec["owner"] = owner[idx]
    rec["seq"] = base + idx
    counts = np.bincount(owner[idx], minlength=world)
    return rec, counts


def _xchg_worker(rank, world, port, out_dir):
    import oracle_ref as O
    from gopacket_amd import flows as FL
    from gopacket_amd import synth
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    try:
        batch = synth.make_mixed(700 + 150 * rank, seed=0x5EED0100 + rank)
        res = O.decode(batch, 17, 0xFFF, ext=False)
        rec, counts = _key_records(batch, res, rank << 32, world)
        recv, rcv = FL.exchange_keys(torch.from_numpy(rec.view(np.int64).reshape(-1, 8)),
                                     [int(c) for c in counts])
        got = recv.numpy().reshape(-1).view(FL.FLOW_KEY_DTYPE)
        ids = torch.from_numpy(((got["seq"] * 7) % 1000003).astype(np.int32))  # stand-in ids
        back = FL.return_ids(ids, rcv, [int(c) for c in counts]).numpy()
        np.savez(os.path.join(out_dir, f"x{rank}.npz"), sent=rec.view(np.uint8), got=got.view(np.uint8),
                 rcv=np.array(rcv), counts=counts, back=back)
    finally:
        dist.destroy_process_group()


def test_flow_key_exchange_routes_every_record_to_its_owner(tmp_path):
    """ShardedFlowTable's all-to-all on gloo, world 3: every rank receives exactly the key
    records it owns from every rank, and the reverse exchange returns each record's id to its
    sender in the order sent."""
    from gopacket_amd import flows as FL
    world = 3
    mp.spawn(_xchg_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    r = [dict(np.load(tmp_path / f"x{k}.npz")) for k in range(world)]
    sent = [x["sent"].view(FL.FLOW_KEY_DTYPE) for x in r]
    got = [x["got"].view(FL.FLOW_KEY_DTYPE) for x in r]
    for k in range(world):
        assert (got[k]["owner"] == k).all()
        want = np.concatenate([s[s["owner"] == k] for s in sent])
        assert np.array_equal(np.sort(got[k]["seq"]), np.sort(want["seq"]))
        assert int(r[k]["rcv"].sum()) == len(got[k])
        assert np.array_equal(r[k]["back"], ((sent[k]["seq"] * 7) % 1000003).astype(np.int32))
    # every owner receives some records, and a flow's two directions share an owner
    assert all(len(g) > 0 for g in got)
