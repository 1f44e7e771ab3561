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
