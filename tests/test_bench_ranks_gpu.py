"""bench.py's N-rank path on the GPU box (one GPU): `--gpus 2` starts two ranks through its own
torch.distributed.run launcher, both on cuda:0 with gloo standing in for RCCL, so the weak-
scaling line and config 5's sharded replay run end to end with real kernels — the same code
the driver's multi-GPU run takes, except where the collective operands live."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(*args, gpus=2, timeout=300):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(gpus), "--dist-backend",
                        "gloo", "--same-device", "--no-cpu-baseline", "--settle-ms", "20", *args],
                       capture_output=True, text=True, timeout=timeout, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-3000:]  # rank 0 alone prints the line
    return json.loads(lines[0])


@pytest.mark.gpu
@pytest.mark.parametrize("gpus", [2, 8])
def test_ranks_weak_scaling_line(gpus):
    """The default line's N-rank path (8 = the driver's node, rehearsed on one GPU)."""
    n = 1 << (20 if gpus == 2 else 18)
    d = _bench("--steps", "3", "--warmup", "1", "--packets", str(n), gpus=gpus)
    assert d["n_gpus"] == gpus and d["scaling"] == "weak"
    assert d["config"]["decode_errors_in_batch"] == 0 and d["config"]["packets_per_gpu"] == n
    # value = packets of all ranks over the max-over-ranks time
    assert abs(d["value"] - gpus * n * 3 / (d["ms_per_step"] * 3 * 1e-3) / 1e6) / d["value"] < 0.02


@pytest.mark.gpu
@pytest.mark.parametrize("gpus,mem", [(2, "auto"), (8, "private"), (8, "shared")])
def test_ranks_sharded_replay(gpus, mem):
    """Config 5's cut and both legs with every rank; `private` is the fallback when /dev/shm
    cannot hold the node's capture (each rank builds its own shard)."""
    n = 3 * (1 << 20) + 12345
    d = _bench("--config", "replay", "--steps", "2", "--warmup", "1", "--packets", str(n),
               "--capture-memory", mem, gpus=gpus)
    assert d["n_gpus"] == gpus and d["scaling"] == "strong"
    ranks = d["per_rank"]
    assert [r["rank"] for r in ranks] == list(range(gpus))
    assert sum(r["packets"] for r in ranks) == n
    assert all(r["decode_errors"] == 0 and r["streamed_equals_resident"] for r in ranks)
    assert len(d["roofline"]["read_frac_per_rank"]) == gpus
    assert d["config"]["capture_memory"].startswith("private" if mem == "private" else "/dev/shm")
