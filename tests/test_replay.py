"""Config 5 (one pcap capture sharded by packet index over the node's GPUs), CPU side.

bench.py --config replay builds ONE seeded capture in host memory (a /dev/shm mapping shared by
the ranks), cuts it into shards [g*N/G, (g+1)*N/G) with gpd_pcap_locate and indexes each shard
chunk by chunk.  These tests run that cut through bench.py's own launcher (`--gpus N` starts N
ranks through torch.distributed.run; gloo, no GPU) and check it against the single-rank index of
the whole capture; they also pin the native capture generator to synth.make_udp64.
"""
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from gopacket_amd import pcap as NP  # noqa: E402
from gopacket_amd import synth  # noqa: E402


def test_native_generator_is_make_udp64():
    n = 3000
    b = synth.make_udp64(n)
    raw = np.zeros(n * 64, np.uint8)
    synth.udp64_native(raw, 0, n, nthreads=3)
    assert np.array_equal(raw, b.data[:n * 64])
    cap = NP.synth_capture(b)
    rec = np.zeros((n - 700) * 80, np.uint8)
    synth.udp64_native(rec, 700, n, records=True, nthreads=5)
    assert np.array_equal(rec, cap[24 + 700 * 80:24 + n * 80])


def _whole_capture(n):
    import struct
    from gopacket_amd.batch import PAD
    cap = np.zeros(24 + 80 * n + PAD, np.uint8)
    cap[:24] = np.frombuffer(struct.pack("<IHHiIII", 0xA1B2C3D4, 2, 4, 0, 0, 262144, 1), np.uint8)
    synth.udp64_native(cap[24:24 + 80 * n], 0, n, 0x5EED0002, records=True, nthreads=4)
    return cap


@pytest.mark.parametrize("world,n,chunk,mem,threads", [
    (2, 200003, 30000, "auto", 2), (3, 100000, 1 << 24, "auto", 2),
    (8, 400009, 20000, "shared", 0), (8, 400009, 20000, "private", 0), (3, 100000, 7000, "private", 2)])
def test_replay_shards_through_the_launcher(tmp_path, world, n, chunk, mem, threads):
    """World 8 is the driver's node: both capture memories (the private one is what a node whose
    /dev/shm cannot hold the 80-GB capture falls back to), threads per rank by default (the
    node's cores shared by its ranks)."""
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(world), "--config", "replay",
           "--packets", str(n), "--chunk", str(chunk), "--threads", str(threads), "--capture-memory", mem,
           "--shard-check", str(tmp_path)]
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    before = set(os.listdir("/dev/shm"))
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    parts = [dict(np.load(tmp_path / f"rank{g}.npz")) for g in range(world)]
    whole = NP.index(_whole_capture(n), nthreads=4)
    assert whole.batch.n == n and whole.err is None
    want = whole.batch.offset.astype(np.uint64) - 16
    # shard g holds records [g*N/G, (g+1)*N/G): disjoint, in order, together the whole index
    for g, p in enumerate(parts):
        assert str(p["mode"]) == ("shared" if mem == "auto" else mem)
        if threads == 0:
            assert 1 <= int(p["threads"]) <= max(1, 16 // world) * 4
        assert (int(p["lo"]), int(p["hi"])) == (n * g // world, n * (g + 1) // world)
        assert int(p["world"]) == world and int(p["cn"]) == int(p["hi"]) - int(p["lo"])
        assert np.array_equal(p["hdr"], want[int(p["lo"]):int(p["hi"])])
        assert int(p["start"]) == int(want[int(p["lo"])])
    cat = np.concatenate([p["hdr"] for p in parts])
    assert len(np.unique(cat)) == n and np.array_equal(cat, want)
    # the shared capture's file name is gone after the run
    assert not [f for f in set(os.listdir("/dev/shm")) - before if f.startswith("gpd_replay_")]


def test_launcher_rejects_a_world_size_mismatch():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4", "--config",
                        "replay", "--shard-check", "/nonexistent"], env=env, capture_output=True,
                       text=True, timeout=120)
    assert r.returncode != 0 and "WORLD_SIZE=2" in r.stderr
