"""F3 flow table (include/gpd_flow.h): the GPU connection map vs the CPU restatement of
tcpassembly's key{NetworkFlow(), TransportFlow()} grouping (oracle/flow_ref.py)."""
import ctypes as C
import os
import sys

import numpy as np
import pytest

import golden_cases as G
import oracle_ref as O
from conftest import ROOT
from gopacket_amd import layers as L
from gopacket_amd import synth
from gopacket_amd.batch import PacketBatch

sys.path.insert(0, os.path.join(ROOT, "oracle"))
import flow_ref as F  # noqa: E402

ALL = 0xFFF


def _hot_batch(n=20000, distinct=300, seed=3):
    """Many packets over few flows (heavy per-record atomics), both directions of some."""
    rng = np.random.default_rng(seed)
    base = synth.make_mixed(distinct)
    pk = [base.packet(i) for i in range(base.n)]
    rev = []
    for p in pk[:50]:  # the reverse direction of a few UDP/IPv4 frames: separate Flow keys
        b = bytearray(p)
        if len(b) >= 42 and b[12:14] == b"\x08\x00" and b[23] == 17:
            b[26:30], b[30:34] = p[30:34], p[26:30]
            b[34:36], b[36:38] = p[36:38], p[34:36]
            rev.append(bytes(b))
    pool = pk + rev
    return PacketBatch.from_packets([pool[int(k)] for k in rng.integers(0, len(pool), n)])


def _burst_batch(n=20000, distinct=200, seed=7):
    """Flows in bursts: runs of 1-150 back-to-back packets of one flow (runs cross wave
    boundaries, unkeyed frames break some), so a wave's lanes share records and the insert
    folds each run before its atomics; a flow recurs in later bursts."""
    rng = np.random.default_rng(seed)
    base = synth.make_mixed(distinct)
    pool = [base.packet(i) for i in range(base.n)]
    out = []
    while len(out) < n:
        out += [pool[int(rng.integers(0, len(pool)))]] * int(rng.integers(1, 151))
    return PacketBatch.from_packets(out[:n])


def test_oracle_flow_keys_directional_and_pcap():
    """The restatement on the reference's own capture: test_ethernet.pcap is one TCP
    conversation, so its packets fall into exactly two directional keys."""
    from gopacket_amd import pcap as NP
    cap = NP.capture_array(open(os.path.join(ROOT, "tests", "golden", "test_ethernet.pcap"), "rb").read())
    pc = NP.index(cap)
    res = O.decode(pc.batch, L.LayerTypeEthernet, ALL, ext=False)
    flows, per = F.group(pc.batch, res)
    assert all(k is not None for k in per)
    assert len(flows) == 2
    a, b = list(flows)
    # reverse keys: src/dst and ports swapped, same types
    ka, kb = np.frombuffer(a, np.uint8), np.frombuffer(b, np.uint8)
    assert (ka[0:4] == kb[16:20]).all() and (ka[16:20] == kb[0:4]).all()
    assert (ka[32:34] == kb[34:36]).all() and (ka[36:39] == kb[36:39]).all() and ka[37] == 4
    assert sum(f["packets"] for f in flows.values()) == pc.batch.n


def _check_table(batch, res, fid, ft, flows_ref, per_ref):
    fid = fid.astype(np.uint32)
    keyed = np.array([k is not None for k in per_ref])
    assert ((fid == 0xFFFFFFFF) == ~keyed).all(), "flow_id NONE exactly where no key"
    assert not (fid[keyed] & 0x80000000).any(), "no fingerprint collisions"
    key_of_id = {}
    for i in np.nonzero(keyed)[0]:
        k = per_ref[i]
        assert key_of_id.setdefault(int(fid[i]), k) == k, "one record, one key"
    assert len(key_of_id) == len(flows_ref), "one record per distinct key"
    recs, idx = ft.Export()
    assert len(recs) == len(flows_ref)
    for r, ix in zip(recs, idx):
        k = F.record_key(r)
        f = flows_ref[k]
        assert key_of_id[int(ix)] == k
        assert (int(r["first"]), int(r["last"]), int(r["packets"]), int(r["bytes"])) == \
            (f["first"], f["last"], f["packets"], f["bytes"])
    assert list(recs["first"]) == sorted(recs["first"])
    st = ft.Stats()
    assert st["flows"] == len(flows_ref) and st["collisions"] == 0 and st["full"] == 0
    assert st["packets"] == int(keyed.sum()) and st["no_key"] == int((~keyed).sum())


def _decode_dev(p, batch):
    from gopacket_amd import parser as P
    db = P.DeviceBatch(batch, 0)
    dr = P.DeviceResult(batch.n, 0)
    p.decode_device(db, dr)
    return db, dr


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["golden_mut", "mixed", "hot", "imix", "burst"])
def test_flow_table_matches_oracle(kind):
    import torch
    from gopacket_amd import flows as FL
    from gopacket_amd import parser as P
    if kind == "golden_mut":
        pk = [G.case_bytes(c) for c in G.load()["cases"]]
        rng = np.random.default_rng(5)
        for p in list(pk):
            for _ in range(200):
                a = np.frombuffer(p[:512], np.uint8).copy()
                pos = rng.integers(0, min(len(a), 80), size=2)
                a[pos] = rng.integers(0, 256, size=2, dtype=np.uint8)
                pk.append(a.tobytes())
        batch = PacketBatch.from_packets(pk)
    elif kind == "mixed":
        batch = synth.make_mixed(30000)
    elif kind == "imix":
        batch = synth.make_imix(1 << 14)
    elif kind == "burst":
        batch = _burst_batch()
    else:
        batch = _hot_batch()
    parser = P.NewDecodingLayerParser(L.LayerTypeEthernet, *[P.DECODER_BY_NAME[k]() for k in P.DECODER_BY_NAME])
    db, dr = _decode_dev(parser, batch)
    ft = FL.NewFlowTable(parser, 4 * batch.n)
    fid = ft.Insert(db, dr)
    torch.cuda.synchronize()
    res = dr.to_host()
    ref = O.decode(batch, L.LayerTypeEthernet, parser.decoders, 0, ext=False, nthreads=8)
    assert (res.hdr_off == ref.hdr_off).all() and (res.status == ref.status).all()
    flows_ref, per_ref = F.group(batch, ref)
    _check_table(batch, res, fid.cpu().numpy().view(np.uint32), ft, flows_ref, per_ref)


@pytest.mark.gpu
def test_flow_table_accumulates_and_resets():
    import torch
    from gopacket_amd import flows as FL
    from gopacket_amd import parser as P
    a, b = _hot_batch(8000, 200, 1), _hot_batch(6000, 200, 2)
    parser = P.NewDecodingLayerParser(L.LayerTypeEthernet, P.Ethernet(), P.Dot1Q(), P.IPv4(), P.IPv6(),
                                      P.TCP(), P.UDP(), P.VXLAN(), P.Payload())
    ft = FL.NewFlowTable(parser, 1 << 12)
    ids = []
    for k, batch in enumerate((a, b)):
        db, dr = _decode_dev(parser, batch)
        ids.append(ft.Insert(db, dr, index_base=k * a.n).cpu().numpy().view(np.uint32))
    torch.cuda.synchronize()
    both = PacketBatch.from_packets([a.packet(i) for i in range(a.n)] + [b.packet(i) for i in range(b.n)])
    ref = O.decode(both, L.LayerTypeEthernet, parser.decoders, 0, ext=False, nthreads=8)
    flows_ref, per_ref = F.group(both, ref)
    _check_table(both, None, np.concatenate(ids), ft, flows_ref, per_ref)
    ft.Reset()
    assert ft.Stats()["flows"] == 0 and len(ft.Export()[0]) == 0


@pytest.mark.gpu
@pytest.mark.parametrize("order", ["ascending", "descending", "same_base_twice"])
def test_flow_table_sequence_bases_in_any_order(order):
    """A record of an earlier call skips its `first` update only when the packet's sequence
    number is above every earlier call's (the host's bound, FlowParams::seen): batches inserted
    with descending index bases (first must still fall) or the same base twice are exact."""
    import torch
    from gopacket_amd import flows as FL
    from gopacket_amd import parser as P
    a, b = _hot_batch(7000, 300, 3), _hot_batch(5000, 300, 4)
    parser = P.NewDecodingLayerParser(L.LayerTypeEthernet, P.Ethernet(), P.Dot1Q(), P.IPv4(), P.IPv6(),
                                      P.TCP(), P.UDP(), P.VXLAN(), P.Payload())
    ft = FL.NewFlowTable(parser, 1 << 12)
    steps = {"ascending": [(a, 0), (b, a.n)], "descending": [(b, a.n), (a, 0)],
             "same_base_twice": [(a, 0), (a, 0)]}[order]
    ids = {}
    for batch, base in steps:
        db, dr = _decode_dev(parser, batch)
        ids.setdefault(base, []).append(ft.Insert(db, dr, index_base=base).cpu().numpy().view(np.uint32))
    torch.cuda.synchronize()
    if order == "same_base_twice":
        # twice the same packets at the same sequence numbers: the records hold every packet twice
        both = PacketBatch.from_packets([a.packet(i) for i in range(a.n)] * 2)
        ref = O.decode(both, L.LayerTypeEthernet, parser.decoders, 0, ext=False, nthreads=8)
        flows_ref, per_ref = F.group(both, ref)
        ex, _ = ft.Export()
        assert len(ex) == len(flows_ref)
        for r in ex:
            f = flows_ref[F.record_key(r)]
            assert (int(r["first"]), int(r["last"]), int(r["packets"]), int(r["bytes"])) == \
                (f["first"], f["last"] - a.n, f["packets"], f["bytes"])
        return
    both = PacketBatch.from_packets([a.packet(i) for i in range(a.n)] + [b.packet(i) for i in range(b.n)])
    ref = O.decode(both, L.LayerTypeEthernet, parser.decoders, 0, ext=False, nthreads=8)
    flows_ref, per_ref = F.group(both, ref)
    _check_table(both, None, np.concatenate([ids[0][0], ids[a.n][0]]), ft, flows_ref, per_ref)


@pytest.mark.gpu
def test_flow_table_full():
    """More distinct keys than records: every lane leaves its probe loop; the overflow is
    counted and flagged, the records that exist stay exact."""
    import torch
    from gopacket_amd import flows as FL
    from gopacket_amd import parser as P
    batch = synth.make_udp64(4096, 0x77)
    parser = P.NewDecodingLayerParser(L.LayerTypeEthernet, P.Ethernet(), P.IPv4(), P.UDP(), P.Payload())
    db, dr = _decode_dev(parser, batch)
    ft = FL.NewFlowTable(parser, 64)
    fid = ft.Insert(db, dr).cpu().numpy().view(np.uint32)
    torch.cuda.synchronize()
    st = ft.Stats()
    assert st["capacity"] == 64 and st["flows"] == 64
    assert st["full"] == int((fid == 0xFFFFFFFE).sum()) == batch.n - st["packets"]
    assert st["packets"] == int((fid < 64).sum())


# ---------------------------------------------------------------- flow-affine sharding (§8(e))
def test_flow_owner_is_direction_symmetric():
    """Both directions of a conversation go to one owner: the owner is computed from
    NetworkFlow().FastHash() ^ TransportFlow().FastHash(), both symmetric (flows.go:167-174)."""
    from gopacket_amd import flows as FL
    batch = _hot_batch(4000, 120, 4)
    ref = O.decode(batch, L.LayerTypeEthernet, ALL, 0, ext=False)
    keyed, keys = F.flow_keys(batch, ref)
    for world in (2, 3, 8):
        own = FL.flow_owner(ref.net_hash, ref.tp_hash, world)
        by_key = {}
        for i in np.nonzero(keyed)[0]:
            k = keys[i]
            rev = np.concatenate([k[16:32], k[0:16], k[34:36], k[32:34], k[36:40]]).tobytes()
            by_key[k.tobytes()] = int(own[i])
            if rev in by_key:
                assert by_key[rev] == int(own[i])
        assert set(own[keyed].tolist()) == set(range(world))


def _global_batch():
    pool = _hot_batch(6000, 400, 6)
    mixed = synth.make_mixed(4000, seed=0x5EED0200)
    burst = _burst_batch(4000, 100, 8)
    return PacketBatch.from_packets([pool.packet(i) for i in range(pool.n)] +
                                    [mixed.packet(i) for i in range(mixed.n)] +
                                    [burst.packet(i) for i in range(burst.n)])


def _shard_worker(rank, world, port, out_dir):
    import torch
    import torch.distributed as dist
    from gopacket_amd import flows as FL
    from gopacket_amd import parser as P
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    try:
        full = _global_batch()
        lo, hi = rank * full.n // world, (rank + 1) * full.n // world
        shard = PacketBatch.from_packets([full.packet(i) for i in range(lo, hi)])
        parser = P.NewDecodingLayerParser(L.LayerTypeEthernet, *[P.DECODER_BY_NAME[k]() for k in P.DECODER_BY_NAME])
        db, dr = _decode_dev(parser, shard)
        st = FL.ShardedFlowTable(parser, 1 << 14)
        owner, fid = st.Insert(db, dr, index_base=lo)
        torch.cuda.synchronize()
        recs, idx = st.Export()
        np.savez(os.path.join(out_dir, f"s{rank}.npz"), owner=owner.cpu().numpy(),
                 fid=fid.cpu().numpy().view(np.uint32), recs=recs.view(np.uint8), idx=idx,
                 stats=np.array(list(st.Stats().values()), np.uint64))
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_sharded_flow_table_two_ranks():
    """ShardedFlowTable with two ranks (gloo, both on the one GPU of the test box): every
    flow lives on exactly one rank, the rank its FastHash pair names; the union of the two
    tables equals the oracle's connection map of the whole batch; each packet's (owner, id)
    names the record holding its key."""
    import subprocess
    import tempfile
    from gopacket_amd import flows as FL
    world = 2
    with tempfile.TemporaryDirectory() as d:
        import socket
        with socket.socket() as s:
            s.bind(("127.0.0.1", 0))
            port = s.getsockname()[1]
        code = ("import sys; sys.path[:0] = [%r, %r]; import test_flow as T; "
                "T._shard_worker(int(sys.argv[1]), %d, %d, %r)" % (ROOT, os.path.join(ROOT, "tests"),
                                                                   world, port, d))
        procs = [subprocess.Popen([sys.executable, "-c", code, str(r)], stdout=subprocess.PIPE,
                                  stderr=subprocess.STDOUT, text=True) for r in range(world)]
        outs = [p.communicate(timeout=100)[0] for p in procs]
        assert all(p.returncode == 0 for p in procs), "\n".join(outs)
        r = [dict(np.load(os.path.join(d, f"s{k}.npz"))) for k in range(world)]
    full = _global_batch()
    ref = O.decode(full, L.LayerTypeEthernet, ALL, 0, ext=False, nthreads=8)
    flows_ref, per_ref = F.group(full, ref)
    own_ref = FL.flow_owner(ref.net_hash, ref.tp_hash, world)
    owner = np.concatenate([x["owner"] for x in r])
    fid = np.concatenate([x["fid"] for x in r])
    tables = []
    for k, x in enumerate(r):
        recs = x["recs"].view(FL.FLOW_REC_DTYPE)
        tables.append({int(i): rec for i, rec in zip(x["idx"], recs)})
        assert int(x["stats"][4]) == 0, "no fingerprint collisions"
    seen = {}
    for i, key in enumerate(per_ref):
        if key is None:
            assert owner[i] == -1 and fid[i] == 0xFFFFFFFF
            continue
        assert owner[i] == own_ref[i]
        assert F.record_key(tables[owner[i]][int(fid[i])]) == key
        seen.setdefault(key, (int(owner[i]), int(fid[i])))
        assert seen[key] == (int(owner[i]), int(fid[i]))
    union = {}
    for k, t in enumerate(tables):
        for rec in t.values():
            key = F.record_key(rec)
            assert key not in union, "a flow on two ranks"
            union[key] = rec
    assert set(union) == set(flows_ref)
    for key, f in flows_ref.items():
        rec = union[key]
        assert (int(rec["first"]), int(rec["last"]), int(rec["packets"]), int(rec["bytes"])) == \
            (f["first"], f["last"], f["packets"], f["bytes"])
    assert all(len(t) > 0 for t in tables)


@pytest.mark.gpu
@pytest.mark.parametrize("bits", [3, 12])
def test_flow_fingerprint_collisions_are_flagged(bits):
    """Fingerprints narrowed to a few bits (test hook): distinct keys now share records.  A
    packet whose key differs from its record's stored key (the claimer's) must carry
    GPD_FLOW_COLLISION, every other packet must not, the collision counter must count exactly
    the flagged packets, and each record's counters still cover every packet mapped to it."""
    import torch
    from gopacket_amd import flows as FL
    from gopacket_amd import parser as P
    batch = synth.make_mixed(20000)
    parser = P.NewDecodingLayerParser(L.LayerTypeEthernet, *[P.DECODER_BY_NAME[k]() for k in P.DECODER_BY_NAME])
    db, dr = _decode_dev(parser, batch)
    ft = FL.NewFlowTable(parser, 1 << 16)
    ft._test_fingerprint_bits(bits)
    fid = ft.Insert(db, dr).cpu().numpy().view(np.uint32)
    torch.cuda.synchronize()
    ref = O.decode(batch, L.LayerTypeEthernet, parser.decoders, 0, ext=False, nthreads=8)
    flows_ref, per_ref = F.group(batch, ref)
    keyed = np.array([k is not None for k in per_ref])
    assert ((fid == 0xFFFFFFFF) == ~keyed).all()
    rec_of = fid & 0x7FFFFFFF
    flagged = (fid & 0x80000000) != 0
    recs, idx = ft.Export()
    st = ft.Stats()
    assert st["flows"] == len(recs) <= (1 << bits) and st["full"] == 0
    assert len(recs) < len(flows_ref)  # keys were merged
    stored = {int(ix): F.record_key(r) for r, ix in zip(recs, idx)}
    ki = np.nonzero(keyed)[0]
    for i in ki:
        assert flagged[i] == (per_ref[i] != stored[int(rec_of[i])])
    assert st["collisions"] == int(flagged.sum()) > 0
    # a key always lands on one record; each record counts every packet that landed on it
    rec_by_key = {}
    for i in ki:
        assert rec_by_key.setdefault(per_ref[i], int(rec_of[i])) == int(rec_of[i])
    for r, ix in zip(recs, idx):
        on = ki[rec_of[ki] == ix]
        assert int(r["packets"]) == len(on)
        assert int(r["bytes"]) == int(batch.caplen[on].astype(np.int64).sum())
        assert (int(r["first"]), int(r["last"])) == (int(on.min()), int(on.max()))


@pytest.mark.gpu
@pytest.mark.parametrize("bits", [1, 7, 12, 57])
def test_flow_counter_spills_are_exact(bits):
    """The packed counter word (packets << B | bytes mod 2^B, one atomicAdd) split at a test
    width (gpd_flow_test_counter_bits): with B = 1..12 nearly every add carries out of the
    byte field, with B = 57 the 7-bit packet field wraps after 128 packets of a flow.  Hot
    flows (~70 packets each per batch) and bursts, accumulated over four batches, so new-flow
    stores, existing-flow adds, carries, wraps and take-back borrows all run; every exported
    record must equal the oracle's group-by."""
    import torch
    from gopacket_amd import flows as FL
    from gopacket_amd import parser as P
    parts = [_hot_batch(20000, 300, 11), _burst_batch(20000, 200, 12), _hot_batch(20000, 300, 11),
             _burst_batch(20000, 200, 12)]
    parser = P.NewDecodingLayerParser(L.LayerTypeEthernet, *[P.DECODER_BY_NAME[k]() for k in P.DECODER_BY_NAME])
    ft = FL.NewFlowTable(parser, 1 << 14)
    ft._test_counter_bits(bits)
    ids, base = [], 0
    for batch in parts:
        db, dr = _decode_dev(parser, batch)
        ids.append(ft.Insert(db, dr, index_base=base).cpu().numpy().view(np.uint32))
        base += batch.n
    torch.cuda.synchronize()
    allp = PacketBatch.from_packets([b.packet(i) for b in parts for i in range(b.n)])
    ref = O.decode(allp, L.LayerTypeEthernet, parser.decoders, 0, ext=False, nthreads=8)
    flows_ref, per_ref = F.group(allp, ref)
    assert max(f["packets"] for f in flows_ref.values()) > 128
    _check_table(allp, None, np.concatenate(ids), ft, flows_ref, per_ref)


@pytest.mark.gpu
@pytest.mark.parametrize("bits", [3, 12])
def test_flow_collisions_across_batches(bits):
    """Records claimed by an earlier insert are updated and key-checked in the insert itself
    (their epoch differs from the call's); with narrowed fingerprints the second batch's packets
    land on the first batch's records and on their own, and every flag, the collision counter
    and every record's counters must still match the restatement over both batches."""
    import torch
    from gopacket_amd import flows as FL
    from gopacket_amd import parser as P
    a, b = synth.make_mixed(12000, 0x5EED0101), _burst_batch(9000, 150, 9)
    parser = P.NewDecodingLayerParser(L.LayerTypeEthernet, *[P.DECODER_BY_NAME[k]() for k in P.DECODER_BY_NAME])
    ft = FL.NewFlowTable(parser, 1 << 16)
    ft._test_fingerprint_bits(bits)
    fids = []
    for k, batch in enumerate((a, b, a)):
        db, dr = _decode_dev(parser, batch)
        fids.append(ft.Insert(db, dr, index_base=k * 20000).cpu().numpy().view(np.uint32))
    torch.cuda.synchronize()
    recs, idx = ft.Export()
    st = ft.Stats()
    stored = {int(ix): F.record_key(r) for r, ix in zip(recs, idx)}
    flagged_total, on_rec = 0, {}
    for k, (batch, fid) in enumerate(zip((a, b, a), fids)):
        ref = O.decode(batch, L.LayerTypeEthernet, parser.decoders, 0, ext=False, nthreads=8)
        _, per_ref = F.group(batch, ref)
        keyed = np.array([x is not None for x in per_ref])
        assert ((fid == 0xFFFFFFFF) == ~keyed).all()
        rec_of = fid & 0x7FFFFFFF
        flagged = (fid & 0x80000000) != 0
        for i in np.nonzero(keyed)[0]:
            assert flagged[i] == (per_ref[i] != stored[int(rec_of[i])])
            on_rec.setdefault(int(rec_of[i]), []).append((k * 20000 + int(i), int(batch.caplen[i])))
        flagged_total += int(flagged.sum())
    assert st["collisions"] == flagged_total > 0 and st["full"] == 0
    for r, ix in zip(recs, idx):
        on = on_rec[int(ix)]
        assert int(r["packets"]) == len(on)
        assert int(r["bytes"]) == sum(c for _, c in on)
        assert (int(r["first"]), int(r["last"])) == (min(s for s, _ in on), max(s for s, _ in on))


@pytest.mark.gpu
def test_flow_table_reads_the_record_form():
    """A batch decoded into gpd_records + hdr_off inserts, keys and shards exactly as the same
    batch decoded into the SoA arrays (status and hashes read from the records)."""
    import torch
    from gopacket_amd import flows as FL
    from gopacket_amd import parser as P
    batch = _burst_batch(12000, 300, 13)
    parser = P.NewDecodingLayerParser(L.LayerTypeEthernet, *[P.DECODER_BY_NAME[k]() for k in P.DECODER_BY_NAME])
    got = []
    for records in (False, True):
        db = P.DeviceBatch(batch, 0)
        dr = P.DeviceResult(batch.n, 0, records=records)
        parser.decode_device(db, dr)
        ft = FL.NewFlowTable(parser, 1 << 15)
        fid = ft.Insert(db, dr).cpu().numpy().view(np.uint32)
        recs, idx = ft.Export()
        st = ft.Stats()
        keys = torch.empty(batch.n * 64, dtype=torch.uint8, device="cuda")
        counts = (C.c_uint64 * 3)()
        b, r = db.c_batch(), dr.c_result()
        FL.check(FL.lib.gpd_flow_keys(ft.h, C.byref(b), C.byref(r), 3, 0, C.c_void_p(keys.data_ptr()),
                                      counts, ft._stream(None)), "gpd_flow_keys")
        m = int(sum(counts))
        kr = keys[:m * 64].cpu().numpy().view(FL.FLOW_KEY_DTYPE)
        torch.cuda.synchronize()
        got.append((fid, recs, idx, st, list(counts), np.sort(kr["seq"]), kr))
    a, b2 = got
    # which record a key lands in depends on the order racing claims resolve (two keys with one
    # home slot), so compare by key: each packet's record key, and the records themselves
    def per_packet_keys(fid, recs, idx):
        key_of = {int(ix): F.record_key(r) for r, ix in zip(recs, idx)}
        return [key_of.get(int(f)) if f < FL.FLOW_FULL else int(f) for f in fid]

    def by_key(recs):
        return sorted((F.record_key(r), int(r["first"]), int(r["last"]), int(r["packets"]), int(r["bytes"]))
                      for r in recs)
    assert per_packet_keys(a[0], a[1], a[2]) == per_packet_keys(b2[0], b2[1], b2[2])
    assert by_key(a[1]) == by_key(b2[1])
    assert a[3] == b2[3] and a[4] == b2[4] and np.array_equal(a[5], b2[5])
    assert np.array_equal(np.sort(a[6], order="seq"), np.sort(b2[6], order="seq"))
