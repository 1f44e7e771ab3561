"""Does config 2's launch time depend on where the buffers land?  One process allocates the batch
and the record array several times over (keeping earlier copies alive so each trial gets new
addresses), settles, and times 50 launches per trial.  Prints one line per trial.

    python tools/mode_probe.py [trials] [config] [tune;tune;...]   (tune: "split=2,grid_rounds=1")
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    import torch
    from gopacket_amd import layers as L
    from gopacket_amd import parser as P
    trials = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    cfg = sys.argv[2] if len(sys.argv) > 2 else "udp64"
    tunes = sys.argv[3].split(";") if len(sys.argv) > 3 else [""]
    torch.cuda.set_device(0)
    _, n = bench.CONFIGS[cfg]
    batch = bench.make_batch(cfg, n, 0)
    layers = [P.Ethernet(), P.Dot1Q(), P.IPv4(), P.IPv6(), P.IPv6ExtensionSkipper(), P.TCP(),
              P.UDP(), P.VXLAN(), P.Payload(), P.Fragment()]
    parser = P.NewDecodingLayerParser(L.LayerTypeEthernet, *layers, device=0)
    stream = torch.cuda.current_stream(0)
    keep = []
    cross = os.environ.get("MODE_CROSS") == "1"  # trials x trials: every batch copy with every record array
    dbs = [P.DeviceBatch(batch, 0) for _ in range(trials)] if cross else []
    drs = [P.DeviceResult(n, 0, ext=False, hdr_off=False, records=True) for _ in range(trials)] if cross else []
    desc = os.environ.get("MODE_DESC") == "1"  # trials x trials: every packet-bytes copy with every offset/caplen copy
    if desc:
        import copy
        dbs = [P.DeviceBatch(batch, 0) for _ in range(trials)]
        drs = [P.DeviceResult(n, 0, ext=False, hdr_off=False, records=True)]
    pack = os.environ.get("MODE_PACK") == "1"  # offsets and caplens in one allocation, caplen at n + pad words
    pads = [int(x) << 18 for x in os.environ.get("MODE_PADS", "0,1,2").split(",")]  # in MiB
    if pack:
        base_db = P.DeviceBatch(batch, 0)
        drs = [P.DeviceResult(n, 0, ext=False, hdr_off=False, records=True)]
    for t in range(trials * len(pads) if pack else trials * trials if cross or desc else trials):
        if pack:
            import copy
            pad = pads[t % len(pads)]
            buf = torch.empty(2 * n + pad, dtype=torch.int32, device="cuda:0")
            buf[:n].copy_(base_db.offset)
            buf[n + pad:].copy_(base_db.caplen)
            keep.append(buf)
            db = copy.copy(base_db)
            db.offset, db.caplen = buf[:n], buf[n + pad:]
            dr = drs[0]
        elif desc:
            db = copy.copy(dbs[t // trials])
            if os.environ.get("MODE_OC") == "1":  # every offset copy with every caplen copy
                db.offset, db.caplen = dbs[t // trials].offset, dbs[t % trials].caplen
                db.data = dbs[0].data
            else:
                db.offset, db.caplen = dbs[t % trials].offset, dbs[t % trials].caplen
            dr = drs[0]
        elif cross:
            db, dr = dbs[t // trials], drs[t % trials]
        else:
            db = P.DeviceBatch(batch, 0)
            if os.environ.get("MODE_ALT") == "1" and t % 2:  # odd trials: separate offset / caplen allocations (the pre-r06 layout)
                db.offset, db.caplen = db.offset.clone(), db.caplen.clone()
            dr = P.DeviceResult(n, 0, ext=False, hdr_off=False, records=True)
            keep.append((db, dr))
        for tu in tunes:
            parser.Tuning = {k: int(v) for k, v in (kv.split("=") for kv in tu.split(",") if kv)}
            bench.settle(lambda: parser.decode_device(db, dr, stream), 250, 0)
            ms = []
            for rep in range(3):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                for _ in range(50):
                    parser.decode_device(db, dr, stream)
                e1.record(stream)
                torch.cuda.synchronize(0)
                ms.append(round(e0.elapsed_time(e1) / 50, 4))
            st = dr.records.view(torch.int32)[0::8].cpu().numpy()
            print(json.dumps({"trial": t, "tune": tu, "layout": "separate" if int(db.caplen.data_ptr()) - int(db.offset.data_ptr()) != 4 * n else "packed", "ms": ms, "errors": int(((st & 3) != 0).sum()),
                              "data": hex(db.data.data_ptr()), "off": hex(db.offset.data_ptr()), "cap": hex(db.caplen.data_ptr()), "rec": hex(dr.records.data_ptr())}),
                  flush=True)


if __name__ == "__main__":
    main()
