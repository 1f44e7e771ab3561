"""Time gpd_ip4_fragments (the F4 hand-off) after a device decode: config 2's
2^24 x 64-B UDP batch (no fragments: the count pass alone) and 2^22 frames of the traffic mix
(3 % fragments).  HIP events on the call's stream; prints one JSON line per workload."""
import json
import sys
import os

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from gopacket_amd import layers as L, synth  # noqa: E402
from gopacket_amd import parser as P, defrag as DF  # noqa: E402


def run(name, batch, reps=20):
    p = P.NewDecodingLayerParser(L.LayerTypeEthernet)
    p._mask = 0xFFF
    db = P.DeviceBatch(batch, 0)
    dr = P.DeviceResult(batch.n, 0, records=True)
    p.decode_device(db, dr)
    out = torch.empty(batch.n * 32, dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream()
    for _ in range(3):
        DF.IPv4Fragments(p, db, dr, out=out)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ms = []
    for _ in range(reps):
        e0.record(s)
        _, cnt = DF.IPv4Fragments(p, db, dr, out=out)
        e1.record(s)
        e1.synchronize()
        ms.append(e0.elapsed_time(e1))
    ms.sort()
    print(json.dumps({"workload": name, "n": batch.n, "fragments": cnt, "ms_median": round(ms[len(ms) // 2], 4),
                      "ms_min": round(ms[0], 4), "gpps": round(batch.n / ms[len(ms) // 2] / 1e6, 2)}), flush=True)


if __name__ == "__main__":
    run("udp64 2^24", synth.make_udp64(1 << 24))
    run("traffic mix 2^22", synth.make_traffic_mix(1 << 22))
