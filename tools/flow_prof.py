"""F3 launch split for rocprofv3 (diagnostic): 2^24 config-2 packets decoded once
with header offsets, then REPS rounds of  reset -> insert(new flows) -> insert(existing flows),
so a kernel trace / PMC pass sees the two cases' flow_insert_kernel and flow_verify_kernel
launches in a fixed order (tools/flow_prof_split.py attributes them).

    rocprofv3 --kernel-trace --stats -d OUT -- python3 tools/flow_prof.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

REPS = int(os.environ.get("FLOW_PROF_REPS", "6"))


def main():
    import torch
    from gopacket_amd import flows as FL
    from gopacket_amd import layers as L
    from gopacket_amd import parser as P
    from gopacket_amd import synth
    n = 1 << 24
    b = synth.make_udp64(n)
    p = P.NewDecodingLayerParser(L.LayerTypeEthernet, P.Ethernet(), P.Dot1Q(), P.IPv4(), P.IPv6(), P.TCP(),
                                 P.UDP(), P.Payload())
    db = P.DeviceBatch(b, 0)
    res = P.DeviceResult(n, 0, ext=False, hdr_off=True)
    s = torch.cuda.current_stream(0)
    p.decode_device(db, res, s)
    ft = FL.NewFlowTable(p, 1 << 25)
    fid = torch.empty(n, dtype=torch.int32, device="cuda:0")
    for _ in range(REPS):
        ft.Reset(s)
        ft.Insert(db, res, fid, 0, s)  # every packet a new flow
        ft.Insert(db, res, fid, n, s)  # every packet an existing flow (next sequence numbers)
    torch.cuda.synchronize()
    st = ft.Stats(s)
    print({k: st[k] for k in ("flows", "packets", "collisions", "full")}, flush=True)


if __name__ == "__main__":
    main()
