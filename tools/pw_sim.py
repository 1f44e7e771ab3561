"""CPU restatement of the device pcap walk's per-segment speculation (gpd_pcapwalk.hip pw_walk)
over a stretch of config 5's synthetic capture: which 2-KiB segments start off the true record
chain, and what the bytes there look like.  Diagnostic for `device_walk_chunks` in bench.py's
replay line.  usage: python tools/pw_sim.py FIRST_RECORD [N_RECORDS]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gopacket_amd import synth  # noqa: E402

SEG, SNAP = 2048, 262144


def main():
    i0 = int(sys.argv[1])
    n = int(sys.argv[2]) if len(sys.argv) > 2 else (64 << 20) // 80
    phase = int(sys.argv[3]) if len(sys.argv) > 3 else 0  # segment starts at phase + k * 2 KiB
    d = np.zeros(n * 80 + 64, np.uint8)
    synth.udp64_native(d, i0, i0 + n, 0x5EED0002, records=True, nthreads=8)
    T = n * 80
    u32 = lambda x: (d[x].astype(np.uint32) | (d[x + 1].astype(np.uint32) << 8) |
                     (d[x + 2].astype(np.uint32) << 16) | (d[x + 3].astype(np.uint32) << 24))

    def plausible(x):
        ok = np.ones(x.shape, bool)
        psec = np.zeros(x.shape, np.uint32)
        pfrac = np.zeros(x.shape, np.uint32)
        for k in range(8):
            end = x >= T
            xs = np.minimum(x, T - 16)
            cap, wire = u32(xs + 8), u32(xs + 12)
            sec, frac = u32(xs), u32(xs + 4)
            step_ok = (x + 16 <= T) & (cap <= SNAP) & (cap <= wire) & (x.astype(np.int64) + 16 + cap <= T)
            nz = (sec | frac | cap | wire) != 0
            mono = ~((sec < psec) | ((sec == psec) & (frac < pfrac)))
            good = step_ok & nz & (frac < 1000000) & mono
            ok &= np.where(end, k > 0, good)
            psec, pfrac = sec, frac
            x = np.where(end, x, x + 16 + np.where(good, cap, 0))
        return ok

    nseg = T // SEG
    lo = phase + np.arange(1, nseg - 1, dtype=np.int64) * SEG  # (segment 0 holds the entry)
    start = np.full(lo.shape, -1, np.int64)
    x = lo.copy()
    todo = np.ones(lo.shape, bool)
    for _ in range(200):
        if not todo.any():
            break
        pl = np.zeros(lo.shape, bool)
        pl[todo] = plausible(x[todo])
        found = todo & pl
        # best of the 8 positions from x (the shortest record), and the 4-byte shift rule
        idx = np.nonzero(found)[0]
        for j in idx:
            xb = int(x[j])
            best, bc = xb, int(u32(np.array([xb + 8]))[0])
            for y in range(xb + 1, min(xb + 8, int(lo[j]) + SEG)):
                if plausible(np.array([y]))[0]:
                    c = int(u32(np.array([y + 8]))[0])
                    if c < bc:
                        best, bc = y, c
            if best >= 4 and plausible(np.array([best - 4]))[0] and int(u32(np.array([best + 4]))[0]) <= bc:
                x[j] = best + 1
                continue
            start[j] = best
            todo[j] = False
        x[todo & ~found] += 1
        x = np.minimum(x, lo + SEG)
        todo &= x < lo + SEG
    true_hdr = (start - 0) % 80 == 0
    bad = np.nonzero((start >= 0) & ~true_hdr)[0]
    print(f"records {i0}..{i0 + n} (segments at {phase} + k 2048): {len(lo)} segments, {len(bad)} start off the chain, "
          f"{int((start < 0).sum())} without a start")
    for j in bad[:8]:
        s = int(start[j])
        r = s - s % 80
        print(f"  segment {j + 1}: start {s} = record {i0 + r // 80} + {s % 80}; bytes there "
              f"{d[s:s + 16].tobytes().hex()} ; record header {d[r:r + 16].tobytes().hex()}")


if __name__ == "__main__":
    main()
