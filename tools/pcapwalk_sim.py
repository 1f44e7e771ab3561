"""Diagnostic (CPU, not product): a Python restatement of gpd_pcapwalk.hip's speculation and
stitch rules (pw_walk / pw_stitch), run over synthetic captures to count the segments whose
speculation the true walk would miss (each one sends a chunk to the host walk).

    python tools/pcapwalk_sim.py
"""
import sys, struct
import numpy as np
import os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, 'tests'))
from gopacket_amd import pcap as NP, synth
from gopacket_amd.batch import PAD
SEG = 2048; snap = 262144
def sim(d, entry, be, nano, last=True, maxfail=5):
    T = len(d); own = T
    fmt = '>I' if be else '<I'
    def rd(p, b=be): return struct.unpack_from('>I' if b else '<I', d, p)[0]
    def step(p):
        if p + 16 > T: return None
        c = rd(p+8); w = rd(p+12)
        if c > snap or c > w: return None
        if p + 16 + c > T: return None
        return c
    def plaus(x):
        pt = (0, 0)
        for k in range(8):
            if x >= T: return k > 0 and (x == T if last else True)
            c = step(x)
            if c is None: return False
            if (rd(x,False)|rd(x+4,False)|rd(x+8,False)|rd(x+12,False)) == 0: return False
            if rd(x+4) >= (10**9 if nano else 10**6): return False
            t = (rd(x), rd(x+4))
            if t < pt: return False
            pt = t
            x += 16 + c
        return True
    nseg = (own + SEG - 1)//SEG
    st=[None]*nseg; ex=[0]*nseg; ct=[0]*nseg; bad=[0]*nseg
    for s in range(nseg):
        lo = s*SEG; hi = min(lo+SEG, own); start=None
        if lo <= entry < hi: start = entry
        elif entry < lo:
            lim = min(hi, lo+16+snap+1)
            x = lo
            while x < lim:
                if plaus(x):
                    best = x; bc = rd(x+8)
                    for y in range(x+1, min(x+8, lim)):
                        if plaus(y) and rd(y+8) < bc: best = y; bc = rd(y+8)
                    if best >= 4 and plaus(best-4) and rd(best-4+8) <= bc:
                        x = best + 1; continue
                    start = best; break
                x += 1
        p = start; c=0; b=0
        if start is not None:
            while p < hi:
                cc = step(p)
                if cc is None: b=1; break
                c+=1; p += 16+cc
        st[s]=start; ex[s]=p if start is not None else 0; ct[s]=c; bad[s]=b
    prev=None; fails=0
    for s in range(nseg):
        lo=s*SEG; hi=min(lo+SEG, own)
        at = entry if prev is None else ex[prev]
        if st[s] is not None:
            if st[s] != at or bad[s]:
                if fails < maxfail: print("seg", s, "start", st[s], "at", at, "bad", bad[s], [rd(st[s]+4*i) for i in range(4)], [rd(at+4*i) for i in range(4)])
                fails += 1
            prev = s
        elif lo <= at < hi:
            if fails < maxfail: print("NONE seg", s, "at", at, lo, hi)
            fails += 1
    print("fails", fails, "nseg", nseg)
# udp64 capture as in pcie_probe (records=True): first 2^16 records
n = 1 << 16
cap = np.empty(24 + 80 * n + PAD, np.uint8)
cap[:24] = np.frombuffer(struct.pack("<IHHiIII", 0xA1B2C3D4, 2, 4, 0, 0, 262144, 1), np.uint8)
synth.udp64_native(cap[24:24 + 80 * n], 0, n, records=True, nthreads=8)
sim(cap[16:24+80*n].tobytes(), 8, False, False)
# BE nano capture from the test
from test_pcap_devwalk_gpu import _capture
c = _capture(1 << 16, 0x54)
dl = c.shape[0] - PAD
pc = NP.index(c, data_len=dl)
be = c.copy()
be[:4] = np.frombuffer(struct.pack("<I", 0x4D3CB2A1), np.uint8)
be[4:24] = np.frombuffer(struct.pack(">HHiIII", 2, 4, 0, 0, 262144, 1), np.uint8)
hdr = pc.batch.offset.astype(np.int64) - 16
for k in range(4):
    idx = hdr[:, None] + 4 * k + np.arange(4)[None, :]
    be[idx] = be[idx][:, ::-1]
sim(be[16:dl].tobytes(), 8, True, True)
sim(c[16:dl].tobytes(), 8, False, False)
inner = NP.synth_capture(synth.make_udp64(40))[24:24 + 40 * 80].tobytes()
eth = bytes(12) + b"\x08\x00" + bytes([0x45]) + bytes(19)
from gopacket_amd.batch import PacketBatch
pk = [eth + inner if i % 3 == 0 else eth + bytes(range(40)) for i in range(6000)]
cc = NP.synth_capture(PacketBatch.from_packets(pk))
sim(cc[16:cc.shape[0]-PAD].tobytes(), 8, False, False)
