"""Generate tests/golden/refsweep.json: every Ethernet frame a reference layers/*_test.go
decodes with gopacket.NewPacket(...) and asserts with checkLayers(p, [...]) — the packet
bytes (extracted from the Go byte literal as data) and the asserted layer list.

Run in the build container only (it reads /root/reference as text):
    python tests/golden/make_refsweep.py [/root/reference]

tests/test_refsweep.py turns each assertion into the DecodingLayerParser expectation it
implies for this engine's decoder set (the asserted prefix up to the first layer this
engine has no decoder for, then UnsupportedLayerType of that layer) and checks the oracle
and the GPU path against it.
"""
import glob
import json
import os
import re
import sys

REF = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))


def byte_literal(src, j):
    """Bytes of the []byte{...} literal whose '{' is at src[j-1]."""
    depth, k = 1, j
    while depth:
        if src[k] == "{":
            depth += 1
        elif src[k] == "}":
            depth -= 1
        k += 1
    body = re.sub(r"//[^\n]*", "", src[j:k - 1])
    return bytes(int(t, 16) for t in re.findall(r"0x([0-9a-fA-F]{1,2})", body))


def main():
    cases = []
    for path in sorted(glob.glob(os.path.join(REF, "layers", "*_test.go"))):
        src = open(path).read()
        rel = os.path.relpath(path, REF)
        # byte-literal variables: top level `var X = []byte{` and local `X := []byte{`
        lits = {}
        for m in re.finditer(r"(?:var\s+(\w+)\s*=|(\w+)\s*:=)\s*\[\]byte\{", src):
            name = m.group(1) or m.group(2)
            lits.setdefault(name, []).append((m.start(), byte_literal(src, m.end())))
        for m in re.finditer(r"(\w+)\s*:?=\s*gopacket\.NewPacket\((\w+),\s*LinkTypeEthernet,", src):
            pvar, var = m.group(1), m.group(2)
            if var not in lits:
                continue
            # the literal in scope: the last definition before the call, inside the same
            # function or at top level (`var`)
            fstart = src.rfind("\nfunc ", 0, m.start())
            defs = [d for d in lits[var] if d[0] < m.start() and
                    (d[0] > fstart or src.startswith("var", d[0]))]
            if not defs:
                continue
            data = defs[-1][1]
            nxt = src.find("gopacket.NewPacket(", m.end())
            region = src[m.end(): nxt if nxt > 0 else len(src)]
            c = re.search(r"checkLayers\(" + re.escape(pvar) + r",\s*\[\]gopacket\.LayerType\{([^}]*)\}", region)
            if not c or not data:
                continue
            names = [t.strip().replace("gopacket.", "").replace("LayerType", "")
                     for t in c.group(1).split(",") if t.strip()]
            line = src[:m.start()].count("\n") + 1
            cline = src[:m.end() + c.start()].count("\n") + 1
            cases.append({"name": f"{os.path.basename(rel)[:-3]}:{line}:{var}", "source": f"{rel}:{line}",
                          "pinned_by": f"{rel}:{cline} checkLayers", "hex": data.hex(),
                          "asserted": names})
    out = {"generated_by": "tests/golden/make_refsweep.py", "reference": "google/gopacket (read as text)",
           "cases": cases}
    with open(os.path.join(OUT, "refsweep.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(f"{len(cases)} asserted frames -> {OUT}/refsweep.json")


if __name__ == "__main__":
    main()
