"""Generate tests/golden/defrag_vectors.json (the F4 fragment hand-off fixtures).

Run in the build container only (it reads /root/reference as text):
    python tests/golden/make_defrag_vectors.py [/root/reference]

What it writes is DATA: the eight Ethernet/IPv4/ICMP fragments ip4defrag's tests feed the
defragmenter (ip4defrag/defrag_test.go testPing1Frag1..4, testPing2Frag1..4, extracted from
their byte literals), the facts those tests assert about them, and the IPv4 header fields of the
tests that build layers.IPv4 structs instead of frames (TestNotFrag, TestDefragTooSmall,
TestDefragFragmentOffset, TestDefragMaxSize) with the outcome each asserts.
"""
import json
import os
import re
import sys

REF = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))
PATH = "ip4defrag/defrag_test.go"


def line_of(path, anchor):
    src = open(os.path.join(REF, path)).read()
    return src[:src.index(anchor)].count("\n") + 1


def frame_at(anchor):
    """The `[]byte{...}` literal at `anchor`; its /* ascii */ comments (which hold braces) removed."""
    src = re.sub(r"/\*.*?\*/", "", open(os.path.join(REF, PATH)).read(), flags=re.S)
    i = src.index(anchor) + len(anchor)
    body = src[i:src.index("}", i)]
    return bytes(int(t, 16) for t in re.findall(r"0x([0-9a-fA-F]{1,2})", body))


def main():
    names = [f"testPing{p}Frag{f}" for p in (1, 2) for f in (1, 2, 3, 4)]
    frames = {}
    for nm in names:
        anchor = f"var {nm} = []byte{{"
        frames[nm] = {"hex": frame_at(anchor).hex(), "source": f"{PATH}:{line_of(PATH, anchor)}"}
    doc = {
        "frames": frames,
        "asserted": {
            # TestDefragPing1 / PingMultipleFrags / Ping1and2: each frame decodes without error
            # (gentestDefrag :262-266), every fragment but the completing one returns nil, the
            # datagram is the frames' bytes [34:] concatenated, 4508 bytes (:49-61, :78-90)
            "payload_from": 34,
            "datagram_payload_len": 4508,
            "completing": {"ping1": "testPing1Frag4", "ping2_after_ping1_and2_order": "testPing2Frag2"},
            "ping1_and2_order": ["testPing1Frag1", "testPing1Frag3", "testPing2Frag3", "testPing2Frag4",
                                 "testPing1Frag2", "testPing2Frag1", "testPing1Frag4", "testPing2Frag2"],
            # TestDefragIDField :245-259: the reassembled Id is BigEndian(testPing1Frag1[18:])
            "id_offset_in_frame": 18,
            "source": f"{PATH}:{line_of(PATH, 'func TestDefragPing1(')}-{line_of(PATH, 'func gentestDefrag(')}",
        },
        # layers.IPv4 structs the tests build (IHL 5 unless absent = 0); `error` = DefragIPv4
        # returned a non-nil error; `unchanged` = it returned the layer itself
        "structs": [
            {"test": "TestNotFrag", "line": line_of(PATH, "func TestNotFrag("), "ihl": 0, "length": 0,
             "flags": 2, "frag_offset": 0, "id": 0, "error": False, "unchanged": True},
            {"test": "TestDefragTooSmall ip1", "line": line_of(PATH, "func TestDefragTooSmall("), "ihl": 5,
             "length": 27, "flags": 1, "frag_offset": 0, "id": 0xcc, "error": True},
            {"test": "TestDefragTooSmall ip1.Length++", "line": line_of(PATH, "ip1.Length++"), "ihl": 5,
             "length": 28, "flags": 1, "frag_offset": 0, "id": 0xcc, "error": False},
            {"test": "TestDefragFragmentOffset ip1", "line": line_of(PATH, "func TestDefragFragmentOffset("),
             "ihl": 5, "length": 512, "flags": 1, "frag_offset": 0, "id": 0xcc, "error": False},
            {"test": "TestDefragFragmentOffset ip2", "line": line_of(PATH, "ip2.FragOffset = 8184"), "ihl": 5,
             "length": 512, "flags": 1, "frag_offset": 8184, "id": 0xcc, "error": True},
            {"test": "TestDefragMaxSize ip1", "line": line_of(PATH, "func TestDefragMaxSize("), "ihl": 5,
             "length": 65535, "flags": 1, "frag_offset": 0, "id": 0xcc, "error": False},
            {"test": "TestDefragMaxSize ip2", "line": line_of(PATH, "ip2.FragOffset = 1"), "ihl": 5,
             "length": 28, "flags": 1, "frag_offset": 1, "id": 0xcc, "error": False},
        ],
        "struct_addrs": {"src": [1, 1, 1, 1], "dst": [2, 2, 2, 2]},
    }
    with open(os.path.join(OUT, "defrag_vectors.json"), "w") as f:
        json.dump(doc, f, indent=1)
        f.write("\n")


if __name__ == "__main__":
    main()
