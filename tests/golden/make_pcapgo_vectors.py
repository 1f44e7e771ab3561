"""Generate tests/golden/pcapgo_vectors.json: the capture bytes pcapgo/read_test.go feeds to
pcapgo.NewReader / ReadPacketData and what those tests assert (DATA only), plus a copy of
pcap/test_loopback.pcap.  Run in the build container only (reads /root/reference as text):
    python tests/golden/make_pcapgo_vectors.py [/root/reference]
"""
import json
import os
import shutil
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import make_golden as MG  # noqa: E402

REF = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
MG.REF = REF
OUT = os.path.dirname(os.path.abspath(__file__))
F = "pcapgo/read_test.go"


def case(fn, expect):
    b = MG.go_bytes_at(F, "func " + fn + "(")
    return {"name": fn, "source": f"{F}:{MG.line_of(F, 'func ' + fn + '(')}", "hex": b.hex(),
            "expect": expect}


# 2014-09-18 12:13:14 UTC = 1411042394 s (read_test.go asserts the time.Date values)
T0 = 1411042394 * 1_000_000_000
cases = [
    case("TestCreatePcapReader", {"header_ok": True, "big_endian": 0, "nano": 0, "snaplen": 65535,
                                  "linktype": 1}),
    case("TestCreatePcapReaderBigEndian", {"header_ok": True, "big_endian": 1, "nano": 0,
                                           "snaplen": 65535, "linktype": 1}),
    case("TestCreatePcapReaderFail", {"header_ok": False}),
    case("TestPacket", {"header_ok": True, "packets": [{"ts_ns": T0 + 1000, "caplen": 4, "length": 8,
                                                         "data": "01020304"}]}),
    case("TestPacketNano", {"header_ok": True, "packets": [{"ts_ns": T0 + 1, "caplen": 4, "length": 8,
                                                             "data": "01020304"}]}),
    case("TestGzipPacket", {"gzip": True, "header_ok": True,
                            "packets": [{"ts_ns": T0 + 1000, "caplen": 4, "length": 8,
                                         "data": "01020304"}]}),
    case("TestTruncatedGzipPacket", {"gzip": True, "header_ok": False}),
    case("TestPacketBufferReuse", {"header_ok": True, "packets_data": ["01020304", "01020304"]}),
]
json.dump({"cases": cases}, open(os.path.join(OUT, "pcapgo_vectors.json"), "w"), indent=1)
shutil.copy(os.path.join(REF, "pcap", "test_loopback.pcap"), os.path.join(OUT, "test_loopback.pcap"))
print(len(cases), "cases")
