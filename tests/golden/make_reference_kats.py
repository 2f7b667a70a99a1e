"""Regenerates reference_kats.json: the reference's own JUnit vectors
(SerializePackedTest.java:20-60, :93-105; SerializeTest.java:90-140, :173-189)
transcribed as data.  Run: python tests/golden/make_reference_kats.py"""
import json
from pathlib import Path

kats = []


def add(line, u, p):
    kats.append({"source": f"runtime/src/test/java/org/capnproto/SerializePackedTest.java:{line}",
                 "unpacked": bytes(u).hex(), "packed": bytes(p).hex()})


add(21, [], [])
add(23, [0] * 8, [0, 0])
add(25, [0, 0, 12, 0, 0, 34, 0, 0], [0x24, 12, 34])
add(27, [1, 3, 2, 4, 5, 7, 6, 8], [0xff, 1, 3, 2, 4, 5, 7, 6, 8, 0])
add(29, [0] * 8 + [1, 3, 2, 4, 5, 7, 6, 8], [0, 0, 0xff, 1, 3, 2, 4, 5, 7, 6, 8, 0])
add(32, [0, 0, 12, 0, 0, 34, 0, 0, 1, 3, 2, 4, 5, 7, 6, 8],
    [0x24, 12, 34, 0xff, 1, 3, 2, 4, 5, 7, 6, 8, 0])
add(35, [1, 3, 2, 4, 5, 7, 6, 8, 8, 6, 7, 4, 5, 2, 3, 1],
    [0xff, 1, 3, 2, 4, 5, 7, 6, 8, 1, 8, 6, 7, 4, 5, 2, 3, 1])
add(38, [1, 2, 3, 4, 5, 6, 7, 8] * 4 + [0, 2, 4, 0, 9, 0, 5, 1],
    [0xff, 1, 2, 3, 4, 5, 6, 7, 8, 3] + [1, 2, 3, 4, 5, 6, 7, 8] * 3 + [0xd6, 2, 4, 9, 5, 1])
add(42, [1, 2, 3, 4, 5, 6, 7, 8, 1, 2, 3, 4, 5, 6, 7, 8, 6, 2, 4, 3, 9, 0, 5, 1,
         1, 2, 3, 4, 5, 6, 7, 8, 0, 2, 4, 0, 9, 0, 5, 1],
    [0xff, 1, 2, 3, 4, 5, 6, 7, 8, 3, 1, 2, 3, 4, 5, 6, 7, 8, 6, 2, 4, 3, 9, 0, 5, 1,
     1, 2, 3, 4, 5, 6, 7, 8, 0xd6, 2, 4, 9, 5, 1])
add(46, [8, 0, 100, 6, 0, 1, 1, 2] + [0] * 24 + [0, 0, 1, 0, 2, 0, 3, 1],
    [0xed, 8, 100, 6, 1, 1, 2, 0, 2, 0xd4, 1, 2, 3, 1])
add(49, [0, 0, 0, 0, 2, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 0] + [0] * 8, [0x10, 2, 0x40, 1, 0, 0])
add(52, [0] * (8 * 200), [0, 199])
ones = [1] * (10 + 8 * 199)
ones[0], ones[9] = 255, 199
add(54, [1] * (8 * 200), ones)

errors = [
    {"source": "runtime/src/test/java/org/capnproto/SerializePackedTest.java:93-98",
     "what": "SerializePacked.read of an empty stream -> DecodeException", "packed": ""},
    {"source": "runtime/src/test/java/org/capnproto/SerializePackedTest.java:100-105",
     "what": "segment 0 claims 127 words, 7-byte input -> DecodeException",
     "packed": bytes([17, 0, 127, 0, 0, 0, 0]).hex()},
]
framing = []
for nseg, line in [(1, 90), (2, 97), (3, 109), (4, 124)]:
    table = [nseg - 1] + list(range(nseg))
    if len(table) % 2:
        table.append(0)
    raw = b"".join(int(v).to_bytes(4, "little") for v in table)
    for i in range(nseg):
        raw += b"".join(int(i).to_bytes(8, "little") for _ in range(i))
    framing.append({"source": f"runtime/src/test/java/org/capnproto/SerializeTest.java:{line}",
                    "segments": nseg, "unpacked_stream": raw.hex()})
overflow = [
    {"source": "runtime/src/test/java/org/capnproto/SerializeTest.java:173-180",
     "unpacked_stream": bytes([0, 0, 0, 0, 255, 255, 255, 0x8f]).hex()},
    {"source": "runtime/src/test/java/org/capnproto/SerializeTest.java:182-189",
     "unpacked_stream": bytes([1, 0, 0, 0, 1, 0, 0, 0, 255, 255, 255, 0x8f, 0, 0, 0, 0]).hex()},
]
out = Path(__file__).with_name("reference_kats.json")
json.dump({"note": "Vectors transcribed (data only) from the reference's JUnit tests; see 'source'.",
           "kats": kats, "decode_errors": errors, "framing": framing, "size_overflow": overflow},
          open(out, "w"), indent=1)
