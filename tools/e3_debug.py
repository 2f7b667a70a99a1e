"""GPU debug aid: encode the reference KATs and random batches through the C
ABI and print the first difference against the oracle."""
import json
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO / "capnproto-java_amd"), str(REPO / "oracle"), str(REPO / "tests")]
import capnp_packed as cp  # noqa: E402
import oracle  # noqa: E402

ctx = cp.Context(0)
GOLD = json.loads((REPO / "tests" / "golden" / "reference_kats.json").read_text())
bad = 0
for k in GOLD["kats"]:
    u, p = bytes.fromhex(k["unpacked"]), bytes.fromhex(k["packed"])
    if not u:
        continue
    pk, off = ctx.encode_host(np.frombuffer(u, np.uint8), np.array([0, len(u) // 8], np.uint64))
    if pk.tobytes() != p:
        bad += 1
        print("KAT", k["source"], "words", len(u) // 8, "\n  want", p.hex()[:120], "\n  got ", pk.tobytes().hex()[:120], off)
print("kats bad", bad)


def first_diff(a, b):
    n = min(len(a), len(b))
    d = np.nonzero(a[:n] != b[:n])[0]
    return int(d[0]) if d.size else (n if len(a) != len(b) else -1)


from test_gpu_parity import _random_words, _swo  # noqa: E402
rng = np.random.default_rng(1)
for mix, probs in {"uniform": [.25, .25, .25, .25], "dense": [.01, .7, .285, .005],
                   "sparse": [.85, .05, .05, .05]}.items():
    for trial in range(3):
        sizes = [int(x) for x in rng.integers(0, 9000, size=12)]
        data = np.concatenate([_random_words(rng, s, probs) for s in sizes]).astype(np.uint8)
        swo = _swo(sizes)
        pk, off = ctx.encode_host(data, swo)
        opk, ooff = oracle.pack_batch(data, swo)
        if not (np.array_equal(off, ooff) and np.array_equal(pk, opk)):
            i = next((j for j in range(len(off)) if off[j] != ooff[j]), None)
            fd = first_diff(pk, opk)
            # which piece / word holds the first differing byte
            pc = int(np.searchsorted(ooff, fd, side="right") - 1)
            print(mix, trial, "sizes", sizes, "first off diff", i, "first byte diff", fd, "piece", pc,
                  "piece off", int(ooff[pc]) if pc < len(ooff) else None)
            lo = max(fd - 16, 0)
            print("  want", opk[lo:fd + 24].tobytes().hex())
            print("  got ", pk[lo:fd + 24].tobytes().hex())
            break
    else:
        print(mix, "ok")
