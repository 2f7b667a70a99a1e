"""Find the first piece/byte where the GPU encoder differs from the oracle."""
import sys
from pathlib import Path
REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO / "capnproto-java_amd"), str(REPO / "oracle"), str(REPO / "tests")]
import numpy as np
import capnp_packed as cp, oracle
from test_gpu_parity import _random_words, _swo
lib = sys.argv[1] if len(sys.argv) > 1 else None
if lib:
    cp.load(Path(lib))
ctx = cp.Context(0)
rng = np.random.default_rng(abs(hash("uniform")) % 2**32)
for trial in range(6):
    sizes = [int(x) for x in rng.integers(1, 8193, size=6)]
    data = np.concatenate([_random_words(rng, s, [.25, .25, .25, .25]) for s in sizes]).astype(np.uint8)
    swo = _swo(sizes)
    pk, off = ctx.encode_host(data, swo)
    opk, ooff = oracle.pack_batch(data, swo)
    for i in range(len(sizes)):
        a = pk[int(off[i]):int(off[i + 1])]; b = opk[int(ooff[i]):int(ooff[i + 1])]
        if not np.array_equal(a, b):
            d = int(np.nonzero(a != b)[0][0]) if len(a) == len(b) else -1
            print(f"trial {trial} piece {i} W={sizes[i]} base={int(off[i])} pad={int(off[i]) & 15} len={len(a)}/{len(b)} first diff byte {d}")
            if d >= 0:
                print("  gpu  ", a[max(0, d - 8):d + 24].tobytes().hex())
                print("  orcl ", b[max(0, d - 8):d + 24].tobytes().hex())
            break
    else:
        print(f"trial {trial}: all {len(sizes)} pieces equal")
