"""Step-by-step GPU bring-up probe (prints after every step, flushes)."""
import sys, time
from pathlib import Path
REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO / "capnproto-java_amd"), str(REPO / "oracle")]
import numpy as np

def log(*a):
    print(f"[{time.strftime('%H:%M:%S')}]", *a, flush=True)

log("import torch")
import torch
log("cuda", torch.cuda.is_available(), torch.cuda.get_device_name(0))
import capnp_packed as cp, oracle
ctx = cp.Context(0)
log("ctx ok")
step = sys.argv[1] if len(sys.argv) > 1 else "all"
def swo_of(sizes):
    return np.concatenate([[0], np.cumsum(sizes)]).astype(np.uint64)
for sizes in ([1], [2], [8], [200], [8192], [8192] * 4, [3, 0, 8192, 17] * 8):
    swo = swo_of(sizes)
    data = oracle.generate(oracle.preset(2), swo)
    log("encode", sizes[:4], len(sizes))
    pk, off = ctx.encode_host(data, swo)
    ref, roff = oracle.pack_batch(data, swo)
    log("  enc equal:", np.array_equal(pk, ref), np.array_equal(off, roff), len(pk), len(ref))
    if not np.array_equal(pk, ref):
        d = np.nonzero(pk[:min(len(pk), len(ref))] != ref[:min(len(pk), len(ref))])[0]
        log("  first diff at", d[:5], "offsets", off[:5], roff[:5])
    log("decode")
    dec, st = ctx.decode_host(ref, roff, swo)
    log("  dec status", np.unique(st), "equal", np.array_equal(dec, data))
log("done")
