"""Does the two-pass encoder's second read of U come from the Infinity Cache
when a batch is encoded in sub-batches small enough for it (256 MiB)?
Config-3-density pieces (1 Mi x 64 KiB, 64 GiB), the two passes forced
(CPK_ENCODER=4); the batch encoded whole, then as consecutive sub-batches of
S pieces (each one cpk_encode_batch: gate, size pass, scan, emit), outputs
packed at 256-byte aligned offsets one after another; every sub-batch's
packed bytes checked against the whole batch's.  For DESIGN.md §5; not the
bench metric.  usage: python tools/mall_probe.py [S ...]"""
import os
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO / "capnproto-java_amd")]
os.environ["CPK_ENCODER"] = "4"
import numpy as np  # noqa: E402
import torch  # noqa: E402
import capnp_packed as cp  # noqa: E402

n = int(os.environ.get("MP_N", "1048576"))
W = 8192
subs = [int(a) for a in sys.argv[1:]] or [16384, 4096, 2048, 1024]
swo = np.arange(0, (n + 1) * W, W, dtype=np.uint64)
d_swo = torch.from_numpy(swo.astype(np.int64)).cuda()
d_in = torch.empty(n * W, dtype=torch.int64, device="cuda")
cap = cp.batch_capacity(swo)
ctx = cp.Context(0)
ctx.generate(cp.preset(3), d_swo, d_in)
d_pk = torch.empty((cap + 255) // 256 * 256 + 256 * (n // min(subs) + 1), dtype=torch.uint8, device="cuda")
d_off = torch.empty(n + 1, dtype=torch.int64, device="cuda")
torch.cuda.synchronize()
U = n * W * 8


def timed(fn, reps=3):
    ts = []
    for r in range(reps + 1):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        if r:
            ts.append(a.elapsed_time(b))
    return float(np.median(ts))


t_full = timed(lambda: ctx.encode_batch(d_in, d_swo, W, d_pk, d_off))
off_full = d_off.cpu().numpy().copy()
P = int(off_full[-1])
ref = d_pk[:P].clone()
print(f"{n} pieces x {W * 8 // 1024} KiB (config-3 density), U = {U / 2**30:.1f} GiB, P/U = {P / U:.4f}")
print(f"  whole batch, two passes:            {t_full:8.2f} ms  ({(2 * U + P) / t_full / 1e6:7.1f} GB/s of 2U+P traffic)")
for S in subs:
    k = n // S
    # sub-batch j's output at a 256-byte aligned offset after the previous ones
    sz = np.diff(off_full[::S]) if S < n else np.array([P])
    pos = np.concatenate([[0], np.cumsum((sz + 255) // 256 * 256)]).astype(np.int64)
    offs = [torch.empty(S + 1, dtype=torch.int64, device="cuda") for _ in range(k)]

    def run():
        for j in range(k):
            ctx.encode_batch(d_in, d_swo[j * S:(j + 1) * S + 1], W, d_pk[int(pos[j]):], offs[j])

    t = timed(run, reps=2)
    ok = True
    for j in (0, k // 2, k - 1):  # spot checks against the whole batch's bytes
        a, b = int(off_full[j * S]), int(off_full[(j + 1) * S])
        ok &= bool(torch.equal(d_pk[int(pos[j]):int(pos[j]) + (b - a)], ref[a:b]))
    print(f"  {k:6d} sub-batches of {S:6d} pieces ({S * W * 8 / 2**20:6.0f} MiB): {t:8.2f} ms"
          f"  ({U / t / 1e6:7.1f} GB/s of U; same bytes: {ok})", flush=True)
