"""Round 6 probe: can the two-pass encoder's second read of U come from the
Infinity Cache (256 MiB) when sub-batches are pipelined across streams, so
that the size pass of sub-batch k+1 runs WHILE the emit pass of sub-batch k
re-reads its words (round 5's r5AD ran the sub-batches one after another and
under-filled the chip)?  K contexts on K streams take sub-batches round-robin
(each cpk_encode_batch: gate, size pass, scan, emit, two passes forced);
every sub-batch's packed bytes are checked against the whole batch's.
Timing probe for DESIGN.md; not the bench metric.
usage: python tools/r6/mall_pipeline.py  (MP_N pieces, MP_CFG density, MP_SUBS, MP_K)"""
import os
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(REPO / "capnproto-java_amd")]
os.environ["CPK_ENCODER"] = "4"
import numpy as np  # noqa: E402
import torch  # noqa: E402
import capnp_packed as cp  # noqa: E402

n = int(os.environ.get("MP_N", "262144"))
cfg = int(os.environ.get("MP_CFG", "3"))
W = 8192
subs = [int(a) for a in os.environ.get("MP_SUBS", "4096,2048,1024,512").split(",")]
Ks = [int(a) for a in os.environ.get("MP_K", "2,3,4").split(",")]
swo = np.arange(0, (n + 1) * W, W, dtype=np.uint64)
d_swo = torch.from_numpy(swo.astype(np.int64)).cuda()
d_in = torch.empty(n * W, dtype=torch.int64, device="cuda")
cap = cp.batch_capacity(swo)
ctxs = [cp.Context(0) for _ in range(max(Ks))]
streams = [torch.cuda.Stream() for _ in range(max(Ks))]
ctx = ctxs[0]
ctx.generate(cp.preset(cfg), d_swo, d_in)
d_pk = torch.empty((cap + 255) // 256 * 256 + 256 * (n // min(subs) + 1), dtype=torch.uint8, device="cuda")
d_off = torch.empty(n + 1, dtype=torch.int64, device="cuda")
torch.cuda.synchronize()
U = n * W * 8


def timed(fn, reps=3):
    ts = []
    for r in range(reps + 1):
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        for s in streams:
            torch.cuda.current_stream().wait_stream(s)
        b.record()
        torch.cuda.synchronize()
        if r:
            ts.append(a.elapsed_time(b))
    return float(np.median(ts)), float(min(ts)), float(max(ts))


t_full = timed(lambda: ctx.encode_batch(d_in, d_swo, W, d_pk, d_off))
off_full = d_off.cpu().numpy().copy()
P = int(off_full[-1])
ref = d_pk[:P].clone()
print(f"{n} pieces x {W * 8 // 1024} KiB (config-{cfg} density), U = {U / 2**30:.1f} GiB, P/U = {P / U:.4f}")
print(f"  whole batch, two passes: {t_full[0]:8.2f} ms (min {t_full[1]:.2f} max {t_full[2]:.2f})", flush=True)
for S in subs:
    k = n // S
    sz = np.diff(off_full[::S])
    pos = np.concatenate([[0], np.cumsum((sz + 255) // 256 * 256)]).astype(np.int64)
    offs = [torch.empty(S + 1, dtype=torch.int64, device="cuda") for _ in range(k)]
    swos = [d_swo[j * S:(j + 1) * S + 1] - int(swo[j * S]) for j in range(k)]
    for K in Ks:
        def run():
            for j in range(k):
                c, s = ctxs[j % K], streams[j % K]
                with torch.cuda.stream(s):
                    c.encode_batch(d_in[j * S * W:], swos[j], W, d_pk[int(pos[j]):], offs[j], stream=s)
        t = timed(run)
        bad = 0
        for j in range(k):
            a = int(off_full[j * S]); L = int(sz[j])
            if not torch.equal(d_pk[int(pos[j]):int(pos[j]) + L], ref[a:a + L]):
                bad += 1
        print(f"  sub-batches of {S:6d} pieces ({S * W * 8 / 2**20:6.0f} MiB) on {K} streams: {t[0]:8.2f} ms"
              f" (min {t[1]:.2f} max {t[2]:.2f})  x{t[0] / t_full[0]:.3f}  bad={bad}", flush=True)
