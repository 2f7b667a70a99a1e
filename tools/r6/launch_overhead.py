"""Per-call host time of a small device-resident cpk_decode_batch: the
default (dec_gate_kernel + three decoder grids, the two not picked return at
their first instruction) against one forced decoder (one grid), and the same
for cpk_decode_host of one small piece.  ADVICE r5: the cost of the extra
launches for small and chunked host decodes."""
import os
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(REPO / "capnproto-java_amd"), str(REPO / "oracle")]
import numpy as np
import torch
import capnp_packed as cp

res = {}
for dec in ("3", "1"):
    os.environ["CPK_DECODER"] = dec
    ctx = cp.Context(0)
    for n, w in ((1, 128), (4, 1024), (64, 1024)):
        swo = np.arange(0, (n + 1) * w, w, dtype=np.uint64)
        gp = cp.preset(2)
        d_swo = torch.from_numpy(swo.astype(np.int64)).cuda()
        d_in = torch.empty(int(swo[-1]), dtype=torch.int64, device="cuda")
        ctx.generate(gp, d_swo, d_in)
        d_pk = torch.empty((cp.batch_capacity(swo) + 255) // 256 * 256, dtype=torch.uint8, device="cuda")
        d_off = torch.empty(n + 1, dtype=torch.int64, device="cuda")
        d_out = torch.empty_like(d_in)
        d_st = torch.empty(n, dtype=torch.int32, device="cuda")
        ctx.encode_batch(d_in, d_swo, w, d_pk, d_off)
        torch.cuda.synchronize()
        for _ in range(20):
            ctx.decode_batch(d_pk, d_off, d_swo, d_out, d_st)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(500):
            ctx.decode_batch(d_pk, d_off, d_swo, d_out, d_st)
            torch.cuda.synchronize()
        dev = (time.perf_counter() - t0) / 500 * 1e6
        assert torch.equal(d_out, d_in) and int(d_st.abs().sum()) == 0
        pk = d_pk[: int(d_off[-1])].cpu().numpy()
        off = d_off.cpu().numpy().astype(np.uint64)
        for _ in range(20):
            ctx.decode_host(pk, off, swo)
        t0 = time.perf_counter()
        for _ in range(500):
            ctx.decode_host(pk, off, swo)
        host = (time.perf_counter() - t0) / 500 * 1e6
        res[(dec, n, w)] = (dev, host)
    ctx.close()
print("# pieces x words: device decode_batch + sync (us), decode_host (us); decoder 3 = gate + 3 grids, 1 = one grid")
for n, w in ((1, 128), (4, 1024), (64, 1024)):
    a, b = res[("3", n, w)], res[("1", n, w)]
    print(f"{n:4d} x {w:5d}: gated {a[0]:7.1f} / {a[1]:7.1f}   one grid {b[0]:7.1f} / {b[1]:7.1f}   "
          f"extra {a[0] - b[0]:6.1f} / {a[1] - b[1]:6.1f} us")
