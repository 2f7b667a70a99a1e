"""Host-form encode and decode of ONE large piece (a big single-segment
message: SerializePacked.write / read through host memory), timed for each
library given, in one process: python tools/one_piece_host_bench.py lib.so ...
(reused output buffers: no first-touch faults in the timing)."""
import os
import sys
import time
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO / "capnproto-java_amd")]
import torch  # noqa: E402
import capnp_packed as cp  # noqa: E402

sizes_mib = [int(x) for x in os.environ.get("OP_MIB", "64,256").split(",")]
handles = []
for lp in sys.argv[1:]:
    cp._lib = None
    L = cp.load(Path(lp), strict=False)
    handles.append((lp.split("/")[-1], L, cp.Context(0)))
for mib in sizes_mib:
    W = mib << 17  # words
    swo = np.array([0, W], dtype=np.uint64)
    d_swo = torch.from_numpy(swo.astype(np.int64)).cuda()
    d_in = torch.empty(W, dtype=torch.int64, device="cuda")
    cp._lib = handles[0][1]
    handles[0][2].generate(cp.preset(2), d_swo, d_in)
    data = d_in.cpu().numpy().view(np.uint8)
    out = np.zeros(cp.batch_capacity(swo), dtype=np.uint8)
    dec = np.zeros(8 * W, dtype=np.uint8)
    ref = None
    for name, L, ctx in handles:
        cp._lib = L
        ctx._lib = L
        te, td = [], []
        for r in range(5):
            t0 = time.perf_counter()
            pk, off = ctx.encode_host(data, swo, out)
            t1 = time.perf_counter()
            d, st = ctx.decode_host(pk, off, swo, dec)
            t2 = time.perf_counter()
            if r:
                te.append(t1 - t0)
                td.append(t2 - t1)
        ok = bool(st[0] == 0 and np.array_equal(d, data))
        if ref is None:
            ref = pk.copy()
        same = bool(np.array_equal(pk, ref))
        U = 8 * W / float(1 << 30)
        print(f"{mib:4d} MiB piece  {name:24s} encode_host {1e3 * np.median(te):7.2f} ms ({U / np.median(te):5.1f} GiB/s)"
              f"  decode_host {1e3 * np.median(td):7.2f} ms ({U / np.median(td):5.1f} GiB/s)  ok={ok} same={same}",
              flush=True)

