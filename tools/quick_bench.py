"""A/B timing of codec builds in one process: python tools/quick_bench.py lib1.so [lib2.so ...]
Each lib is loaded in a subprocess-free way via ctypes (separate handles)."""
import ctypes, sys, time
from pathlib import Path
REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO / "capnproto-java_amd")]
import numpy as np, torch
import capnp_packed as cp

n = int(__import__("os").environ.get("QB_N", "131072"))
cfgs = [int(c) for c in __import__("os").environ.get("QB_CFG", "2").split(",")]
libs = sys.argv[1:]
hint = int(__import__("os").environ.get("QB_HINT", "8192"))  # 0: tiled encoder path
swo = np.arange(0, (n + 1) * 8192, 8192, dtype=np.uint64)
d_swo = torch.from_numpy(swo.astype(np.int64)).cuda()
d_in = torch.empty(n * 8192, dtype=torch.int64, device="cuda")
cap = cp.batch_capacity(swo)
d_pk = torch.empty((cap + 255) // 256 * 256, dtype=torch.uint8, device="cuda")
d_off = torch.empty(n + 1, dtype=torch.int64, device="cuda")
d_out = torch.empty_like(d_in)
d_st = torch.empty(n, dtype=torch.int32, device="cuda")
cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
handles = []
import os
for spec in libs:
    # "lib.so@1": context created with CPK_ENCODER=1 (workgroup-per-piece encoder)
    lp, _, enc = spec.partition("@")
    os.environ["CPK_ENCODER"] = enc or "1"
    cp._lib = None
    L = cp.load(Path(lp), strict=False)
    ctx = cp.Context(0)
    handles.append((Path(lp).name + (f"@{enc}" if enc else ""), L, ctx))
for cfg in cfgs:
    cp._lib = handles[0][1]
    handles[0][2].generate(cp.preset(cfg), d_swo, d_in)
    torch.cuda.synchronize()
    res = {h[0]: ([], []) for h in handles}
    for rnd in range(6):
        for name, L, ctx in handles:
            cp._lib = L
            ctx._lib = L
            e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
            ctx._lib = L
            e[0].record(); ctx.encode_batch(d_in, d_swo, hint, d_pk, d_off); e[1].record()
            ctx.decode_batch(d_pk, d_off, d_swo, d_out, d_st); e[2].record()
            torch.cuda.synchronize()
            if rnd:
                res[name][0].append(e[0].elapsed_time(e[1])); res[name][1].append(e[1].elapsed_time(e[2]))
    U = n * 65536
    P = int(d_off[-1].item())
    cnt.zero_(); handles[-1][2].count_mismatch(d_in, d_out, n * 8192, cnt)
    print(f"config {cfg}: n={n} P/U={P / U:.4f} mismatch={int(cnt.item())} badst={int((d_st != 0).sum().item())}")
    for name, (te, td) in res.items():
        me, md = np.median(te), np.median(td)
        print(f"  {name:36s} enc {me:8.3f} ms ({U / me / 1e6:7.1f} GB/s)  dec {md:8.3f} ms ({U / md / 1e6:7.1f} GB/s)"
              f"  rt {U / (me + md) / 1e6 / 1.073741824:7.1f} GiB/s")
