"""A/B timing of codec builds in one process: python tools/quick_bench.py lib1.so [lib2.so ...]
Each lib is loaded in a subprocess-free way via ctypes (separate handles).
Spec "lib.so@E[:K=V,...]": CPK_ENCODER=E for that library's context -- 0 the
dense single pass (no device gate: CPK_SP_FORM is ignored), 4 the two
passes, 5 the library's default (the device gate: single pass, its sparse
form for mostly-zero batches, or the two passes) -- plus env knobs read at
context creation."""
import ctypes, sys, time
from pathlib import Path
REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO / "capnproto-java_amd")]
import numpy as np, torch
import capnp_packed as cp

n = int(__import__("os").environ.get("QB_N", "131072"))
cfgs = [int(c) for c in __import__("os").environ.get("QB_CFG", "2").split(",")]
libs = sys.argv[1:]
hint = int(__import__("os").environ.get("QB_HINT", __import__("os").environ.get("QB_W", "8192")))  # 0: tiled encoder path
W = int(__import__("os").environ.get("QB_W", "8192"))  # words per piece
swo = np.arange(0, (n + 1) * W, W, dtype=np.uint64)
if __import__("os").environ.get("QB_MIXED"):
    # config-3 segment sizes (4-256 KiB, bench.CFG3_SEG_WORDS), seeded; W = mean
    _sz = np.random.default_rng(3).choice([512, 1024, 2048, 4096, 8192, 16384, 32768], size=n).astype(np.uint64)
    swo = np.concatenate([[0], np.cumsum(_sz)]).astype(np.uint64)
    hint = 32768
    W = int(swo[-1]) // n
d_swo = torch.from_numpy(swo.astype(np.int64)).cuda()
d_in = torch.empty(int(swo[-1]), dtype=torch.int64, device="cuda")
cap = cp.batch_capacity(swo)
d_pk = torch.empty((cap + 255) // 256 * 256, dtype=torch.uint8, device="cuda")
d_off = torch.empty(n + 1, dtype=torch.int64, device="cuda")
d_out = torch.empty_like(d_in)
d_st = torch.empty(n, dtype=torch.int32, device="cuda")
cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
handles = []
import os
for spec in libs:
    # "lib.so@0": context created with CPK_ENCODER=0 (single-pass encoder)
    # "lib.so@4:CPK_DECODER=2": encoder 4 plus env knobs read at ctx creation
    lp, _, enc = spec.partition("@")
    enc, _, envs = enc.partition(":")
    os.environ["CPK_ENCODER"] = enc or "0"
    os.environ.pop("CPK_DECODER", None)
    for kv in filter(None, envs.split(",")):
        k, _, v = kv.partition("=")
        os.environ[k] = v
    cp._lib = None
    L = cp.load(Path(lp), strict=False)
    ctx = cp.Context(0)
    handles.append((spec.split("/")[-1], L, ctx))
# QB_DENS="z:lz:q,...": custom densities (zero-word fraction, mean zero run,
# zero-byte fraction of nonzero words), one run each, instead of QB_CFG's presets
dens = [tuple(float(x) for x in d.split(":")) for d in os.environ.get("QB_DENS", "").split(",") if d]
for cfg in (dens or cfgs):
    cp._lib = handles[0][1]
    if dens:
        gp = cp.gen_params(2, *cfg)
    else:
        gp = cp.preset(cfg)
    if __import__("os").environ.get("QB_Z"):  # (a custom density: QB_Z zero fraction, QB_LZ mean zero run)
        _e = __import__("os").environ
        gp = cp.gen_params(cfg, float(_e["QB_Z"]), float(_e.get("QB_LZ", "16")), 0.25)
    handles[0][2].generate(gp, d_swo, d_in)
    torch.cuda.synchronize()
    U = int(swo[-1]) * 8
    print(f"config {cfg}: n={n}", flush=True)
    for name, L, ctx in handles:
        cp._lib = L
        ctx._lib = L
        te, td = [], []
        for rnd in range(6):
            e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
            e[0].record(); ctx.encode_batch(d_in, d_swo, hint, d_pk, d_off); e[1].record()
            ctx.decode_batch(d_pk, d_off, d_swo, d_out, d_st); e[2].record()
            torch.cuda.synchronize()
            if rnd:
                te.append(e[0].elapsed_time(e[1])); td.append(e[1].elapsed_time(e[2]))
        err = ctx.take_error() if hasattr(L, "cpk_ctx_take_error") else 0
        cnt.zero_(); ctx.count_mismatch(d_in, d_out, int(swo[-1]), cnt)
        P = int(d_off[-1].item())
        me, md = np.median(te), np.median(td)
        print(f"  {name:44s} enc {me:8.3f} ms ({U / me / 1e6:7.1f} GB/s)  dec {md:8.3f} ms ({U / md / 1e6:7.1f} GB/s)"
              f"  rt {U / (me + md) / 1e6 / 1.073741824:7.1f} GiB/s  P/U={P / U:.4f} mism={int(cnt.item())}"
              f" bad={int((d_st != 0).sum().item())} err={err}", flush=True)
