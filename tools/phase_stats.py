"""Per-phase cycle shares of the single-pass encoder (diagnostic stats build:
tools/build_variant.sh stats -DCPK_PHASE_STATS).  Per-wave s_memtime sums,
read them as shares, not times (the stamps cost cycles themselves).
Usage: python tools/phase_stats.py [config] [pieces] [lib]"""
import ctypes
import os
import sys
from pathlib import Path
REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO / "capnproto-java_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
import capnp_packed as cp  # noqa: E402

cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 2
n = int(sys.argv[2]) if len(sys.argv) > 2 else 65536
os.environ["CPK_ENCODER"] = "0"
L = cp.load(Path(sys.argv[3]) if len(sys.argv) > 3 else REPO / "build" / "variants" / "stats.so", strict=False)
L.cpk_debug_phase_stats.argtypes = [ctypes.c_void_p]
ctx = cp.Context(0)
swo = np.arange(0, (n + 1) * 8192, 8192, dtype=np.uint64)
d_swo = torch.from_numpy(swo.astype(np.int64)).cuda()
d_in = torch.empty(n * 8192, dtype=torch.int64, device="cuda")
ctx.generate(cp.preset(cfg), d_swo, d_in)
cap = cp.batch_capacity(swo)
d_pk = torch.empty((cap + 255) // 256 * 256, dtype=torch.uint8, device="cuda")
d_off = torch.empty(n + 1, dtype=torch.int64, device="cuda")
for _ in range(2):
    ctx.encode_batch(d_in, d_swo, 8192, d_pk, d_off)
torch.cuda.synchronize()
buf = np.zeros(64, dtype=np.uint64)
L.cpk_debug_phase_stats(buf.ctypes.data)
ctx.encode_batch(d_in, d_swo, 8192, d_pk, d_off)
torch.cuda.synchronize()
L.cpk_debug_phase_stats(buf.ctypes.data)
names = ["ticket + barriers", "barrier + A2 + barrier", "look-back + barrier", "loop top", "B emit",
         "B: look-back (wave 0)", "B: wait for offset (waves 1-3)", "A1 (loads, tags, ballots)"]
v = buf[32:40].astype(float)
tot = v.sum()
print(f"sp_encode config {cfg}: {tot / 1e6:.1f} Mcycles over all waves; per piece per wave {tot / n / 4:.0f} cyc")
for nm, x in zip(names, v):
    print(f"   {nm:30s} {100 * x / max(tot, 1):6.2f} %   {x / n / 4:8.0f} cyc/piece/wave")
print(f"look-back: {buf[40] / n:.2f} polls per piece, {buf[42] / n:.2f} of them retried")

# ---- decoder phases (decode_kernel WPH slots 16..22) ----
d_out = torch.empty_like(d_in)
d_st = torch.empty(n, dtype=torch.int32, device="cuda")
ctx.decode_batch(d_pk, d_off, d_swo, d_out, d_st)
torch.cuda.synchronize()
L.cpk_debug_phase_stats(buf.ctypes.data)
ctx.decode_batch(d_pk, d_off, d_swo, d_out, d_st)
torch.cuda.synchronize()
L.cpk_debug_phase_stats(buf.ctypes.data)
dnames = ["ticket+piece", "window load", "chunk walks", "lane chain", "count walk", "errors+blk map | index", "expand+store"]
v = buf[16:16 + len(dnames)].astype(float)
tot = v.sum()
print(f"decode config {cfg}: total {tot / 1e6:.1f} Mcycles over all waves; per piece {tot / n:.0f} cyc")
for nm, x in zip(dnames, v):
    print(f"   {nm:22s} {100 * x / max(tot, 1):6.2f} %   {x / n:8.0f} cyc/piece")
print("bad status", int((d_st != 0).sum().item()))
