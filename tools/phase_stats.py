"""Per-phase cycle shares of the codec kernels (diagnostic stats build).
Usage: python tools/phase_stats.py [config] [segments] [lib]"""
import ctypes, sys
from pathlib import Path
REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO / "capnproto-java_amd")]
import numpy as np, torch
import capnp_packed as cp

cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 2
n = int(sys.argv[2]) if len(sys.argv) > 2 else 65536
L = cp.load(Path(sys.argv[3]) if len(sys.argv) > 3 else REPO / "build" / "variants" / "stats.so")
L.cpk_debug_phase_stats.argtypes = [ctypes.c_void_p]
ctx = cp.Context(0)
swo = np.arange(0, (n + 1) * 8192, 8192, dtype=np.uint64)
d_swo = torch.from_numpy(swo.astype(np.int64)).cuda()
d_in = torch.empty(n * 8192, dtype=torch.int64, device="cuda")
ctx.generate(cp.preset(cfg), d_swo, d_in)
cap = cp.batch_capacity(swo)
d_pk = torch.empty((cap + 255) // 256 * 256, dtype=torch.uint8, device="cuda")
d_off = torch.empty(n + 1, dtype=torch.int64, device="cuda")
d_out = torch.empty_like(d_in)
d_st = torch.empty(n, dtype=torch.int32, device="cuda")
for _ in range(2):
    ctx.encode_batch(d_in, d_swo, 8192, d_pk, d_off)
    ctx.decode_batch(d_pk, d_off, d_swo, d_out, d_st)
torch.cuda.synchronize()
buf = np.zeros(64, dtype=np.uint64)
L.cpk_debug_phase_stats(buf.ctypes.data)
ctx.encode_batch(d_in, d_swo, 8192, d_pk, d_off)
ctx.decode_batch(d_pk, d_off, d_swo, d_out, d_st)
torch.cuda.synchronize()
L.cpk_debug_phase_stats(buf.ctypes.data)
e1names = ["ticket", "load+classify", "roles", "long stretches", "bytes+zero stage", "strings to LDS", "look-back", "store"]
v = buf[0:len(e1names)].astype(float)
tot = v.sum()
print(f"encode (v1, wave 0 of each workgroup): total {tot / 1e6:.1f} Mcycles; per piece {tot / n:.0f} cyc")
for nm, x in zip(e1names, v):
    print(f"   {nm:22s} {100 * x / max(tot, 1):6.2f} %   {x / n:8.0f} cyc/piece")
e2names = ["ticket+setup", "load+classify", "exit/entry state", "roles", "look-back", "strings+store"]
v = buf[32:32 + len(e2names)].astype(float)
tot = v.sum()
print(f"encode2: total {tot / 1e6:.1f} Mcycles over all waves; per piece {tot / n:.0f} cyc")
for nm, x in zip(e2names, v):
    print(f"   {nm:22s} {100 * x / max(tot, 1):6.2f} %   {x / n:8.0f} cyc/piece")
dnames = ["ticket+piece", "window load", "chunk walks", "lane chain", "count walk", "errors+blk map", "expand+store"]
v = buf[16:16 + len(dnames)].astype(float)
tot = v.sum()
print(f"decode: total {tot / 1e6:.1f} Mcycles over all waves; per piece {tot / n:.0f} cyc")
for nm, x in zip(dnames, v):
    print(f"   {nm:22s} {100 * x / max(tot, 1):6.2f} %   {x / n:8.0f} cyc/piece")
print("P/U =", int(d_off[-1].item()) / (8.0 * n * 8192), "bad status", int((d_st != 0).sum().item()))
