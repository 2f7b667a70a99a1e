"""Per-phase wave-cycle shares of encode3_kernel (stats build:
tools/build_variant.sh stats -DCPK_PHASE_STATS).
usage: python tools/e3_stats.py [config] [pieces] [lib]"""
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
lib = sys.argv[3] if len(sys.argv) > 3 else str(REPO / "build" / "variants" / "stats.so")
os.environ["CPK_ENCODER"] = "3"
L = cp.load(Path(lib))
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
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
ctx.encode_batch(d_in, d_swo, 8192, d_pk, d_off)
e1.record()
torch.cuda.synchronize()
L.cpk_debug_phase_stats(buf.ctypes.data)
names = ["front (load, tags, roles)", "B2 barrier", "look-back (wave 0)", "B3 barrier",
         "strings + stores", "end barrier"]
v = buf[40:40 + len(names)].astype(float)
tot = v.sum()
tiles = n * 2
print(f"encode3 cfg {cfg}: {e0.elapsed_time(e1):.3f} ms; {tot / 1e6:.1f} Mcycles over all waves; "
      f"per tile-wave {tot / tiles / 4:.0f} cyc")
for nm, x in zip(names, v):
    print(f"   {nm:28s} {100 * x / max(tot, 1):6.2f} %   {x / tiles / 4:8.0f} cyc/tile-wave")
