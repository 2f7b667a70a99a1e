"""Per-phase cycle shares of the block-map decoder (decode_kernel<false>),
diagnostic stats build: tools/build_variant.sh stats -DCPK_PHASE_STATS.
Per-wave s_memtime sums: read them as shares, not times (the stamps cost
cycles themselves).
Usage: python tools/dec_phase_stats.py [config] [pieces] [lib]"""
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
os.environ["CPK_DECODER"] = "1"
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
ctx.encode_batch(d_in, d_swo, 8192, d_pk, d_off)
d_out = torch.empty_like(d_in)
d_st = torch.empty(n, dtype=torch.int32, device="cuda")
for _ in range(2):
    ctx.decode_batch(d_pk, d_off, d_swo, d_out, d_st)
torch.cuda.synchronize()
buf = np.zeros(64, dtype=np.uint64)
L.cpk_debug_phase_stats(buf.ctypes.data)
ctx.decode_batch(d_pk, d_off, d_swo, d_out, d_st)
torch.cuda.synchronize()
L.cpk_debug_phase_stats(buf.ctypes.data)
assert torch.equal(d_out, d_in)
names = ["piece / window loop", "window load", "1-2: chunk + landing walks", "3: chain",
         "4: own words + scan", "5: map walk + checks + fill", "5: expansion"]
v = buf[16:23].astype(float)
tot = v.sum()
windows = float(d_off[-1].item()) / 3072
print(f"decode_kernel config {cfg}: {tot / 1e6:.1f} Mcycles over all waves; per window {tot / windows:.0f} cyc")
for nm, x in zip(names, v):
    print(f"  {nm:34s} {100 * x / tot:5.1f} %  {x / windows:7.0f} cyc/window")
