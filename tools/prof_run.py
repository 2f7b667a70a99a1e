"""Profiling driver: device-resident encode + decode of one synthetic batch,
repeated; run under rocprofv3 (kernel trace / PMC passes).
usage: python tools/prof_run.py [config] [pieces] [reps]"""
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO / "capnproto-java_amd")]
import torch  # noqa: E402
import capnp_packed as cp  # noqa: E402

cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 2
n = int(sys.argv[2]) if len(sys.argv) > 2 else 131072
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
sw = 8192
swo = np.arange(0, (n + 1) * sw, sw, dtype=np.uint64)
d_swo = torch.from_numpy(swo.astype(np.int64)).cuda()
d_in = torch.empty(n * sw, dtype=torch.int64, device="cuda")
ctx = cp.Context(0)
ctx.generate(cp.preset(cfg), d_swo, d_in)
cap = cp.batch_capacity(swo)
d_pk = torch.empty((cap + 255) // 256 * 256, dtype=torch.uint8, device="cuda")
d_off = torch.empty(n + 1, dtype=torch.int64, device="cuda")
d_out = torch.empty_like(d_in)
d_st = torch.empty(n, dtype=torch.int32, device="cuda")
for _ in range(reps):
    ctx.encode_batch(d_in, d_swo, sw, d_pk, d_off)
    ctx.decode_batch(d_pk, d_off, d_swo, d_out, d_st)
torch.cuda.synchronize()
cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
ctx.count_mismatch(d_in, d_out, n * sw, cnt)
U, P = 8 * n * sw, int(d_off[-1].item())
print(f"config {cfg} n={n} U={U} P={P} mismatch={int(cnt.item())} bad={int((d_st != 0).sum().item())}")
