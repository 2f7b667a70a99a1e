"""Message batches on config-3 shaped messages (4 segments of 4-256 KiB,
dense data, each message preceded by its packed segment table):
cpk_encode_messages (tables built and packed on the device) against
cpk_encode_batch with the table pieces supplied, and cpk_decode_messages
(tables read and validated on the device) against cpk_decode_batch with
every piece's packed offsets known.  For DESIGN.md; not the bench metric.
usage: python tools/msg_bench.py [messages]"""
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO / "capnproto-java_amd")]
import torch  # noqa: E402
import capnp_packed as cp  # noqa: E402

nm = int(sys.argv[1]) if len(sys.argv) > 1 else 32768
rng = np.random.default_rng(3)
import os  # noqa: E402
maxw = int(os.environ.get("MB_MAXW", "32768"))  # (largest segment size drawn)
seg = rng.choice([w for w in (512, 1024, 2048, 4096, 8192, 16384, 32768) if w <= maxw],
                 size=(nm, 4)).astype(np.uint64)
sizes = np.concatenate([np.full((nm, 1), 3, np.uint64), seg], axis=1).reshape(-1)
swo = np.concatenate([[0], np.cumsum(sizes)]).astype(np.uint64)
n = len(sizes)
if os.environ.get("MB_LIB"):  # (A/B: a variant build of the library)
    cp.load(Path(os.environ["MB_LIB"]), strict=False)
ctx = cp.Context(0)
d_swo = torch.from_numpy(swo.astype(np.int64)).cuda()
d_in = torch.empty(int(swo[-1]) + 1, dtype=torch.int64, device="cuda")
ctx.generate(cp.preset(3), d_swo, d_in)
# the table pieces: [count - 1 = 3, size0 | size1, size2 | size3, pad]
tab = np.zeros((nm, 6), np.uint32)
tab[:, 0] = 3
tab[:, 1:5] = seg
tw = torch.from_numpy(tab.view(np.int64).reshape(-1).copy()).cuda()
tpos = torch.from_numpy(swo[:-1:5].astype(np.int64)).cuda()
idx = (tpos[:, None] + torch.arange(3, device="cuda")[None, :]).reshape(-1)
d_in[idx] = tw
cap = (cp.batch_capacity(swo) + 63) // 16 * 16
d_pk = torch.zeros(cap, dtype=torch.uint8, device="cuda")
d_off = torch.empty(n + 1, dtype=torch.int64, device="cuda")
ctx.encode_batch(d_in, d_swo, maxw, d_pk, d_off)
assert ctx.take_error() == 0
torch.cuda.synchronize()
d_moff = d_off[::5].contiguous()  # message m starts at its table piece; [nm] = total
assert d_moff.numel() == nm + 1
U = int(8 * seg.sum())
P = int(d_off[-1].item())

d_mseg = torch.zeros(nm + 1, dtype=torch.int64, device="cuda")
d_mst = torch.zeros(nm, dtype=torch.int32, device="cuda")
S = 4 * nm
d_out = torch.empty(U // 8 + 1, dtype=torch.int64, device="cuda")
d_sw = torch.empty(S + 1, dtype=torch.int64, device="cuda")
d_si = torch.empty(S + 1, dtype=torch.int64, device="cuda")
d_ss = torch.empty(S, dtype=torch.int32, device="cuda")


def run_msgs():
    return ctx.decode_messages(d_pk, d_moff, d_out, d_sw, d_si, d_ss, d_mseg, d_mst)


rc, W, S2 = run_msgs()
assert rc == 0 and W == U // 8 and S2 == S
assert int((d_mst != 0).sum().item()) == 0
# decoded segments == the input's segment words (boolean-mask gather: kept
# to moderate sizes)
if nm > 32768:
    sys.exit("use at most 32768 messages (verification gather)")
mask = torch.ones(int(swo[-1]), dtype=torch.bool, device="cuda")
mask[idx] = False
exp = d_in[: int(swo[-1])][mask]
cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
ctx.count_mismatch(exp, d_out, U // 8, cnt)
torch.cuda.synchronize()
assert int(cnt.item()) == 0
del exp, mask

d_bout = torch.empty_like(d_in)
d_bst = torch.empty(n, dtype=torch.int32, device="cuda")


def timed(f, reps=5):
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        a.record()
        f()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) / 1e3)
    return sorted(ts)[len(ts) // 2]


# message encode: the segments alone (tables built on the device); bytes
# must equal the piece encode with the table pieces supplied
segmask = torch.ones(int(swo[-1]), dtype=torch.bool, device="cuda")
segmask[idx] = False
d_seg = torch.empty(U // 8 + 1, dtype=torch.int64, device="cuda")
d_seg[: U // 8] = d_in[: int(swo[-1])][segmask]
del segmask
sswo = np.concatenate([[0], np.cumsum(seg.reshape(-1))]).astype(np.int64)
d_sswo = torch.from_numpy(sswo).cuda()
d_msegs = torch.arange(0, 4 * nm + 1, 4, dtype=torch.int64, device="cuda")
d_pk2 = torch.zeros_like(d_pk)
d_off2 = torch.empty(n + 1, dtype=torch.int64, device="cuda")
ctx.encode_messages(d_seg, d_sswo, d_msegs, maxw, d_pk2, d_off2)
assert ctx.take_error() == 0
assert torch.equal(d_off2, d_off) and torch.equal(d_pk2[:P], d_pk[:P])
t_em = timed(lambda: ctx.encode_messages(d_seg, d_sswo, d_msegs, maxw, d_pk2, d_off2))
t_eb = timed(lambda: ctx.encode_batch(d_in, d_swo, maxw, d_pk2, d_off2))

t_m = timed(run_msgs)
t_b = timed(lambda: ctx.decode_batch(d_pk, d_off, d_swo, d_bout, d_bst))
G = float(1 << 30)
print(f"{nm} messages x 4 segments, U = {U / G:.2f} GiB, P/U = {P / U:.4f}")
print(f"  encode_messages (tables built on device):                   {U / G / t_em:8.1f} GiB/s"
      f"  ({t_em * 1e3:.2f} ms)")
print(f"  encode_batch (table pieces supplied):                       {U / G / t_eb:8.1f} GiB/s"
      f"  ({t_eb * 1e3:.2f} ms)")
print(f"  decode_messages (tables on device, one stream per message): {U / G / t_m:8.1f} GiB/s"
      f"  ({t_m * 1e3:.2f} ms, incl. one host sync)")
print(f"  decode_batch (every piece's offsets known):                 {U / G / t_b:8.1f} GiB/s"
      f"  ({t_b * 1e3:.2f} ms)")
