"""Does an encode launch overlapping a decode launch raise throughput?
Config-2 batch of n pieces split in two halves A and B (own buffers, own
context each); times (1) the whole batch encoded then decoded, (2) A then B
each encoded then decoded on one stream, (3) decode(A) on a second stream
concurrently with encode(B).  usage: python tools/overlap_probe.py [cfg] [n]"""
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO / "capnproto-java_amd")]
import torch  # noqa: E402
import capnp_packed as cp  # noqa: E402

cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 2
n = int(sys.argv[2]) if len(sys.argv) > 2 else 131072
W = 8192


class Half:
    def __init__(self, m, ctx):
        self.m = m
        self.ctx = ctx
        swo = np.arange(0, (m + 1) * W, W, dtype=np.uint64)
        self.swo = torch.from_numpy(swo.astype(np.int64)).cuda()
        self.inp = torch.empty(m * W, dtype=torch.int64, device="cuda")
        cap = cp.batch_capacity(swo)
        self.pk = torch.empty((cap + 255) // 256 * 256, dtype=torch.uint8, device="cuda")
        self.off = torch.empty(m + 1, dtype=torch.int64, device="cuda")
        self.out = torch.empty_like(self.inp)
        self.st = torch.empty(m, dtype=torch.int32, device="cuda")
        ctx.generate(cp.preset(cfg), self.swo, self.inp)

    def enc(self, s):
        self.ctx.encode_batch(self.inp, self.swo, W, self.pk, self.off, stream=s)

    def dec(self, s):
        self.ctx.decode_batch(self.pk, self.off, self.swo, self.out, self.st, stream=s)

    def check(self):
        cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
        self.ctx.count_mismatch(self.inp, self.out, self.m * W, cnt)
        torch.cuda.synchronize()
        return int(cnt.item()) + int((self.st != 0).sum().item())


def timed(fn, reps=6):
    ts = []
    for r in range(reps):
        torch.cuda.synchronize()
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        if r:
            ts.append(a.elapsed_time(b))
    return float(np.median(ts))


s0 = torch.cuda.current_stream()
s1 = torch.cuda.Stream()
c1, c2, c3 = cp.Context(0), cp.Context(0), cp.Context(0)
full = Half(n, c3)
A, B = Half(n // 2, c1), Half(n // 2, c2)
torch.cuda.synchronize()
U = n * W * 8


def seq_full():
    full.enc(s0)
    full.dec(s0)


def seq_halves():
    A.enc(s0)
    A.dec(s0)
    B.enc(s0)
    B.dec(s0)


def pipelined():
    A.enc(s0)
    ea = torch.cuda.Event()
    ea.record(s0)
    B.enc(s0)  # encode(B) follows encode(A) on s0 ...
    s1.wait_event(ea)
    A.dec(s1)  # ... while decode(A) runs on s1
    eb = torch.cuda.Event()
    eb.record(s0)
    s1.wait_event(eb)
    B.dec(s1)
    s0.wait_stream(s1)


for name, fn in (("full batch enc+dec", seq_full), ("halves, one stream", seq_halves),
                 ("halves, dec(A) || enc(B)", pipelined), ("full batch enc+dec", seq_full),
                 ("halves, dec(A) || enc(B)", pipelined)):
    t = timed(fn)
    print(f"{name:28s} {t:8.3f} ms  {U / t / 1e6 / 1.073741824:8.1f} GiB/s", flush=True)
print("errors:", full.check(), A.check(), B.check())
