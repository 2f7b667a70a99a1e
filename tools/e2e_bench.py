"""End-to-end (host-resident, PCIe-inclusive) rates for DESIGN.md: the
C ABI's host forms (cpk_encode_host / cpk_decode_host: pageable buffers,
chunked through pinned staging by the library, host_pipe.hip), and the
pinned-memory copy rates
that bound any host path.  Not the bench metric (that is device-resident).
usage: python tools/e2e_bench.py [config] [pieces]"""
import sys
import time
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO / "capnproto-java_amd"), str(REPO / "oracle")]
import torch  # noqa: E402
import capnp_packed as cp  # noqa: E402

cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 2
n = int(sys.argv[2]) if len(sys.argv) > 2 else 16384
sw = 8192
GIB = float(1 << 30)
swo = np.arange(0, (n + 1) * sw, sw, dtype=np.uint64)
ctx = cp.Context(0)
d_swo = torch.from_numpy(swo.astype(np.int64)).cuda()
d_in = torch.empty(n * sw, dtype=torch.int64, device="cuda")
ctx.generate(cp.preset(cfg), d_swo, d_in)
host = d_in.cpu().numpy().view(np.uint8)
U = host.size

def best(f, reps=3):
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        r = f()
        ts.append(time.perf_counter() - t0)
    return min(ts), r

t_enc, (pk, off) = best(lambda: ctx.encode_host(host, swo))
t_dec, (dec, st) = best(lambda: ctx.decode_host(pk, off, swo))
assert (st == 0).all() and np.array_equal(dec, host)
print(f"config {cfg}: {n} pieces x 64 KiB, U = {U / GIB:.2f} GiB, P/U = {pk.size / U:.4f}")
print(f"  host forms, fresh outputs:  encode {U / GIB / t_enc:7.2f} GiB/s  decode {U / GIB / t_dec:7.2f} GiB/s"
      f"  round trip {U / GIB / (t_enc + t_dec):7.2f} GiB/s")
# reused (already faulted-in) output buffers, as a server reusing its buffers
ob = np.ones(cp.batch_capacity(swo), np.uint8)
db = np.ones(U, np.uint8)
pk = pk.copy()
t_enc, (pk2, _) = best(lambda: ctx.encode_host(host, swo, out=ob))
t_dec, (dec, st) = best(lambda: ctx.decode_host(pk, off, swo, out=db))
assert np.array_equal(pk2, pk) and (st == 0).all() and np.array_equal(dec, host)
print(f"  host forms, reused outputs: encode {U / GIB / t_enc:7.2f} GiB/s  decode {U / GIB / t_dec:7.2f} GiB/s"
      f"  round trip {U / GIB / (t_enc + t_dec):7.2f} GiB/s")
# gather form: every piece in its own host allocation (builder segments)
parts = [host[i * sw * 8:(i + 1) * sw * 8].view(np.uint64).copy() for i in range(n)]
pk3, off3 = ctx.encode_host_gather(parts, out=ob)
assert np.array_equal(pk3, pk) and np.array_equal(off3, off)
# the C call alone (the Python wrapper's per-piece pointer list is not the
# JNI path's cost)
import ctypes  # noqa: E402
ptrs = (ctypes.c_void_p * n)(*[x.ctypes.data for x in parts])
off3 = np.zeros(n + 1, dtype=np.uint64)
t_g, rc = best(lambda: ctx._lib.cpk_encode_host_gather(ctx.handle, ptrs, swo.ctypes.data, n,
                                                        ob.ctypes.data, ob.size, off3.ctypes.data))
assert rc == 0 and np.array_equal(off3, off)
print(f"  gather encode (separate piece buffers), reused output: {U / GIB / t_g:7.2f} GiB/s")
del parts
# pinned copy rates (the PCIe bound of any pipelined host path)
pin = torch.empty(U, dtype=torch.uint8).pin_memory()
dev = torch.empty(U, dtype=torch.uint8, device="cuda")
for name, f in (("H2D pinned", lambda: dev.copy_(pin, non_blocking=True)),
                ("D2H pinned", lambda: pin.copy_(dev, non_blocking=True))):
    f(); torch.cuda.synchronize()
    t0 = time.perf_counter(); f(); torch.cuda.synchronize(); t = time.perf_counter() - t0
    print(f"  {name}: {U / GIB / t:7.2f} GiB/s")
