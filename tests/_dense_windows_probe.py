"""Helper for tests/test_gpu_parity.py::test_dense_batches_serial_windows
(not collected by pytest): decodes a packed batch with the diagnostics
library (CPK_LIB = libcapnp_packed_hip_diag.so, -DCPK_DEC_CNT=1) and prints
the dense decoder form's counters (windows walked serially, serial walks
given back) after checking the words.
usage: python tests/_dense_windows_probe.py DIR   (DIR/{pk,off,swo,data}.npy)"""
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "capnproto-java_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import capnp_packed as cp  # noqa: E402

d = Path(sys.argv[1])
pk, off, swo, data = (np.load(d / f"{k}.npy") for k in ("pk", "off", "swo", "data"))
ctx = cp.Context(0)
d_pk = torch.zeros(len(pk) + 64, dtype=torch.uint8, device="cuda")
d_pk[: len(pk)] = torch.from_numpy(pk)
d_off = torch.from_numpy(off.astype(np.int64)).cuda()
d_swo = torch.from_numpy(swo.astype(np.int64)).cuda()
d_out = torch.zeros(int(swo[-1]) + 1, dtype=torch.int64, device="cuda")
d_st = torch.full((len(swo) - 1,), 99, dtype=torch.int32, device="cuda")
ctx.decode_batch(d_pk, d_off, d_swo, d_out, d_st)
torch.cuda.synchronize()
assert (d_st.cpu().numpy() == 0).all()
assert d_out.cpu().numpy()[: int(swo[-1])].view(np.uint8).tobytes() == data.tobytes()
ser, back = ctx.dense_windows()
print(f"dense_windows {ser} {back}")
