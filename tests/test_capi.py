"""C-ABI boundary checks that need no GPU: the library loads, exports every
symbol include/capnp_packed.h declares, and its host-only helpers agree with
the oracle.  No compute call is made here."""
import ctypes
import re
from pathlib import Path

import numpy as np
import pytest

REPO = Path(__file__).resolve().parents[1]


def _declared():
    hdr = (REPO / "include" / "capnp_packed.h").read_text()
    return sorted(set(re.findall(r"\b(cpk_[a-z_]+)\s*\(", hdr)))


def test_header_and_binding_agree():
    import capnp_packed as cp
    assert sorted(cp.EXPORTS) == _declared()


def test_library_exports_every_declared_symbol():
    import capnp_packed as cp
    L = ctypes.CDLL(str(cp.LIB_PATH))
    for name in _declared():
        assert hasattr(L, name), name
    assert cp.load().cpk_abi_version() == 1


def test_packed_bound_matches_oracle(oracle):
    import capnp_packed as cp
    L = cp.load()
    for w in [0, 1, 2, 3, 255, 256, 8191, 8192, 1 << 28]:
        assert L.cpk_packed_bound(w) == oracle.packed_bound(w) == cp.packed_bound(w)
    swo = np.array([0, 1, 4, 4, 8196], dtype=np.uint64)
    assert L.cpk_batch_packed_capacity(swo.ctypes.data, 4) == cp.batch_capacity(swo)


def test_status_strings():
    import capnp_packed as cp
    for s in (cp.OK, cp.EINVAL, cp.ETRUNC, cp.EOVERRUN, cp.ETRAILING, cp.ENOMEM, cp.EDEVICE,
              cp.EUNSUPPORTED):
        assert cp.status_string(s) != "unknown status"


def test_ctx_without_device_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    import capnp_packed as cp
    with pytest.raises(cp.CodecError):
        cp.Context(0)
