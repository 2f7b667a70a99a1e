import sys
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parents[1]
for p in (REPO, REPO / "oracle", REPO / "capnproto-java_amd", REPO / "tools"):
    if str(p) not in sys.path:
        sys.path.insert(0, str(p))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run with -m gpu)")
    config.addinivalue_line("markers", "slow: longer CPU test")


@pytest.fixture(scope="session")
def oracle():
    import oracle as o
    o.build()
    return o


@pytest.fixture(scope="module", params=[("5", "3"), ("0", "2"), ("4", "1")],
                ids=["enc-auto+dec-auto", "enc-single-pass+dec-index", "enc-two-pass+dec-block-map"])
def ctx(request):
    """A context per encoder / decoder pair (CPK_ENCODER, CPK_DECODER are read
    at context creation): every parity case runs through the default choice
    (the single pass for like-sized pieces of 4 Ki words or more, the two-pass
    encoder, encode_v4.hip, otherwise; the record-index decoder,
    decode_v2.hip, for sparse batches, the block-map decoder, decode_kernel,
    otherwise), through the single-pass encoder (encode_sp.hip) forced
    for every batch with the record-index decoder forced, and through the
    two-pass encoder with the block-map decoder forced (so sparse batches,
    whose windows expand in several rounds, reach the block map too)."""
    import os
    import torch
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    import capnp_packed as cp
    saved = {k: os.environ.get(k) for k in ("CPK_ENCODER", "CPK_DECODER")}
    os.environ["CPK_ENCODER"], os.environ["CPK_DECODER"] = request.param
    try:
        c = cp.Context(0)
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k)
            else:
                os.environ[k] = v
    yield c
    c.close()


def pytest_assertrepr_compare(op, left, right):
    """Short report for unequal large byte strings: pytest's default diff
    of megabytes (difflib) runs for minutes and trips the GPU tests' time
    limit before the failure is shown."""
    if op == "==" and isinstance(left, (bytes, bytearray)) and isinstance(right, (bytes, bytearray)) \
            and max(len(left), len(right)) > 4096:
        n = min(len(left), len(right))
        first = next((i for i in range(n) if left[i] != right[i]), n)
        return [f"byte strings differ: lengths {len(left)} / {len(right)}, first difference at byte {first}",
                f"left[{first}:{first + 16}] = {bytes(left[first:first + 16]).hex()}",
                f"right[{first}:{first + 16}] = {bytes(right[first:first + 16]).hex()}"]
    return None
