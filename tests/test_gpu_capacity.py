"""The device encoders' output capacity (cpk_encode_batch_cap,
cpk_encode_messages_cap): the reference's sink refuses a write that does not
fit (ArrayOutputStream.write throws IOException when `available < size`,
/root/reference/runtime/src/main/java/org/capnproto/ArrayOutputStream.java:36-44).
Here a piece whose packed bytes would pass the capacity is reported
(cpk_ctx_take_error -> CPK_ENOMEM) and no byte at or past the capacity is
stored: a sentinel after it stays intact, and the pieces wholly below it are
the oracle's bytes.  Every encoder form runs through the `ctx` fixture (the
device gate, the single pass forced, the two passes forced) and the gate's
sparse form through the config-4 batch."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SENTINEL = 0xA5
PAD = 4096  # sentinel bytes after the capacity


def _swo(sizes):
    return np.concatenate([[0], np.cumsum(np.asarray(sizes, dtype=np.uint64))]).astype(np.uint64)


def _check_capped(ctx, cp, torch, d_in, d_swo, maxw, want, woff, cap, encode):
    """Encode into a buffer of `cap` bytes followed by PAD sentinel bytes."""
    d_pk = torch.full((cap + PAD,), SENTINEL, dtype=torch.uint8, device="cuda")
    d_off = torch.zeros(len(woff), dtype=torch.int64, device="cuda")
    encode(d_pk, cap, d_off)
    rc = ctx.take_error()
    got = d_pk.cpu().numpy()
    assert (got[cap:] == SENTINEL).all(), f"bytes stored past the capacity at {cap + np.flatnonzero(got[cap:] != SENTINEL)[:8]}"
    if cap >= int(woff[-1]):
        assert rc == cp.OK
        assert got[:cap][: len(want)].tobytes() == want
        return
    assert rc == cp.ENOMEM
    # the pieces wholly below the capacity are written as usual
    fit = int(np.searchsorted(woff, cap, side="right")) - 1  # pieces [0, fit) end at or before cap
    end = int(woff[fit])
    assert got[:end].tobytes() == want[:end]
    # the error is cleared by take_error
    assert ctx.take_error() == cp.OK


@pytest.mark.parametrize("cfg", [2, 3, 4])
@pytest.mark.parametrize("short", [0, 1, 4097, "half"])
def test_encode_batch_capacity(ctx, oracle, cfg, short):
    """Like-sized 64 KiB pieces (configs 2 / 4: the single pass and its
    sparse form under the gate; config 3: the two passes) plus ragged ones;
    the capacity exactly the packed size, one byte short, a page short, half."""
    import torch
    import capnp_packed as cp
    swo = _swo([8192] * 40 + [8191, 17, 4096, 0, 8192])
    data = oracle.generate(oracle.preset(cfg), swo)
    want, woff = oracle.pack_batch(data, swo, threads=8)
    want = want.tobytes()
    total = int(woff[-1])
    cap = total // 2 if short == "half" else total - short
    d_in = torch.from_numpy(data.view(np.int64).copy()).cuda()
    d_swo = torch.from_numpy(swo.astype(np.int64)).cuda()
    _check_capped(ctx, cp, torch, d_in, d_swo, 8192, want, woff, cap,
                  lambda d_pk, c, d_off: ctx.encode_batch_cap(d_in, d_swo, 8192, d_pk, c, d_off))


@pytest.mark.parametrize("nmsg", [60, 300])
@pytest.mark.parametrize("short", [0, 1, "half"])
def test_encode_messages_capacity(ctx, oracle, short, nmsg):
    """Message batches (tables built on the device): 60 messages (at most
    1,024 pieces: the single pass with the tables' descriptors) and 300
    (the two passes) of mixed segments; the table pieces are refused like
    the segments."""
    import torch
    import capnp_packed as cp
    rng = np.random.default_rng(77 + nmsg)
    msgs = []
    for i in range(nmsg):
        nseg = int(rng.choice([1, 2, 3, 4, 9]))
        sizes = [int(rng.choice([0, 1, 17, 300, 2000, 9000])) for _ in range(nseg)]
        msgs.append([(rng.integers(0, 256, size=8 * s, dtype=np.uint8)
                      * (rng.random(8 * s) < 0.6)).astype(np.uint8).tobytes() for s in sizes])
    segs = [s for m in msgs for s in m]
    swo = _swo([len(s) // 8 for s in segs])
    mseg = _swo([len(m) for m in msgs])
    data = np.frombuffer(b"".join(segs) + b"\0" * 8, np.uint8)
    d_in = torch.from_numpy(data.view(np.int64).copy()).cuda()
    d_swo = torch.from_numpy(swo.astype(np.int64)).cuda()
    d_mseg = torch.from_numpy(mseg.astype(np.int64)).cuda()
    # piece offsets in message order (table, segments) from the oracle
    woff, o = [0], 0
    for m in msgs:
        nseg = len(m)
        tb = ((nseg - 1) & 0xffffffff).to_bytes(4, "little") + b"".join(
            (len(s) // 8).to_bytes(4, "little") for s in m)
        tb += b"\0" * (-len(tb) % 8)
        for piece in [tb] + m:
            o += len(oracle.pack(piece))
            woff.append(o)
    woff = np.asarray(woff, dtype=np.uint64)
    want = b"".join(oracle.write_message(m) for m in msgs)
    assert len(want) == int(woff[-1])
    cap = len(want) // 2 if short == "half" else len(want) - short
    _check_capped(ctx, cp, torch, d_in, d_swo, 9000, want, woff, cap,
                  lambda d_pk, c, d_off: ctx.encode_messages_cap(d_in, d_swo, d_mseg, 9000, d_pk, c, d_off))
