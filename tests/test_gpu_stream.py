"""Stream decode (cpk_decode_stream / cpk_decode_stream_host): pieces back to
back in one packed stream, each read() stopping when its piece is full
(PackedInputStream.java:35-140, Serialize.java:165-175).  Streams of 384 KiB
and more take the parallel block path (csrc/stream_split.hip); each case is
checked against the oracle piece by piece AND against the one-wave decoder
(CPK_STREAM_ONE_WAVE=1), errors included.
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _swo(sizes):
    return np.concatenate([[0], np.cumsum(np.asarray(sizes, dtype=np.uint64))]).astype(np.uint64)


def _oracle_stream(oracle, stream: bytes, swo):
    """PackedInputStream.read per piece over one stream (the oracle's unpack
    of each piece from where the previous one stopped).  A failed piece stops
    the stream: it and every later piece carry its status."""
    n = len(swo) - 1
    st = np.zeros(n, np.int32)
    bounds = [0]
    out = []
    pos, fail = 0, 0
    for i in range(n):
        w = int(swo[i + 1] - swo[i])
        if fail:
            st[i] = fail
            continue
        if w == 0:
            bounds.append(pos)
            out.append(b"")
            continue
        s, data, used = oracle.unpack(stream[pos: pos + 10 * w + 16], 8 * w)
        if s != oracle.OK:
            fail = s
            st[i] = s
            continue
        pos += used
        bounds.append(pos)
        out.append(data)
    return st, bounds, out


def _decode_both(ctx, stream: bytes, swo, parallel_only=False):
    """-> (parallel path result, one-wave result).  parallel_only: the
    parallel path may not hand the stream to the one-wave decoder (a stream
    it gives up on then reads CPK_EUNSUPPORTED)."""
    arr = np.frombuffer(stream, np.uint8)
    if parallel_only:
        os.environ["CPK_STREAM_NO_FALLBACK"] = "1"
    try:
        fast = ctx.decode_stream_host(arr, swo)
    finally:
        os.environ.pop("CPK_STREAM_NO_FALLBACK", None)
    os.environ["CPK_STREAM_ONE_WAVE"] = "1"
    try:
        slow = ctx.decode_stream_host(arr, swo)
    finally:
        os.environ.pop("CPK_STREAM_ONE_WAVE")
    return fast, slow


def _check(ctx, oracle, stream: bytes, swo, expect_ok=None):
    # a stream that decodes cleanly must be decoded by the parallel path alone
    (dec, bounds, st), (sdec, sbounds, sst) = _decode_both(ctx, stream, swo, parallel_only=bool(expect_ok))
    ost, obounds, oout = _oracle_stream(oracle, stream, swo)
    assert np.array_equal(st, ost), (st[st != ost][:8], ost[st != ost][:8])
    assert np.array_equal(st, sst)
    good = int(np.argmax(ost != 0)) if (ost != 0).any() else len(ost)
    assert [int(b) for b in bounds[: good + 1]] == obounds[: good + 1]
    assert np.array_equal(bounds[: good + 1], sbounds[: good + 1])
    for i in range(good):
        a, b = 8 * int(swo[i]), 8 * int(swo[i + 1])
        assert dec[a:b].tobytes() == oout[i], f"piece {i}"
    assert np.array_equal(dec[: 8 * int(swo[good])], sdec[: 8 * int(swo[good])])
    if expect_ok is not None:
        assert bool((ost == 0).all()) == expect_ok
    return bounds, st


def _stream_of(oracle, data, swo):
    pk, off = oracle.pack_batch(data, swo, threads=8)
    return pk.tobytes(), off


@pytest.mark.parametrize("cfg", [2, 3, 4])
def test_parallel_stream_configs(ctx, oracle, cfg):
    """64 pieces of 64 KiB of the bench data (dense config 3: literal runs of
    up to 255 words span several 1 KiB blocks), plus trailing bytes of a
    following message that the stream must not consume."""
    swo = _swo([8192] * 64)
    data = oracle.generate(oracle.preset(cfg), swo)
    stream, off = _stream_of(oracle, data, swo)
    rng = np.random.default_rng(cfg)
    tail = bytes(rng.integers(0, 256, size=3000, dtype=np.uint8))
    bounds, st = _check(ctx, oracle, stream + tail, swo, expect_ok=True)
    assert np.array_equal(bounds, off)


def test_parallel_stream_one_long_piece(ctx, oracle):
    """One 4 MiB segment (SerializePacked.read of a message with one large
    segment): the case the one-wave decoder serialises completely."""
    swo = _swo([8192 * 64])
    data = oracle.generate(oracle.preset(2), _swo([8192] * 64))
    stream, _ = _stream_of(oracle, data, swo)
    bounds, _ = _check(ctx, oracle, stream, swo, expect_ok=True)
    assert int(bounds[-1]) == len(stream)


def test_parallel_stream_ragged_mixes(ctx, oracle):
    """500 ragged pieces (empty ones included) of mixed word classes."""
    from test_gpu_parity import _random_words
    rng = np.random.default_rng(21)
    sizes = [int(s) for s in rng.integers(0, 3000, size=500)]
    sizes[::37] = [0] * len(sizes[::37])
    probs = [.3, .3, .2, .2]
    data = np.concatenate([_random_words(rng, s, probs) for s in sizes]).astype(np.uint8)
    swo = _swo(sizes)
    stream, off = _stream_of(oracle, data, swo)
    bounds, _ = _check(ctx, oracle, stream, swo, expect_ok=True)
    assert np.array_equal(bounds, off)


def test_parallel_stream_literal_and_zero_runs(ctx, oracle):
    """All-nonzero words (0xFF runs of 255 literal words, 2 KiB records),
    all-zero words (2-byte records of 256 words) and alternations, followed by
    1 MiB of junk so the bounded reach still cuts blocks past the end."""
    rng = np.random.default_rng(4)
    pieces = [rng.integers(1, 256, size=8 * 40000, dtype=np.uint8),
              np.zeros(8 * 300000, np.uint8),
              np.tile(np.concatenate([np.zeros(8 * 3, np.uint8), np.full(8 * 5, 9, np.uint8)]), 5000),
              rng.integers(1, 256, size=8 * 1000, dtype=np.uint8)]
    data = np.concatenate(pieces)
    swo = _swo([p.size // 8 for p in pieces])
    stream, off = _stream_of(oracle, data, swo)
    junk = bytes(rng.integers(0, 256, size=1 << 20, dtype=np.uint8))
    bounds, _ = _check(ctx, oracle, stream + junk, swo, expect_ok=True)
    assert np.array_equal(bounds, off)


def test_parallel_stream_errors_match_one_wave(ctx, oracle):
    """Truncated, corrupted and mis-sized streams: the statuses (ETRUNC,
    EOVERRUN) equal the oracle's and the one-wave decoder's."""
    swo = _swo([8192] * 48)
    data = oracle.generate(oracle.preset(2), swo)
    stream, off = _stream_of(oracle, data, swo)
    rng = np.random.default_rng(8)
    # truncated in the middle of piece 30
    cut = int(off[30]) + 777
    _check(ctx, oracle, stream[:cut], swo, expect_ok=False)
    # bytes flipped at random places
    for _ in range(6):
        b = bytearray(stream)
        for i in rng.integers(0, len(b), size=3):
            b[int(i)] = int(rng.integers(0, 256))
        _check(ctx, oracle, bytes(b), swo)
    # piece sizes that do not match the stream: runs across piece boundaries
    sizes = [8192] * 48
    sizes[10] -= 3
    sizes[11] += 3
    _check(ctx, oracle, stream, _swo(sizes))
    sizes = [8192] * 48
    sizes[47] += 100
    _check(ctx, oracle, stream, _swo(sizes), expect_ok=False)


def test_device_stream_decode(ctx, oracle):
    """cpk_decode_stream on device buffers (the path SerializePacked.read takes
    once the bytes are in HBM)."""
    import torch
    swo = _swo([8192] * 32 + [0, 5, 70000])
    data = oracle.generate(oracle.preset(3), swo)
    stream, off = _stream_of(oracle, data, swo)
    pad = (len(stream) + 64 + 15) // 16 * 16
    d_pk = torch.zeros(pad, dtype=torch.uint8, device="cuda")
    d_pk[: len(stream)] = torch.from_numpy(np.frombuffer(stream, np.uint8).copy()).cuda()
    d_swo = torch.from_numpy(swo.astype(np.int64)).cuda()
    d_out = torch.zeros(int(swo[-1]) + 1, dtype=torch.int64, device="cuda")
    d_io = torch.zeros(len(swo), dtype=torch.int64, device="cuda")
    d_st = torch.full((len(swo) - 1,), 99, dtype=torch.int32, device="cuda")
    ctx.decode_stream(d_pk, len(stream), d_swo, d_out, d_io, d_st)
    torch.cuda.synchronize()
    assert int((d_st != 0).sum().item()) == 0
    assert np.array_equal(d_io.cpu().numpy().astype(np.uint64), off)
    got = d_out.cpu().numpy().view(np.uint8)[: data.size]
    assert np.array_equal(got, data)


def test_parallel_stream_garbage_matches_one_wave(ctx, oracle):
    """Random bytes as a packed stream (mostly malformed: truncations, runs
    across piece ends) and valid streams with random byte flips, at sizes
    that take the parallel path: every status, boundary and decoded word
    equals the one-wave decoder's and the oracle's."""
    rng = np.random.default_rng(77)
    for trial in range(6):
        n = int(rng.integers(1, 40))
        sizes = [int(x) for x in rng.integers(0, 30000, size=n)]
        swo = _swo(sizes)
        if trial % 2 == 0:
            stream = bytes(rng.integers(0, 256, size=400_000, dtype=np.uint8))
        else:
            data = oracle.generate(oracle.preset(int(rng.integers(2, 5))), swo)
            b = bytearray(_stream_of(oracle, data, swo)[0])
            for i in rng.integers(0, len(b), size=int(rng.integers(1, 5))):
                b[int(i)] = int(rng.integers(0, 256))
            stream = bytes(b) + bytes(rng.integers(0, 256, size=300_000, dtype=np.uint8))
        _check(ctx, oracle, stream, swo)



@pytest.mark.parametrize("cfg", [2, 3, 4])
def test_mid_size_stream_workgroup_path(ctx, oracle, cfg):
    """Streams of 6-384 KiB reachable bytes take the one-workgroup decoder
    (decode_mw.hip): one piece, ragged pieces with empty ones, junk behind
    the stream, cuts, flips and mis-sized pieces -- statuses, boundaries and
    words equal to the oracle's and to the one-wave decoder's."""
    rng = np.random.default_rng(20 + cfg)
    for sizes in ([3000], [9000], [0, 1, 700, 0, 2500, 64, 3], [int(x) for x in rng.integers(0, 1500, size=20)]):
        swo = _swo(sizes)
        data = oracle.generate(oracle.preset(cfg), swo)
        stream, off = _stream_of(oracle, data, swo)
        junk = bytes(rng.integers(0, 256, size=3000, dtype=np.uint8))
        bounds, _ = _check(ctx, oracle, stream + junk, swo)
        assert np.array_equal(bounds, off)
        for cut in rng.integers(1, len(stream), size=5):
            _check(ctx, oracle, stream[: int(cut)], swo)
        for _ in range(4):
            b = bytearray(stream)
            for i in rng.integers(0, len(b), size=2):
                b[int(i)] = int(rng.integers(0, 256))
            _check(ctx, oracle, bytes(b), swo)
        if len(sizes) > 2 and sizes[1] > 3:
            bad = list(sizes)
            bad[1] -= 3
            bad[2] += 3
            _check(ctx, oracle, stream, _swo(bad))
