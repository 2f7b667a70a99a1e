"""cpk_read_message / cpk_read_message_host: Serialize.read over
PackedInputStream (Serialize.java:119-178) for ONE message at the front of a
packed stream whose length is not known in advance -- the table read and
validated on the device, then every segment decoded back to back, in one
enqueue.  Each case is checked against the oracle's Serialize.read
(oracle/packed_oracle.c:cpko_read_message): status, segments and the bytes
consumed; streams reaching 64 KiB and more take the parallel block path, and the
one-wave decoder (CPK_STREAM_ONE_WAVE=1) must agree with it.
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _rd(ctx, data: bytes, **kw):
    return ctx.read_message_host(np.frombuffer(data, np.uint8), **kw)


def _expect(oracle, data: bytes, limit=8 * 1024 * 1024):
    # (an output capacity for any table, up to a 2^28-word segment: the
    # oracle's CPK_EINVAL for a short buffer would hide the real status;
    # the zero pages are never touched beyond the message's words)
    st, segs, used = oracle.read_message(data, traversal_limit_words=limit, out_cap=(1 << 31) + 4096)
    return st, segs, used


def _check(ctx, oracle, data: bytes, both=False, limit=8 * 1024 * 1024):
    st, segs, used, _ = _rd(ctx, data, traversal_limit_words=limit)
    ost, osegs, oused = _expect(oracle, data, limit)
    assert st == ost, (st, ost)
    if st == 0:
        assert used == oused
        assert segs == osegs
    if both:
        os.environ["CPK_STREAM_ONE_WAVE"] = "1"
        try:
            st2, segs2, used2, _ = _rd(ctx, data, traversal_limit_words=limit)
        finally:
            os.environ.pop("CPK_STREAM_ONE_WAVE")
        assert (st2, used2) == (st, used) and segs2 == segs
    return st, segs, used


def _msg(rng, oracle, sizes, probs=(.4, .3, .2, .1)):
    from test_gpu_parity import _random_words
    segs = [_random_words(rng, s, list(probs)).tobytes() for s in sizes]
    return segs, oracle.write_message(segs)


def test_read_message_small_followed_by_more(ctx, oracle):
    """Messages of 1-512 segments (empty ones included), each followed by the
    next message: only the first is consumed."""
    rng = np.random.default_rng(5)
    for sizes in ([3], [0], [1, 0, 7], [5] * 7, [int(x) for x in rng.integers(0, 40, size=512)],
                  [0] * 512, [int(x) for x in rng.integers(0, 3000, size=9)]):
        segs, pk = _msg(rng, oracle, sizes)
        _, nxt = _msg(rng, oracle, [4, 4])
        st, got, used = _check(ctx, oracle, pk + nxt)
        assert st == 0 and got == segs and used == len(pk)


def test_read_message_large_single_segment(ctx, oracle):
    """A 4 MiB single-segment message of config-2 data (the parallel stream
    path), followed by a second message; and a dense config-3 one."""
    rng = np.random.default_rng(6)
    for cfg in (2, 3):
        swo = np.array([0, 8192 * 64], np.uint64)
        data = oracle.generate(oracle.preset(cfg), np.arange(65, dtype=np.uint64) * 8192)
        seg = data[: 8 * int(swo[1])].tobytes()
        pk = oracle.write_message([seg])
        _, nxt = _msg(rng, oracle, [100, 3])
        st, got, used = _check(ctx, oracle, pk + nxt, both=True)
        assert st == 0 and got == [seg] and used == len(pk)


def test_read_message_many_segments_large(ctx, oracle):
    """Four config-3 segments of mixed sizes (SerializePacked.write of a
    config-3 message) with trailing junk."""
    rng = np.random.default_rng(7)
    sizes = [512, 32768, 2048, 16384]
    swo = np.concatenate([[0], np.cumsum(sizes)]).astype(np.uint64)
    data = oracle.generate(oracle.preset(3), swo)
    segs = [data[8 * int(swo[i]): 8 * int(swo[i + 1])].tobytes() for i in range(4)]
    pk = oracle.write_message(segs)
    junk = bytes(rng.integers(0, 256, size=100_000, dtype=np.uint8))
    st, got, used = _check(ctx, oracle, pk + junk, both=True)
    assert st == 0 and got == segs and used == len(pk)


def test_read_message_truncated_everywhere(ctx, oracle):
    """Every cut of a small message ends inside it: ETRUNC (the channel
    reader's cue to take more bytes), as Serialize.read's premature EOF."""
    rng = np.random.default_rng(8)
    segs, pk = _msg(rng, oracle, [2, 0, 9, 1])
    for cut in range(len(pk)):
        st, _, _ = _check(ctx, oracle, pk[:cut])
        assert st == -2, cut
    # and a few cuts of a large one (parallel path)
    data = oracle.generate(oracle.preset(2), np.arange(65, dtype=np.uint64) * 8192)
    big = oracle.write_message([data[: 8 * 8192 * 64].tobytes()])
    for cut in (9, 4000, len(big) // 2, len(big) - 1):
        st, _, _ = _check(ctx, oracle, big[:cut], both=True)
        assert st == -2


def test_read_message_bad_tables(ctx, oracle):
    """Segment tables Serialize.read rejects (Serialize.java:125-163, :45-53):
    count over 512, negative sizes, over the traversal limit, a segment over
    2^28 - 1 words -- each CPK_EFRAME like the oracle."""
    import struct
    rng = np.random.default_rng(9)
    cases = []
    cases.append(struct.pack("<iI", 512, 1))                      # 513 segments
    cases.append(struct.pack("<ii", 0, -1))                        # negative seg 0
    cases.append(struct.pack("<iiii", 2, 1, -5, 0))                # negative seg 2
    cases.append(struct.pack("<iI", 0, (1 << 28)))                 # over 2^28 - 1
    for raw in cases:
        words = raw + b"\0" * (-len(raw) % 8)
        pk = oracle.pack(words) + bytes(rng.integers(0, 256, size=64, dtype=np.uint8))
        st, _, _ = _check(ctx, oracle, pk, limit=1 << 40)
        assert st == -7
    segs, pk = _msg(rng, oracle, [100, 100])
    st, _, _ = _check(ctx, oracle, pk, limit=150)  # over the traversal limit
    assert st == -7


def test_read_message_corrupted_matches_oracle(ctx, oracle):
    """Byte flips anywhere in a message (tables and segments): status,
    segments and consumed bytes equal the oracle's Serialize.read."""
    rng = np.random.default_rng(10)
    for trial in range(40):
        segs, pk = _msg(rng, oracle, [int(x) for x in rng.integers(0, 400, size=int(rng.integers(1, 6)))])
        b = bytearray(pk + oracle.write_message([b"\1" * 64]))
        for i in rng.integers(0, len(pk), size=int(rng.integers(1, 3))):
            b[int(i)] = int(rng.integers(0, 256))
        _check(ctx, oracle, bytes(b))


def test_read_message_capacity(ctx, oracle):
    """Segments over the caller's capacity: CPK_ENOMEM with the count and
    words needed, nothing decoded; the sized call then succeeds."""
    rng = np.random.default_rng(11)
    segs, pk = _msg(rng, oracle, [300, 200])
    st, _, _, info = _rd(ctx, pk, out_cap_words=499)
    assert st == -5 and int(info[2]) == 2 and int(info[3]) == 500
    st, got, used, _ = _rd(ctx, pk, out_cap_words=500)
    assert st == 0 and got == segs and used == len(pk)


@pytest.mark.parametrize("sizes", [[4000, 0, 70000, 9], [3000, 0, 9000, 5]])
def test_read_message_device_form(ctx, oracle, sizes):
    """cpk_read_message on device buffers: the info row and the decoded
    words in HBM, the segments after the table's words (the parallel block
    path, and the one-workgroup decoder for the mid-size stream)."""
    import torch
    import capnp_packed as cp
    rng = np.random.default_rng(12)
    segs, pk = _msg(rng, oracle, sizes)
    stream = pk + bytes(rng.integers(0, 256, size=5000, dtype=np.uint8))
    d_pk = torch.zeros((len(stream) + 64 + 15) // 16 * 16, dtype=torch.uint8, device="cuda")
    d_pk[: len(stream)] = torch.from_numpy(np.frombuffer(stream, np.uint8).copy()).cuda()
    words = sum(len(s) for s in segs) // 8
    d_out = torch.zeros(words + cp.MSG_HEAD_WORDS, dtype=torch.int64, device="cuda")
    d_info = torch.zeros(cp.MSG_INFO_WORDS, dtype=torch.int64, device="cuda")
    ctx.read_message(d_pk, len(stream), d_out, d_info)
    torch.cuda.synchronize()
    info = d_info.cpu().numpy()
    assert info[0] == 0 and info[1] == len(pk) and info[2] == len(sizes) and info[3] == words
    out = d_out.cpu().numpy().view(np.uint8)
    got = [out[8 * int(info[4 + i]): 8 * int(info[5 + i])].tobytes() for i in range(4)]
    assert got == segs


def test_small_host_paths_back_to_back(ctx, oracle):
    """The one-launch host paths (read and write under 64 KiB) return once
    their kernel's completion flag turns, with no stream synchronisation:
    back-to-back calls whose pinned input changes every time must each see
    their own bytes (a kernel must not read lines an earlier call left in
    L2) and hand back their own results."""
    rng = np.random.default_rng(13)
    msgs = [_msg(rng, oracle, [int(x) for x in rng.integers(1, 600, size=int(rng.integers(1, 4)))])
            for _ in range(6)]
    f0 = ctx.small_fallbacks()
    for k in range(300):
        segs, pk = msgs[k % len(msgs)]
        st, got, used, _ = _rd(ctx, pk)
        assert st == 0 and got == segs and used == len(pk), k
        packed, _ = ctx.encode_messages_host([segs])
        assert bytes(packed) == pk, k
    # no call lost its kernel's completion flag (a late launch may take the
    # 5 ms stream-sync fallback on a busy box; that is not counted)
    assert ctx.small_fallbacks() == f0


def test_read_message_mid_size_workgroup_path(ctx, oracle):
    """Streams of 6-128 KiB from host memory (6-512 KiB device-resident) take
    the one-launch workgroup decoder (decode_mw.hip: a piece's windows spread
    over 16 waves, entries chained between them): clean messages of 1-9
    segments (empty ones included) with the next message behind them, cuts
    anywhere (ETRUNC), byte flips (status, segments and bytes consumed equal
    the oracle's Serialize.read) and both dense and sparse data.  Host
    streams of 128-512 KiB, which now take the block path, are also read
    through a context whose workgroup bound is 512 KiB (CPK_RM_MW_MAX_KB)."""
    import capnp_packed as cp
    os.environ["CPK_RM_MW_MAX_KB"] = "512"
    try:
        ctx512 = cp.Context(0)
    finally:
        os.environ.pop("CPK_RM_MW_MAX_KB")
    rng = np.random.default_rng(14)
    for cfg_probs in ((.4, .3, .2, .1), (.05, .05, .1, .8), (.9, .05, .03, .02)):
        for sizes in ([3000], [8192 * 4], [0, 5000, 0, 12000], [int(x) for x in rng.integers(0, 6000, size=9)],
                      [int(x) if x > 40 else 0 for x in rng.integers(0, 400, size=300)]):
            segs, pk = _msg(rng, oracle, sizes, cfg_probs)
            if not 6 * 1024 <= len(pk) < 512 * 1024:
                continue
            _, nxt = _msg(rng, oracle, [7, 0, 3])
            st, got, used = _check(ctx, oracle, pk + nxt)
            assert st == 0 and got == segs and used == len(pk)
            if len(pk) >= 128 * 1024:
                st, got, used = _check(ctx512, oracle, pk + nxt)
                assert st == 0 and got == segs and used == len(pk)
                for cut in (len(pk) // 2, len(pk) - 1):
                    assert _check(ctx512, oracle, pk[:cut])[0] == -2, cut
            for cut in sorted(set([1, 8, 9, 17, len(pk) // 3, len(pk) // 2, len(pk) - 1] +
                                  [int(c) for c in rng.integers(1, len(pk), size=12)])):
                st, _, _ = _check(ctx, oracle, pk[:cut])
                assert st == -2, cut
            for _ in range(6):
                b = bytearray(pk + nxt)
                for i in rng.integers(0, len(pk), size=int(rng.integers(1, 4))):
                    b[int(i)] = int(rng.integers(0, 256))
                _check(ctx, oracle, bytes(b))
