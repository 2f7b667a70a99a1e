"""The CPU oracle pinned against the reference's own known-answer tests.

Vectors: tests/golden/reference_kats.json, transcribed from
SerializePackedTest.java:20-60 / :93-105 and SerializeTest.java:90-140 /
:173-189.  assertPacksTo (SerializePackedTest.java:63-91) checks both
directions; so do we.
"""
import json
from pathlib import Path

import numpy as np
import pytest

GOLD = json.loads((Path(__file__).parent / "golden" / "reference_kats.json").read_text())


@pytest.mark.parametrize("kat", GOLD["kats"], ids=[k["source"].split(":")[-1] for k in GOLD["kats"]])
def test_assert_packs_to(oracle, kat):
    u, p = bytes.fromhex(kat["unpacked"]), bytes.fromhex(kat["packed"])
    assert oracle.pack(u) == p
    st, out, used = oracle.unpack(p, len(u))
    assert st == oracle.OK and out == u and used == len(p)


def test_empty_stream_is_decode_error(oracle):
    st, segs, _ = oracle.read_message(b"")
    assert st == oracle.ETRUNC


def test_truncated_stream_is_decode_error(oracle):
    st, segs, _ = oracle.read_message(bytes([17, 0, 127, 0, 0, 0, 0]))
    assert st != oracle.OK


@pytest.mark.parametrize("fr", GOLD["framing"], ids=lambda f: str(f["segments"]))
def test_framing_roundtrip(oracle, fr):
    raw = bytes.fromhex(fr["unpacked_stream"])
    n = fr["segments"]
    segs = [b"".join(int(i).to_bytes(8, "little") for _ in range(i)) for i in range(n)]
    packed = oracle.write_message(segs)
    # pack(table) || pack(seg_i) == packing the unpacked stream piece by piece
    table_len = 4 * ((n + 2) & ~1)
    expect = oracle.pack(raw[:table_len])
    o = table_len
    for s in segs:
        expect += oracle.pack(raw[o:o + len(s)])
        o += len(s)
    assert packed == expect
    st, got, used = oracle.read_message(packed)
    assert st == oracle.OK and got == segs and used == len(packed)


@pytest.mark.parametrize("ov", GOLD["size_overflow"])
def test_negative_segment_size(oracle, ov):
    raw = bytes.fromhex(ov["unpacked_stream"])
    st, _, _ = oracle.read_message(oracle.pack(raw))
    assert st == oracle.EFRAME


def test_segment_over_max_words(oracle):
    """A size over MAX_SEGMENT_WORDS (2^28 - 1) passes the traversal check
    when the limit is raised, then makeByteBufferForWords throws when that
    segment is allocated (Serialize.java:45-53, :165-175); an earlier
    segment is still read first."""
    import struct
    table = struct.pack("<Iii", 1, 1, 1 << 28) + b"\0" * 4
    stream = oracle.pack(table) + oracle.pack(b"\1" * 8)
    st, _, _ = oracle.read_message(stream, traversal_limit_words=1 << 30, out_cap=1 << 12)
    assert st == oracle.EINVAL  # (the oracle's own output bound is checked first)
    st, _, _ = oracle.read_message(stream, traversal_limit_words=1 << 30, out_cap=(1 << 31) + 64)
    assert st == oracle.EFRAME
    table = struct.pack("<Iii", 1, 1, (1 << 28) - 1) + b"\0" * 4
    st, _, _ = oracle.read_message(oracle.pack(table) + oracle.pack(b"\1" * 8),
                                   traversal_limit_words=1 << 30, out_cap=(1 << 31) + 64)
    assert st == oracle.ETRUNC  # allowed size, data missing


def test_misaligned_read(oracle):
    st, _, _ = oracle.unpack(b"\x00\x00", 7)
    assert st == oracle.EINVAL


def test_overrun_and_trailing(oracle):
    # zero run of 3 more words into a 2-word output -> exception in the reference
    st, _, _ = oracle.unpack(bytes([0, 3]), 16)
    assert st == oracle.EOVERRUN
    st, _, _ = oracle.unpack(bytes([0xff] + [1] * 8 + [2] + [1] * 16), 16)
    assert st == oracle.EOVERRUN
    # literal run truncated by end of input: documented divergence -> ETRUNC
    st, _, _ = oracle.unpack(bytes([0xff] + [1] * 8 + [1] + [1] * 3), 16)
    assert st == oracle.ETRUNC


def _classes(words):
    b = words.view(np.uint8).reshape(-1, 8)
    nz = (b != 0).sum(1)
    return nz


def test_roundtrip_random_mixes(oracle):
    rng = np.random.default_rng(7)
    for trial in range(300):
        n = int(rng.integers(0, 700))
        kind = rng.integers(0, 4, size=n)
        w = rng.integers(1, 256, size=(n, 8), dtype=np.uint8)
        for i in range(n):
            if kind[i] == 0:
                w[i] = 0
            elif kind[i] == 1:
                w[i, rng.integers(0, 8)] = 0
            elif kind[i] == 2:
                w[i, rng.choice(8, size=int(rng.integers(2, 8)), replace=False)] = 0
        u = w.tobytes()
        p = oracle.pack(u)
        assert len(p) <= oracle.packed_bound(n)
        st, out, used = oracle.unpack(p, len(u))
        if n == 0:
            assert p == b"" and st == oracle.OK
            continue
        assert st == oracle.OK and out == u and used == len(p)


def test_generator_presets(oracle):
    swo = np.arange(0, 8193 * 4, 8192, dtype=np.uint64)
    for cfg, (zlo, zhi) in {2: (0.4, 0.6), 3: (0.0, 0.12), 4: (0.8, 0.97)}.items():
        d = oracle.generate(oracle.preset(cfg), swo)
        z = (d.view(np.uint64) == 0).mean()
        assert zlo < z < zhi, (cfg, z)
        # deterministic
        assert np.array_equal(d, oracle.generate(oracle.preset(cfg), swo))
        # a single segment generated alone equals its slice of the batch
        one = oracle.generate(oracle.preset(cfg), swo, first=2, count=1)
        assert np.array_equal(one, d[2 * 65536:3 * 65536])


def _run_lengths(z):
    """Lengths of the maximal runs of True in a boolean vector."""
    d = np.diff(np.concatenate([[0], z.astype(np.int8), [0]]))
    return np.flatnonzero(d == -1) - np.flatnonzero(d == 1)


def test_generator_matches_survey_workload(oracle):
    """q (zero byte in a nonzero word) 0.25 / (1/256) / 0.25,
    mean zero run Lz 4 / 1.5 / 64 for configs 2 / 3 / 4, on 64 pieces of
    8192 words.  FastRand.nextInt() is never negative (Common.java:31-38),
    so thresholds are out of 2^31 (round 3's 2^32 doubled every probability)."""
    swo = np.arange(0, 8192 * 65, 8192, dtype=np.uint64)
    spec = {2: (0.25, 0.01, 4.0), 3: (1 / 256, 0.001, 1.5), 4: (0.25, 0.01, 64.0)}
    for cfg, (q, qtol, lz) in spec.items():
        w = oracle.generate(oracle.preset(cfg), swo).view(np.uint64).reshape(64, 8192)
        b = w.view(np.uint8).reshape(64, 8192, 8)
        nzw = w != 0
        qm = (b[nzw] == 0).mean()
        assert abs(qm - q) <= qtol, (cfg, qm)
        runs = np.concatenate([_run_lengths(~nzw[i]) for i in range(64)])
        # runs cut by a piece's first or last word are shorter: keep interior runs
        inner = np.concatenate([_run_lengths(~nzw[i][1:-1]) for i in range(64)])
        assert runs.size and abs(inner.mean() - lz) <= 0.1 * lz, (cfg, inner.mean())


def test_batch_threads_agree(oracle):
    swo = np.concatenate([[0], np.cumsum(np.array([0, 1, 3, 8192, 100, 7, 5000, 0, 2], np.uint64))]).astype(np.uint64)
    d = oracle.generate(oracle.preset(2), swo)
    p1, o1 = oracle.pack_batch(d, swo, threads=1)
    p4, o4 = oracle.pack_batch(d, swo, threads=4)
    assert np.array_equal(p1, p4) and np.array_equal(o1, o4)
    dec, st = oracle.unpack_batch(p1, o1, swo, threads=3)
    assert (st == 0).all() and np.array_equal(dec, d)
