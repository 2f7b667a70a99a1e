"""Parity of the HIP codec with the CPU oracle (which is pinned by the
reference's KATs, tests/test_oracle.py).  Bit-exact: this is byte work.

Mirrors SerializePackedTest.assertPacksTo (SerializePackedTest.java:63-91):
every case is checked in both directions, through the C ABI.
"""
import json
from pathlib import Path

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

GOLD = json.loads((Path(__file__).parent / "golden" / "reference_kats.json").read_text())


def _swo(sizes):
    return np.concatenate([[0], np.cumsum(np.asarray(sizes, dtype=np.uint64))]).astype(np.uint64)


def _check_batch(ctx, oracle, data, swo):
    """Encode on the GPU, compare with the oracle byte for byte, decode back."""
    pk, off = ctx.encode_host(data, swo)
    opk, ooff = oracle.pack_batch(data, swo, threads=8)
    assert np.array_equal(off, ooff), "piece offsets differ"
    assert np.array_equal(pk, opk), "packed bytes differ"
    dec, st = ctx.decode_host(pk, off, swo)
    assert (st == 0).all(), st[st != 0][:8]
    assert np.array_equal(dec, data)
    return pk, off


def test_assert_packs_to_kats(ctx, oracle):
    """Each SerializePackedTest.java:20-60 vector as a piece, then all of them
    as one batch (pieces are independent write() calls)."""
    import capnp_packed as cp
    datas = []
    for k in GOLD["kats"]:
        u, p = bytes.fromhex(k["unpacked"]), bytes.fromhex(k["packed"])
        a = np.frombuffer(u, dtype=np.uint8)
        swo = _swo([len(u) // 8])
        pk, off = ctx.encode_host(a, swo)
        assert pk.tobytes() == p, k["source"]
        dec, st = ctx.decode_host(np.frombuffer(p, np.uint8), np.array([0, len(p)], np.uint64), swo)
        assert st[0] == cp.OK and dec.tobytes() == u, k["source"]
        datas.append(u)
    data = np.frombuffer(b"".join(datas), dtype=np.uint8)
    _check_batch(ctx, oracle, data, _swo([len(d) // 8 for d in datas]))


def _random_words(rng, n, probs):
    kind = rng.choice(4, size=n, p=probs)
    w = rng.integers(1, 256, size=(n, 8), dtype=np.uint8)
    w[kind == 0] = 0
    one = np.where(kind == 1)[0]
    w[one, rng.integers(0, 8, size=one.size)] = 0
    for i in np.where(kind == 2)[0]:
        w[i, rng.choice(8, size=int(rng.integers(2, 8)), replace=False)] = 0
    return w.reshape(-1)


@pytest.mark.parametrize("mix", ["uniform", "dense", "sparse", "lonely_ff"])
def test_random_class_mixes(ctx, oracle, mix):
    rng = np.random.default_rng(abs(hash(mix)) % 2**32)
    probs = {"uniform": [.25, .25, .25, .25], "dense": [.01, .7, .285, .005],
             "sparse": [.85, .05, .05, .05], "lonely_ff": [.45, .05, .05, .45]}[mix]
    sizes = list(rng.integers(0, 8193, size=40)) + [0, 1, 2, 255, 256, 257, 8191, 8192]
    rng.shuffle(sizes)
    # ragged pieces so that piece starts land at every byte phase
    data = np.concatenate([_random_words(rng, int(s), probs) for s in sizes]).astype(np.uint8)
    _check_batch(ctx, oracle, data, _swo(sizes))


def test_long_literal_chains(ctx, oracle):
    """D/L stretches far longer than 256 words: the 0xFF-run chain
    (PackedOutputStream.java:145-161), incl. the 255 cap and L heads."""
    rng = np.random.default_rng(3)
    pieces = []
    for n, pl in [(8192, 0.0), (8192, 0.3), (8192, 0.9), (5000, 0.5), (600, 0.99), (300, 0.0)]:
        w = rng.integers(1, 256, size=(n, 8), dtype=np.uint8)
        lmask = rng.random(n) < pl
        w[lmask, rng.integers(0, 8, size=int(lmask.sum()))] = 0
        pieces.append(w.reshape(-1))
    # one all-ones piece: 200 words -> 0xFF, 199 (SerializePackedTest.java:54-60)
    pieces.append(np.ones(8 * 8192, dtype=np.uint8))
    pieces.append(np.zeros(8 * 8192, dtype=np.uint8))   # 0x00 runs capped at 255
    data = np.concatenate(pieces)
    _check_batch(ctx, oracle, data, _swo([len(p) // 8 for p in pieces]))


@pytest.mark.parametrize("cfg", [2, 3, 4])
def test_synthetic_configs(ctx, oracle, cfg):
    """The bench workloads at 64 KiB pieces (configs 2/4; dense 3 at 64 KiB),
    host-generated here and device-generated below."""
    swo = _swo([8192] * 64 + [8191, 17, 4096])
    data = oracle.generate(oracle.preset(cfg), swo)
    _check_batch(ctx, oracle, data, swo)


def test_device_generator_matches_host(ctx, oracle):
    import torch
    import capnp_packed as cp
    swo = _swo([8192] * 8 + [3, 100, 0, 5000])
    for cfg in (2, 3, 4):
        d_swo = torch.from_numpy(swo.astype(np.int64)).cuda()
        d = torch.zeros(int(swo[-1]) + 1, dtype=torch.int64, device="cuda")
        ctx.generate(cp.preset(cfg), d_swo, d)
        torch.cuda.synchronize()
        host = oracle.generate(oracle.preset(cfg), swo)
        assert np.array_equal(d.cpu().numpy().view(np.uint8)[: host.size], host)


def test_device_resident_roundtrip(ctx, oracle):
    """The bench path: device generator -> encode_batch -> decode_batch."""
    import torch
    import capnp_packed as cp
    n = 512
    swo = _swo([8192] * n)
    d_swo = torch.from_numpy(swo.astype(np.int64)).cuda()
    d_in = torch.empty(n * 8192, dtype=torch.int64, device="cuda")
    ctx.generate(cp.preset(2), d_swo, d_in)
    cap = cp.batch_capacity(swo)
    d_pk = torch.empty((cap + 15) // 16 * 16, dtype=torch.uint8, device="cuda")
    d_off = torch.empty(n + 1, dtype=torch.int64, device="cuda")
    ctx.encode_batch(d_in, d_swo, 8192, d_pk, d_off)
    d_out = torch.empty_like(d_in)
    d_st = torch.empty(n, dtype=torch.int32, device="cuda")
    ctx.decode_batch(d_pk, d_off, d_swo, d_out, d_st)
    cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
    ctx.count_mismatch(d_in, d_out, n * 8192, cnt)
    torch.cuda.synchronize()
    assert int(cnt.item()) == 0
    assert int((d_st != 0).sum().item()) == 0
    off = d_off.cpu().numpy().astype(np.uint64)
    host = oracle.generate(oracle.preset(2), swo)
    opk, ooff = oracle.pack_batch(host, swo, threads=8)
    assert np.array_equal(off, ooff)
    assert np.array_equal(d_pk[: int(off[-1])].cpu().numpy(), opk)


def _corrupt_cases(oracle, rng):
    """Valid packed pieces with bytes flipped / truncated / extended."""
    cases = []
    for _ in range(300):
        n = int(rng.integers(1, 64))
        u = _random_words(rng, n, [.3, .3, .2, .2]).tobytes()
        p = bytearray(oracle.pack(u))
        r = rng.integers(0, 4)
        if r == 0 and len(p) > 1:
            p = p[: int(rng.integers(0, len(p)))]                   # truncate
        elif r == 1:
            p += bytes(rng.integers(0, 256, size=int(rng.integers(1, 12)), dtype=np.uint8))
        elif r == 2 and len(p):
            i = int(rng.integers(0, len(p)))
            p[i] = int(rng.integers(0, 256))                       # flip one byte
        else:
            n = max(1, n + int(rng.integers(-2, 3)))               # wrong piece size
        cases.append((bytes(p), n))
    return cases


def test_malformed_streams_match_reference_errors(ctx, oracle):
    """Per-piece status equals the oracle's for corrupted input (the reference
    throws exactly when the oracle reports an error, SURVEY.md 8a policy)."""
    rng = np.random.default_rng(11)
    cases = _corrupt_cases(oracle, rng)
    packed = b"".join(p for p, _ in cases)
    in_off = _swo([len(p) for p, _ in cases])
    swo = _swo([n for _, n in cases])
    dec, st = ctx.decode_host(np.frombuffer(packed, np.uint8), in_off, swo)
    for i, (p, n) in enumerate(cases):
        ost, out, used = oracle.unpack(p, 8 * n)
        if ost == oracle.OK and used != len(p):
            ost = oracle.ETRAILING
        assert st[i] == ost, (i, p.hex(), n, st[i], ost)
        if ost == oracle.OK:
            assert dec[8 * int(swo[i]): 8 * int(swo[i + 1])].tobytes() == out


def test_malformed_long_pieces_match_reference_errors(ctx, oracle):
    """Multi-window pieces (up to 8192 words, up to ~80 KB packed) corrupted
    anywhere, and pieces ending in a 255-word literal run (a 2,050-byte
    record) cut short by every distance up to and past that record: the
    decoder checks errors only in windows within one window plus one record
    of the piece's end or reaching its last word, so the statuses must still
    equal the oracle's wherever the damage lies."""
    rng = np.random.default_rng(23)
    cases = []
    for k in range(120):
        n = int(rng.integers(600, 8193))
        probs = [[.3, .3, .2, .2], [.02, .6, .37, .01], [.05, .0, .0, .95]][k % 3]
        u = _random_words(rng, n, probs).tobytes()
        p = bytearray(oracle.pack(u))
        r = k % 4
        if r == 0:
            p = p[: int(rng.integers(max(0, len(p) - 6000), len(p)))]          # truncate near the end
        elif r == 1:
            p += bytes(rng.integers(0, 256, size=int(rng.integers(1, 40)), dtype=np.uint8))
        elif r == 2:
            for _ in range(int(rng.integers(1, 4))):
                i = int(rng.integers(0, len(p)))
                p[i] = int(rng.integers(0, 256))                               # flip anywhere
        else:
            n = max(1, n + int(rng.integers(-300, 301)))                       # wrong piece size
        cases.append((bytes(p), n))
    # a tail of 255 all-nonzero words after mixed words: its 0xFF record is
    # the piece's last, 2,050 bytes long; cut it by 1 .. 2,100 bytes
    for cut in (1, 2, 7, 8, 9, 10, 11, 100, 1000, 2040, 2049, 2050, 2051, 2100):
        head = _random_words(rng, 3000, [.3, .3, .2, .2]).tobytes()
        tail = rng.integers(1, 256, size=8 * 256, dtype=np.uint8).tobytes()
        p = oracle.pack(head + tail)
        cases.append((p[: len(p) - cut], 3256))
        cases.append((p, 3256 - int(rng.integers(1, 300))))                   # run past the piece
    packed = b"".join(p for p, _ in cases)
    in_off = _swo([len(p) for p, _ in cases])
    swo = _swo([n for _, n in cases])
    dec, st = ctx.decode_host(np.frombuffer(packed, np.uint8), in_off, swo)
    for i, (p, n) in enumerate(cases):
        ost, out, used = oracle.unpack(p, 8 * n)
        if ost == oracle.OK and used != len(p):
            ost = oracle.ETRAILING
        assert st[i] == ost, (i, len(p), n, st[i], ost)
        if ost == oracle.OK:
            assert dec[8 * int(swo[i]): 8 * int(swo[i + 1])].tobytes() == out


def test_serialize_packed_message(ctx, oracle):
    """SerializePacked.write = pack(table) || pack(seg0) || ... (Serialize.java
    :256-288): the table is one more piece of the batch."""
    rng = np.random.default_rng(5)
    segs = [_random_words(rng, int(s), [.4, .2, .2, .2]).tobytes() for s in (0, 1, 7, 4000, 33)]
    n = len(segs)
    table = (n - 1).to_bytes(4, "little") + b"".join((len(s) // 8).to_bytes(4, "little") for s in segs)
    if len(table) % 8:
        table += b"\0" * 4
    pieces = [table] + segs
    data = np.frombuffer(b"".join(pieces), np.uint8)
    swo = _swo([len(p) // 8 for p in pieces])
    pk, off = _check_batch(ctx, oracle, data, swo)
    assert pk.tobytes() == oracle.write_message(segs)
    st, got, _ = oracle.read_message(pk.tobytes())
    assert st == 0 and got == segs


def test_stream_decode_message(ctx, oracle):
    """SerializePacked.read: the reader knows each segment's size from the
    table but not where its packed bytes end -- each read() stops when its
    piece is full (PackedInputStream.java:35-140, Serialize.java:165-175)."""
    rng = np.random.default_rng(9)
    for trial in range(20):
        nseg = int(rng.integers(1, 6))
        segs = [_random_words(rng, int(rng.integers(0, 9000)), [.3, .3, .2, .2]).tobytes()
                for _ in range(nseg)]
        stream = oracle.write_message(segs)
        table = (nseg - 1).to_bytes(4, "little") + b"".join((len(s) // 8).to_bytes(4, "little") for s in segs)
        if len(table) % 8:
            table += b"\0" * 4
        pieces = [table] + segs
        swo = _swo([len(p) // 8 for p in pieces])
        extra = bytes(rng.integers(0, 256, size=int(rng.integers(0, 40)), dtype=np.uint8))
        dec, bounds, st = ctx.decode_stream_host(np.frombuffer(stream + extra, np.uint8), swo)
        assert (st == 0).all(), st
        assert dec.tobytes() == b"".join(pieces)
        assert int(bounds[-1]) == len(stream)
    # truncated stream -> DecodeException (SerializePackedTest.java:100-105)
    dec, bounds, st = ctx.decode_stream_host(np.frombuffer(bytes([17, 0, 127, 0, 0, 0, 0]), np.uint8),
                                             _swo([1, 127]))
    assert st[0] != 0 or st[1] != 0


# ---- pieces larger than one 8192-word tile (tiled encoder) -----------------
D8 = np.full(8, 7, np.uint8)
L8 = np.array([0, 1, 2, 3, 4, 5, 6, 7], np.uint8)
Z8 = np.zeros(8, np.uint8)


def _runs_piece(rng, n):
    """Long Z / D / L / D-L runs placed to cross tile boundaries."""
    import step_model
    return np.frombuffer(step_model.rand_piece(rng, n), np.uint8)


def test_tiled_pieces_random(ctx, oracle):
    rng = np.random.default_rng(21)
    sizes = [8193, 16384, 16385, 20000, 8192 * 5 + 3, 70000] + list(rng.integers(8193, 60000, size=10))
    sizes += [0, 5, 8192]
    pieces = [_runs_piece(rng, int(s)) if s else np.zeros(0, np.uint8) for s in sizes]
    data = np.concatenate(pieces)
    _check_batch(ctx, oracle, data, _swo(sizes))


def test_tiled_boundary_runs(ctx, oracle):
    """Runs that start / end at, just before and just after tile boundaries,
    whole tiles of one run (zero: phase carried; all-D: head distance
    min(d, 256); D/L with L words: chain carried)."""
    T = 8192
    pieces = [
        [Z8] * (5 * T + 17), [D8] * (4 * T + 300), [L8] * (3 * T + 1),
        [L8] * (T - 100) + [D8] + [L8] * (2 * T), [D8] * (T - 1) + [L8] * (T + 5) + [D8] * (T + 7),
        [Z8] * (T - 255) + [D8] * (T + 256) + [Z8] * (T + 257),
        [L8] * (T - 256) + [D8] * 2 + [L8] * (T + 3),
        [D8] * (T + 1), [Z8] * (T + 1), [Z8] * T + [D8] * T + [L8] * T + [Z8] * 3,
        [L8] * (2 * T - 255) + [D8] + [L8] * 600,
        [D8] * 100 + [Z8] * (2 * T) + [D8] * (T + 40),
    ]
    rng = np.random.default_rng(4)
    for lead in (0, 1, 255, 256, 257):   # shift every boundary pattern
        parts = [np.concatenate([rng.integers(1, 256, size=8 * lead, dtype=np.uint8)] + p) for p in pieces]
        data = np.concatenate(parts)
        _check_batch(ctx, oracle, data, _swo([len(p) // 8 for p in parts]))


def test_like_sized_large_pieces(ctx, oracle):
    """Like-sized pieces over one 8192-word chunk (the default choice sends
    them to the single pass as several units each, chained by their run
    state): random sizes within a factor of two, runs crossing every chunk
    boundary, and dense config-3 pieces of 64 Ki words."""
    rng = np.random.default_rng(31)
    sizes = [int(s) for s in rng.integers(12000, 24000, size=20)]
    pieces = [_runs_piece(rng, s) for s in sizes]
    T = 8192
    pieces += [np.concatenate([Z8] * (2 * T + 5)), np.concatenate([D8] * (2 * T - 3)),
               np.concatenate([L8] * (T - 100) + [D8] + [L8] * (T + 200)),
               np.concatenate([D8] * (T + 300) + [Z8] * (T - 300) + [D8] * 20)]
    data = np.concatenate(pieces)
    _check_batch(ctx, oracle, data, _swo([len(p) // 8 for p in pieces]))
    swo = _swo([65536] * 6)
    _check_batch(ctx, oracle, oracle.generate(oracle.preset(3), swo), swo)


def test_config3_messages(ctx, oracle):
    """messages of 4 segments of 4-256 KiB, dense
    (<10 % zero words), each preceded by its segment-table piece."""
    rng = np.random.default_rng(8)
    sizes = []
    for m in range(12):
        segs = [int(rng.choice([512, 1024, 2048, 4096, 8192, 16384, 32768])) for _ in range(4)]
        sizes += [3] + segs   # table: (4 segments) -> 1 + 4 u32 = 20 B -> 3 words
    swo = _swo(sizes)
    data = oracle.generate(oracle.preset(3), swo)
    _check_batch(ctx, oracle, data, swo)


def test_tiled_path_for_small_pieces(ctx, oracle):
    """max_seg_words = 0 (unknown) takes the tiled path for any batch."""
    import torch
    rng = np.random.default_rng(12)
    sizes = list(rng.integers(0, 20000, size=30)) + [8192, 1, 0]
    swo = _swo(sizes)
    data = oracle.generate(oracle.preset(2), swo)
    d_swo = torch.from_numpy(swo.astype(np.int64)).cuda()
    d_in = torch.from_numpy(np.concatenate([data, np.zeros(8, np.uint8)]).view(np.int64).copy()).cuda()
    cap = batch_capacity_16(swo)
    d_pk = torch.zeros(cap, dtype=torch.uint8, device="cuda")
    d_off = torch.zeros(len(sizes) + 1, dtype=torch.int64, device="cuda")
    ctx.encode_batch(d_in, d_swo, 0, d_pk, d_off)
    assert ctx.take_error() == 0
    opk, ooff = oracle.pack_batch(data, swo, threads=8)
    off = d_off.cpu().numpy().astype(np.uint64)
    assert np.array_equal(off, ooff)
    assert np.array_equal(d_pk[: int(off[-1])].cpu().numpy(), opk)


def batch_capacity_16(swo):
    import capnp_packed as cp
    return (cp.batch_capacity(swo) + 15) // 16 * 16


def test_wrong_size_hint_is_reported(ctx, oracle):
    """A piece larger than max_seg_words: no fault, reported by take_error."""
    import torch
    import capnp_packed as cp
    # (the last case: many pieces far over a hint above one chunk -- the
    # unit table is sized from the hint, so no slack may hide an overrun)
    for sizes, hint in (([9000, 10], 100), ([30000, 10], 9000), ([40000] * 1000, 9000)):
        swo = _swo(sizes)
        d_swo = torch.from_numpy(swo.astype(np.int64)).cuda()
        d_in = torch.ones(int(swo[-1]), dtype=torch.int64, device="cuda")
        d_pk = torch.zeros(batch_capacity_16(swo), dtype=torch.uint8, device="cuda")
        d_off = torch.zeros(len(sizes) + 1, dtype=torch.int64, device="cuda")
        ctx.encode_batch(d_in, d_swo, hint, d_pk, d_off)
        assert ctx.take_error() == cp.EINVAL
        assert ctx.take_error() == cp.OK


def test_short_stretch_after_long(ctx, oracle):
    """A short D/L stretch whose 0xFF head lies within 255 words of a long
    stretch's last head: the head is not a member of the other stretch's run
    (PackedOutputStream.java:133-161 scan is per stretch)."""
    pieces = []
    for sep in ([Z8], [np.array([1, 0, 0, 2, 0, 3, 0, 0], np.uint8)]):
        for gap in (0, 5, 100, 250):
            p = [D8] * 300 + sep + [L8] * gap + [D8] + [L8] * 3 + sep + [D8] * 2
            pieces.append(np.concatenate(p))
            p = [L8] * 10 + [D8] * 700 + sep + [L8] * gap + [D8] * 3
            pieces.append(np.concatenate(p))
    data = np.concatenate(pieces)
    _check_batch(ctx, oracle, data, _swo([len(p) // 8 for p in pieces]))


@pytest.mark.parametrize("enc", ["default", "0", "4"])
def test_every_encoder_matches_oracle(oracle, enc, monkeypatch):
    """Every encoder on one mixed batch: pieces of 0..20000 words, long D/L
    stretches, long zero runs."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    import capnp_packed as cp
    if enc != "default":
        monkeypatch.setenv("CPK_ENCODER", enc)
    c = cp.Context(0)
    try:
        rng = np.random.default_rng(1234)
        sizes = [0, 1, 63, 64, 65, 255, 256, 257, 8191, 8192, 8193, 20000] + \
            list(rng.integers(0, 3000, size=24))
        parts = []
        for i, n in enumerate(sizes):
            probs = [[.25, .25, .25, .25], [.01, .7, .285, .005], [.9, .04, .03, .03]][i % 3]
            w = _random_words(rng, int(n), probs).reshape(-1, 8)
            if i % 4 == 1 and n > 800:  # a D/L stretch of 600 words
                w[100:700] = rng.integers(1, 256, size=(600, 8), dtype=np.uint8)
                w[100:700:7, 3] = 0
            parts.append(w.reshape(-1))
        data = np.concatenate(parts)
        _check_batch(c, oracle, data, _swo(sizes))
    finally:
        c.close()


def test_large_single_pieces(ctx, oracle):
    """Pieces of 2^21 and 3 * 2^20 + 17 words (the default encoder walks a
    piece with one wave; its step / word indices are 32-bit) and the decoder's
    many windows per piece."""
    rng = np.random.default_rng(77)
    sizes = [1 << 21, 3 * (1 << 20) + 17, 5]
    parts = []
    for i, n in enumerate(sizes):
        probs = [[.5, .2, .2, .1], [.05, .6, .3, .05], [.9, .04, .03, .03]][i % 3]
        parts.append(_random_words(rng, n, probs))
    _check_batch(ctx, oracle, np.concatenate(parts), _swo(sizes))


@pytest.mark.parametrize("chunk_kb", ["1", "64"])
def test_host_forms_pipelined_chunks(ctx, oracle, chunk_kb, monkeypatch):
    """cpk_encode_host / cpk_decode_host cut a batch into chunks of whole
    pieces that flow through two pinned staging slots (host_pipe.hip): many
    chunks, a piece larger than a chunk, empty pieces, a malformed tail."""
    monkeypatch.setenv("CPK_HOST_CHUNK_KB", chunk_kb)
    rng = np.random.default_rng(int(chunk_kb))
    sizes = [0, 3, 9000, 0, 1] + list(rng.integers(0, 2500, size=60)) + [20000, 7, 0]
    parts = [_random_words(rng, int(s), [.4, .3, .2, .1]) for s in sizes]
    _check_batch(ctx, oracle, np.concatenate(parts), _swo(sizes))
    # per-piece statuses survive the chunking
    cases = _corrupt_cases(oracle, rng)
    packed = b"".join(p for p, _ in cases)
    dec, st = ctx.decode_host(np.frombuffer(packed, np.uint8), _swo([len(p) for p, _ in cases]),
                              _swo([n for _, n in cases]))
    for i, (p, n) in enumerate(cases):
        ost, _, used = oracle.unpack(p, 8 * n)
        if ost == oracle.OK and used != len(p):
            ost = oracle.ETRAILING
        assert st[i] == ost, (i, st[i], ost)


@pytest.mark.parametrize("chunk_kb", [None, "1"])
def test_encode_host_first_offset_above_zero(ctx, oracle, chunk_kb, monkeypatch):
    """cpk_encode_host with seg_word_off[0] > 0: the pieces are words
    [swo[i], swo[i+1]) of the caller's buffer, on the one-launch small path
    (no CPK_HOST_CHUNK_KB) and on the pipelined chunks alike (the
    small path once copied from word 0)."""
    if chunk_kb:
        monkeypatch.setenv("CPK_HOST_CHUNK_KB", chunk_kb)
    rng = np.random.default_rng(17)
    data = _random_words(rng, 300, [.4, .3, .2, .1])
    swo = np.array([5, 105, 300], dtype=np.uint64)
    pk, off = ctx.encode_host(data, swo)
    want = [oracle.pack(data[8 * int(swo[i]):8 * int(swo[i + 1])]) for i in range(2)]
    assert off.tolist() == [0, len(want[0]), len(want[0]) + len(want[1])]
    assert pk.tobytes() == b"".join(want)


@pytest.mark.parametrize("chunk_kb", ["1", "64"])
def test_encode_host_gather_matches_contiguous(ctx, oracle, chunk_kb, monkeypatch):
    """cpk_encode_host_gather (pieces left in their own host buffers, SURVEY.md
    §8f row 4) writes the bytes and offsets of cpk_encode_host over the
    concatenation, and those are the oracle's."""
    monkeypatch.setenv("CPK_HOST_CHUNK_KB", chunk_kb)
    rng = np.random.default_rng(77 + int(chunk_kb))
    sizes = [0, 5, 3000, 0, 1] + list(rng.integers(0, 4000, size=80)) + [30000, 0]
    parts = [_random_words(rng, int(s), [.4, .3, .2, .1]) for s in sizes]
    got, goff = ctx.encode_host_gather([p.view(np.uint64) for p in parts])
    ref, roff = ctx.encode_host(np.concatenate(parts), _swo(sizes))
    assert np.array_equal(goff, roff)
    assert got.tobytes() == ref.tobytes()
    for i in (0, 1, 2, 7, len(parts) - 2):
        assert got[int(goff[i]):int(goff[i + 1])].tobytes() == oracle.pack(parts[i].tobytes())


def test_gather_threaded_split_large(ctx, oracle):
    """Over 8 MiB of ragged pieces (empty ones passed as NULL) under the
    default chunk size, so the host threads' byte-balanced gather split runs:
    cpk_encode_host_gather and cpk_encode_messages_host_gather against the
    oracle byte for byte."""
    rng = np.random.default_rng(808)
    sizes = [int(s) for s in rng.integers(0, 30000, size=90)]
    sizes[::9] = [0] * len(sizes[::9])
    parts = [oracle.generate(oracle.preset(int(rng.integers(2, 5))), _swo([s])) for s in sizes]
    assert sum(p.size for p in parts) >= 8 << 20
    got, goff = ctx.encode_host_gather([p.view(np.uint64) for p in parts])
    opk, ooff = oracle.pack_batch(np.concatenate(parts), _swo(sizes), threads=8)
    assert np.array_equal(goff, ooff)
    assert got.tobytes() == opk.tobytes()
    # the same segments as 30 messages of 3
    msgs = [[parts[3 * m + j].tobytes() for j in range(3)] for m in range(30)]
    pkg, _ = ctx.encode_messages_host_gather(msgs)
    assert pkg == b"".join(oracle.write_message(m) for m in msgs)


def _message_cases(oracle, rng, limit):
    """Packed messages (SerializePacked.write) and broken ones: truncated,
    trailing bytes, flipped table bytes, segment count over 512, negative
    sizes, over the traversal limit."""
    import struct
    msgs = []
    for i in range(400):
        nseg = int(rng.choice([1, 1, 2, 3, 4, 7, 40])) if i != 5 else 512
        sizes = [int(rng.choice([0, 1, 3, 50, 700, 3000])) for _ in range(nseg)]
        segs = [_random_words(rng, s, [.4, .3, .2, .1]).tobytes() for s in sizes]
        m = bytearray(oracle.write_message(segs))
        r = int(rng.integers(0, 12))
        if r == 0 and len(m) > 1:
            m = m[: int(rng.integers(1, len(m)))]
        elif r == 1:
            m += bytes(rng.integers(0, 256, size=int(rng.integers(1, 9)), dtype=np.uint8))
        elif r == 2:
            j = int(rng.integers(0, min(len(m), 12)))
            m[j] = int(rng.integers(0, 256))
        elif r in (3, 4, 5):
            # a hand-made table: count over 512 / a negative size / over the limit
            cnt = {3: 600, 4: 2, 5: 2}[r]
            vals = {3: [0], 4: [5, -3], 5: [limit, 1]}[r]
            words = ((cnt + 2) & ~1) // 2 if r != 3 else 1
            tb = struct.pack("<I", cnt - 1) + b"".join(struct.pack("<i", v) for v in vals)
            tb = (tb + b"\0" * (8 * words))[: 8 * words]
            m = bytearray(oracle.pack(tb)) + m[8:]
        msgs.append(bytes(m))
    return msgs


def test_decode_messages_matches_serialize_read(ctx, oracle):
    """cpk_decode_messages (segment tables read and validated on the device,
    Serialize.java:119-178) against the oracle's Serialize.read, per message."""
    import torch
    import capnp_packed as cp
    rng = np.random.default_rng(31)
    limit = 1 << 16
    msgs = _message_cases(oracle, rng, limit)
    moff = _swo([len(m) for m in msgs])
    blob = b"".join(msgs) + b"\0" * 48
    d_pk = torch.from_numpy(np.frombuffer(blob, np.uint8).copy()).cuda()
    d_moff = torch.from_numpy(moff.astype(np.int64)).cuda()
    nm = len(msgs)
    d_mseg = torch.zeros(nm + 1, dtype=torch.int64, device="cuda")
    d_mst = torch.zeros(nm, dtype=torch.int32, device="cuda")
    # sizing call: capacities of 0 -> CPK_ENOMEM with the totals
    rc, W, S = ctx.decode_messages(d_pk, d_moff, None, None, None, None, d_mseg, d_mst,
                                   traversal_limit_words=limit)
    assert rc == cp.ENOMEM and S > 0
    d_out = torch.zeros(W + 1, dtype=torch.int64, device="cuda")
    d_swo = torch.zeros(S + 1, dtype=torch.int64, device="cuda")
    d_sin = torch.zeros(S + 1, dtype=torch.int64, device="cuda")
    d_sst = torch.zeros(S, dtype=torch.int32, device="cuda")
    rc, W2, S2 = ctx.decode_messages(d_pk, d_moff, d_out, d_swo, d_sin, d_sst, d_mseg, d_mst,
                                     traversal_limit_words=limit)
    torch.cuda.synchronize()
    assert rc == cp.OK and (W2, S2) == (W, S)
    out = d_out.cpu().numpy().view(np.uint8)
    swo = d_swo.cpu().numpy()
    mseg = d_mseg.cpu().numpy()
    mst = d_mst.cpu().numpy()
    kinds = set()
    for i, m in enumerate(msgs):
        ost, segs, used = oracle.read_message(m, traversal_limit_words=limit,
                                              out_cap=8 * limit + 4096)
        if ost == oracle.OK and used != len(m):
            ost = oracle.ETRAILING
        kinds.add(ost)
        assert mst[i] == ost, (i, mst[i], ost, m[:16].hex())
        if ost == oracle.OK:
            got = [out[8 * swo[j]: 8 * swo[j + 1]].tobytes() for j in range(mseg[i], mseg[i + 1])]
            assert got == segs, i
    assert {oracle.OK, oracle.ETRAILING, oracle.ETRUNC, cp.EFRAME} <= kinds, kinds


@pytest.mark.parametrize("hint", ["exact", "huge"])
def test_encode_messages_matches_serialize_write(ctx, oracle, hint):
    """cpk_encode_messages (segment tables built and packed on the device)
    == SerializePacked.write per message, back to back; then the device
    message decode reads them back.  hint "huge": a max_seg_words of 2^30,
    whose per-segment step rows would pass 4 GiB, so the two-pass encoder
    packs them by word offset instead."""
    import torch
    import capnp_packed as cp
    rng = np.random.default_rng(41)
    msgs = []
    for i in range(300):
        nseg = int(rng.choice([1, 1, 2, 3, 4, 5, 40])) if i not in (7, 8) else (512 if i == 7 else 600)
        sizes = [int(rng.choice([0, 1, 2, 17, 300, 2000, 9000])) for _ in range(nseg)]
        if i % 50 == 3:
            sizes = [0x1ff01, 70000][: nseg] if nseg <= 2 else sizes  # table bytes with runs
        msgs.append([_random_words(rng, s, [.4, .3, .2, .1]).tobytes() for s in sizes])
    segs = [s for m in msgs for s in m]
    swo = _swo([len(s) // 8 for s in segs])
    mseg = _swo([len(m) for m in msgs])
    data = np.frombuffer(b"".join(segs) + b"\0" * 8, np.uint8)
    d_in = torch.from_numpy(data.view(np.int64).copy()).cuda()
    d_swo = torch.from_numpy(swo.astype(np.int64)).cuda()
    d_mseg = torch.from_numpy(mseg.astype(np.int64)).cuda()
    cap = cp.batch_capacity(swo) + sum(10 * ((len(m) + 2) // 2 + 1) for m in msgs)
    d_pk = torch.zeros((cap + 63) // 16 * 16, dtype=torch.uint8, device="cuda")
    d_off = torch.zeros(len(msgs) + len(segs) + 1, dtype=torch.int64, device="cuda")
    maxw = int(max(np.diff(swo))) if hint == "exact" else 1 << 30
    ctx.encode_messages(d_in, d_swo, d_mseg, maxw, d_pk, d_off)
    assert ctx.take_error() == cp.OK
    off = d_off.cpu().numpy()
    want = b"".join(oracle.write_message(m) for m in msgs)
    assert int(off[-1]) == len(want)
    assert d_pk[: len(want)].cpu().numpy().tobytes() == want
    # piece offsets: table, then segments, per message
    o, k = 0, 0
    for m in msgs:
        nseg = len(m)
        tb = ((nseg - 1) & 0xffffffff).to_bytes(4, "little") + b"".join(
            (len(s) // 8).to_bytes(4, "little") for s in m)
        tb += b"\0" * (-len(tb) % 8)
        for piece in [tb] + m:
            assert int(off[k]) == o, k
            o += len(oracle.pack(piece))
            k += 1
    # and back: the message ranges are the table pieces' offsets
    starts = off[(mseg[:-1] + np.arange(len(msgs))).astype(np.int64)]
    d_moff = torch.from_numpy(np.append(starts, off[-1]).astype(np.int64)).cuda()
    nm = len(msgs)
    d_mso = torch.zeros(nm + 1, dtype=torch.int64, device="cuda")
    d_mst = torch.zeros(nm, dtype=torch.int32, device="cuda")
    d_out = torch.zeros(int(swo[-1]) + 1, dtype=torch.int64, device="cuda")
    S = len(segs)
    d_sw = torch.zeros(S + 1, dtype=torch.int64, device="cuda")
    d_si = torch.zeros(S + 1, dtype=torch.int64, device="cuda")
    d_ss = torch.zeros(S, dtype=torch.int32, device="cuda")
    rc, W, S2 = ctx.decode_messages(d_pk, d_moff, d_out, d_sw, d_si, d_ss, d_mso, d_mst,
                                    traversal_limit_words=1 << 24)
    torch.cuda.synchronize()
    st = d_mst.cpu().numpy()
    assert rc == cp.OK
    for i, m in enumerate(msgs):
        # over 512 segments: Serialize.read rejects what Serialize.write wrote
        assert st[i] == (cp.EFRAME if len(m) > 512 else cp.OK), i
    ok = [len(m) <= 512 for m in msgs]
    assert S2 == sum(len(m) for m, g in zip(msgs, ok) if g)
    got = d_out.cpu().numpy().view(np.uint8)[: 8 * W].tobytes()
    assert got == b"".join(s for m, g in zip(msgs, ok) if g for s in m)


@pytest.mark.parametrize("chunk_kb", [None, "4", "64"])
def test_message_host_forms(ctx, oracle, chunk_kb, monkeypatch):
    """cpk_encode_messages_host / cpk_decode_messages_host: the JNI facade's
    SerializePacked batch path, against the oracle's Serialize.write/read;
    whole messages flow through the pinned slots in chunks (small chunks:
    many chunks, slot growth mid-batch)."""
    if chunk_kb:
        monkeypatch.setenv("CPK_HOST_CHUNK_KB", chunk_kb)
    rng = np.random.default_rng(43)
    msgs = [[_random_words(rng, int(rng.choice([0, 1, 9, 500, 4000])), [.4, .3, .2, .1]).tobytes()
             for _ in range(int(rng.integers(1, 6)))] for _ in range(60)]
    pk, off = ctx.encode_messages_host(msgs)
    assert pk == b"".join(oracle.write_message(m) for m in msgs)
    pkg, offg = ctx.encode_messages_host_gather(msgs)  # segments where they lie
    assert pkg == pk and np.array_equal(offg, off)
    mso = np.concatenate([[0], np.cumsum([len(m) for m in msgs])])
    moff = off[(mso[:-1] + np.arange(len(msgs))).astype(np.int64)]
    moff = np.append(moff, off[-1])
    st, got = ctx.decode_messages_host(pk, moff)
    assert (st == 0).all() and got == msgs
    # a broken message in the middle: its status, the others intact
    bad = bytearray(pk)
    j = int(moff[7])
    bad[j: j + 1] = b"\x0f"  # first tag of message 7's table: 4 bytes follow
    st, got = ctx.decode_messages_host(bytes(bad), moff)
    ost, _, used = oracle.read_message(bytes(bad[j: int(moff[8])]))
    if ost == oracle.OK and used != int(moff[8]) - j:
        ost = oracle.ETRAILING
    assert st[7] == ost and ost != oracle.OK
    assert all(st[i] == 0 and got[i] == msgs[i] for i in range(len(msgs)) if i != 7)


@pytest.mark.parametrize("chunk_kb", [None, "4"])
def test_message_host_forms_all_broken(ctx, oracle, chunk_kb, monkeypatch):
    """A batch made only of broken messages (no segment anywhere): the
    sizing call has no segment array and must still return the statuses
    (it wrote the segment offsets through NULL)."""
    if chunk_kb:
        monkeypatch.setenv("CPK_HOST_CHUNK_KB", chunk_kb)
    for pk, moff in [(b"\x0f", [0, 1]),
                     (b"\x0f" * 4, [0, 1, 2, 3, 4]),
                     (b"\x01\x05" * 3000, list(range(0, 6001, 2)))]:
        st, got = ctx.decode_messages_host(pk, np.array(moff, np.uint64))
        for i in range(len(moff) - 1):
            ost, _, used = oracle.read_message(pk[moff[i]: moff[i + 1]])
            if ost == oracle.OK and used != moff[i + 1] - moff[i]:
                ost = oracle.ETRAILING
            assert ost != oracle.OK and st[i] == ost, (i, st[i], ost)
            assert got[i] == []


@pytest.mark.parametrize("cfg", [2, 3, 4])
@pytest.mark.parametrize("words", [2048, 4095, 4096, 8192, 12288])
def test_gate_edges_and_sparse_form(ctx, oracle, cfg, words):
    """The device gate's edges (encode_v4.hip, e4_gate_kernel): like-sized
    pieces just under and at the single pass's 4 Ki-word threshold, one
    chunk, and 1.5 chunks (two units each); config-4 data (~90 % zero
    words) sends the single-pass batches to its sparse form
    (cpk_sparse::sp_encode_kernel), config-2 data to the dense one, and
    config-3 data (sampled packed bytes >= 90 % of the words') to the two
    passes (round 5)."""
    n = max(8, (1 << 22) // words)  # ~32 MiB per batch
    swo = _swo([words] * n)
    _check_batch(ctx, oracle, oracle.generate(oracle.preset(cfg), swo), swo)


@pytest.mark.parametrize("cfg", [2, 3, 4])
def test_gate_big_piece_takes_single_pass(ctx, oracle, cfg):
    """A batch with one piece over a unit and at least 1/2048 of the words
    (a single message's segments, the last as large as all before it) goes
    to the single pass whatever its density (round 6: the two passes would
    give that piece one wave) -- dense (config 3), config-2 and sparse data,
    the big piece first, in the middle and last."""
    for order in range(3):
        sizes = [17, 300, 4096, 1, 9000]
        sizes.insert([0, 3, 5][order], 70000 + order)
        swo = _swo(sizes)
        _check_batch(ctx, oracle, oracle.generate(oracle.preset(cfg), swo), swo)


def test_decode_host_few_large_pieces(ctx, oracle):
    """cpk_decode_host with a few large pieces (>= 8 MiB of words each on
    average) decodes them as one stream in parallel and keeps that result
    only when every piece ended exactly at its given packed boundary; a
    piece with a trailing byte in its range (the reference's read() leaves
    it unread: CPK_ETRAILING in the batch form) falls back to the batch
    decoder, so the statuses are the batch form's."""
    W = 3 << 19  # 1.5 Mi words = 12 MiB per piece
    swo = _swo([W, W + 5, W - 7])
    data = oracle.generate(oracle.preset(2), swo)
    pk, off = _check_batch(ctx, oracle, data, swo)
    # a trailing zero byte after piece 0's packed bytes, inside its range
    pk2 = np.concatenate([pk[: off[1]], np.zeros(1, np.uint8), pk[off[1]:]])
    off2 = off.copy()
    off2[1:] += 1
    dec, st = ctx.decode_host(pk2, off2, swo)
    ost = oracle.unpack_batch(pk2, off2, swo, threads=8)[1]
    assert list(st) == list(ost) and st[0] != 0 and (st[1:] == 0).all(), (st, ost)
    assert np.array_equal(dec[8 * int(swo[1]):], data[8 * int(swo[1]):])


def test_message_host_one_large_message(ctx, oracle):
    """One message of one 40 MiB segment through cpk_encode_messages_host:
    a single chunk, whose transfers are pipelined in 16 MiB sub-chunks;
    the bytes equal the oracle's Serialize.write."""
    swo = _swo([5 << 20])
    seg = oracle.generate(oracle.preset(2), swo).tobytes()
    pk, off = ctx.encode_messages_host([[seg]])
    assert pk == oracle.write_message([seg])


def test_decode_batch_few_large_pieces_device(ctx, oracle):
    """Device-resident cpk_decode_batch of a few large pieces (>= 8 MiB of
    words each on average; the default decoder choice): decoded as one
    stream in parallel when every piece ends exactly at its packed range's
    end; a trailing byte inside piece 0's range sends the batch to the batch
    decoders, whose statuses are the batch form's (the oracle's)."""
    import torch
    W = 3 << 19
    swo = _swo([W, W + 3, W - 9])
    data = oracle.generate(oracle.preset(2), swo)
    opk, ooff = oracle.pack_batch(data, swo, threads=8)
    d_swo = torch.from_numpy(swo.astype(np.int64)).cuda()
    for trailing in (False, True):
        pk, off = opk, ooff.copy()
        if trailing:
            pk = np.concatenate([opk[: ooff[1]], np.zeros(1, np.uint8), opk[ooff[1]:]])
            off[1:] += 1
        d_pk = torch.zeros((pk.size + 64) // 16 * 16, dtype=torch.uint8, device="cuda")
        d_pk[: pk.size] = torch.from_numpy(pk).cuda()
        d_off = torch.from_numpy(off.astype(np.int64)).cuda()
        d_out = torch.zeros(int(swo[-1]), dtype=torch.int64, device="cuda")
        d_st = torch.full((3,), -99, dtype=torch.int32, device="cuda")
        ctx.decode_batch(d_pk, d_off, d_swo, d_out, d_st)
        torch.cuda.synchronize()
        st = d_st.cpu().numpy()
        ost = oracle.unpack_batch(pk, off, swo, threads=8)[1]
        assert list(st) == list(ost), (trailing, st, ost)
        out = d_out.cpu().numpy().view(np.uint8)
        if trailing:
            assert st[0] != 0 and np.array_equal(out[8 * int(swo[1]):], data[8 * int(swo[1]):])
        else:
            assert (st == 0).all() and np.array_equal(out, data)


@pytest.mark.parametrize("kind", ["runs", "tagged", "mixed"])
def test_dense_batches_serial_windows(ctx, oracle, kind):
    """Dense batches (packed >= 80 % of the words) decode in the block map's
    dense form: windows of few, long records walked by one lane
    (decode_body<.., kSerial>), the rest in parallel.  Covered: 0xFF runs
    (the serial walk's case), dense data of tagged words (one zero byte per
    word: a serial walk passes its record cap and gives the window back,
    then the cooldown), and both mixed, over pieces of many windows, ragged
    sizes and a piece ending mid-window; device-resident and host forms,
    against the oracle."""
    rng = np.random.default_rng({"runs": 21, "tagged": 22, "mixed": 23}[kind])
    sizes = [8192, 8191, 300, 16384, 1, 40000, 5000, 0, 8192, 777]
    parts = []
    for n in sizes:
        w = rng.integers(1, 256, size=(n, 8), dtype=np.uint8)
        if kind == "tagged":
            w[np.arange(n), rng.integers(0, 8, size=n)] = 0          # L words: a record each
        elif kind == "mixed":
            sel = rng.random(n) < 0.5
            w[np.where(sel)[0], rng.integers(0, 8, size=int(sel.sum()))] = 0
            w[rng.random(n) < 0.02] = 0
        else:
            w[rng.random(n) < 0.03] = 0                              # rare zero words end the runs
        parts.append(w.reshape(-1))
    data = np.concatenate(parts)
    swo = _swo(sizes)
    pk, off = _check_batch(ctx, oracle, data, swo)
    assert len(pk) >= 0.8 * len(data)  # (the dense form's batches)
    # device-resident batch decode (dec_gate_kernel picks the dense form)
    import torch
    d_pk = torch.zeros(len(pk) + 64, dtype=torch.uint8, device="cuda")
    d_pk[: len(pk)] = torch.from_numpy(pk)
    d_off = torch.from_numpy(off.astype(np.int64)).cuda()
    d_swo = torch.from_numpy(swo.astype(np.int64)).cuda()
    d_out = torch.zeros(int(swo[-1]) + 1, dtype=torch.int64, device="cuda")
    d_st = torch.full((len(sizes),), 99, dtype=torch.int32, device="cuda")
    ctx.decode_batch(d_pk, d_off, d_swo, d_out, d_st)
    torch.cuda.synchronize()
    assert (d_st.cpu().numpy() == 0).all()
    assert d_out.cpu().numpy()[: int(swo[-1])].view(np.uint8).tobytes() == data.tobytes()
    # the serial walk really ran (and, on tagged words, gave windows back):
    # a change to its heuristics must not quietly turn it off.  Counted by
    # the diagnostics build (the same sources with -DCPK_DEC_CNT=1; the
    # counters cost the product's dense forms ~2 %), in a child process
    if not ctx.decoder_forced:
        import subprocess
        import sys
        import tempfile
        repo = Path(__file__).resolve().parents[1]
        diag = repo / "capnproto-java_amd" / "lib" / "libcapnp_packed_hip_diag.so"
        assert diag.exists(), "diagnostics library not built (build_native.build_diag)"
        with tempfile.TemporaryDirectory() as td:
            for k, v in (("pk", pk), ("off", off), ("swo", swo), ("data", data)):
                np.save(Path(td) / f"{k}.npy", v)
            import os
            r = subprocess.run([sys.executable, str(repo / "tests" / "_dense_windows_probe.py"), td],
                               capture_output=True, text=True, timeout=120,
                               env=dict(os.environ, CPK_LIB=str(diag)))
        assert r.returncode == 0, r.stdout + r.stderr
        ser, back = (int(x) for x in r.stdout.split("dense_windows")[1].split())
        if kind == "runs":
            assert ser > 0, (ser, back)
        elif kind == "tagged":
            assert back > 0, (ser, back)
        else:
            assert ser + back > 0, (ser, back)
    # corrupted dense pieces (a flipped byte mid-piece, cuts, a trailing
    # byte): statuses are the oracle's, whichever walk saw the window
    cases = []
    p0 = bytes(pk[int(off[0]):int(off[1])])
    n0 = sizes[0]
    for k in range(12):
        b = bytearray(p0)
        r = k % 4
        if r == 0:
            i = int(rng.integers(0, len(b)))
            b[i] = int(rng.integers(0, 256))
        elif r == 1:
            b = b[: int(rng.integers(1, len(b)))]
        elif r == 2:
            b += b"\x00"
        else:
            i = int(rng.integers(len(b) // 4, len(b) // 2))
            b[i] = 0xFF
        cases.append(bytes(b))
    packed = b"".join(cases)
    dec, st = ctx.decode_host(np.frombuffer(packed, np.uint8), _swo([len(c) for c in cases]),
                              _swo([n0] * len(cases)))
    for i, c in enumerate(cases):
        ost, out, used = oracle.unpack(c, 8 * n0)
        if ost == oracle.OK and used != len(c):
            ost = oracle.ETRAILING
        assert st[i] == ost, (kind, i, st[i], ost)
        if ost == oracle.OK:
            assert dec[8 * n0 * i: 8 * n0 * (i + 1)].tobytes() == out
