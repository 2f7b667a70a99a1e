"""The bench workloads (bench.py) checked against
the oracle at their own shapes: the same layout code, device generator and
entry points as the timed run, on a slice of the job small enough for the
oracle (2048 pieces / messages)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _dev(a):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a).astype(np.int64)).cuda()


@pytest.mark.parametrize("cfg", [2, 4])
def test_bench_batch_shape(ctx, oracle, cfg):
    """Configs 2 / 4: 64 KiB pieces through encode_batch / decode_batch,
    every byte compared with the oracle's pack of the host-generated data."""
    import torch
    import bench
    import capnp_packed as cp
    args = bench.parse(["--config", str(cfg), "--segments", "2048"])
    swo, _ = bench.rank_shard(args, bench.global_layout(args, 1), 0)
    n, words = len(swo) - 1, int(swo[-1])
    d_swo = _dev(swo)
    d_in = torch.empty(words, dtype=torch.int64, device="cuda")
    ctx.generate(cp.preset(cfg), d_swo, d_in)
    cap = cp.batch_capacity(swo)
    d_pk = torch.empty((cap + 255) // 256 * 256, dtype=torch.uint8, device="cuda")
    d_off = torch.empty(n + 1, dtype=torch.int64, device="cuda")
    ctx.encode_batch(d_in, d_swo, args.seg_words, d_pk, d_off)
    d_out = torch.empty_like(d_in)
    d_st = torch.empty(n, dtype=torch.int32, device="cuda")
    ctx.decode_batch(d_pk, d_off, d_swo, d_out, d_st)
    torch.cuda.synchronize()
    assert ctx.take_error() == 0
    host = oracle.generate(oracle.preset(cfg), swo)
    opk, ooff = oracle.pack_batch(host, swo, threads=8)
    off = d_off.cpu().numpy().astype(np.uint64)
    assert np.array_equal(off, ooff)
    assert np.array_equal(d_pk[: int(off[-1])].cpu().numpy(), opk)
    assert int((d_st != 0).sum().item()) == 0
    assert np.array_equal(d_out.cpu().numpy().view(np.uint8), host)


def test_bench_messages_shape(ctx, oracle):
    """Config 3: messages of 4 segments of 4-256 KiB (bench layout, seeded)
    through encode_messages / decode_messages; the packed stream equals the
    oracle's Serialize.write per message and decodes back."""
    import torch
    import bench
    import capnp_packed as cp
    args = bench.parse(["--config", "3", "--segments", "2048"])
    swo, mso = bench.rank_shard(args, bench.global_layout(args, 1), 0)
    nseg, nm, words = len(swo) - 1, len(mso) - 1, int(swo[-1])
    d_swo, d_mso = _dev(swo), _dev(mso)
    d_in = torch.empty(words + 1, dtype=torch.int64, device="cuda")
    ctx.generate(cp.preset(3), d_swo, d_in)
    cap = cp.batch_capacity(swo) + nm * 10 * ((4 + 2) // 2 + 1)
    d_pk = torch.zeros((cap + 255) // 256 * 256, dtype=torch.uint8, device="cuda")
    d_off = torch.empty(nm + nseg + 1, dtype=torch.int64, device="cuda")
    ctx.encode_messages(d_in, d_swo, d_mso, int(bench.CFG3_SEG_WORDS.max()), d_pk, d_off)
    torch.cuda.synchronize()
    assert ctx.take_error() == 0
    off = d_off.cpu().numpy().astype(np.uint64)
    pk = d_pk[: int(off[-1])].cpu().numpy()
    host = oracle.generate(oracle.preset(3), swo)
    # messages start at piece mso[m] + m (table, then its segments)
    starts = [int(off[int(mso[m]) + m]) for m in range(nm)] + [int(off[-1])]
    expect = []
    for m in range(nm):
        segs = [host[8 * int(swo[s]): 8 * int(swo[s + 1])].tobytes() for s in range(int(mso[m]), int(mso[m + 1]))]
        expect.append(oracle.write_message(segs))
    assert b"".join(expect) == pk.tobytes()
    assert [len(e) for e in expect] == list(np.diff(starts))
    # decode_messages back
    d_moff = _dev(np.array(starts, np.uint64))
    d_out = torch.empty(words + 1, dtype=torch.int64, device="cuda")
    d_sw = torch.empty(nseg + 1, dtype=torch.int64, device="cuda")
    d_si = torch.empty(nseg + 1, dtype=torch.int64, device="cuda")
    d_ss = torch.empty(nseg, dtype=torch.int32, device="cuda")
    d_ms = torch.empty(nm + 1, dtype=torch.int64, device="cuda")
    d_mst = torch.empty(nm, dtype=torch.int32, device="cuda")
    rc, tw, ts = ctx.decode_messages(d_pk, d_moff, d_out, d_sw, d_si, d_ss, d_ms, d_mst)
    torch.cuda.synchronize()
    assert rc == cp.OK and tw == words and ts == nseg
    assert int((d_mst != 0).sum().item()) == 0
    assert np.array_equal(d_sw.cpu().numpy().astype(np.uint64), swo)
    assert np.array_equal(d_out[:words].cpu().numpy().view(np.uint8), host)


def test_sparse_messages_multi_round(ctx, oracle):
    """Messages of sparse segments (config-4 data, ~90 % zero words, 4-256
    KiB) through encode_messages / decode_messages: the stream-form decoder's
    windows then hold more words than one expansion round (zero runs of up
    to 256 words per 2-byte record), so later rounds and their block maps
    are exercised; the packed bytes equal the oracle's Serialize.write and
    the words come back."""
    import torch
    import capnp_packed as cp
    rng = np.random.default_rng(44)
    nm = 96
    seg = rng.choice([512, 2048, 8192, 32768], size=(nm, 4)).astype(np.uint64)
    swo = np.concatenate([[0], np.cumsum(seg.reshape(-1))]).astype(np.uint64)
    mso = np.arange(0, 4 * nm + 1, 4, dtype=np.uint64)
    nseg, words = 4 * nm, int(swo[-1])
    d_swo, d_mso = _dev(swo), _dev(mso)
    d_in = torch.empty(words + 1, dtype=torch.int64, device="cuda")
    ctx.generate(cp.preset(4), d_swo, d_in)
    cap = cp.batch_capacity(swo) + nm * 10 * 4
    d_pk = torch.zeros((cap + 255) // 256 * 256, dtype=torch.uint8, device="cuda")
    d_off = torch.empty(nm + nseg + 1, dtype=torch.int64, device="cuda")
    ctx.encode_messages(d_in, d_swo, d_mso, 32768, d_pk, d_off)
    torch.cuda.synchronize()
    assert ctx.take_error() == 0
    off = d_off.cpu().numpy().astype(np.uint64)
    pk = d_pk[: int(off[-1])].cpu().numpy()
    host = oracle.generate(oracle.preset(4), swo)
    assert np.array_equal(d_in[:words].cpu().numpy().view(np.uint8), host)
    expect = []
    for m in range(nm):
        segs = [host[8 * int(swo[s]): 8 * int(swo[s + 1])].tobytes() for s in range(4 * m, 4 * m + 4)]
        expect.append(oracle.write_message(segs))
    assert b"".join(expect) == pk.tobytes()
    starts = np.concatenate([[0], np.cumsum([len(e) for e in expect])]).astype(np.uint64)
    assert len(pk) < 0.2 * 8 * words  # sparse: windows of many words
    d_moff = _dev(starts)
    d_out = torch.empty(words + 1, dtype=torch.int64, device="cuda")
    d_sw = torch.empty(nseg + 1, dtype=torch.int64, device="cuda")
    d_si = torch.empty(nseg + 1, dtype=torch.int64, device="cuda")
    d_ss = torch.empty(nseg, dtype=torch.int32, device="cuda")
    d_ms = torch.empty(nm + 1, dtype=torch.int64, device="cuda")
    d_mst = torch.empty(nm, dtype=torch.int32, device="cuda")
    rc, tw, ts = ctx.decode_messages(d_pk, d_moff, d_out, d_sw, d_si, d_ss, d_ms, d_mst)
    torch.cuda.synchronize()
    assert rc == cp.OK and tw == words and ts == nseg
    assert int((d_mst != 0).sum().item()) == 0 and int((d_ss != 0).sum().item()) == 0
    assert np.array_equal(d_sw.cpu().numpy().astype(np.uint64), swo)
    assert np.array_equal(d_out[:words].cpu().numpy().view(np.uint8), host)


@pytest.mark.parametrize("config,segments", [(2, 4096), (3, 512)])
def test_bench_two_ranks_same_device(config, segments):
    """bench.py's real GPU rank path at N = 2 (config 5 readiness) on a
    one-GPU box: both ranks on cuda:0 (--same-device).  Every mode uses the
    same gloo group, so shard planning, per-rank generation, the
    barrier-bracketed timing and the max/sum reduction are exactly the code
    the 8-GPU run takes but for torch.cuda.set_device; both shards must round-trip bit-exact and rank 0's
    oracle sample must equal the device bytes."""
    import json
    import os
    import subprocess
    import sys
    from pathlib import Path
    repo = Path(__file__).resolve().parents[1]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    out = subprocess.run([sys.executable, str(repo / "bench.py"), "--gpus", "2", "--same-device",
                          "--config", str(config), "--segments", str(segments), "--steps", "3",
                          "--warmup", "1", "--no-cpu", "--sample-check", "16"],
                         env=env, capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-3000:]
    line = json.loads(out.stdout.strip().splitlines()[-1])
    print(json.dumps(line))
    assert line["n_gpus"] == 2 and line["per_rank"]["backend"] == "gloo"
    assert line["parity"]["mismatched_words_plus_bad_status"] == 0
    assert line["parity"]["oracle_sample_equal"] is True
    per = 8 * 8192 * segments if config == 2 else None
    if per:
        assert line["per_rank"]["unpacked_bytes_total"] == 2 * per
    assert line["value"] > 0
