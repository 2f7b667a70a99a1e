#!/usr/bin/env python3
"""Packed-stream codec benchmark: device-resident encode+decode GiB/s.

Metric (BASELINE.json): "GiB/s packed encode+decode (device-resident
segments) at 1/2/4/8 MI355X".  One step = one PackedOutputStream.write per
piece (encode) + one PackedInputStream.read per piece (decode) over the whole
batch, i.e. a round trip of every segment, inputs already resident in HBM.
value = unpacked bytes of all ranks / (max over ranks of the timed wall time
per step); encode_ms / decode_ms are the medians of the HIP-event times.

Workloads (synthetic Markov generator on the device):
  --config 2 (default, configs[1]): 1 Mi pieces x 64 KiB per GPU, ~50 % zero
             words, cpk_encode_batch / cpk_decode_batch;
  --config 3: 256 Ki messages x 4 segments per GPU, segment sizes uniform over
             {4..256} KiB, dense; SerializePacked.write / read per message
             (cpk_encode_messages / cpk_decode_messages: tables included);
  --config 4: 1 Mi pieces x 64 KiB per GPU, ~90 % zero words.
Multi-GPU (config 5 = config 2 per GPU): one shard per rank, contiguous
piece ranges of the global batch (capnp_packed.shard.plan_shards), no
collective on the data path (pieces are independent, Serialize.java:283-287).

Run:  python bench.py [--gpus N --steps K --warmup W --config C]
  --gpus N without a torch.distributed launcher starts N rank processes
  itself (before any GPU call); under torchrun WORLD_SIZE must equal N.
  --stub: CPU-only rehearsal of the multi-rank path (gloo, the oracle as
  the "kernel"), used by tests/test_shard.py.
  --same-device: every rank on cuda:0 (the real GPU rank path at N > 1 on a
  one-GPU box, tests/test_gpu_bench_shapes.py); use a small --segments so
  the shards fit.  Ranks talk over gloo in every mode: no RCCL anywhere.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parent
sys.path.insert(0, str(REPO / "capnproto-java_amd"))

GIB = float(1 << 30)
PEAK_HBM_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
SEED = 0x1D2ACD47
CFG3_SEG_WORDS = np.array([512, 1024, 2048, 4096, 8192, 16384, 32768], dtype=np.uint64)


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", type=int, default=2, choices=[2, 3, 4])
    ap.add_argument("--segments", type=int, default=None,
                    help="pieces per GPU (config 3: messages per GPU)")
    ap.add_argument("--seg-words", type=int, default=8192)
    ap.add_argument("--cpu-seconds", type=float, default=10.0,
                    help="time budget of each CPU-baseline sample (1 thread, then all threads)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--sample-check", type=int, default=64,
                    help="pieces re-packed on the host oracle and compared")
    ap.add_argument("--stub", action="store_true", help="CPU rehearsal (gloo, no GPU)")
    ap.add_argument("--same-device", action="store_true",
                    help="all ranks on cuda:0, gloo group (N > 1 rehearsal on one GPU)")
    return ap.parse_args(argv)


# ---------------------------------------------------------------- launcher
def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def spawn(args) -> int:
    """Start args.gpus rank processes (this process never touches the GPU)
    and return the worst exit code."""
    port = _free_port()
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus),
                   LOCAL_WORLD_SIZE=str(args.gpus), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, str(Path(__file__).resolve())] + sys.argv[1:],
                                      env=env))
    rc = 0
    for p in procs:
        p.wait()
        rc = rc or p.returncode
    return rc


# ---------------------------------------------------------------- workloads
def global_layout(args, world):
    """The whole job's batch (all ranks) and each rank's shard boundaries.
    Config 3: message segment counts / sizes from a seeded RNG (identical on
    every rank); configs 2/4: uniform pieces."""
    from capnp_packed.shard import plan_shards
    if args.config == 3:
        nm = (args.segments or (1 << 18)) * world
        rng = np.random.default_rng(SEED)
        seg_words = CFG3_SEG_WORDS[rng.integers(0, len(CFG3_SEG_WORDS), size=4 * nm)]
        msg_words = seg_words.reshape(nm, 4).sum(1)
        mwo = np.concatenate([[0], np.cumsum(msg_words)]).astype(np.uint64)
        bounds = plan_shards(mwo, world)  # messages per rank, balanced by bytes
        return dict(seg_words=seg_words, bounds=bounds)
    n = (args.segments or (1 << 20)) * world
    swo = np.arange(0, (n + 1) * args.seg_words, args.seg_words, dtype=np.uint64)
    return dict(swo=swo, bounds=plan_shards(swo, world))


def rank_shard(args, lay, rank):
    """This rank's pieces: (seg_word_off from 0, msg_seg_off or None)."""
    b0, b1 = int(lay["bounds"][rank]), int(lay["bounds"][rank + 1])
    if args.config == 3:
        sw = lay["seg_words"][4 * b0: 4 * b1]
        swo = np.concatenate([[0], np.cumsum(sw)]).astype(np.uint64)
        mso = np.arange(0, 4 * (b1 - b0) + 1, 4, dtype=np.uint64)
        return swo, mso
    swo = lay["swo"][b0: b1 + 1] - lay["swo"][b0]
    return swo.astype(np.uint64), None


# ---------------------------------------------------------------- GPU rank
def run_rank(args, rank, world, local):
    import torch
    import capnp_packed as cp

    dist = None
    if args.same_device:
        local = 0
    torch.cuda.set_device(local)
    if world > 1:
        import torch.distributed as dist
        # gloo in every mode: the data path has no collective (pieces are
        # independent, Serialize.java:283-287); the group only carries the
        # barrier around the timed region and the max / sum of a few host
        # scalars, so an N-GPU run takes exactly the code the one-GPU
        # --same-device rehearsal tests, but for the device each rank sets
        dist.init_process_group("gloo")
    dev = torch.device("cuda", local)
    ctx = cp.Context(local)

    lay = global_layout(args, world)
    swo, mso = rank_shard(args, lay, rank)
    n = len(swo) - 1
    words = int(swo[-1])
    U = 8 * words
    maxw = int(np.diff(swo).max()) if n else 0
    d_swo = torch.from_numpy(swo.astype(np.int64)).to(dev)
    d_in = torch.empty(words, dtype=torch.int64, device=dev)
    params = cp.preset(args.config)
    params.cfg = args.config | (rank << 8)          # distinct shard per rank
    ctx.generate(params, d_swo, d_in)
    d_out = torch.empty(words + 1, dtype=torch.int64, device=dev)
    stream = torch.cuda.current_stream(dev)

    if mso is None:
        cap = cp.batch_capacity(swo)
        d_pk = torch.empty((cap + 255) // 256 * 256, dtype=torch.uint8, device=dev)
        d_off = torch.empty(n + 1, dtype=torch.int64, device=dev)
        d_st = torch.empty(n, dtype=torch.int32, device=dev)

        def encode():
            ctx.encode_batch(d_in, d_swo, maxw, d_pk, d_off, stream)

        def decode():
            ctx.decode_batch(d_pk, d_off, d_swo, d_out, d_st, stream)

        def piece_range(i):
            return int(offs[i]), int(offs[i + 1])
    else:
        nm = len(mso) - 1
        d_mso = torch.from_numpy(mso.astype(np.int64)).to(dev)
        segs_per = np.diff(mso)
        cap = cp.batch_capacity(swo) + int(sum(10 * ((c + 2) // 2 + 1) for c in segs_per))
        d_pk = torch.empty((cap + 255) // 256 * 256, dtype=torch.uint8, device=dev)
        d_off = torch.empty(nm + n + 1, dtype=torch.int64, device=dev)
        # message m starts at piece mso[m] + m (its table), the last entry is the total
        d_msg_idx = d_mso + torch.arange(nm + 1, device=dev, dtype=torch.int64)
        d_moff = torch.empty(nm + 1, dtype=torch.int64, device=dev)
        d_swo_o = torch.empty(n + 1, dtype=torch.int64, device=dev)
        d_sio = torch.empty(n + 1, dtype=torch.int64, device=dev)
        d_sst = torch.empty(n, dtype=torch.int32, device=dev)
        d_mso_o = torch.empty(nm + 1, dtype=torch.int64, device=dev)
        d_st = torch.empty(nm, dtype=torch.int32, device=dev)
        msg_fail = [0]

        def encode():
            ctx.encode_messages(d_in, d_swo, d_mso, maxw, d_pk, d_off, stream)

        def decode():
            torch.index_select(d_off, 0, d_msg_idx, out=d_moff)
            rc, tw, ts = ctx.decode_messages(d_pk, d_moff, d_out, d_swo_o, d_sio, d_sst,
                                             d_mso_o, d_st, stream=stream)
            if rc != cp.OK or tw != words or ts != n:
                msg_fail[0] += 1

        def piece_range(i):
            # segment i of message i // 4 is piece mso[m] + m + 1 + (i - mso[m])
            p = i + i // 4 + 1
            return int(offs[p]), int(offs[p + 1])
    torch.cuda.synchronize(dev)

    def step(ev=None):
        if ev is not None:
            ev[0].record(stream)
        encode()
        if ev is not None:
            ev[1].record(stream)
        decode()
        if ev is not None:
            ev[2].record(stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)

    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(args.steps)]
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(evs[k])
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    wall = time.perf_counter() - t0
    enc_t = [e[0].elapsed_time(e[1]) for e in evs]
    dec_t = [e[1].elapsed_time(e[2]) for e in evs]
    enc_ms, dec_ms = float(np.median(enc_t)), float(np.median(dec_t))

    # ---- parity: decoded == input, statuses, sample vs the host oracle ----
    cnt = torch.zeros(1, dtype=torch.int64, device=dev)
    ctx.count_mismatch(d_in, d_out, words, cnt, stream)
    bad_status = int((d_st != 0).sum().item())
    if mso is not None:
        bad_status += int((d_sst != 0).sum().item()) + msg_fail[0]
    mism = int(cnt.item())
    offs = d_off.cpu().numpy().astype(np.uint64)
    P = int(offs[-1])
    sample_ok = None
    if rank == 0 and args.sample_check > 0:
        sys.path.insert(0, str(REPO / "oracle"))
        import oracle  # checker only, after the timed region
        rng = np.random.default_rng(0)
        idx = np.unique(np.concatenate([[0, n - 1], rng.integers(0, n, size=args.sample_check)]))
        op = oracle.preset(args.config)
        op.cfg = params.cfg
        sample_ok = True
        for i in idx:
            host = oracle.generate(op, swo, first=int(i), count=1)
            a, b = piece_range(int(i))
            if oracle.pack(host) != d_pk[a:b].cpu().numpy().tobytes():
                sample_ok = False
                break
        if mso is not None and sample_ok:
            # whole messages = SerializePacked.write bytes (Serialize.java:256-288)
            for m in np.unique(rng.integers(0, len(mso) - 1, size=8)):
                s0, s1 = int(mso[m]), int(mso[m + 1])
                segs = [oracle.generate(op, swo, first=s, count=1).tobytes() for s in range(s0, s1)]
                a, b = int(offs[s0 + m]), int(offs[s1 + m + 1])
                if oracle.write_message(segs) != d_pk[a:b].cpu().numpy().tobytes():
                    sample_ok = False
                    break

    if dist:
        from capnp_packed.shard import reduce_max_sum
        mx, sm = reduce_max_sum([wall, enc_ms, dec_ms, float(mism + bad_status), float(P), float(U)])
        wall, enc_ms, dec_ms = mx[0], mx[1], mx[2]
        errors = int(sm[3])
        P_total, U_total = sm[4], sm[5]
        per_rank = {"encode_ms_max": round(mx[1], 4), "decode_ms_max": round(mx[2], 4),
                    "wall_s_max": round(mx[0], 4), "unpacked_bytes_total": int(U_total),
                    "packed_bytes_total": int(P_total),
                    "backend": dist.get_backend(), "same_device": bool(args.same_device)}
    else:
        errors = mism + bad_status
        P_total, U_total = float(P), float(U)
        per_rank = None

    if rank != 0:
        if dist:
            dist.destroy_process_group()
        return

    ms_per_step = 1e3 * wall / args.steps
    value = U_total / GIB / (wall / args.steps)
    r = P / U
    # Roofline of the dominant kernel: the longer stage, each one launch of
    # its main kernel (the single-pass encoder, sp_encode_kernel, or
    # decode_kernel; U+P algorithmic bytes either way); the other stage is
    # reported beside it.  HIP events on the launch stream, median of K.
    # (the library's choice: the single pass for like-sized 64 KiB pieces,
    # the two passes for message batches; CPK_ENCODER forces one)
    forced = os.environ.get("CPK_ENCODER", "")[:1]
    # (like-sized pieces whose sampled words are >= 85 % zero, config 4: the
    # single pass's sparse form, cpk_sparse::sp_encode_kernel)
    enc_kernel = "e4_size_kernel+e4_emit_kernel" if forced == "4" or (mso is not None and forced != "0") \
        else "cpk_sparse::sp_encode_kernel" if forced != "0" and args.config == 4 else "sp_encode_kernel"
    # (the batch decoder: the record-index one for sparse batches, packed
    # under 15 % of the words' bytes, else the block map; messages: block map)
    forced_d = os.environ.get("CPK_DECODER", "")[:1]
    # (and the block map's dense form, decode_kernel<.., true>, for batches
    # packed at >= 80 % of the words' bytes: dense windows walked by one lane)
    dec_kernel = "decode2_kernel" if forced_d == "2" or (forced_d != "1" and mso is None and 100 * P < 15 * U) \
        else "decode_kernel<dense>" if forced_d not in ("1", "2") and 100 * P >= 80 * U else "decode_kernel"
    dom_enc = enc_ms > dec_ms
    dom_ms = enc_ms if dom_enc else dec_ms
    achieved = (U + P) / (dom_ms * 1e-3) / 1e9
    traffic = {"encode": None, "decode": None}
    pmc = REPO / "profiles" / "pmc_traffic.json"
    workload_key = f"config{args.config}:{n}x{args.seg_words if mso is None else 'mixed'}"
    if pmc.exists():
        # PMC-measured HBM bytes per launch (tools/pmc_summary.py --json),
        # keyed by the workload they were measured on
        try:
            t = json.loads(pmc.read_text()).get(workload_key) or {}
            for k in traffic:
                if k in t:
                    traffic[k] = int(t[k]["hbm_bytes"])
        except (ValueError, KeyError, TypeError, AttributeError):
            pass

    # (rank 0 at N = 1 only: at N > 1 the other ranks would wait on it and
    # the host cores are shared by all ranks)
    cpu = None
    if not args.no_cpu and world == 1:
        cpu = cpu_baseline(args, params)

    if mso is None:
        workload = (f"config{args.config}: {n} pieces x {8 * args.seg_words // 1024} KiB per GPU, "
                    + {2: "~50% zero words", 4: "~90% zero words"}[args.config])
    else:
        workload = (f"config3: {len(mso) - 1} messages x 4 segments (4-256 KiB) per GPU, dense "
                    "(<10% zero words), SerializePacked.write/read incl. segment tables")
    line = {
        "metric": "GiB/s packed encode+decode (device-resident segments)",
        "value": round(value, 2),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (device Markov generator, SURVEY.md 8d)",
        "config": {
            "workload": workload,
            "pieces_per_gpu": n, "unpacked_bytes_per_gpu": U,
            "packed_bytes_per_gpu": P, "packed_ratio": round(r, 4),
            "parallelism": f"shard x{world} (no collective)",
        },
        "encode_ms": round(enc_ms, 4),
        "decode_ms": round(dec_ms, 4),
        "timing": "encode_ms/decode_ms: median of the K steps' HIP events; value: wall time of K steps",
        "encode_GiBps": round(U / GIB / (enc_ms * 1e-3), 2),
        "decode_GiBps": round(U / GIB / (dec_ms * 1e-3), 2),
        "roofline": {
            "kernel": enc_kernel if dom_enc else dec_kernel,
            "bound": "hbm",
            "achieved": round(achieved, 1),
            "peak": PEAK_HBM_GBS,
            "unit": "GB/s",
            "frac": round(achieved / PEAK_HBM_GBS, 4),
            "traffic": traffic["encode" if dom_enc else "decode"],
            "algorithmic_bytes_per_launch": U + P,
        },
        ("decode_stage_roofline" if dom_enc else "encode_stage_roofline"): {
            "kernel": dec_kernel if dom_enc else enc_kernel,
            "ms": round(dec_ms if dom_enc else enc_ms, 3),
            "achieved": round((U + P) / ((dec_ms if dom_enc else enc_ms) * 1e-3) / 1e9, 1),
            "frac": round((U + P) / ((dec_ms if dom_enc else enc_ms) * 1e-3) / 1e9 / PEAK_HBM_GBS, 4),
            "traffic": traffic["decode" if dom_enc else "encode"],
            "note": "algorithmic U+P over the other stage's event time",
        },
        "roundtrip_roofline_frac": round(2 * (U + P) / ((enc_ms + dec_ms) * 1e-3) / 1e9 / PEAK_HBM_GBS, 4),
        "parity": {"mismatched_words_plus_bad_status": errors, "oracle_sample_equal": sample_ok},
        "cpu_baseline": cpu,
    }
    if per_rank:
        line["per_rank"] = per_rank
    print(json.dumps(line), flush=True)
    if dist:
        dist.destroy_process_group()


# ---------------------------------------------------------------- CPU baseline
def cpu_model() -> str:
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_threads() -> int:
    """Threads for the multi-core leg: the CPUs this process may use, capped
    at 16 (a one-GPU box's share of its host)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(16, n))


def cpu_baseline(args, params):
    """The oracle's scalar restatement of the Java loops ("port") on a bounded
    sample of the same workload (same generator + seeds): 1 thread, then
    cpu_threads() threads over independent pieces."""
    sys.path.insert(0, str(REPO / "oracle"))
    import oracle
    op = oracle.preset(args.config)
    op.cfg = params.cfg
    if args.config == 3:
        # the bench's own message layout: the first messages of the seeded
        # 4 x (4-256 KiB) layout, each = table piece + 4 segment pieces
        # (SerializePacked.write = Serialize.java:256-288), ~32 MiB per pass
        seg_words = global_layout(args, 1)["seg_words"]
        gswo = np.concatenate([[0], np.cumsum(seg_words)]).astype(np.uint64)
        nm = int(np.searchsorted(gswo[4::4], 4 << 20)) + 1
        segs = oracle.generate(op, gswo[: 4 * nm + 1])
        table = np.zeros((nm, 3), np.uint64)  # [count - 1 | size0], [size1 | size2], [size3 | pad]
        sw32 = seg_words[: 4 * nm].reshape(nm, 4).astype(np.uint64)
        table[:, 0] = 3 | (sw32[:, 0] << 32)
        table[:, 1] = sw32[:, 1] | (sw32[:, 2] << 32)
        table[:, 2] = sw32[:, 3]
        parts, sizes = [], []
        for k in range(nm):
            parts.append(table[k].view(np.uint8))
            sizes.append(3)
            a0, a1 = 8 * int(gswo[4 * k]), 8 * int(gswo[4 * k + 4])
            parts.append(segs[a0:a1])
            sizes.extend(int(x) for x in sw32[k])
        data = np.concatenate(parts).astype(np.uint8)
        swo = np.concatenate([[0], np.cumsum(sizes)]).astype(np.uint64)
        m, U1 = len(sizes), 8 * int(gswo[4 * nm])
        sample_desc = f"{nm} messages x (table + 4 segments, 4-256 KiB) of the config3 layout"
    else:
        sw = args.seg_words
        m = 512  # 32 MiB per pass
        swo = np.arange(0, (m + 1) * sw, sw, dtype=np.uint64)
        data = oracle.generate(op, swo)
        U1 = 8 * int(swo[-1])
        sample_desc = f"{m} pieces x {8 * sw // 1024} KiB (config{args.config} generator)"

    def leg(threads, budget):
        t_enc = t_dec = 0.0
        passes = 0
        t_start = time.perf_counter()
        while True:
            t0 = time.perf_counter()
            pk, off = oracle.pack_batch(data, swo, threads=threads)
            t1 = time.perf_counter()
            dec, st = oracle.unpack_batch(pk, off, swo, threads=threads)
            t2 = time.perf_counter()
            assert (st == 0).all() and np.array_equal(dec, data)
            t_enc += t1 - t0
            t_dec += t2 - t1
            passes += 1
            if time.perf_counter() - t_start >= budget:
                break
        U = passes * U1
        return passes, U / GIB / (t_enc + t_dec), U / GIB / t_enc, U / GIB / t_dec

    p1, v1, e1, d1 = leg(1, args.cpu_seconds)
    T = cpu_threads()
    pT, vT, eT, dT = leg(T, args.cpu_seconds / 2) if T > 1 else (p1, v1, e1, d1)
    return {
        "value": round(vT, 3),
        "unit": "GiB/s",
        "cores": T,
        "kind": "port",
        "cpu_model": cpu_model(),
        "sample": f"{pT} passes x {sample_desc}, "
                  f"scalar C restatement of PackedOutputStream/PackedInputStream, {T} threads over "
                  f"independent pieces; single thread: {p1} passes",
        "encode_GiBps": round(eT, 3),
        "decode_GiBps": round(dT, 3),
        "single_thread": {"value": round(v1, 3), "encode_GiBps": round(e1, 3),
                          "decode_GiBps": round(d1, 3), "cores": 1},
    }


# ---------------------------------------------------------------- CPU stub
def run_stub(args, rank, world):
    """The multi-rank path with the oracle as the kernel (gloo): shard
    planning, per-rank generation, round trip, barrier-bracketed timing and
    the max/sum reduction -- what the GPU ranks do, without a GPU."""
    import torch.distributed as dist
    sys.path.insert(0, str(REPO / "oracle"))
    import oracle
    from capnp_packed.shard import reduce_max_sum
    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    lay = global_layout(args, world)
    swo, mso = rank_shard(args, lay, rank)
    op = oracle.preset(args.config)
    op.cfg = args.config | (rank << 8)
    data = oracle.generate(op, swo)
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    errs = 0
    for _ in range(args.steps):
        pk, off = oracle.pack_batch(data, swo)
        dec, st = oracle.unpack_batch(pk, off, swo)
        errs += int((st != 0).sum()) + int(not np.array_equal(dec, data))
    if world > 1:
        dist.barrier()
    wall = time.perf_counter() - t0
    U = float(8 * int(swo[-1]))
    vals = [wall, float(errs), U, float(len(swo) - 1)]
    if world > 1:
        mx, sm = reduce_max_sum(vals)
        dist.destroy_process_group()
    else:
        mx, sm = vals, vals
    if rank == 0:
        print(json.dumps({"metric": "stub", "n_gpus": world, "steps": args.steps,
                          "value": sm[2] / GIB / (mx[0] / args.steps), "errors": int(sm[1]),
                          "pieces_total": int(sm[3]), "unpacked_bytes_total": int(sm[2]),
                          "shard_bounds": [int(b) for b in lay["bounds"]]}), flush=True)


def main():
    args = parse()
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        sys.exit(spawn(args))
    world = int(env_world or 1)
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.stub:
        run_stub(args, rank, world)
    else:
        run_rank(args, rank, world, local)


if __name__ == "__main__":
    main()
