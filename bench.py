#!/usr/bin/env python3
"""Packed-stream codec benchmark: device-resident encode+decode GiB/s.

Metric (BASELINE.json): "GiB/s packed encode+decode (device-resident
segments) at 1/2/4/8 MI355X".  One step = one PackedOutputStream.write per
piece (encode) + one PackedInputStream.read per piece (decode) over the whole
batch, i.e. a round trip of every segment, inputs already resident in HBM.
value = unpacked bytes of all ranks / (max over ranks of the timed wall time).

Workload (configs[1]): 1 Mi pieces x 64 KiB (8192 words), ~50 % zero words
(z=0.5, Lz=4, q=0.25), synthetic, one shard per GPU (weak
scaling, no collective: pieces are independent, Serialize.java:283-287).

Run:  python bench.py [--gpus N --steps K --warmup W --config 2 --segments S]
Multi-GPU: torch.distributed.run, one rank per GPU (RCCL only for the
barrier and the max-over-ranks reduction of the timings).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parent
sys.path.insert(0, str(REPO / "capnproto-java_amd"))

GIB = float(1 << 30)
PEAK_HBM_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", type=int, default=2, choices=[2, 3, 4])
    ap.add_argument("--segments", type=int, default=1 << 20, help="pieces per GPU")
    ap.add_argument("--seg-words", type=int, default=8192)
    ap.add_argument("--cpu-seconds", type=float, default=10.0,
                    help="time budget of the CPU baseline sample")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--sample-check", type=int, default=64,
                    help="pieces re-packed on the host oracle and compared")
    return ap.parse_args()


def main():
    args = parse()
    import torch
    import capnp_packed as cp

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    ctx = cp.Context(local)
    n = args.segments
    sw = args.seg_words
    swo = np.arange(0, (n + 1) * sw, sw, dtype=np.uint64)
    d_swo = torch.from_numpy(swo.astype(np.int64)).to(dev)
    words = n * sw
    U = 8 * words
    d_in = torch.empty(words, dtype=torch.int64, device=dev)
    params = cp.preset(args.config)
    params.cfg = args.config | (rank << 8)          # distinct shard per rank
    ctx.generate(params, d_swo, d_in)
    cap = cp.batch_capacity(swo)
    d_pk = torch.empty((cap + 255) // 256 * 256, dtype=torch.uint8, device=dev)
    d_off = torch.empty(n + 1, dtype=torch.int64, device=dev)
    d_out = torch.empty(words, dtype=torch.int64, device=dev)
    d_st = torch.empty(n, dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream(dev)
    torch.cuda.synchronize(dev)

    def step(ev=None):
        if ev is not None:
            ev[0].record(stream)
        ctx.encode_batch(d_in, d_swo, sw, d_pk, d_off, stream)
        if ev is not None:
            ev[1].record(stream)
        ctx.decode_batch(d_pk, d_off, d_swo, d_out, d_st, stream)
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
    enc_ms = float(np.mean([e[0].elapsed_time(e[1]) for e in evs]))
    dec_ms = float(np.mean([e[1].elapsed_time(e[2]) for e in evs]))

    # ---- parity: decoded == input, statuses, sample vs the host oracle ----
    cnt = torch.zeros(1, dtype=torch.int64, device=dev)
    ctx.count_mismatch(d_in, d_out, words, cnt, stream)
    bad_status = int((d_st != 0).sum().item())
    mism = int(cnt.item())
    P = int(d_off[-1].item())
    sample_ok = None
    if rank == 0 and args.sample_check > 0:
        sys.path.insert(0, str(REPO / "oracle"))
        import oracle  # checker only
        rng = np.random.default_rng(0)
        idx = np.unique(np.concatenate([[0, n - 1], rng.integers(0, n, size=args.sample_check)]))
        off = d_off.cpu().numpy().astype(np.uint64)
        op = oracle.preset(args.config)
        op.cfg = params.cfg
        sample_ok = True
        for i in idx:
            host = oracle.generate(op, swo, first=int(i), count=1)
            ref = oracle.pack(host)
            got = d_pk[int(off[i]): int(off[i + 1])].cpu().numpy().tobytes()
            if ref != got:
                sample_ok = False
                break

    if dist:
        from capnp_packed.shard import reduce_max_sum
        mx, sm = reduce_max_sum([wall, enc_ms, dec_ms, float(mism + bad_status), float(P)])
        wall, enc_ms, dec_ms = mx[0], mx[1], mx[2]
        errors = int(sm[3])
        P_total = sm[4]
    else:
        errors = mism + bad_status
        P_total = float(P)

    if rank != 0:
        if dist:
            dist.destroy_process_group()
        return

    ms_per_step = 1e3 * wall / args.steps
    value = world * U / GIB / (wall / args.steps)
    r = P / U
    # Roofline of the dominant kernel.  The encode stage is two kernels (the
    # size pass e4_size_kernel and the emit pass e4_emit_kernel, plus a scan
    # of a few microseconds) and the decode stage one (decode_kernel); each
    # of the three reads or writes U+P algorithmic bytes (the size pass: U).
    # decode_kernel is the longest single launch (rocprofv3 summaries under
    # profiles/), so the roofline object is decode_kernel's: U+P per launch
    # over its HIP-event time; the encode stage's figure is reported beside it.
    dom = "decode"
    dom_ms = dec_ms
    achieved = (U + P) / (dom_ms * 1e-3) / 1e9
    # HBM bytes per launch of the dominant kernel from the committed PMC
    # passes (tools/profile.sh + tools/pmc_summary.py), when they were taken
    # on this same workload
    traffic = None
    pmc = REPO / "profiles" / "pmc_traffic.json"
    workload_key = f"config{args.config}:{n}x{sw}"
    if pmc.exists():
        try:
            t = json.loads(pmc.read_text())
            if t.get("workload") == workload_key and dom in t:
                traffic = int(t[dom]["hbm_bytes"])
        except (ValueError, KeyError, TypeError):
            traffic = None

    cpu = None
    if not args.no_cpu:
        cpu = cpu_baseline(args, params)

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
            "workload": f"config{args.config}: {n} pieces x {8 * sw // 1024} KiB per GPU, "
                        + {2: "~50% zero words", 3: "dense (<10% zero words)", 4: "~90% zero words"}[args.config],
            "pieces_per_gpu": n, "piece_bytes": 8 * sw, "unpacked_bytes_per_gpu": U,
            "packed_bytes_per_gpu": P, "packed_ratio": round(r, 4),
            "parallelism": f"shard x{world} (no collective)",
        },
        "encode_ms": round(enc_ms, 4),
        "decode_ms": round(dec_ms, 4),
        "encode_GiBps": round(U / GIB / (enc_ms * 1e-3), 2),
        "decode_GiBps": round(U / GIB / (dec_ms * 1e-3), 2),
        "roofline": {
            "kernel": f"{dom}_kernel",
            "bound": "hbm",
            "achieved": round(achieved, 1),
            "peak": PEAK_HBM_GBS,
            "unit": "GB/s",
            "frac": round(achieved / PEAK_HBM_GBS, 4),
            "traffic": traffic,
            "algorithmic_bytes_per_launch": U + P,
        },
        "encode_stage_roofline": {
            "kernels": ["e4_size_kernel", "e4_scan_*", "e4_emit_kernel"],
            "achieved": round((U + P) / (enc_ms * 1e-3) / 1e9, 1),
            "frac": round((U + P) / (enc_ms * 1e-3) / 1e9 / PEAK_HBM_GBS, 4),
            "note": "algorithmic U+P over the stage's event time; the stage reads U twice",
        },
        "roundtrip_roofline_frac": round(2 * (U + P) / ((enc_ms + dec_ms) * 1e-3) / 1e9 / PEAK_HBM_GBS, 4),
        "parity": {"mismatched_words_plus_bad_status": errors, "oracle_sample_equal": sample_ok},
        "cpu_baseline": cpu,
    }
    print(json.dumps(line), flush=True)
    if dist:
        dist.destroy_process_group()


def cpu_baseline(args, params):
    """The oracle's scalar restatement of the Java loops ("port"), 1 thread,
    on a bounded sample of the same workload (same generator + seeds)."""
    sys.path.insert(0, str(REPO / "oracle"))
    import oracle
    sw = args.seg_words
    m = 512  # 32 MiB per pass
    swo = np.arange(0, (m + 1) * sw, sw, dtype=np.uint64)
    op = oracle.preset(args.config)
    op.cfg = params.cfg
    data = oracle.generate(op, swo)
    t_enc = t_dec = 0.0
    passes = 0
    t_start = time.perf_counter()
    while True:
        t0 = time.perf_counter()
        pk, off = oracle.pack_batch(data, swo, threads=1)
        t1 = time.perf_counter()
        dec, st = oracle.unpack_batch(pk, off, swo, threads=1)
        t2 = time.perf_counter()
        assert (st == 0).all() and np.array_equal(dec, data)
        t_enc += t1 - t0
        t_dec += t2 - t1
        passes += 1
        if time.perf_counter() - t_start >= args.cpu_seconds:
            break
    U = passes * 8 * int(swo[-1])
    return {
        "value": round(U / GIB / (t_enc + t_dec), 3),
        "unit": "GiB/s",
        "cores": 1,
        "kind": "port",
        "sample": f"{passes} passes x {m} pieces x {8 * sw // 1024} KiB (config{args.config} generator), "
                  f"scalar C restatement of PackedOutputStream/PackedInputStream, 1 thread",
        "encode_GiBps": round(U / GIB / t_enc, 3),
        "decode_GiBps": round(U / GIB / t_dec, 3),
    }


if __name__ == "__main__":
    main()
