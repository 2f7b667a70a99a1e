"""Timing of the stream decode (Serialize.read shape: one message, its segments
back to back, boundaries unknown) -- python tools/stream_bench.py [MiB ...]

For a stream of about the given packed size (config-2 data, one segment):
  device   cpk_decode_stream on HBM-resident bytes, parallel block path
  1-wave   the same call with CPK_STREAM_ONE_WAVE=1 (the round-1 path)
  host     cpk_decode_stream_host from/to pageable host memory (what
           SerializePacked::read in csrc/host/packed_stream.hpp calls)
"""
import os
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO / "capnproto-java_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
import capnp_packed as cp  # noqa: E402


def main():
    sizes = [float(a) for a in sys.argv[1:]] or [64]
    if os.environ.get("SB_LIB"):  # (A/B of builds)
        cp.load(Path(os.environ["SB_LIB"]))
    ctx = cp.Context(0)
    for mib in sizes:
        # config 2 packs to ~0.375 of its words: words for ~mib MiB packed
        words = int(mib * (1 << 20) / 8 / 0.375)
        words = (words + 8191) // 8192 * 8192
        gswo = np.arange(0, words + 1, 8192, dtype=np.uint64)
        d_gswo = torch.from_numpy(gswo.astype(np.int64)).cuda()
        d_in = torch.empty(words, dtype=torch.int64, device="cuda")
        ctx.generate(cp.preset(2), d_gswo, d_in)
        # one piece of all the words
        swo = np.array([0, words], np.uint64)
        d_swo = torch.from_numpy(swo.astype(np.int64)).cuda()
        cap = cp.batch_capacity(swo)
        d_pk = torch.zeros((cap + 255) // 256 * 256, dtype=torch.uint8, device="cuda")
        d_off = torch.zeros(2, dtype=torch.int64, device="cuda")
        ctx.encode_batch(d_in, d_swo, words, d_pk, d_off)
        torch.cuda.synchronize()
        P = int(d_off[1].item())
        d_out = torch.empty_like(d_in)
        d_io = torch.zeros(2, dtype=torch.int64, device="cuda")
        d_st = torch.zeros(1, dtype=torch.int32, device="cuda")
        cnt = torch.zeros(1, dtype=torch.int64, device="cuda")

        def run_dev(reps):
            ts = []
            for _ in range(reps):
                d_out.zero_()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                ctx.decode_stream(d_pk, P, d_swo, d_out, d_io, d_st)
                torch.cuda.synchronize()
                ts.append(time.perf_counter() - t0)
            cnt.zero_()
            ctx.count_mismatch(d_in, d_out, words, cnt)
            torch.cuda.synchronize()
            ok = int(cnt.item()) == 0 and int(d_st.item()) == 0 and int(d_io[1].item()) == P
            return float(np.median(ts)), ok

        td, okd = run_dev(10)
        os.environ["CPK_STREAM_ONE_WAVE"] = "1"
        t1, ok1 = run_dev(1)
        os.environ.pop("CPK_STREAM_ONE_WAVE")
        h_pk = d_pk[:P].cpu().numpy()
        h_out = np.zeros(words * 8 + 8, np.uint8)  # (reused: no first-touch faults in the timing)
        th = []
        for _ in range(5):
            t0 = time.perf_counter()
            dec, bounds, st = ctx.decode_stream_host(h_pk, swo, out=h_out)
            th.append(time.perf_counter() - t0)
        okh = bool((st == 0).all()) and int(bounds[-1]) == P and \
            np.array_equal(dec.view(np.int64), d_in.cpu().numpy())
        U = words * 8
        gib = 1 << 30
        print(f"stream {P / (1 << 20):8.3f} MiB packed ({U / (1 << 20):7.1f} MiB words):"
              f"  device {td * 1e3:8.3f} ms ({P / td / gib:7.1f} GiB/s packed, {U / td / gib:7.1f} GiB/s words) ok={okd}"
              f"  1-wave {t1 * 1e3:9.1f} ms ({P / t1 / gib:6.2f} GiB/s) ok={ok1}"
              f"  host {np.median(th) * 1e3:8.2f} ms ({P / np.median(th) / gib:6.2f} GiB/s packed,"
              f" {U / np.median(th) / gib:6.2f} GiB/s words) ok={okh}", flush=True)


if __name__ == "__main__":
    main()
