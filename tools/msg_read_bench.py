"""SerializePacked.read of ONE single-segment message (config-2 words) from a
packed stream: python tools/msg_read_bench.py [packed MiB ...]

  device     cpk_read_message on HBM-resident bytes (one enqueue, no host sync
             inside; timed to the stream's completion)
  host       cpk_read_message_host from/to pageable host memory (reused
             output buffer: no first-touch faults in the timing)
  3-call     round 2's Java path: cpk_decode_stream_host for the first word,
             then for the segments (the table's remaining words are none for
             one segment) -- two staged calls here, three for 2+ segments
"""
import ctypes
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO / "capnproto-java_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
import capnp_packed as cp  # noqa: E402


def med(f, reps):
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        f()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts))


def main():
    sizes = [int(a) for a in sys.argv[1:]] or [4, 16, 64, 256]
    ctx = cp.Context(0)
    lib = ctx._lib
    gib = 1 << 30
    for mib in sizes:
        words = int(mib * (1 << 20) / 8 / 0.375)
        words = (words + 8191) // 8192 * 8192
        gswo = np.arange(0, words + 1, 8192, dtype=np.uint64)
        d_in = torch.empty(words, dtype=torch.int64, device="cuda")
        ctx.generate(cp.preset(2), torch.from_numpy(gswo.astype(np.int64)).cuda(), d_in)
        swo = np.array([0, words], np.uint64)
        d_swo = torch.from_numpy(swo.astype(np.int64)).cuda()
        d_mso = torch.tensor([0, 1], dtype=torch.int64, device="cuda")
        cap = cp.batch_capacity(swo) + 64
        d_pk = torch.zeros((cap + 255) // 256 * 256, dtype=torch.uint8, device="cuda")
        d_off = torch.zeros(3, dtype=torch.int64, device="cuda")
        ctx.encode_messages(d_in, d_swo, d_mso, words, d_pk, d_off)
        torch.cuda.synchronize()
        P = int(d_off[2].item())
        U = 8 * words
        # ---- device form
        d_out = torch.zeros(words + cp.MSG_HEAD_WORDS, dtype=torch.int64, device="cuda")
        d_info = torch.zeros(cp.MSG_INFO_WORDS, dtype=torch.int64, device="cuda")

        def dev():
            ctx.read_message(d_pk, P, d_out, d_info, traversal_limit_words=1 << 31)
            torch.cuda.synchronize()
        dev()
        td = med(dev, 10)
        info = d_info.cpu().numpy()
        cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
        s0 = int(info[4])
        ctx.count_mismatch(d_in, d_out[s0: s0 + words], words, cnt)
        torch.cuda.synchronize()
        okd = info[0] == 0 and info[1] == P and info[3] == words and int(cnt.item()) == 0
        # ---- host form
        h_pk = d_pk[:P].cpu().numpy()
        h_out = np.zeros(words + 1, np.uint64)
        h_info = np.zeros(cp.MSG_INFO_WORDS, np.uint64)

        def host():
            rc = lib.cpk_read_message_host(ctx.handle, h_pk.ctypes.data, P, 8 << 20 << 8, h_out.ctypes.data,
                                           words, h_info.ctypes.data)
            assert rc == 0, rc
        host()
        th = med(host, 5)
        ref = d_in.cpu().numpy().view(np.uint64)
        okh = h_info[1] == P and np.array_equal(h_out[int(h_info[4]): int(h_info[4]) + words], ref)
        # ---- round 2's staged calls: first word, then the segments
        one = np.array([0, 1], np.uint64)
        w_out = np.zeros(16, np.uint8)
        s_out = np.zeros(U + 8, np.uint8)

        def three():
            _, b1, st1 = ctx.decode_stream_host(h_pk, one, out=w_out)
            first = int(b1[-1])
            dec, b2, st2 = ctx.decode_stream_host(h_pk[first:], swo, out=s_out)
            return dec, first + int(b2[-1])
        dec, used = three()
        t3 = med(three, 5)
        ok3 = used == P and np.array_equal(dec.view(np.uint64), ref)
        print(f"message {P / (1 << 20):7.1f} MiB packed ({U / (1 << 20):7.1f} MiB words):"
              f"  device {td * 1e3:7.3f} ms ({U / td / gib:6.1f} GiB/s words) ok={okd}"
              f"  host {th * 1e3:7.2f} ms ({U / th / gib:5.2f} GiB/s) ok={okh}"
              f"  3-call {t3 * 1e3:7.2f} ms ({U / t3 / gib:5.2f} GiB/s) ok={ok3}", flush=True)


if __name__ == "__main__":
    main()
