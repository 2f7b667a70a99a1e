"""CPU model of the tiled encoder's carried run state (packed_codec.hip
enc_tile_state): encodes a piece tile by tile, each tile seeing only its own
words, a 256-word look-ahead and the state published by earlier tiles, and
checks the bytes against the oracle.  Validates the state algebra (Z phase,
D/L head distance, PASS tiles) independent of the GPU."""
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "oracle"))
import oracle  # noqa: E402

NOHEAD = None


def groups(words):
    nz = (words.reshape(-1, 8) != 0).sum(1)
    g = np.where(nz == 0, 0, np.where(nz >= 7, 1, 2))
    return g, nz


def encode_tiled(data: bytes, TS: int):
    w = np.frombuffer(data, np.uint8).reshape(-1, 8)
    N = len(w)
    g, nz = groups(w)
    out = bytearray()
    states = []  # per tile: ("LOCAL", grp, val) | ("PASS", kind)
    ntiles = max(1, -(-N // TS))
    for t in range(ntiles):
        a, b = t * TS, min(N, (t + 1) * TS)
        W = b - a
        last = b >= N
        # local view: words [a, b) + look-ahead 256 + the word before
        def grp(k):  # local index
            p = a + k
            return g[p] if 0 <= p < N else 3
        # run starts within the tile
        starts = [k for k in range(W) if grp(k) != grp(k - 1)]
        # look-ahead run end after the tile
        look = W
        if not last:
            look = W + 256
            for k in range(W, W + 256):
                if grp(k) != grp(k - 1):
                    look = k
                    break
        def run_end(k):
            nxt = [s for s in starts if s > k]
            return nxt[0] if nxt else look
        isD = lambda k: 0 <= k < W and nz[a + k] == 8  # noqa: E731
        def first_d(x, lim):
            for k in range(max(x, 0), lim):
                if isD(k):
                    return k
            return lim
        def chain(x, lim):
            hs = []
            h = first_d(x, lim)
            while h < lim:
                hs.append(h)
                h = first_d(h + 256, lim)
            return hs
        cont = t > 0 and W > 0 and grp(0) == grp(-1)
        # entry state: nearest LOCAL, composing PASS tiles
        rs_in, hl_in = -1, NOHEAD
        if cont and grp(0) != 2:
            q = t - 1
            sawD = False
            while states[q][0] == "PASS":
                sawD |= states[q][1] == "D"
                q -= 1
            _, sg, val = states[q]
            assert sg == grp(0)
            if sg == 0:
                rs_in = -val
            else:
                dist = val
                if sawD:
                    dist = 256 if (dist == 0 or dist > 256) else dist
                hl_in = -dist if dist else NOHEAD
        # exit state
        if not last:
            gF = grp(W - 1)
            sF = starts[-1] if starts else -1
            if gF == 2:
                states.append(("LOCAL", 2, 0))
            elif sF >= 0:
                if gF == 0:
                    states.append(("LOCAL", 0, (-sF) % 256))
                else:
                    hs = chain(sF, W)
                    states.append(("LOCAL", 1, W - hs[-1] if hs else 0))
            elif gF == 0:
                states.append(("PASS", "Z"))
            elif all(isD(k) for k in range(W)):
                states.append(("PASS", "D"))
            else:
                hs = chain(max((hl_in if hl_in is not None else -10**9) + 256, 0), W)
                states.append(("LOCAL", 1, W - hs[-1] if hs else 0))
        # roles
        heads = set()
        member_until = -1
        run_of = {}
        for si, s0 in enumerate([0] if cont else []):
            pass
        # D/L heads per run
        runs = []
        s_list = ([0] if cont and 0 not in starts else []) + starts
        for i, s0 in enumerate(s_list):
            e0 = s_list[i + 1] if i + 1 < len(s_list) else look
            runs.append((s0, e0, cont and s0 == 0 and 0 not in starts))
        for s0, e0, c in runs:
            if grp(s0) != 1:
                continue
            if c:
                if hl_in is not None:
                    member_until = hl_in + 255
                hs = chain(max((hl_in if hl_in is not None else -10**9) + 256, 0), min(e0, W))
            else:
                hs = chain(s0, min(e0, W))
            for h in hs:
                heads.add((h, e0))
        mem = np.zeros(W, bool)
        for h, e0 in heads:
            mem[h + 1: min(h + 255, e0 - 1) + 1] = True
        if member_until >= 0:
            first_end = runs[0][1]
            mem[: min(member_until + 1, first_end, W)] = True
        hd = {h: e0 for h, e0 in heads}
        for s0, e0, c in runs:
            rs = rs_in if c else s0
            for k in range(s0, min(e0, W)):
                word = bytes(w[a + k])
                gk = grp(k)
                if gk == 0:
                    if (k - rs) % 256 == 0:
                        out += bytes([0, min(255, e0 - k - 1)])
                elif gk == 2:
                    m = sum(1 << i for i in range(8) if word[i])
                    out += bytes([m]) + bytes(x for x in word if x)
                else:
                    if mem[k]:
                        out += word
                    elif k in hd:
                        out += bytes([0xFF]) + word + bytes([min(255, e0 - k - 1)])
                    else:  # L head
                        m = sum(1 << i for i in range(8) if word[i])
                        out += bytes([m]) + bytes(x for x in word if x)
    return bytes(out)


def rand_piece(rng, n):
    out = []
    while len(out) < n:
        kind = rng.integers(0, 6)
        ln = int(rng.choice([1, 3, 100, 255, 256, 257, 300, 511, 513, 700, 1500]))
        if kind == 0:
            out += [np.zeros(8, np.uint8)] * ln
        elif kind == 1:
            out += [rng.integers(1, 256, 8, dtype=np.uint8) for _ in range(ln)]
        elif kind == 2:  # D/L mix
            for _ in range(ln):
                x = rng.integers(1, 256, 8, dtype=np.uint8)
                if rng.random() < 0.3:
                    x[rng.integers(0, 8)] = 0
                out.append(x)
        elif kind == 3:  # mostly L with rare D
            for _ in range(ln):
                x = rng.integers(1, 256, 8, dtype=np.uint8)
                if rng.random() < 0.97:
                    x[rng.integers(0, 8)] = 0
                out.append(x)
        elif kind == 4:
            for _ in range(min(ln, 5)):
                x = rng.integers(1, 256, 8, dtype=np.uint8)
                x[rng.choice(8, 3, replace=False)] = 0
                out.append(x)
        else:
            out.append(rng.integers(0, 256, 8, dtype=np.uint8))
    return np.concatenate(out[:n]).tobytes()


if __name__ == "__main__":
    rng = np.random.default_rng(int(sys.argv[1]) if len(sys.argv) > 1 else 1)
    trials = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    bad = 0
    for trial in range(trials):
        n = int(rng.integers(1, 5000))
        d = rand_piece(rng, n)
        ref = oracle.pack(d)
        for TS in (256, 512):
            got = encode_tiled(d, TS)
            if got != ref:
                bad += 1
                i = next((i for i in range(min(len(got), len(ref))) if got[i] != ref[i]), None)
                print("MISMATCH trial", trial, "n", n, "TS", TS, "first diff", i, len(got), len(ref))
                break
    print("bad", bad, "of", trials)
