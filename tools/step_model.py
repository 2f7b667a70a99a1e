"""CPU model of the single-pass encoder's mask algebra (csrc/encode_sp.hip).

The kernel never walks a piece word by word: it classifies 64-word steps
into 64-bit masks (Z: zero word, DL: <= 1 zero byte, D: tag 0xff) and derives
every word's role in PackedOutputStream.write (PackedOutputStream.java:64-193)
from mask arithmetic plus a small carried state:

  zl  length of the zero run ending at the step start (0: none);
  dlo the word before the step is a D/L word (its stretch may continue);
  hd  distance from the step start back to that stretch's last 0xFF head
      (0: no head yet), capped at 256.

roles() below is the per-step function the kernel runs (SALU); state_at()
recomputes the state entering any step from the masks of the steps before it
(what each wave does for its first step); encode_model() drives both the way
the kernel does -- chunks of CS steps, waves of WS steps, per-step run-end
masks for the counts -- and returns the packed bytes, which tests compare
with the oracle (tests/test_step_model.py).
"""
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "oracle"))

M64 = (1 << 64) - 1


def ctz(x):
    return (x & -x).bit_length() - 1 if x else 64


def hibit(x):
    return x.bit_length() - 1  # -1 for 0


def clz(x):
    return 64 - x.bit_length()


def step_masks(tags, W, s):
    """(V, Z, DL, D) of step s from per-word nonzero-byte tags."""
    V = Z = DL = D = 0
    for j in range(64):
        k = 64 * s + j
        if k >= W:
            break
        m = int(tags[k])
        V |= 1 << j
        pc = bin(m).count("1")
        if m == 0:
            Z |= 1 << j
        if pc >= 7:
            DL |= 1 << j
        if m == 0xFF:
            D |= 1 << j
    return V, Z, DL, D


def roles(Z, DL, D, st):
    """Role masks of one step and the state entering the next.
    -> (Zh, Mem, Dh, (zl', dlo', hd'))."""
    zl, dlo, hd = st
    # zero runs: a head at every run start and every 256 words after it
    Zh = Z & ~(((Z << 1) | (1 if zl > 0 else 0)) & M64)
    if zl > 0 and (Z & 1):
        j0 = (256 - zl % 256) % 256
        if j0 < 64:
            pre = (2 << j0) - 1
            if Z & pre == pre:
                Zh |= 1 << j0
    nz = ~Z & M64
    zl2 = zl + 64 if nz == 0 else clz(nz)
    # D/L stretches: members follow a head for up to 255 words
    # (PackedOutputStream.java:133-193); carry-add smear from each D
    if dlo and (DL & 1) and hd >= 193:
        f = ctz(~DL & M64)
        rng = (1 << f) - 1
        A = (D << 1) & M64 & DL
        C = ((DL + A) ^ DL ^ A) & M64
        Mem = DL & (A | C) & ~rng
        c = 255 - hd                     # last lane the carried head covers
        cm = ((1 << min(c + 1, f)) - 1) if c >= 0 else 0
        x = max(c + 1, 0)
        dc = D & rng & ~((1 << x) - 1)   # next head: first D >= old head + 256
        if dc:
            h1 = ctz(dc)
            cm |= rng & ~((2 << h1) - 1)
        Mem |= cm
    else:
        cin = 1 if (dlo and (DL & 1) and hd > 0) else 0
        A = (((D << 1) & M64) | cin) & DL
        C = ((DL + A) ^ DL ^ A) & M64
        Mem = DL & (A | C)
    Dh = D & ~Mem
    if (DL >> 63) & 1:
        nd = ~DL & M64
        t = 64 - clz(nd) if nd else 0    # start of the run reaching bit 63
        H = Dh & (M64 & ~((1 << t) - 1))
        if H:
            hd2 = 64 - hibit(H)
        elif t == 0 and dlo and hd > 0:
            hd2 = min(hd + 64, 256)
        else:
            hd2 = 0
        return Zh, Mem, Dh, (zl2, True, hd2)
    return Zh, Mem, Dh, (zl2, False, 0)


def first_d(masks, x, lim):
    """first D word at position >= x and < lim (positions relative to the
    chunk), else lim."""
    if x >= lim:
        return lim
    q = x >> 6
    m = masks[q][3] & (M64 & ~((1 << (x & 63)) - 1))
    while not m:
        q += 1
        if q * 64 >= lim:
            return lim
        m = masks[q][3]
    return min(q * 64 + ctz(m), lim)


def state_at(masks, s0, cst):
    """State entering step s0 of a chunk from the masks of steps < s0 and the
    chunk's entering state cst (the kernel's per-wave entry)."""
    if s0 == 0:
        return cst
    _, Zp, DLp, _ = masks[s0 - 1]
    zl = 0
    if (Zp >> 63) & 1:
        q = s0 - 1
        while q >= 0 and masks[q][1] == M64:
            zl += 64
            q -= 1
        if q >= 0:
            zl += clz(~masks[q][1] & M64)
        else:
            zl += cst[0]
    if not (DLp >> 63) & 1:
        return (zl, False, 0)
    # stretch start (chunk-relative; None = continues from the previous chunk)
    q = s0 - 1
    while q >= 0 and masks[q][2] == M64:
        q -= 1
    P = 64 * s0
    if q >= 0:
        start = 64 * q + 64 - clz(~masks[q][2] & M64)
        h = first_d(masks, start, P)
        if h >= P:
            return (zl, True, 0)
    else:
        if not cst[1]:
            h = first_d(masks, 0, P)
            if h >= P:
                return (zl, True, 0)
        elif cst[2] > 0:
            h = -cst[2]
        else:
            h = first_d(masks, 0, P)
            if h >= P:
                return (zl, True, 0)
    while True:
        h2 = first_d(masks, max(h + 256, 0), P)
        if h2 >= P:
            break
        h = h2
    return (zl, True, min(P - h, 256))


def encode_model(data, WS=32, NW=4):
    """Packed bytes of one piece (uint8 array, len % 8 == 0) the way the
    single-pass kernel produces them: chunks of CS = WS * NW steps, each
    wave's first state from state_at, the rest sequential."""
    w = np.frombuffer(bytes(data), np.uint8).reshape(-1, 8)
    W = len(w)
    if W == 0:
        return b""
    nzb = w != 0
    tags = (nzb * (1 << np.arange(8))).sum(1)
    CS = WS * NW
    nsteps = (W + 63) // 64
    all_masks = [step_masks(tags, W, s) for s in range(nsteps + 5)]
    out = bytearray()
    cst = (0, False, 0)
    for c0 in range(0, nsteps, CS):
        c1 = min(c0 + CS, nsteps)
        masks = all_masks[c0:c1]
        nxt = all_masks[c1:c1 + 5]   # look-ahead (next chunk's first steps)
        roles_of = {}
        end_state = None
        for wv in range(NW):
            s_a, s_b = wv * WS, min((wv + 1) * WS, c1 - c0)
            if s_a >= s_b:
                continue
            st = state_at(masks, s_a, cst)
            for s in range(s_a, s_b):
                V, Z, DL, D = masks[s]
                Zh, Mem, Dh, st = roles(Z, DL, D, st)
                roles_of[s] = (Zh, Mem, Dh)
            if s_b == c1 - c0:
                end_state = st
        seq = masks + nxt
        for s in range(c1 - c0):
            V, Z, DL, D = masks[s]
            Zh, Mem, Dh = roles_of[s]
            nV, nZ, nDL, nD = seq[s + 1] if s + 1 < len(seq) else (0, 0, 0, 0)
            E = (Z & ~(((Z >> 1) | ((nZ & 1) << 63)) & M64)) | \
                (DL & ~(((DL >> 1) | ((nDL & 1) << 63)) & M64))
            # X: run continuation past the step end, minus one (counts cap at 255)
            X = 0
            cls = 1 if (Z >> 63) & 1 else 2 if (DL >> 63) & 1 else 0
            if cls:
                r, q = 0, s + 1
                while q < len(seq) and r < 256:
                    cm = seq[q][cls]
                    if cm == M64:
                        r += 64
                        q += 1
                        continue
                    r += ctz(~cm & M64)
                    break
                X = max(min(r, 256) - 1, 0)
            for j in range(64):
                k = 64 * (c0 + s) + j
                if k >= W:
                    break
                if (Mem >> j) & 1:
                    out += bytes(w[k])
                    continue
                if (Z >> j) & 1 and not (Zh >> j) & 1:
                    continue
                m = int(tags[k])
                out.append(m)
                out += bytes(b for b in w[k] if b)
                if ((Zh | Dh) >> j) & 1:
                    e = E >> j
                    ne = 64 * (c0 + s) + j + ctz(e) if e else 64 * (c0 + s + 1) + X
                    out.append(min(255, ne - k))
        cst = end_state
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
            for _ in range(min(ln, 40)):
                x = rng.integers(0, 256, 8, dtype=np.uint8)
                x[rng.random(8) < 0.5] = 0
                out.append(x)
    return np.concatenate(out[:n]).tobytes()


def roles_parallel(wmasks, st):
    """The lane-parallel form of a wave's roles (csrc/encode_sp.hip sp_a2p):
    step j's Zh / Mem from its own masks plus ballots over the wave's steps.
    wmasks: [(V, Z, DL, D)] of the wave's steps; st: state entering the first.
    -> [(Zh, Mem)] or None when a D/L stretch over 192 words enters a step
    (the kernel then runs the sequential form)."""
    cnt = len(wmasks)
    Zs = [m[1] for m in wmasks]
    DLs = [m[2] for m in wmasks]
    Ds = [m[3] for m in wmasks]
    zl_in, dlo_in, hd_in = st
    notall_dl = [DLs[j] != M64 for j in range(cnt)]
    topdl = [64 if DLs[j] == M64 else clz(~DLs[j] & M64) for j in range(cnt)]
    anyD = [Ds[j] != 0 for j in range(cnt)]
    topd = [topdl[j] > 0 and (Ds[j] >> (64 - topdl[j])) != 0 for j in range(cnt)]
    notall_z = [Zs[j] != M64 for j in range(cnt)]
    topz = [64 if Zs[j] == M64 else clz(~Zs[j] & M64) for j in range(cnt)]
    out = []
    for j in range(cnt):
        Z, DL, D = Zs[j], DLs[j], Ds[j]
        dlo = (DLs[j - 1] >> 63) & 1 if j else (1 if dlo_in else 0)
        kd = max([k for k in range(j) if notall_dl[k]], default=-1)
        ln = topdl[kd] + 64 * (j - 1 - kd) if kd >= 0 else (hd_in if dlo_in else 0) + 64 * j
        cont = dlo and (DL & 1)
        if cont and ln > 192:
            return None
        btw = any(anyD[k] for k in range(kd + 1, j))
        head = btw or (topd[kd] if kd >= 0 else bool(dlo_in and hd_in))
        cin = 1 if (cont and head) else 0
        A = (((D << 1) & M64) | cin) & DL
        C = ((DL + A) ^ DL ^ A) & M64
        Mem = DL & (A | C)
        zc = (Zs[j - 1] >> 63) & 1 if j else (1 if zl_in else 0)
        Zh = Z & ~(((Z << 1) | zc) & M64)
        kz = max([k for k in range(j) if notall_z[k]], default=-1)
        zl = topz[kz] + 64 * (j - 1 - kz) if kz >= 0 else zl_in + 64 * j
        j0 = (256 - (zl & 255)) & 255
        if zc and (Z & 1) and j0 < 64:
            pre = (2 << j0) - 1
            if Z & pre == pre:
                Zh |= 1 << j0
        out.append((Zh, Mem))
    return out
