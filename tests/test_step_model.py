"""The single-pass encoder's mask algebra (tools/step_model.py, the model of
csrc/encode_sp.hip's role pass) against the oracle: per-step role masks from
a carried state, per-wave entry states recomputed from earlier steps' masks,
pieces processed in chunks with the state carried between them.  Small wave /
chunk sizes put many wave and chunk seams inside each piece."""
import numpy as np
import pytest

import step_model as sm


@pytest.mark.parametrize("ws,nw", [(32, 4), (1, 2), (2, 3), (4, 1)])
@pytest.mark.parametrize("seed", [1, 2])
def test_mask_algebra_matches_oracle(oracle, ws, nw, seed):
    rng = np.random.default_rng(seed * 100 + ws)
    for _ in range(6):
        d = sm.rand_piece(rng, int(rng.integers(1, 3000)))
        assert sm.encode_model(d, ws, nw) == oracle.pack(d)


@pytest.mark.parametrize("ws,nw", [(32, 4), (1, 1), (2, 2), (3, 1)])
def test_mask_algebra_edge_pieces(oracle, ws, nw):
    D = np.full(8, 7, np.uint8)
    L = np.array([0, 1, 2, 3, 4, 5, 6, 7], np.uint8)
    Z = np.zeros(8, np.uint8)
    M = np.array([0, 0, 9, 0, 1, 0, 0, 0], np.uint8)
    cases = [
        [Z] * 2000, [D] * 2000, [L] * 2000, [Z] * 256, [Z] * 257, [Z] * 512 + [M],
        [L] * 300 + [D] + [L] * 1700, [D] * 511 + [L] * 700 + [D] * 900,
        [Z] * 255 + [D] * 1030 + [Z] * 257, [L] * 255 + [D] * 2 + [L] * 1000,
        [D] * 256 + [L] * 3 + [D] * 300, [D] * 193 + [M] + [D] * 70,
        [L] * 64 + [D] + [L] * 255 + [D] * 2 + [L] * 600 + [D] * 5,
        [M, D, Z, D, L, L, Z, Z, M] * 40,
    ]
    for c in cases:
        d = np.concatenate(c).tobytes()
        assert sm.encode_model(d, ws, nw) == oracle.pack(d), [len(x) for x in c][:4]


def test_state_at_equals_sequential_state():
    rng = np.random.default_rng(7)
    for _ in range(5):
        d = sm.rand_piece(rng, int(rng.integers(200, 2500)))
        w = np.frombuffer(d, np.uint8).reshape(-1, 8)
        tags = ((w != 0) * (1 << np.arange(8))).sum(1)
        ns = (len(w) + 63) // 64
        masks = [sm.step_masks(tags, len(w), s) for s in range(ns)]
        st = (0, False, 0)
        for s in range(ns):
            assert sm.state_at(masks, s, (0, False, 0)) == st, s
            _, Z, DL, D = masks[s]
            st = sm.roles(Z, DL, D, st)[3]


@pytest.mark.parametrize("ws", [32, 5, 2])
def test_parallel_roles_equal_sequential(oracle, ws):
    """sp_a2p's ballot formulation (tools/step_model.roles_parallel) gives the
    sequential roles on every wave it accepts, from any entry state."""
    rng = np.random.default_rng(ws)
    accepted = fallbacks = 0
    pieces = [sm.rand_piece(rng, int(rng.integers(100, 4000))) for _ in range(8)]
    for cfg in (2, 3, 4):
        swo = np.array([0, 8192], dtype=np.uint64)
        op = oracle.preset(cfg)
        op.cfg = cfg | (ws << 8)
        pieces.append(oracle.generate(op, swo).tobytes())
    for d in pieces:
        w = np.frombuffer(d, np.uint8).reshape(-1, 8)
        tags = ((w != 0) * (1 << np.arange(8))).sum(1)
        ns = (len(w) + 63) // 64
        masks = [sm.step_masks(tags, len(w), s) for s in range(ns)]
        for a in range(0, ns, ws):
            st = sm.state_at(masks, a, (0, False, 0))
            par = sm.roles_parallel(masks[a:a + ws], st)
            if par is None:
                fallbacks += 1
                continue
            accepted += 1
            s2 = st
            for j, (V, Z, DL, D) in enumerate(masks[a:a + ws]):
                Zh, Mem, _, s2 = sm.roles(Z, DL, D, s2)
                assert par[j] == (Zh, Mem), (a, j)
    assert accepted > 10


def _group(m, valid):
    return 3 if not valid else (0 if m == 0 else (1 if bin(m).count("1") >= 7 else 2))


@pytest.mark.parametrize("seed", range(4))
def test_size_pass_boundary_masks(seed):
    """encode_v4.hip's size pass (CPK_E4_MASKROLES) derives the emit pass's
    run-boundary rows from the step's Z / D-or-L masks: BV = past the end |
    M words | a Z word after a non-Z | a D/L word after a non-D/L (the word
    before the step: the carried group gl).  Checked against e4_classify's
    per-lane rule (!valid || g != g_prev || g == 2) and its gl update."""
    rng = np.random.default_rng(seed)
    M64 = (1 << 64) - 1
    for _ in range(400):
        nvalid = int(rng.integers(1, 65))
        gl = int(rng.integers(0, 3))
        kind = rng.choice(["zero", "dense", "mixed"], p=[0.3, 0.3, 0.4])
        tags = []
        for lane in range(64):
            r = rng.random()
            if kind == "zero" and r < 0.7 or kind == "mixed" and r < 0.3:
                tags.append(0)
            elif kind == "dense" and r < 0.7 or kind == "mixed" and r < 0.6:
                tags.append(int(rng.choice([0xFF, 0x7F, 0xFE, 0xBF])))
            else:
                tags.append(int(rng.integers(1, 256)))
        valid = [lane < nvalid for lane in range(64)]
        tags = [t if v else 0 for t, v in zip(tags, valid)]
        # per-lane rule (e4_classify)
        g = [_group(t, v) for t, v in zip(tags, valid)]
        bv_ref = 0
        for lane in range(64):
            gp = gl if lane == 0 else g[lane - 1]
            if not valid[lane] or g[lane] != gp or g[lane] == 2:
                bv_ref |= 1 << lane
        gl_ref = min(g[63], 2)
        # mask form (e4_size_kernel, CPK_E4_MASKROLES)
        Z = sum(1 << i for i in range(64) if valid[i] and tags[i] == 0)
        DL = sum(1 << i for i in range(64) if bin(tags[i]).count("1") >= 7)
        V = M64 if nvalid >= 64 else (1 << nvalid) - 1
        Zp = ((Z << 1) & M64) | (1 if gl == 0 else 0)
        DLp = ((DL << 1) & M64) | (1 if gl == 1 else 0)
        bv = ((~V & M64) | (V & ~Z & ~DL & M64) | (Z & ~Zp & M64) | (DL & ~DLp & M64))
        gl_new = 0 if Z >> 63 else (1 if DL >> 63 else 2)
        assert bv == bv_ref
        assert gl_new == gl_ref
