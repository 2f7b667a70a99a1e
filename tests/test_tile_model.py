"""The tiled encoder's carried run state (packed_codec.hip enc_tile_state),
modelled on the CPU at small tile sizes (multiples of 256 like the kernel's
8192) and checked against the oracle: each tile sees only its words, a
256-word look-ahead and the states earlier tiles published."""
import numpy as np
import pytest

import tile_model


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_tile_state_algebra_matches_oracle(oracle, seed):
    rng = np.random.default_rng(seed)
    for _ in range(15):
        d = tile_model.rand_piece(rng, int(rng.integers(1, 4000)))
        ref = oracle.pack(d)
        for ts in (256, 512):
            assert tile_model.encode_tiled(d, ts) == ref


def test_tile_state_edge_pieces(oracle):
    D = np.full(8, 7, np.uint8)
    L = np.array([0, 1, 2, 3, 4, 5, 6, 7], np.uint8)
    Z = np.zeros(8, np.uint8)
    cases = [
        [Z] * 2000, [D] * 2000, [L] * 2000,
        [L] * 300 + [D] + [L] * 1700, [D] * 511 + [L] * 700 + [D] * 900,
        [Z] * 255 + [D] * 1030 + [Z] * 257, [L] * 255 + [D] * 2 + [L] * 1000,
    ]
    for c in cases:
        d = np.concatenate(c).tobytes()
        for ts in (256, 512):
            assert tile_model.encode_tiled(d, ts) == oracle.pack(d)
