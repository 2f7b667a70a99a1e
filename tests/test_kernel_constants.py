"""Host checks of integer tricks the HIP kernels rely on (no GPU needed).

The block-map decoder (csrc/packed_codec.hip: chunk_div) finds the lane
whose chunk holds a window position r as floor(r / C) computed by a 24-bit
multiply and a shift (v_mul_u32_u24, full rate) instead of the compiler's
quarter-rate division by a constant; window positions are < 2^13 (kWin <=
4096).  The decoders check errors only in windows within one window plus the
longest record of the piece's end: a 0xFF tag, its word, the count byte and
255 literal words (PackedOutputStream.java:133-193).
"""
import pytest


def chunk_div(r, c):
    km = ((1 << 20) + c - 1) // c
    return ((r * km) & 0xFFFFFFFF) >> 20  # __umul24 keeps the low 32 bits


@pytest.mark.parametrize("c", [28, 32, 40, 48, 56, 60, 64])
def test_chunk_div_is_exact_for_window_positions(c):
    km = ((1 << 20) + c - 1) // c
    assert (km * c - (1 << 20)) * (1 << 13) < (1 << 20)  # the kernel's static_assert
    assert km < (1 << 24)                                  # a 24-bit operand
    for r in range(1 << 13):
        assert chunk_div(r, c) == r // c, (r, c)


def test_longest_record_fits_the_check_reach():
    longest = 1 + 8 + 1 + 8 * 255  # 0xFF tag, word, count, 255 verbatim words
    assert longest == 2050
    k_win = 64 * 56
    assert k_win + 2064 >= k_win + longest  # CPK_DEC_CHK_REACH default
