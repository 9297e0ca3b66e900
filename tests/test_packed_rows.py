"""k_expand's packed row view (gs_window.hip pk_byte, k_pack_rows): row v of
a stride-8 sealed table lives at byte 128 * (v / 5) + 24 * (v mod 5), with v / 5
computed as (v * 0xCCCCCCCD) >> 34, and is read as two 16-B loads from the
row's 16-B aligned base.  CPU restatement of the index arithmetic and the
two-load selection over all five offsets in a line."""
import numpy as np


def pk_byte(v):
    v = np.asarray(v, dtype=np.uint64)
    line = (v * np.uint64(0xCCCCCCCD)) >> np.uint64(34)
    return line * np.uint64(128) + (v - line * np.uint64(5)) * np.uint64(24)


def test_div5_by_multiply_shift_exact_for_32_bit_ids():
    rng = np.random.default_rng(5)
    v = np.concatenate([np.arange(0, 1 << 20, dtype=np.uint64),
                        rng.integers(0, 1 << 32, 1 << 20, dtype=np.uint64),
                        np.arange((1 << 32) - (1 << 16), 1 << 32, dtype=np.uint64)])
    line = (v * np.uint64(0xCCCCCCCD)) >> np.uint64(34)
    assert np.array_equal(line, v // np.uint64(5))


def test_rows_never_straddle_a_line_and_two_aligned_loads_cover_them():
    v = np.arange(0, 100_000, dtype=np.uint64)
    b = pk_byte(v)
    assert np.all(b // 128 == (b + 23) // 128)          # inside one 128-B line
    assert len(np.unique(b)) == len(b)                    # no two rows overlap
    base = b & ~np.uint64(15)
    assert np.all(base + 32 >= b + 24) and np.all((b & 7) == 0)
    assert np.all(base // 128 == (base + 31) // 128)      # both loads in the same line


def test_packed_view_round_trip():
    rng = np.random.default_rng(9)
    n = 1003
    ids = rng.integers(0, 1 << 30, (n, 8), dtype=np.uint32)
    pk = np.zeros(((n + 4) // 5) * 32, dtype=np.uint32)  # u32 words, 32 per line
    for v in range(n):  # k_pack_rows: slots 0..5 of row v
        w = int(pk_byte(v)) // 4
        pk[w:w + 6] = ids[v, :6]
    for v in range(n):  # load_row's packed path: two uint4 loads + a select
        b = int(pk_byte(v))
        x = pk[(b & ~15) // 4:(b & ~15) // 4 + 8]
        row = x[2:8] if b & 8 else x[0:6]
        assert np.array_equal(row, ids[v, :6])
