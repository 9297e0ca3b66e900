"""k_part2's tiles dealt by XCD (gs_window.hip tiles_by_xcd): k_plan writes
the tile prefix in the order (bin & 7, bin >> 3, sub-region); workgroup b of a
grid that is a multiple of 8 takes XCD b & 7's run of tiles, strided by
grid / 8.  CPU restatement: every tile of every region is taken exactly once,
by a workgroup of the XCD its bin is dealt to, and maps back to its region."""
import numpy as np
import pytest

SUB, REG = 8, 2048


def pos(c):
    return (c & 7) * 32 + (c >> 3)


def bin_of(pc):
    return (pc & 31) * 8 + (pc >> 5)


def plan(fills, tile):
    """k_plan block 0: tprefix indexed by rho = pos(c) * 8 + sub."""
    ntile = (fills + tile - 1) // tile
    per_bin = ntile.reshape(256, SUB).sum(1)
    s_pt = np.zeros(256, np.int64)
    s_pt[[pos(c) for c in range(256)]] = per_bin
    pre = np.concatenate([[0], np.cumsum(s_pt)])
    tp = np.zeros(REG + 1, np.int64)
    for c in range(256):
        a = pre[pos(c)]
        for x in range(SUB):
            tp[pos(c) * SUB + x] = a
            a += ntile[c * SUB + x]
    tp[REG] = pre[256]
    return tp, ntile


def test_bin_order_is_a_permutation():
    assert sorted(pos(c) for c in range(256)) == list(range(256))
    assert all(bin_of(pos(c)) == c for c in range(256))


@pytest.mark.parametrize("grid", [8, 64, 2304, 8192])
@pytest.mark.parametrize("ncoarse", [1, 7, 239, 256])
def test_every_tile_once_on_its_xcd(grid, ncoarse):
    rng = np.random.default_rng(grid + ncoarse)
    tile = 16384
    fills = rng.integers(0, 5 * tile, REG)
    fills[ncoarse * SUB:] = 0
    tp, ntile = plan(fills, tile)
    seen = {}
    for b in range(grid):
        x = b & 7
        g0, g1, step = tp[x * 256] + (b >> 3), tp[(x + 1) * 256], grid >> 3
        for g in range(g0, g1, step):
            rho = int(np.searchsorted(tp[:REG], g, side="right") - 1)
            r = bin_of(rho // SUB) * SUB + rho % SUB
            assert (r // SUB) & 7 == x                 # dealt to its bin's XCD
            k = (r, g - tp[rho])
            assert 0 <= k[1] < ntile[r] and k not in seen
            seen[k] = b
    assert len(seen) == int(ntile.sum())
