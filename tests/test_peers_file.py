import numpy as np
import pytest

from gossip_simulator_amd import peers


@pytest.mark.parametrize("n,stride", [(1, 2), (7, 6), (1000, 19), (4133, 6)])
def test_roundtrip(tmp_path, n, stride):
    rng = np.random.default_rng(n)
    deg = rng.integers(0, stride + 1, n).astype(np.uint8)
    ids = rng.integers(0, n, (n, stride)).astype(np.uint32)
    path = str(tmp_path / "x.peers")
    peers.write(path, deg, ids)
    d2, i2 = peers.read(path)
    assert np.array_equal(deg, d2) and np.array_equal(ids, i2)
    with open(path, "rb") as f:
        head = f.read(24)
    assert head[:8] == b"GSPEERS1"
    assert int.from_bytes(head[8:16], "little") == n


def test_rejects_garbage(tmp_path):
    path = tmp_path / "bad"
    path.write_bytes(b"NOTPEERS" + bytes(32))
    with pytest.raises(ValueError):
        peers.read(str(path))
