"""Injected peer-table file ("GSPEERS1"): the shared artefact for bit-exact
replays between implementations.

Layout (little-endian):
  0   8 B  magic b"GSPEERS1"
  8   u64  n
  16  u32  stride (row length; friends beyond deg[v] are ignored)
  20  u32  reserved (0)
  24  u8   deg[n]            (friends-list lengths, simulator.go:45)
  ..  pad to a multiple of 4
  ..  u32  ids[n * stride]   (row-major friends, simulator.go:45)
The CLI (`gossip_sim -peers FILE`) reads the same format.
"""
from __future__ import annotations

import numpy as np

MAGIC = b"GSPEERS1"


def write(path: str, deg: np.ndarray, ids: np.ndarray) -> None:
    deg = np.ascontiguousarray(deg, dtype=np.uint8)
    ids = np.ascontiguousarray(ids, dtype=np.uint32)
    n, stride = ids.shape
    if deg.shape != (n,):
        raise ValueError("deg must have n entries")
    with open(path, "wb") as f:
        f.write(MAGIC)
        f.write(np.array([n], dtype="<u8").tobytes())
        f.write(np.array([stride, 0], dtype="<u4").tobytes())
        f.write(deg.tobytes())
        f.write(b"\0" * ((4 - (n & 3)) & 3))
        f.write(ids.astype("<u4").tobytes())


def read(path: str):
    with open(path, "rb") as f:
        data = f.read()
    if data[:8] != MAGIC:
        raise ValueError(f"{path}: not a GSPEERS1 file")
    n = int(np.frombuffer(data, "<u8", 1, 8)[0])
    stride = int(np.frombuffer(data, "<u4", 1, 16)[0])
    deg = np.frombuffer(data, np.uint8, n, 24).copy()
    off = 24 + n + ((4 - (n & 3)) & 3)
    ids = np.frombuffer(data, "<u4", n * stride, off).astype(np.uint32).reshape(n, stride)
    if deg.max(initial=0) > stride:
        raise ValueError(f"{path}: a friends-list length exceeds the stride")
    return deg, ids
