"""CPU-side checks of libgossip_hip.so: it loads, exports every symbol that
include/gossip.h declares, and its host-only helpers (Go formatting, Go
quantisation, Philox) are right.  No compute call needs a GPU here."""
from __future__ import annotations

import json
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def L():
    from gossip_simulator_amd import _lib
    return _lib


def header_symbols():
    with open(os.path.join(ROOT, "include", "gossip.h")) as f:
        src = f.read()
    return sorted(set(re.findall(r"\b(gs_[a-z0-9_]+)\s*\(", src)))


def test_exports_every_declared_symbol(L):
    lib = L.load()
    syms = header_symbols()
    assert len(syms) >= 20
    for s in syms:
        assert hasattr(lib, s), f"{s} declared in include/gossip.h but not exported"
    assert sorted(L.EXPORTS) == syms
    assert lib.gs_version() == 6


def test_header_constants_match_binding(L):
    """Every #define GS_* / enum GS_* value in include/gossip.h equals the
    ctypes binding's constant of the same name."""
    with open(os.path.join(ROOT, "include", "gossip.h")) as f:
        src = f.read()
    defs = dict((k, int(v)) for k, v in re.findall(r"#define (GS_[A-Z0-9_]+) (\d+)u?\b", src))
    defs.update((k, int(v)) for k, v in re.findall(r"\b(GS_[A-Z0-9_]+) = (-?\d+)", src))
    assert len(defs) >= 15
    missing = [k for k in defs if not hasattr(L, k)]
    assert not [k for k in missing if k.startswith("GS_FLAG_") or k.startswith("GS_MODEL_")], missing
    for k, v in defs.items():
        if hasattr(L, k):
            assert getattr(L, k) == v, (k, getattr(L, k), v)


def test_struct_sizes_match_header(L):
    import ctypes as C
    assert C.sizeof(L.Params) == 8 + 4 * 4 + 8 + 8 + 8 + 4 + 4 + 4 + 4 + 8 + 8 + 4 * 8
    assert C.sizeof(L.TickStats) == 7 * 8
    assert C.sizeof(L.Window) == 3 * 8
    assert C.sizeof(L.TrialStats) == 8 * 8 + 2 * 4


@pytest.mark.parametrize("x,s", [
    (99.61, "99.61"), (100.0, "100"), (0.0, "0"), (49.998, "49.998"),
    (1e-7, "1e-07"), (0.002, "0.002"), (0.0001, "0.0001"), (0.00001, "1e-05"),
    (12.5, "12.5"), (33.333332, "33.333332"), (1234567.0, "1.234567e+06"),
])
def test_go_float32_format(L, x, s):
    assert L.format_float32(x) == s


def test_go_float32_one_node_of_a_billion(L):
    import numpy as np
    pct = np.float32(1) / np.float32(1e9)
    assert L.format_float32(float(np.float32(pct * np.float32(100)))) == "9.9999994e-08"


@pytest.mark.parametrize("x,s", [(0.1, "0.1"), (0.001, "0.001"), (0.01, "0.01"),
                                 (1e-05, "1e-05"), (1.0, "1"), (1e21, "1e+21"),
                                 (123456.0, "123456"), (1e6, "1e+06")])
def test_go_float64_format(L, x, s):
    assert L.format_float64(x) == s


@pytest.mark.parametrize("ns,s", [
    (0, "0s"), (1, "1ns"), (999, "999ns"), (1500, "1.5µs"), (10_000_000, "10ms"),
    (120_500_000, "120.5ms"), (1_000_000_000, "1s"), (1_500_000_000, "1.5s"),
    (60_000_000_000, "1m0s"), (3_723_000_000_000, "1h2m3s"), (-2_000_000, "-2ms"),
    (290_000_000, "290ms"), (1_230_000_000, "1.23s"),
])
def test_go_duration_format(L, ns, s):
    assert L.format_duration(ns) == s


@pytest.mark.parametrize("rate,k", [(0.001, 0), (0.1, 10), (0.29, 28), (0.57, 56),
                                    (0.58, 57), (0.01, 1), (1.0, 100), (-1.0, 0)])
def test_threshold(L, rate, k):
    assert L.threshold(rate) == k


def test_product_philox_matches_kat(L):
    with open(os.path.join(ROOT, "tests", "golden", "philox_kat.json")) as f:
        kat = json.load(f)
    for v in kat:
        assert L.philox(v["ctr"], v["key"]) == v["out"]


def test_stride_magic_division_exact():
    # gs_api.cpp: q / S == umulhi(q, floor(2^32/S) + 1) for q < 1024*255, S in [2, 255]
    import numpy as np
    q = np.arange(0, 1024 * 255 + 1, dtype=np.uint64)
    for S in range(2, 256):
        M = np.uint64((1 << 32) // S + 1)
        assert np.array_equal((q * M) >> np.uint64(32), q // np.uint64(S)), S


def test_create_without_gpu_fails_loudly(L):
    import ctypes as C
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    p = L.Params()
    p.n, p.fanout, p.fanin, p.delay_low, p.delay_high = 100, 5, 6, 10, 20
    h = C.c_void_p()
    assert L.load().gs_create(C.byref(p), C.byref(h)) == L.GS_EDEVICE
    assert not h.value


def test_create_rejects_reference_panics(L):
    import ctypes as C
    p = L.Params()
    p.n, p.fanout, p.fanin, p.delay_low, p.delay_high = 0, 5, 6, 10, 20
    h = C.c_void_p()
    assert L.load().gs_create(C.byref(p), C.byref(h)) == L.GS_EINVAL  # :240 Intn(0)
    p.n, p.delay_low, p.delay_high = 10, 20, 20
    assert L.load().gs_create(C.byref(p), C.byref(h)) == L.GS_EINVAL  # :167 Intn(0)
