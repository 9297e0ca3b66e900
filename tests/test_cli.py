"""The gossip_sim CLI keeps simulator.go's flag set, defaults, usage text and
stdout lines (simulator.go:186-253)."""
from __future__ import annotations

import os
import re
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(ROOT, "gossip_simulator_amd", "bin", "gossip_sim")

PARAMS_DEFAULT = """=== Parameters ===
crashrate=0.001
delayhigh=20ms
delaylow=10ms
droprate=0.1
fanin=6
fanout=5
n=50000
"""


def run(*args, timeout=300):
    return subprocess.run([CLI, *args], capture_output=True, text=True, timeout=timeout)


def test_usage_lists_reference_flags_go_style():
    r = run("-h")
    assert r.returncode == 0
    u = r.stderr
    assert u.startswith("Usage of ")
    for block in ["  -crashrate float\n    \tmachine crash rate (default 0.001)",
                  "  -delayhigh int\n    \tdelay high (ms) (default 20)",
                  "  -delaylow int\n    \tdelay low (ms) (default 10)",
                  "  -droprate float\n    \tmessage drop rate (default 0.1)",
                  "  -fanin int\n    \tfanin (default 6)",
                  "  -fanout int\n    \tfanout (default 5)",
                  "  -n int\n    \ttotal number of nodes (default 50000)"]:
        assert block in u
    names = re.findall(r"^  -(\w+)", u, flags=re.M)
    assert names == sorted(names)


def test_bad_flags_exit_2():
    r = run("-bogus")
    assert r.returncode == 2 and "flag provided but not defined: -bogus" in r.stderr
    r = run("-n", "abc")
    assert r.returncode == 2 and 'invalid value "abc" for flag -n: parse error' in r.stderr
    r = run("-n")
    assert r.returncode == 2 and "flag needs an argument: -n" in r.stderr


def test_parameter_echo_before_device():
    r = run("-n=1000")  # no GPU here: echo first, then a loud device failure
    assert r.stdout.startswith(PARAMS_DEFAULT.replace("n=50000", "n=1000"))
    if r.returncode != 0:
        assert "gs_create" in r.stderr


def test_echo_formats_floats_like_go():
    r = run("-droprate", "0.25", "-crashrate=1e-5", "--fanin", "9")
    assert "crashrate=1e-05\n" in r.stdout and "droprate=0.25\n" in r.stdout
    assert "fanin=9\n" in r.stdout


@pytest.mark.gpu
def test_cli_full_run_reference_shape(tmp_path):
    r = run("-n", "50000")
    assert r.returncode == 0, r.stderr
    out = r.stdout
    assert out.startswith(PARAMS_DEFAULT)
    assert "\n\n=== Constructing Overlay ===\n" in out
    assert re.search(r"^break \d+ makeup \d+ elasped \d+(\.\d+)?(ms|s)$", out, re.M)
    assert re.search(r"^--- Took \S+ to stabilize ---\n\n=== Broadcast one message ===$", out, re.M)
    cov = re.findall(r"^([0-9.e+-]+)% covered, took (\S+)$", out, re.M)
    assert cov and float(cov[-1][0]) >= 99.0
    assert all(float(a[0]) <= float(b[0]) for a, b in zip(cov, cov[1:]))
    assert re.search(r"^--- Took \S+ to get 99% ---\n\nTotal message \d+ Total Crashed 0\n$", out,
                     re.M)


@pytest.mark.gpu
@pytest.mark.parametrize("crash,fanout", [("0.02", 4), ("0.01", 5)])
def test_cli_injected_peers_matches_oracle(tmp_path, oracle, crash, fanout):
    from gossip_simulator_amd import peers
    kw = dict(n=20000, fanout=fanout, fanin=6, delay_low=10, delay_high=20, drop_rate=0.1,
              crash_rate=float(crash), seed=9, trial=0)
    p = oracle.make_params(**kw)
    deg, ids, _, _ = oracle.overlay(p)
    path = str(tmp_path / "t.peers")
    peers.write(path, deg, ids)
    rows, _ = oracle.run_to_coverage(p, deg, ids)
    r = run("-n", "20000", "-fanout", str(fanout), "-crashrate", crash, "-seed", "9", "-peers", path)
    cov = re.findall(r"^([0-9.e+-]+)% covered", r.stdout, re.M)
    assert len(cov) == len(rows) // 10
    if not oracle.covered(int(rows[-1, 4]), kw["n"]):
        # the flood died out below 99 %: the reference would poll forever
        assert r.returncode == 3 and "no broadcast left in flight" in r.stderr
        return
    assert r.returncode == 0, r.stderr
    tot = re.search(r"Total message (\d+) Total Crashed (\d+)", r.stdout)
    assert int(tot.group(1)) == int(rows[:, 3].sum()) and int(tot.group(2)) == int(rows[-1, 5])
    last = np.float32(rows[-1, 4]) / np.float32(kw["n"]) * np.float32(100)
    from gossip_simulator_amd import _lib
    assert cov[-1] == _lib.format_float32(float(last))
