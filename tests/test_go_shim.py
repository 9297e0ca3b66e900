"""The committed cgo shim (go/simulator_hip.go) against the C ABI.

No Go toolchain ships in this image, so the shim cannot be compiled here;
instead every C.gs_* / C.GS_* name it uses must be declared in
include/gossip.h (and every function exported by libgossip_hip.so), and every
gs_params / gs_tick_stats / gs_window field it touches must exist.  The Go
globals it reads are the reference's flag variables (simulator.go:12-20)."""
from __future__ import annotations

import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GO = os.path.join(ROOT, "go", "simulator_hip.go")


def _read(p):
    with open(p) as f:
        return f.read()


def _struct_fields(header, name):
    m = re.search(r"typedef struct %s \{(.*?)\} %s;" % (name, name), header, re.S)
    assert m, name
    body = re.sub(r"/\*.*?\*/", "", m.group(1), flags=re.S)
    fields = set()
    for decl in body.split(";"):
        decl = decl.strip()
        if not decl:
            continue
        for part in decl.split(","):
            w = re.findall(r"([A-Za-z_][A-Za-z0-9_]*)\s*(?:\[[^\]]*\])?\s*$", part.strip())
            if w:
                fields.add(w[-1])
    return fields


def test_shim_names_exist_in_header_and_library():
    go, hdr = _read(GO), _read(os.path.join(ROOT, "include", "gossip.h"))
    funcs = set(re.findall(r"\bC\.(gs_[a-z0-9_]+)\s*\(", go))
    assert {"gs_create", "gs_create_multi", "gs_create_rank", "gs_comm_unique_id", "gs_build_overlay",
            "gs_broadcast_begin", "gs_step", "gs_totals", "gs_run", "gs_trial_results"} <= funcs
    declared = set(re.findall(r"\b(gs_[a-z0-9_]+)\s*\(", hdr))
    assert funcs <= declared, funcs - declared
    consts = set(re.findall(r"\bC\.(GS_[A-Z0-9_]+)", go))
    for c in consts:
        assert re.search(r"#define %s\b|\b%s\s*=" % (c, c), hdr), c
    from gossip_simulator_amd import _lib
    lib = _lib.load()
    for f in funcs:
        assert hasattr(lib, f), f


def test_shim_struct_fields_exist():
    go, hdr = _read(GO), _read(os.path.join(ROOT, "include", "gossip.h"))
    params = _struct_fields(hdr, "gs_params")
    used = set(re.findall(r"\b([a-z_]+):\s*C\.", go)) | set(re.findall(r"\bp\.([a-z_]+)\s*=", go))
    assert used and used <= params, used - params
    stats = _struct_fields(hdr, "gs_tick_stats")
    assert set(re.findall(r"\btot\.([a-z_]+)", go)) <= stats
    win = _struct_fields(hdr, "gs_window")
    assert set(re.findall(r"\bw\.([a-z_]+)", go)) <= win


def test_shim_uses_reference_flag_globals():
    go = _read(GO)
    for g in ("N", "Fanout", "Fanin", "DelayLow", "DelayHigh", "DropRate", "CrashRate"):
        assert re.search(r"\b%s\b" % g, go), g
    assert "package main" in go and "//go:build hip" in go
