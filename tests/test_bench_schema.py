"""bench.py's line carries BASELINE.json's 8-GPU target as measured: a
top-level `strong_scaling` block (ONE N = 1e9 broadcast sharded over the
GPUs, total work fixed) beside the weak-scaling headline `value` (verdict r04,
item 4).  CPU-only: the block is assembled by a pure function from the
headline and the extension legs."""
from __future__ import annotations

import importlib.util
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


LINE = {"value": 8.4e10, "unit": "msgs/s", "ms_per_step": 57.9, "scaling": "weak",
        "config": {"status": "quiescent"}, "roofline": {"broadcast_device_ms": 56.3}}


def test_one_gpu_block_is_the_headline_and_the_unsharded_pushpull():
    b = _bench().strong_scaling_block(1, LINE, {"pushpull": {"value": 9.7e10, "unit": "msgs/s",
                                                             "ms_per_step": 116.6, "rounds_to_99": 40,
                                                             "status": "covered"}})
    assert b["scaling"] == "strong" and b["n_gpus"] == 1
    assert b["flood"]["value"] == LINE["value"] and b["flood"]["ms_per_step"] == 57.9
    assert b["flood"]["device_ms_per_rank"] == [56.3]
    assert b["pushpull"]["ms_per_step"] == 116.6 and b["pushpull"]["rounds_to_99"] == 40


def test_eight_gpu_block_is_the_sharded_single_run_with_every_rank():
    ext = {"c5_flood_sharded": {"value": 4e11, "unit": "msgs/s", "ms_per_step": 12.2, "device_ms_per_step": 9.9,
                                "device_ms_per_rank": [9.9, 10.1, 9.8, 10.0, 9.7, 10.2, 9.9, 10.0],
                                "wall_over_device": 1.23, "status": "quiescent", "shards": 8},
           "c5_pushpull_sharded": {"value": 3e11, "unit": "msgs/s", "ms_per_step": 38.0, "rounds_to_99": 40,
                                   "status": "covered", "placement": "ranks"}}
    b = _bench().strong_scaling_block(8, LINE, ext)
    assert b["n_gpus"] == 8 and b["scaling"] == "strong"
    assert len(b["flood"]["device_ms_per_rank"]) == 8
    assert b["flood"]["ms_per_step"] == 12.2 and b["flood"]["wall_over_device"] == 1.23
    assert b["pushpull"]["placement"] == "ranks"
    # the weak-scaling headline is not touched
    assert LINE["scaling"] == "weak"


def test_a_failed_leg_is_reported_not_hidden():
    b = _bench().strong_scaling_block(8, LINE, {"c5_flood_sharded": {"error": "RuntimeError: boom"}})
    assert b["flood"] == {"error": "RuntimeError: boom"} and b["pushpull"] == {}


def test_main_puts_the_block_in_the_line():
    src = open(os.path.join(ROOT, "bench.py")).read()
    assert 'out.line["strong_scaling"] = strong_scaling_block(world, out.line, ext)' in src
    assert '"device_ms_per_rank": per_rank' in src
