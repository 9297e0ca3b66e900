"""bench.py's extension-leg deadline (CPU): a leg that blocks -- as a
multi-rank collective would, waiting on a failed peer -- must not swallow the
headline line.  The watchdog prints the line once, marks the unfinished leg and
exits the process with status 3 (bench.DEADLINE_EXIT): the line is printed,
but the run is reported as not finished."""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = r"""
import sys, time
sys.path.insert(0, ROOT)
import bench
out = bench.Emitter(0)
ext = {"done_leg": {"value": 1}}
out.line = {"metric": "m", "value": 2.0, "extensions": ext}
out.arm(0.5, ext)
bench.guarded("stuck_leg", lambda: time.sleep(30))
out.disarm()
out.emit()
print("NOT REACHED", flush=True)
"""


def test_deadline_prints_line_once_and_exits():
    t0 = time.time()
    r = subprocess.run([sys.executable, "-c", "ROOT = %r\n" % ROOT + SCRIPT], capture_output=True, text=True,
                       timeout=60)
    assert r.returncode == 3, (r.returncode, r.stderr)
    assert time.time() - t0 < 20
    lines = [l for l in r.stdout.splitlines() if l.strip()]
    assert len(lines) == 1 and "NOT REACHED" not in r.stdout
    d = json.loads(lines[0])
    assert d["value"] == 2.0 and d["extensions"]["done_leg"] == {"value": 1}
    assert "deadline" in d["extensions"]["stuck_leg"]["error"]


def test_no_deadline_prints_once():
    script = SCRIPT.replace("time.sleep(30)", "{'value': 3}").replace('print("NOT REACHED", flush=True)', "")
    r = subprocess.run([sys.executable, "-c", "ROOT = %r\n" % ROOT + script], capture_output=True, text=True,
                       timeout=60)
    assert r.returncode == 0, r.stderr
    lines = [l for l in r.stdout.splitlines() if l.strip()]
    assert len(lines) == 1
    assert json.loads(lines[0])["extensions"] == {"done_leg": {"value": 1}}
