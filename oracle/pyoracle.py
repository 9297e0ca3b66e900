"""ctypes binding of the CPU restatement (oracle/gsoracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py, always as the checker -- never by the product
package.  Parity with the reference is unpinned by reference artefacts (see
gsoracle.h); the pins are the hand-derived known answers under tests/.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "libgsoracle.so")
_OMP_PATH = os.path.join(_HERE, "_build", "libgsomp.so")
OR_EOVERFLOW = -6  # gsoracle.h: > 65535 arrivals at one node in one tick


def build() -> str:
    """Compile the restatement (gcc) into oracle/_build/."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


class Params(C.Structure):
    _fields_ = [
        ("n", C.c_uint64),
        ("fanout", C.c_int32),
        ("fanin", C.c_int32),
        ("delay_low", C.c_int32),
        ("delay_high", C.c_int32),
        ("drop_rate", C.c_double),
        ("crash_rate", C.c_double),
        ("seed", C.c_uint64),
        ("trial", C.c_uint32),
        ("model", C.c_uint32),  # 0 flood (reference), 1 push-pull (extension)
    ]


class TickStats(C.Structure):
    _fields_ = [(f, C.c_uint64) for f in
                ("tick", "fired", "sent", "messages", "received", "crashed", "pending")]


class Window(C.Structure):
    _fields_ = [(f, C.c_uint64) for f in ("tick", "makeups", "breakups")]


class RefsimResult(C.Structure):
    _fields_ = [(f, C.c_uint64) for f in
                ("tick_99", "poll_99", "messages", "crashed", "received", "sent",
                 "overlay_ticks")] + [
        ("deg_hist", C.c_uint64 * 256),
        ("reached", C.c_int32),
        ("pad_", C.c_int32),
    ]


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = C.CDLL(_LIB_PATH)
        P = C.POINTER
        L.or_threshold.argtypes = [C.c_double]
        L.or_threshold.restype = C.c_int32
        L.or_philox.argtypes = [P(C.c_uint32), P(C.c_uint32), P(C.c_uint32)]
        L.or_uniform.argtypes = [C.c_uint32, C.c_uint32]
        L.or_uniform.restype = C.c_uint32
        L.or_drop_crash.argtypes = [C.c_uint32, P(C.c_uint32), P(C.c_uint32)]
        L.or_first_crash.argtypes = [P(C.c_uint32), C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32,
                                     C.c_uint32]
        L.or_first_crash.restype = C.c_uint32
        L.or_pick_sender.argtypes = [P(Params)]
        L.or_pick_sender.restype = C.c_uint64
        L.or_overlay.argtypes = [P(Params), C.c_void_p, C.c_void_p, P(Window), C.c_size_t,
                                 P(C.c_size_t), C.c_uint64, P(C.c_uint64)]
        L.or_engine_new.argtypes = [P(Params), C.c_void_p, C.c_void_p, C.c_uint32]
        L.or_engine_new.restype = C.c_void_p
        L.or_engine_free.argtypes = [C.c_void_p]
        L.or_engine_begin.argtypes = [C.c_void_p, C.c_int64]
        L.or_engine_step.argtypes = [C.c_void_p, C.c_uint32, P(TickStats)]
        L.or_engine_read_received.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t]
        L.or_engine_read_crashed.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t]
        L.or_engine_set_failed.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t]
        L.or_engine_tick.argtypes = [C.c_void_p]
        L.or_engine_tick.restype = C.c_uint64
        L.or_engine_set_range.argtypes = [C.c_void_p, C.c_uint64, C.c_uint64]
        L.or_engine_get_slot.argtypes = [C.c_void_p, C.c_uint64, C.c_void_p, C.c_size_t]
        L.or_engine_set_slot.argtypes = [C.c_void_p, C.c_uint64, C.c_void_p, C.c_size_t]
        L.or_refsim.argtypes = [P(Params), C.c_uint64, C.c_uint64, P(RefsimResult)]
        L.or_refsim_broadcast.argtypes = [P(Params), C.c_void_p, C.c_void_p, C.c_uint32,
                                          C.c_uint64, C.c_uint64, P(RefsimResult)]
        _lib = L
    return _lib


MODEL_FLOOD, MODEL_PUSHPULL = 0, 1


def make_params(n=50000, fanout=5, fanin=6, delay_low=10, delay_high=20,
                drop_rate=0.1, crash_rate=0.001, seed=0x5EED, trial=0, model=0) -> Params:
    return Params(n, fanout, fanin, delay_low, delay_high, drop_rate, crash_rate,
                  seed, trial, model)


def threshold(rate: float) -> int:
    return lib().or_threshold(rate)


def first_crash(key, trial, u, t, k, ones):
    """Rule A6's keyed first-crash position (gsoracle.h or_first_crash)."""
    kk = (C.c_uint32 * 2)(*[int(x) & 0xFFFFFFFF for x in key])
    return int(lib().or_first_crash(kk, trial, u, t, k, ones))


def philox(ctr, key):
    c = (C.c_uint32 * 4)(*[int(x) & 0xFFFFFFFF for x in ctr])
    k = (C.c_uint32 * 2)(*[int(x) & 0xFFFFFFFF for x in key])
    o = (C.c_uint32 * 4)()
    lib().or_philox(c, k, o)
    return [int(x) for x in o]


def pick_sender(p: Params) -> int:
    return int(lib().or_pick_sender(C.byref(p)))


class OverlayError(RuntimeError):
    pass


def overlay(p: Params, max_ticks: int = 1_000_000, wcap: int = 100000):
    """Tick-model overlay.  Returns (deg u8[n], ids u32[n, stride], windows, final_tick)."""
    stride = max(p.fanout, p.fanin, 1)
    deg = np.zeros(p.n, dtype=np.uint8)
    ids = np.zeros((p.n, stride), dtype=np.uint32)
    win = (Window * wcap)()
    nwin = C.c_size_t(0)
    ft = C.c_uint64(0)
    rc = lib().or_overlay(C.byref(p), deg.ctypes.data, ids.ctypes.data, win, wcap,
                          C.byref(nwin), max_ticks, C.byref(ft))
    if rc != 0:
        raise OverlayError(f"or_overlay failed: {rc}")
    ws = [(win[i].tick, win[i].makeups, win[i].breakups) for i in range(min(nwin.value, wcap))]
    return deg, ids, ws, int(ft.value)


class Engine:
    """Tick-model broadcast engine (bit-exact spec of the HIP engine)."""

    def __init__(self, p: Params, deg: np.ndarray, ids: np.ndarray):
        self.p = p
        self.n = int(p.n)
        self.W = (self.n + 63) // 64
        deg = np.ascontiguousarray(deg, dtype=np.uint8)
        ids = np.ascontiguousarray(ids, dtype=np.uint32)
        self.stride = ids.shape[1]
        self._keep = (deg, ids)
        self.h = lib().or_engine_new(C.byref(p), deg.ctypes.data, ids.ctypes.data, self.stride)
        if not self.h:
            raise ValueError("or_engine_new rejected the parameters/table")

    def __del__(self):
        if getattr(self, "h", None):
            lib().or_engine_free(self.h)
            self.h = None

    def begin(self, sender: int = -1):
        if lib().or_engine_begin(self.h, sender) != 0:
            raise ValueError("or_engine_begin failed")

    def set_failed(self, words: np.ndarray):
        words = np.ascontiguousarray(words, dtype=np.uint64)
        if lib().or_engine_set_failed(self.h, words.ctypes.data, words.size) != 0:
            raise ValueError("or_engine_set_failed failed")

    def step(self, ticks: int = 1) -> np.ndarray:
        out = (TickStats * ticks)()
        rc = lib().or_engine_step(self.h, ticks, out)
        if rc == OR_EOVERFLOW:
            raise OverflowError("or_engine_step: more than 65535 arrivals at one node in one tick")
        if rc != 0:
            raise RuntimeError("or_engine_step failed")
        return np.array([[out[i].tick, out[i].fired, out[i].sent, out[i].messages,
                          out[i].received, out[i].crashed, out[i].pending]
                         for i in range(ticks)], dtype=np.uint64).reshape(ticks, 7)

    def received(self) -> np.ndarray:
        w = np.zeros(self.W, dtype=np.uint64)
        lib().or_engine_read_received(self.h, w.ctypes.data, self.W)
        return w

    def crashed(self) -> np.ndarray:
        w = np.zeros(self.W, dtype=np.uint64)
        lib().or_engine_read_crashed(self.h, w.ctypes.data, self.W)
        return w

    @property
    def tick(self) -> int:
        return int(lib().or_engine_tick(self.h))

    def set_range(self, lo: int, hi: int):
        if lib().or_engine_set_range(self.h, lo, hi) != 0:
            raise ValueError("or_engine_set_range failed")

    def get_slot(self, tick: int) -> np.ndarray:
        w = np.zeros(self.W, dtype=np.uint64)
        lib().or_engine_get_slot(self.h, tick, w.ctypes.data, self.W)
        return w

    def set_slot(self, tick: int, words: np.ndarray):
        words = np.ascontiguousarray(words, dtype=np.uint64)
        if lib().or_engine_set_slot(self.h, tick, words.ctypes.data, words.size) != 0:
            raise ValueError("or_engine_set_slot failed")


STAT_FIELDS = ("tick", "fired", "sent", "messages", "received", "crashed", "pending")

_omp = None


def omp_lib():
    """The all-core OpenMP port (gsomp.c): bench.py's cpu_baseline."""
    global _omp
    if _omp is None:
        if not os.path.exists(_OMP_PATH):
            build()
        L = C.CDLL(_OMP_PATH)
        P = C.POINTER
        L.om_engine_new.argtypes = [P(Params), C.c_void_p, C.c_void_p, C.c_uint32, C.c_int]
        L.om_engine_new.restype = C.c_void_p
        L.om_engine_free.argtypes = [C.c_void_p]
        L.om_engine_begin.argtypes = [C.c_void_p, C.c_int64]
        L.om_engine_step.argtypes = [C.c_void_p, C.c_uint32, P(TickStats)]
        L.om_engine_read_received.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t]
        L.om_engine_read_crashed.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t]
        L.om_engine_set_failed.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t]
        L.om_threads.argtypes = [C.c_void_p]
        L.om_threads.restype = C.c_int
        _omp = L
    return _omp


class OmpEngine:
    """The tick engine on every core (gsomp.c); same results as Engine."""

    def __init__(self, p: Params, deg: np.ndarray, ids: np.ndarray, threads: int = 0):
        self.p = p
        self.n = int(p.n)
        self.W = (self.n + 63) // 64
        deg = np.ascontiguousarray(deg, dtype=np.uint8)
        ids = np.ascontiguousarray(ids, dtype=np.uint32)
        self.h = omp_lib().om_engine_new(C.byref(p), deg.ctypes.data, ids.ctypes.data, ids.shape[1], threads)
        if not self.h:
            raise ValueError("om_engine_new rejected the parameters/table")
        self.threads = int(omp_lib().om_threads(self.h))

    def __del__(self):
        if getattr(self, "h", None):
            omp_lib().om_engine_free(self.h)
            self.h = None

    def begin(self, sender: int = -1):
        if omp_lib().om_engine_begin(self.h, sender) != 0:
            raise ValueError("om_engine_begin failed")

    def set_failed(self, words: np.ndarray):
        words = np.ascontiguousarray(words, dtype=np.uint64)
        if omp_lib().om_engine_set_failed(self.h, words.ctypes.data, words.size) != 0:
            raise ValueError("om_engine_set_failed failed")

    def step(self, ticks: int = 1) -> np.ndarray:
        out = (TickStats * ticks)()
        rc = omp_lib().om_engine_step(self.h, ticks, out)
        if rc == OR_EOVERFLOW:
            raise OverflowError("om_engine_step: more than 65535 arrivals at one node in one tick")
        if rc != 0:
            raise RuntimeError("om_engine_step failed")
        return np.array([[out[i].tick, out[i].fired, out[i].sent, out[i].messages,
                          out[i].received, out[i].crashed, out[i].pending]
                         for i in range(ticks)], dtype=np.uint64).reshape(ticks, 7)

    def received(self) -> np.ndarray:
        w = np.zeros(self.W, dtype=np.uint64)
        omp_lib().om_engine_read_received(self.h, w.ctypes.data, self.W)
        return w

    def crashed(self) -> np.ndarray:
        w = np.zeros(self.W, dtype=np.uint64)
        omp_lib().om_engine_read_crashed(self.h, w.ctypes.data, self.W)
        return w


def covered(recv: int, n: int) -> bool:
    """simulator.go:246-248 in float32."""
    return bool(np.float32(recv) / np.float32(n) >= np.float32(0.99))


def run_to_coverage(p: Params, deg, ids, sender=-1, poll=10, max_ticks=100000,
                    failed=None):
    """Poll every `poll` ticks like simulator.go:243-251; returns (stats rows, engine)."""
    e = Engine(p, deg, ids)
    if failed is not None:
        e.set_failed(failed)
    e.begin(sender)
    rows = []
    r0 = int(sum(bin(int(x)).count("1") for x in e.received()))  # informed at begin (push-pull)
    while True:
        s = e.step(poll)
        rows.append(s)
        last = s[-1]
        if covered(int(last[4]), p.n) or int(last[6]) == 0 or int(last[0]) >= max_ticks:
            break
        # gs_run's push-pull stop: a poll informed nobody new and no call can
        # change the informed set any more
        if p.model == MODEL_PUSHPULL and int(last[4]) == r0 and \
                pp_stalled(p, deg, ids, e.received(), e.crashed()):
            break
        r0 = int(last[4])
    return np.concatenate(rows), e


def _bits(words, idx):
    return ((words[idx >> 6] >> (idx & 63).astype(np.uint64)) & np.uint64(1)).astype(bool)


def pp_stalled(p: Params, deg, ids, recv, failed) -> bool:
    """Push-pull quiescence: no live informed node has a live uninformed friend
    and no live uninformed node has an informed friend (or every call is lost)."""
    if threshold(p.drop_rate) >= 100:
        return True
    n = int(p.n)
    v = np.arange(n, dtype=np.int64)
    deg = np.asarray(deg, dtype=np.int64)
    ids = np.asarray(ids, dtype=np.int64)
    live = ~_bits(failed, v)
    iv = _bits(recv, v)
    slot = np.arange(ids.shape[1])[None, :] < deg[:, None]
    iu = _bits(recv, ids)
    fu = _bits(failed, ids)
    useful = np.where(iv[:, None], ~iu & ~fu, iu) & slot & live[:, None]
    return not useful.any()


def refsim(p: Params, rng_seed: int, max_ms: int = 10_000_000) -> RefsimResult:
    r = RefsimResult()
    rc = lib().or_refsim(C.byref(p), rng_seed, max_ms, C.byref(r))
    if rc != 0:
        raise RuntimeError(f"or_refsim failed: {rc}")
    return r


def refsim_broadcast(p: Params, deg, ids, rng_seed: int, max_ms: int = 10_000_000):
    deg = np.ascontiguousarray(deg, dtype=np.uint8)
    ids = np.ascontiguousarray(ids, dtype=np.uint32)
    r = RefsimResult()
    rc = lib().or_refsim_broadcast(C.byref(p), deg.ctypes.data, ids.ctypes.data,
                                   ids.shape[1], rng_seed, max_ms, C.byref(r))
    if rc != 0:
        raise RuntimeError(f"or_refsim_broadcast failed: {rc}")
    return r
