"""Python host API over the C ABI: the operator-level mirror of simulator.go.

`Simulator` keeps the reference's parameter names (simulator.go:11-20,
186-193) and phases: `build_overlay()` = main :214-235, `broadcast_begin()` =
:239-241, `step()` / `run()` = the receive/broadcast actors plus the poll loop
:243-251.  All compute runs in libgossip_hip.so on a gfx950 device.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field

import numpy as np

from . import _lib
from ._lib import GossipError, Params, TickStats, Timing, TrialStats, Window

STAT_FIELDS = ("tick", "fired", "sent", "messages", "received", "crashed", "pending")
TRIAL_FIELDS = ("trial", "tick_99", "tick", "fired", "sent", "messages", "received", "crashed",
                "status")


@dataclass
class Config:
    """The reference's flags (simulator.go:187-193) plus additive knobs."""
    n: int = 50000
    fanout: int = 5
    fanin: int = 6          # Fanout+1 evaluated before Parse -> always 6 (:189)
    delaylow: int = 10
    delayhigh: int = 20
    droprate: float = 0.1
    crashrate: float = 0.001
    seed: int = 1
    trial: int = 0
    device: int = 0
    timing: bool = False
    engine: str = "window"  # "window" (default) or "tick" (per-tick atomic engine)
    model: str = "flood"    # "flood" (the reference) or "pushpull" (extension)
    trials: int = 1         # batched independent trials trial .. trial+trials-1 (config C3)
    pp_l2_only: bool = False  # push-pull: force the no-LDS summary path (tests)
    pp_rounds: str = "auto"   # push-pull: "auto" (sparse early rounds while |I| <= n/256, dense
                              # rounds bottom-up once |I| >= 96n/256), "dense" (every round streams the
                              # table top-down), "early" (sparse at any |I|), "topdown" (auto, but
                              # dense rounds never bottom-up nor pull-answer), "bottom" (every dense round
                              # bottom-up), "answer" (every dense round below the bottom-up threshold
                              # pull-answer)

    PP_ROUNDS = ("auto", "dense", "early", "topdown", "bottom", "answer")

    def flags(self, timing: bool | None = None) -> int:
        if self.pp_rounds not in self.PP_ROUNDS:
            raise ValueError(f"pp_rounds must be one of {self.PP_ROUNDS}, not {self.pp_rounds!r}")
        t = self.timing if timing is None else timing
        return (_lib.GS_FLAG_TIMING if t else 0) | \
            (_lib.GS_FLAG_TICK_ENGINE if self.engine == "tick" else 0) | \
            (_lib.GS_FLAG_PP_L2_ONLY if self.pp_l2_only else 0) | \
            (_lib.GS_FLAG_PP_DENSE if self.pp_rounds == "dense" else 0) | \
            (_lib.GS_FLAG_PP_EARLY if self.pp_rounds == "early" else 0) | \
            (_lib.GS_FLAG_PP_TOPDOWN if self.pp_rounds == "topdown" else 0) | \
            (_lib.GS_FLAG_PP_BOTTOM if self.pp_rounds == "bottom" else 0) | \
            (_lib.GS_FLAG_PP_ANSWER if self.pp_rounds == "answer" else 0)

    def to_params(self) -> Params:
        p = Params()
        p.n, p.fanout, p.fanin = self.n, self.fanout, self.fanin
        p.delay_low, p.delay_high = self.delaylow, self.delayhigh
        p.drop_rate, p.crash_rate = self.droprate, self.crashrate
        p.seed, p.trial, p.device = self.seed, self.trial, self.device
        if self.model not in ("flood", "pushpull"):
            raise ValueError(f"model must be 'flood' or 'pushpull', not {self.model!r}")
        p.model = _lib.GS_MODEL_PUSHPULL if self.model == "pushpull" else _lib.GS_MODEL_FLOOD
        p.flags = self.flags()
        p.trials = max(1, int(self.trials))
        return p


def _stats_array(buf, k: int) -> np.ndarray:
    return np.array([[getattr(buf[i], f) for f in STAT_FIELDS] for i in range(k)],
                    dtype=np.uint64).reshape(k, len(STAT_FIELDS))


class Simulator:
    """One broadcast (or one batch of trials) behind a gs_ctx.

    devices=None: one GPU (cfg.device), gs_create.  devices=[d0, d1, ...]:
    gs_create_multi -- a node-range-sharded broadcast over those devices
    (entries may repeat), or the trials split over them when cfg.trials > 1.
    Simulator.rank(...): one rank of a multi-process run (gs_create_rank)."""

    def __init__(self, cfg: Config, devices=None, _rank=None):
        self.cfg = cfg
        self.L = _lib.load()
        self._p = cfg.to_params()
        h = C.c_void_p()
        if _rank is not None and len(_rank) == 5:  # host exchange: (nranks, rank, all_gather, all_reduce, all_to_allv)
            nranks, rank, ag, ar, av = _rank
            self._xfns = self._exchange_fns(nranks, ag, ar, av)  # kept alive with the context
            rc = self.L.gs_create_rank_exchange(C.byref(self._p), cfg.device, nranks, rank,
                                                C.byref(self._xfns[-1]), C.byref(h))
            what = "gs_create_rank_exchange"
        elif _rank is not None:
            nranks, rank, cid = _rank
            rc = self.L.gs_create_rank(C.byref(self._p), cfg.device, nranks, rank, cid, C.byref(h))
            what = "gs_create_rank"
        elif devices is not None:
            devs = (C.c_int * len(devices))(*[int(d) for d in devices])
            rc = self.L.gs_create_multi(C.byref(self._p), devs, len(devices), C.byref(h))
            what = "gs_create_multi"
        else:
            rc = self.L.gs_create(C.byref(self._p), C.byref(h))
            what = "gs_create"
        if rc != 0:
            raise GossipError(rc, f"{what} failed: {self.L.gs_strerror(rc).decode()}")
        self.h = h
        self.n = cfg.n
        self.trials = max(1, int(cfg.trials))
        self.words = (cfg.n + 63) // 64

    @classmethod
    def rank(cls, cfg: Config, nranks: int, rank: int, comm_id: bytes | None):
        """Rank `rank` of `nranks` processes (gs_create_rank); comm_id from
        comm_unique_id() on rank 0, shipped to every rank by the caller.  With
        cfg.trials > 1 the rank gets its share of the trials (no comm_id)."""
        sim = cls(cfg, _rank=(nranks, rank, comm_id))
        if cfg.trials > 1:  # this rank's trials
            t0 = cfg.trials * rank // nranks
            sim.trials = cfg.trials * (rank + 1) // nranks - t0
        return sim

    @classmethod
    def rank_exchange(cls, cfg: Config, nranks: int, rank: int, all_gather, all_reduce_sum, all_to_allv=None):
        """Rank `rank` of `nranks` processes with the exchange done by the caller
        (gs_create_rank_exchange): all_gather(send: np.uint8 array) -> np.uint8
        array of nranks * len(send) bytes, rank-major; all_reduce_sum(x:
        np.uint64 array) -> the element-wise sum over the ranks;
        all_to_allv(send: np.uint8 array, send_sizes, recv_sizes) -> np.uint8
        array of sum(recv_sizes) bytes (blocks back to back in rank order; a
        flood run needs it)."""
        return cls(cfg, _rank=(nranks, rank, all_gather, all_reduce_sum, all_to_allv))

    @staticmethod
    def _exchange_fns(nranks, all_gather, all_reduce_sum, all_to_allv):
        def ag(_user, send, recv, nbytes):
            try:
                src = np.ctypeslib.as_array((C.c_uint8 * nbytes).from_address(send))
                out = np.asarray(all_gather(src.copy()), dtype=np.uint8).ravel()
                C.memmove(recv, out.ctypes.data, out.nbytes)
                return 0
            except Exception:  # noqa: BLE001 -- reported to the engine as a failed exchange
                import traceback
                traceback.print_exc()
                return 1

        def ar(_user, buf, count):
            try:
                x = np.ctypeslib.as_array(buf, shape=(count,))
                x[:] = np.asarray(all_reduce_sum(x.copy()), dtype=np.uint64)
                return 0
            except Exception:  # noqa: BLE001
                import traceback
                traceback.print_exc()
                return 1

        def av(_user, send, send_bytes, recv, recv_bytes):
            try:
                sb = [int(send_bytes[i]) for i in range(nranks)]
                rb = [int(recv_bytes[i]) for i in range(nranks)]
                src = np.ctypeslib.as_array((C.c_uint8 * sum(sb)).from_address(send)) if sum(sb) else \
                    np.zeros(0, np.uint8)
                out = np.asarray(all_to_allv(src.copy(), sb, rb), dtype=np.uint8).ravel()
                if out.nbytes != sum(rb):
                    raise ValueError(f"all_to_allv returned {out.nbytes} bytes, expected {sum(rb)}")
                if out.nbytes:
                    C.memmove(recv, out.ctypes.data, out.nbytes)
                return 0
            except Exception:  # noqa: BLE001
                import traceback
                traceback.print_exc()
                return 1

        f1, f2 = _lib.ALL_GATHER_FN(ag), _lib.ALL_REDUCE_FN(ar)
        f3 = _lib.ALL_TO_ALLV_FN(av) if all_to_allv is not None else _lib.ALL_TO_ALLV_FN()
        return f1, f2, f3, _lib.Exchange(None, f1, f2, f3)

    # -- plumbing --------------------------------------------------------
    def _check(self, rc: int, what: str):
        if rc != 0:
            msg = self.L.gs_last_error(self.h).decode(errors="replace")
            raise GossipError(rc, f"{what}: {msg}")

    def close(self):
        if getattr(self, "h", None):
            self.L.gs_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    # -- overlay (simulator.go:62-106, 127-164, 214-235) -------------------
    def load_peers(self, deg: np.ndarray, ids: np.ndarray):
        """deg [n], ids [n, stride]; batched trials: the trials' tables back to
        back (deg [trials*n], ids [trials*n, stride], ids local to the trial)."""
        deg = np.ascontiguousarray(deg, dtype=np.uint8)
        ids = np.ascontiguousarray(ids, dtype=np.uint32)
        m = self.n * self.trials
        if deg.shape != (m,) or ids.ndim != 2 or ids.shape[0] != m:
            raise ValueError("deg must be [trials*n], ids [trials*n, stride]")
        self._check(self.L.gs_load_peers(self.h, deg.ctypes.data, ids.ctypes.data, ids.shape[1]),
                    "gs_load_peers")

    def load_peers_device(self, deg_ptr: int, ids_ptr: int, stride: int):
        self._check(self.L.gs_load_peers_device(self.h, deg_ptr, ids_ptr, stride),
                    "gs_load_peers_device")

    def build_overlay(self, max_ticks: int = 10_000_000, wcap: int = 1 << 16):
        win = (Window * wcap)()
        nwin = C.c_size_t(0)
        ft = C.c_uint64(0)
        self._check(self.L.gs_build_overlay(self.h, max_ticks, win, wcap, C.byref(nwin),
                                            C.byref(ft)), "gs_build_overlay")
        ws = [(win[i].tick, win[i].makeups, win[i].breakups)
              for i in range(min(nwin.value, wcap))]
        return ws, int(ft.value)

    def read_peers(self):
        stride = C.c_uint32(0)
        self._check(self.L.gs_read_peers(self.h, None, None, C.byref(stride)), "gs_read_peers")
        deg = np.zeros(self.n * self.trials, dtype=np.uint8)
        ids = np.zeros((self.n * self.trials, stride.value), dtype=np.uint32)
        self._check(self.L.gs_read_peers(self.h, deg.ctypes.data, ids.ctypes.data, C.byref(stride)),
                    "gs_read_peers")
        return deg, ids

    def set_failed(self, words: np.ndarray):
        words = np.ascontiguousarray(words, dtype=np.uint64)
        self._check(self.L.gs_set_failed(self.h, words.ctypes.data, words.size), "gs_set_failed")

    # -- broadcast (simulator.go:107-123, 140-149, 237-253) ----------------
    def broadcast_begin(self, sender: int = -1):
        self._check(self.L.gs_broadcast_begin(self.h, sender), "gs_broadcast_begin")

    def step(self, ticks: int = 1) -> np.ndarray:
        buf = (TickStats * ticks)()
        self._check(self.L.gs_step(self.h, ticks, buf), "gs_step")
        return _stats_array(buf, ticks)

    def run(self, poll: int = 10, max_ticks: int = 10_000_000, cap: int = 1 << 16):
        buf = (TickStats * cap)()
        nout = C.c_size_t(0)
        status = C.c_int32(0)
        self._check(self.L.gs_run(self.h, poll, max_ticks, buf, cap, C.byref(nout),
                                  C.byref(status)), "gs_run")
        return _stats_array(buf, min(nout.value, cap)), int(status.value)

    def totals(self) -> dict:
        t = TickStats()
        self._check(self.L.gs_totals(self.h, C.byref(t)), "gs_totals")
        return {f: int(getattr(t, f)) for f in STAT_FIELDS}

    def received(self) -> np.ndarray:
        """ceil(n/64) words (batched trials: [trials, ceil(n/64)])."""
        w = np.zeros(self.words * self.trials, dtype=np.uint64)
        self._check(self.L.gs_read_received(self.h, w.ctypes.data, w.size), "gs_read_received")
        return w if self.trials == 1 else w.reshape(self.trials, self.words)

    def crashed(self) -> np.ndarray:
        w = np.zeros(self.words * self.trials, dtype=np.uint64)
        self._check(self.L.gs_read_crashed(self.h, w.ctypes.data, w.size), "gs_read_crashed")
        return w if self.trials == 1 else w.reshape(self.trials, self.words)

    def trial_results(self) -> np.ndarray:
        """[trials, len(TRIAL_FIELDS)] int64: per trial its number, first
        covered tick, stopping poll's tick and counters there, and status."""
        buf = (TrialStats * self.trials)()
        k = C.c_size_t(0)
        self._check(self.L.gs_trial_results(self.h, buf, self.trials, C.byref(k)), "gs_trial_results")
        return np.array([[int(getattr(buf[i], f)) for f in TRIAL_FIELDS] for i in range(k.value)],
                        dtype=np.int64).reshape(k.value, len(TRIAL_FIELDS))

    def shard_info(self):
        """[(lo, hi)] node range of every shard."""
        ns = C.c_uint32(0)
        lo, hi = C.c_uint64(0), C.c_uint64(0)
        self._check(self.L.gs_shard_info(self.h, 0, C.byref(ns), C.byref(lo), C.byref(hi)), "gs_shard_info")
        out = []
        for i in range(ns.value):
            self._check(self.L.gs_shard_info(self.h, i, None, C.byref(lo), C.byref(hi)), "gs_shard_info")
            out.append((int(lo.value), int(hi.value)))
        return out

    def set_flags(self, timing: bool):
        flags = self.cfg.flags(timing)
        self._check(self.L.gs_set_flags(self.h, flags), "gs_set_flags")

    def reset(self):
        self._check(self.L.gs_reset(self.h), "gs_reset")

    def set_trial(self, trial: int):
        """Renumber the trial(s) (then build_overlay again), keeping the buffers."""
        self._check(self.L.gs_set_trial(self.h, trial), "gs_set_trial")
        self.cfg.trial = trial

    def set_stream(self, hip_stream: int | None):
        self._check(self.L.gs_set_stream(self.h, hip_stream), "gs_set_stream")

    def timing(self) -> dict:
        t = Timing()
        self._check(self.L.gs_timing_get(self.h, C.byref(t)), "gs_timing_get")
        return {f: getattr(t, f) for f, _ in Timing._fields_}

    def shard_timing(self, index: int) -> dict:
        """Kernel timing of shard `index` (GS_FLAG_TIMING)."""
        t = Timing()
        self._check(self.L.gs_shard_timing(self.h, index, C.byref(t)), "gs_shard_timing")
        return {f: getattr(t, f) for f, _ in Timing._fields_}


def comm_unique_id() -> bytes:
    """RCCL unique id for gs_create_rank (rank 0 makes it, every rank uses it)."""
    L = _lib.load()
    b = C.create_string_buffer(_lib.GS_COMM_ID_BYTES)
    rc = L.gs_comm_unique_id(b)
    if rc != 0:
        raise GossipError(rc, "gs_comm_unique_id failed")
    return b.raw


def trim(device: int = -1) -> int:
    """Return the library's free cached device blocks to the driver (gs_trim);
    returns the bytes released."""
    L = _lib.load()
    out = C.c_size_t(0)
    rc = L.gs_trim(int(device), C.byref(out))
    if rc != 0:
        raise GossipError(rc, "gs_trim failed")
    return int(out.value)


MEMORY_FIELDS = ("alloc_ms", "largest_alloc_ms", "free_ms", "alloc_calls", "alloc_cache_hits", "cached_bytes")


def memory_stats() -> dict:
    """The library's process-wide device-memory figures (gs_memory_stats)."""
    L = _lib.load()
    t = Timing()
    rc = L.gs_memory_stats(C.byref(t))
    if rc != 0:
        raise GossipError(rc, "gs_memory_stats failed")
    return {f: getattr(t, f) for f in MEMORY_FIELDS}


def covered(recv: int, n: int) -> bool:
    """simulator.go:246-248 in float32."""
    return bool(np.float32(recv) / np.float32(n) >= np.float32(0.99))
