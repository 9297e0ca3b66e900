"""gossip_simulator_amd -- MI355X-native engine for the broadcast round loop of
go-distributed/gossip_simulator (simulator.go).

Layers:
  include/gossip.h          C ABI (the drop-in seam; cgo binding in INTEGRATION.md)
  csrc/gs_broadcast.hip     tick kernels: delivery, infection, crash, stats
  csrc/gs_window.hip        window engine: expand, partition, resolve (default)
  csrc/gs_pushpull.hip      push-pull rounds (extension, config C5)
  csrc/gs_overlay.hip       overlay construction (makeup/breakup) on the GPU
  csrc/gs_api.cpp           C ABI implementation (device state, stream, polling)
  csrc/gs_devmem.cpp        process-wide cache of large device blocks (gs_trim)
  csrc/gossip_sim.cpp       CLI with the reference's flags and stdout
  engine.py                 Python host API (ctypes)
  peers.py                  injected peer-table file format
  dist.py                   multi-GPU sharding (trials; node ranges)
"""
from ._lib import (GS_RUN_COVERED, GS_RUN_MAX_TICKS, GS_RUN_QUIESCENT,  # noqa: F401
                   GossipError, load)
from .engine import Config, Simulator, covered, memory_stats, trim  # noqa: F401

__all__ = ["Config", "Simulator", "GossipError", "covered", "load", "trim", "memory_stats", "GS_RUN_COVERED",
           "GS_RUN_QUIESCENT", "GS_RUN_MAX_TICKS"]
