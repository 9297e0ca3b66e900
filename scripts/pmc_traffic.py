"""HBM traffic of the window pipeline (k_expand, k_part2, k_resolve_small,
k_resolve, k_resolve_rolled) from a PMC summary (scripts/pmc.sh ->
summary.csv over ONE broadcast: bench.py --steps 1 --warmup 0).

Read bytes, calibrated (profiles/r03_fetch_calibration.json, the known-byte
micro kernels of scripts/micro/fetch_calib.hip): on gfx950 every read request
the L2 sends to memory was a 128-B request (TCC_EA0_RDREQ_128B = RDREQ) for
every pattern measured -- coalesced streams, random 128-B lines, random 64-,
32-, 16- and 4-B accesses and k_expand's uint4 + uint2 row load -- while
FETCH_SIZE tallies 64 B per request.  So bytes read = 128 * RDREQ_128B +
64 * RDREQ_64B + 32 * RDREQ_32B when those counters were collected, else
2 * FETCH_SIZE (the same number for these patterns).  WRITE_SIZE matched the
known bytes of every write pattern (partial 32-B sectors count whole).
Infinity-Cache hits are counted as traffic.
Usage: python scripts/pmc_traffic.py <summary.csv> <out.json> [passes] [windows]
(passes: rocprofv3 runs in the summary, each over one broadcast; windows: the
broadcast's real windows; the device-driven loop also issues no-op launches
past the last window, which the dispatch count includes)"""
import csv
import json
import sys

KERNELS = ("gs::k_expand", "gs::k_part2", "gs::k_resolve_small", "gs::k_resolve", "gs::k_resolve_rolled")


def main():
    rows = {r["kernel"]: r for r in csv.DictReader(open(sys.argv[1]))}
    out = {"source": sys.argv[1], "calibration": "profiles/r03_fetch_calibration.json",
           "unit": "bytes per broadcast", "kernels": {}}
    total = 0.0
    for k in KERNELS:
        if k not in rows:
            continue
        r = rows[k]
        g = lambda c: float(r.get(c, 0) or 0)
        req = 128 * g("TCC_EA0_RDREQ_128B_sum") + 64 * g("TCC_EA0_RDREQ_64B_sum") + 32 * g("TCC_EA0_RDREQ_32B_sum")
        fetch2 = g("FETCH_SIZE") * 1024 * 2.0
        fetch = req if req > 0 else fetch2
        write = g("WRITE_SIZE") * 1024
        out["kernels"][k] = {"read": fetch, "read_from": "RDREQ sizes" if req > 0 else "2 x FETCH_SIZE",
                             "read_2xFETCH_SIZE": fetch2, "write": write,
                             "dram_read": 32 * g("TCC_EA0_RDREQ_DRAM_32B_sum"),
                             "dram_write": 32 * g("TCC_EA0_WRREQ_WRITE_DRAM_32B_sum")}
        total += fetch + write
    out["pipeline_bytes"] = total
    passes = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    out["launches"] = int(sys.argv[4]) if len(sys.argv) > 4 else int(rows["gs::k_resolve"]["dispatches"]) // passes
    out["bytes_per_launch"] = total / max(out["launches"], 1)
    json.dump(out, open(sys.argv[2], "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
