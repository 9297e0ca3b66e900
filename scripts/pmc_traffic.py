"""HBM traffic of the window pipeline (k_expand, k_part2, k_resolve_small, k_resolve) from a PMC summary (scripts/pmc.sh ->
summary.csv over ONE broadcast: bench.py --steps 1 --warmup 0).

rocprofv3 reports FETCH_SIZE / WRITE_SIZE in KiB.  MI355X_MICROARCH.md (HBM
section): on gfx950 FETCH_SIZE counts 64 B per 128-B read request, i.e. half
the bytes of a coalesced streaming read, so FETCH_SIZE is doubled here;
WRITE_SIZE is taken as is.  Infinity-Cache hits are counted as traffic.
Usage: python scripts/pmc_traffic.py <summary.csv> <out.json> [passes=5] [windows]
(windows: the broadcast's real windows; the device-driven loop also issues
no-op launches past the last window, which the dispatch count includes)"""
import csv
import json
import sys

KERNELS = ("gs::k_expand", "gs::k_part2", "gs::k_resolve_small", "gs::k_resolve", "gs::k_resolve_rolled")


def main():
    rows = {r["kernel"]: r for r in csv.DictReader(open(sys.argv[1]))}
    out = {"source": sys.argv[1], "fetch_correction": 2.0, "unit": "bytes per broadcast",
           "kernels": {}}
    total = 0.0
    for k in KERNELS:
        if k not in rows:
            continue
        r = rows[k]
        fetch = float(r["FETCH_SIZE"]) * 1024 * 2.0
        write = float(r["WRITE_SIZE"]) * 1024
        out["kernels"][k] = {"fetch": fetch, "write": write}
        total += fetch + write
    out["pipeline_bytes"] = total
    # pmc.sh makes one rocprofv3 pass per counter group over the same broadcast
    passes = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    out["launches"] = int(sys.argv[4]) if len(sys.argv) > 4 else int(rows["gs::k_resolve"]["dispatches"]) // passes
    out["bytes_per_launch"] = total / max(out["launches"], 1)
    json.dump(out, open(sys.argv[2], "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
