"""Counter bytes per known byte for each micro pattern of
scripts/micro/fetch_calib.hip (scripts/calib.sh).  For every kernel: the known
bytes it touches, and what each counter formula reports:
  FETCH_SIZE / WRITE_SIZE       rocprofv3's derived counters (KiB -> bytes)
  req_bytes                     32*RDREQ_32B + 64*RDREQ_64B + 128*RDREQ_128B
  dram_bytes                    32 * TCC_EA0_RDREQ_DRAM_32B (32-B units, DRAM only)
  wr_req_bytes                  64*WRREQ_64B + 32*(WRREQ - WRREQ_64B)
  wr_dram_bytes                 32 * TCC_EA0_WRREQ_WRITE_DRAM_32B
Usage: python scripts/calib_summary.py <plain.txt> <summary.csv>"""
import csv
import json
import sys


def main():
    known = {}
    for line in open(sys.argv[1]):
        if line.startswith("CALIB "):
            _, name, kb, acc, ms = line.split()
            known[name] = (float(kb), float(acc), float(ms))
    rows = {r["kernel"].split("::")[-1]: r for r in csv.DictReader(open(sys.argv[2]))}
    out = {}
    for name, (kb, acc, ms) in known.items():
        key = name if name in rows else None
        r = rows.get(key, {})
        g = lambda c: float(r.get(c, 0) or 0)
        d = {"known_bytes": kb, "accesses": acc, "ms": ms, "GBps_known": round(kb / ms / 1e6, 1),
             "dispatches_of_kernel": int(float(r.get("dispatches", 0) or 0))}
        if r:
            d["FETCH_SIZE"] = g("FETCH_SIZE") * 1024
            d["WRITE_SIZE"] = g("WRITE_SIZE") * 1024
            d["req_bytes"] = 32 * g("TCC_EA0_RDREQ_32B_sum") + 64 * g("TCC_EA0_RDREQ_64B_sum") + \
                128 * g("TCC_EA0_RDREQ_128B_sum")
            d["rdreq"] = g("TCC_EA0_RDREQ_sum")
            d["rdreq_32_64_128"] = [g("TCC_EA0_RDREQ_32B_sum"), g("TCC_EA0_RDREQ_64B_sum"), g("TCC_EA0_RDREQ_128B_sum")]
            d["bubble"] = g("TCC_BUBBLE_sum")
            d["dram_bytes"] = 32 * g("TCC_EA0_RDREQ_DRAM_32B_sum")
            d["wr_req_bytes"] = 64 * g("TCC_EA0_WRREQ_64B_sum") + 32 * (g("TCC_EA0_WRREQ_sum") - g("TCC_EA0_WRREQ_64B_sum"))
            d["wr_dram_bytes"] = 32 * g("TCC_EA0_WRREQ_WRITE_DRAM_32B_sum")
            for f in ("FETCH_SIZE", "req_bytes", "dram_bytes", "WRITE_SIZE", "wr_req_bytes", "wr_dram_bytes"):
                d[f + "_per_access"] = round(d[f] / acc, 2) if acc else None
        out[name] = d
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
