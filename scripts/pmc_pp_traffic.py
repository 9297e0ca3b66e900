"""HBM traffic of ONE C5 push-pull broadcast per kernel kind, from a PMC
summary (scripts/pmc_pp.sh -> summary.csv, every pass one broadcast of
scripts/pp_once.py).  Read bytes = the L2's memory read requests by size
(128 * RDREQ_128B + 64 * RDREQ_64B + 32 * RDREQ_32B: every read request was
128 B on gfx950 in the calibration, profiles/r03_fetch_calibration.json),
writes = WRITE_SIZE.  The algorithmic figure it is compared with is SURVEY.md
8(d)'s 8 B per delivered push-pull message (the messages come from the
pp_once log).  Usage: python scripts/pmc_pp_traffic.py <summary.csv> <out.json> <pp_once log>"""
import csv
import json
import re
import sys

ROUNDS = {"sparse early rounds": ("k_ppe_round", "k_ppe_commit"),
          "pull-answer rounds": ("k_ppa_round",),
          "bottom-up rounds": ("k_ppb_round",),
          "top-down rounds": ("k_pp_round",),
          "deferred-set partition + apply": ("k_ppd_part", "k_ppd_apply"),
          "summaries, commit, mode": ("k_pp_summary", "k_pp_summary2", "k_pp_commit", "k_pp_mode", "k_pp_count",
                                      "k_pp_live_edges", "k_pp_set_mode")}


def main():
    rows = {r["kernel"]: r for r in csv.DictReader(open(sys.argv[1]))}
    log = open(sys.argv[3]).read()
    m = re.search(r"rounds=(\d+) messages=(\d+) calls=(\d+)", log)
    rounds, msgs, calls = (int(m.group(1)), int(m.group(2)), int(m.group(3))) if m else (0, 0, 0)
    out = {"source": sys.argv[1], "unit": "bytes per broadcast", "rounds": rounds, "messages": msgs,
           "calls": calls, "kinds": {}, "kernels": {}}
    total = 0.0
    for kind, names in ROUNDS.items():
        rd = wr = 0.0
        disp = 0
        for k, r in rows.items():
            base = k.split("::")[-1]
            if not any(base == nm or base.startswith(nm + "_") for nm in names):
                continue
            g = lambda c: float(r.get(c, 0) or 0)  # noqa: E731
            req = 128 * g("TCC_EA0_RDREQ_128B_sum") + 64 * g("TCC_EA0_RDREQ_64B_sum") + 32 * g("TCC_EA0_RDREQ_32B_sum")
            read = req if req > 0 else 2048.0 * g("FETCH_SIZE")
            write = 1024.0 * g("WRITE_SIZE")
            out["kernels"][k] = {"read": read, "write": write, "dispatches": int(r["dispatches"])}
            rd += read
            wr += write
            disp += int(r["dispatches"])
        out["kinds"][kind] = {"read": rd, "write": wr, "dispatches": disp}
        total += rd + wr
    out["round_bytes"] = total
    out["algorithmic_bytes"] = 8 * msgs
    out["traffic_ratio"] = round(total / (8 * msgs), 3) if msgs else None
    json.dump(out, open(sys.argv[2], "w"), indent=1)
    print(json.dumps({k: out[k] for k in ("rounds", "messages", "round_bytes", "algorithmic_bytes",
                                          "traffic_ratio")}, indent=1))
    for kind, v in out["kinds"].items():
        print(f"{kind:32s} read {v['read'] / 1e9:8.2f} GB  write {v['write'] / 1e9:7.2f} GB  ({v['dispatches']} launches)")


if __name__ == "__main__":
    main()
