"""Summarise a rocprofv3 run (rocpd SQLite .db or kernel_stats.csv) per kernel:
calls, total ms, average us, share.  Usage: python tools_profsummary.py <db|csv> [top]"""
import csv
import re
import sqlite3
import sys


def short(n):
    n = n.replace("(anonymous namespace)::", "").replace("void ", "")
    if "rocprim" in n:
        k = re.findall(r"detail::(\w+?)(?:<|\()", n)
        return "rocprim::" + (k[0] if k else "?")
    n = re.sub(r"\(.*", "", n)
    n = re.sub(r"<.*", "", n)
    return n[-56:]


def rows_of(path):
    if path.endswith(".db"):
        db = sqlite3.connect(path)
        q = "select name, count(*), sum(end-start) from kernels group by name"
        return [(short(n), c, float(s)) for n, c, s in db.execute(q)]
    return [(short(r["Name"]), int(r["Calls"]), float(r["TotalDurationNs"]))
            for r in csv.DictReader(open(path))]


def main():
    agg = {}
    for n, c, s in rows_of(sys.argv[1]):
        a = agg.setdefault(n, [0, 0.0])
        a[0] += c
        a[1] += s
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 25
    tot = sum(v[1] for v in agg.values())
    print(f"{'kernel':56s} {'calls':>7s} {'total':>11s} {'avg':>11s} {'share':>6s}")
    for n, (c, s) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
        print(f"{n:56s} {c:7d} {s / 1e6:8.3f} ms {s / c / 1e3:8.2f} us {100 * s / tot:5.1f}%")
    print(f"{'TOTAL':56s} {sum(v[0] for v in agg.values()):7d} {tot / 1e6:8.3f} ms")


if __name__ == "__main__":
    main()
