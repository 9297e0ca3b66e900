"""Aggregate rocprofv3 --pmc CSV output (counter_collection.csv) per kernel:
sum of every counter over that kernel's dispatches, plus dispatch count.
Usage: python scripts/pmc_summary.py <dir-with-pN-subdirs> > summary.csv"""
import csv
import glob
import os
import re
import sys
from collections import defaultdict


def short(n):
    n = n.replace("(anonymous namespace)::", "").replace("void ", "")
    if "rocprim" in n:
        k = re.findall(r"detail::(\w+?)(?:<|\()", n)
        return "rocprim::" + (k[0] if k else "?")
    n = re.sub(r"\(.*", "", n)
    return re.sub(r"<.*", "", n)[-56:]


def main():
    root = sys.argv[1]
    acc = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[k].add((f, r["Dispatch_Id"]))
    names = sorted({c for v in acc.values() for c in v})
    w = csv.writer(sys.stdout)
    w.writerow(["kernel", "dispatches"] + names)
    for k in sorted(acc, key=lambda k: -acc[k].get("SQ_BUSY_CYCLES", acc[k].get("FETCH_SIZE", 0))):
        w.writerow([k, len(disp[k])] + [f"{acc[k].get(c, 0):.6g}" for c in names])


if __name__ == "__main__":
    main()
