import csv, sys, re
rows = list(csv.DictReader(open(sys.argv[1])))
def short(n):
    n = n.replace("gs::(anonymous namespace)::", "").replace("void ", "")
    n = re.sub(r"\(.*", "", n)
    if "rocprim" in n: n = "rocprim::" + (re.findall(r"detail::(\w+)", n) or ["?"])[-1]
    return n[:48]
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:25]:
    print(f'{short(r["Name"]):50s} {int(r["Calls"]):7d} {float(r["TotalDurationNs"])/1e6:9.3f} ms {float(r["AverageNs"])/1e3:9.2f} us {100*float(r["TotalDurationNs"])/tot:6.2f}%')
