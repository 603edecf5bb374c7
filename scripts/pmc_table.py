"""Per-kernel averages of rocprofv3 --pmc counter CSVs: python scripts/pmc_table.py DIR [name-filter ...]"""
import collections
import csv
import glob
import sys

root = sys.argv[1]
filt = sys.argv[2:]
per = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(f"{root}/**/run_counter_collection.csv", recursive=True)):
    disp = collections.defaultdict(float)
    names = {}
    for r in csv.DictReader(open(f)):
        k = (r["Dispatch_Id"], r["Counter_Name"])
        disp[k] += float(r["Counter_Value"])
        names[r["Dispatch_Id"]] = r["Kernel_Name"]
    for (d, c), v in disp.items():
        per[names[d]][c].append(v)
for name, cs in per.items():
    if filt and not any(x in name for x in filt):
        continue
    print(name[:90])
    for c, v in sorted(cs.items()):
        print(f"   {c:28s} {sum(v) / len(v):16.0f}  (n={len(v)})")
