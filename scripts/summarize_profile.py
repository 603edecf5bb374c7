#!/usr/bin/env python3
"""Turn a gpurun_out/prof_<tag> directory (scripts/profile.sh) into committed summaries:
profiles/<round>_kernel_stats.csv (rocprofv3 --kernel-trace --stats) and
profiles/<round>_pmc.json (per-kernel average FETCH_SIZE / WRITE_SIZE per launch, with the gfx950
correction of MI355X_MICROARCH.md 'HBM': FETCH_SIZE counts half the bytes of wide coalesced reads,
so read bytes = 2 x FETCH_SIZE KiB; write bytes = WRITE_SIZE KiB)."""
import csv
import json
import os
import shutil
import sys
from collections import defaultdict

src, rnd = sys.argv[1], sys.argv[2]
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
dst = os.path.join(root, "profiles")
os.makedirs(dst, exist_ok=True)
shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"), os.path.join(dst, f"{rnd}_kernel_stats.csv"))
out = {}
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    acc = defaultdict(list)
    for r in csv.DictReader(open(os.path.join(src, f"pmc_{c}", "run_counter_collection.csv"))):
        acc[r["Kernel_Name"].split("(")[0].replace("void ", "")].append(float(r["Counter_Value"]))
    for k, v in acc.items():
        out.setdefault(k, {})[c + "_KiB_avg"] = sum(v) / len(v)
        out[k]["launches"] = len(v)
for k, v in out.items():
    if "FETCH_SIZE_KiB_avg" in v and "WRITE_SIZE_KiB_avg" in v:
        v["hbm_bytes_per_launch"] = (2 * v["FETCH_SIZE_KiB_avg"] + v["WRITE_SIZE_KiB_avg"]) * 1024
stats = {}
for r in csv.DictReader(open(os.path.join(src, "trace", "run_kernel_stats.csv"))):
    stats[r["Name"].split("(")[0].replace("void ", "")] = {"calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"]),
                                                             "pct": float(r["Percentage"])}
# steady state: the average of each frequently launched kernel's last 64 launches (the last rollout
# iteration at T = 64; early iterations run slower while clocks and episode states settle)
trace_csv = os.path.join(src, "trace", "run_kernel_trace.csv")
if os.path.exists(trace_csv):
    durs = defaultdict(list)
    for r in csv.DictReader(open(trace_csv)):
        durs[r["Kernel_Name"].split("(")[0].replace("void ", "")].append(
            int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    timed = int(os.environ.get("TIMED_LAUNCHES", "10"))  # profile.sh's --steps: the bench's timed iterations
    for k, v in durs.items():
        if k in stats and len(v) >= 128:
            stats[k]["last64_avg_ns"] = sum(v[-64:]) / 64
        if k in stats and "k_rollout_steps" in k and len(v) > timed:
            # the bench's timed region: the last `timed` launches (graph replays + the eager one),
            # after the warm-up, capture and capture-warm-up launches
            stats[k]["timed_avg_ns"] = sum(v[-timed:]) / timed
            stats[k]["timed_min_ns"] = min(v[-timed:])
            stats[k]["timed_launches"] = timed
json.dump({"pmc": out, "kernel_stats": stats, "source": os.path.basename(src)},
          open(os.path.join(dst, f"{rnd}_pmc.json"), "w"), indent=1)
print(json.dumps({k: v for k, v in out.items() if "uavhip" in k}, indent=1))
