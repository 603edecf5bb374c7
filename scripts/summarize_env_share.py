#!/usr/bin/env python3
"""gpurun_out/envshare_<tag> (scripts/profile_env_share.sh, or the product / noenv directories of
scripts/profile_env_attrib.sh's gpurun_out/envattr_<tag>) -> profiles/<round>_env_share.json: per
step of k_rollout_steps (launch / T) the average duration and the HBM bytes (FETCH_SIZE x 2 +
WRITE_SIZE, the gfx950 correction of MI355X_MICROARCH.md 'HBM') of the product build and of the build
without the env step; their differences are the env step's time and traffic per step (all E envs)."""
import csv
import json
import os
import sys

src, rnd = sys.argv[1], sys.argv[2]
T, E = int(os.environ.get("T", "64")), int(os.environ.get("E", "4096"))
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNEL = "k_rollout_steps"
out = {}
for b in ("product", "noenv"):
    d = {}
    durs = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            for r in csv.DictReader(open(os.path.join(src, b, "trace", "run_kernel_trace.csv")))
            if KERNEL in r["Kernel_Name"]]
    d["launches"] = len(durs)
    warm = durs[len(durs) // 2:] if len(durs) > 2 else durs[1:]  # steady state: the later half of the launches
    d["avg_ns_per_step"] = sum(warm) / max(1, len(warm)) / T
    for i, c in enumerate(("FETCH_SIZE", "WRITE_SIZE")):
        d_ = os.path.join(src, b, f"pmc_{c}")
        if not os.path.isdir(d_):  # scripts/profile_env_attrib.sh's layout: pmc_1 = FETCH, pmc_2 = WRITE
            d_ = os.path.join(src, b, f"pmc_{i + 1}")
        v = [float(r["Counter_Value"]) for r in csv.DictReader(open(os.path.join(d_, "run_counter_collection.csv")))
             if KERNEL in r["Kernel_Name"] and r.get("Counter_Name", c) == c]
        d[c + "_KiB_per_step"] = sum(v) / len(v) / T
    d["hbm_bytes_per_step"] = (2 * d["FETCH_SIZE_KiB_per_step"] + d["WRITE_SIZE_KiB_per_step"]) * 1024
    out[b] = d
res = {"kernel": KERNEL, "T": T, "E": E, "builds": out,
       "env_ns_per_step": out["product"]["avg_ns_per_step"] - out["noenv"]["avg_ns_per_step"],
       "env_bytes_per_step": out["product"]["hbm_bytes_per_step"] - out["noenv"]["hbm_bytes_per_step"],
       "source": os.path.basename(src)}
res["env_bytes_per_env_step"] = res["env_bytes_per_step"] / E
json.dump(res, open(os.path.join(root, "profiles", f"{rnd}_env_share.json"), "w"), indent=1)
print(json.dumps(res, indent=1))
