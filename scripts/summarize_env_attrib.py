#!/usr/bin/env python3
"""gpurun_out/envattr_<tag> (scripts/profile_env_attrib.sh) -> profiles/<round>_env_attrib.json: per
build (product, NOENV, the attribution builds EXP=21..27) and per step of k_rollout_steps (launch / T):
the average duration, HBM bytes (FETCH_SIZE x 2 + WRITE_SIZE, the gfx950 correction of
MI355X_MICROARCH.md 'HBM'), L2 hits / misses and memory-side read requests; and for each build its
difference from the product build (what the compiled-out accesses cost)."""
import csv
import json
import os
import sys

src, rnd = sys.argv[1], sys.argv[2]
T, E = int(os.environ.get("T", "64")), int(os.environ.get("E", "4096"))
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNEL = "k_rollout_steps"
WHAT = {"noenv": "the whole env step", "exp21": "scene values (tgt_value / uav_cost / p_pen, both buffers)",
        "exp22": "per-target / per-UAV state loads (nh_final, nh_pure, t_cost, n_lock, assigned)",
        "exp23": "istate / dstate row loads", "exp24": "the env's own window load",
        "exp25": "the env-state stores", "exp26": "the step outputs (obs, reward, done, info)",
        "exp27": "the dependent p_dmg load of the new pointer pair",
        "exp32": "the ring rows' L2 misses (every ring load reads one hot row; policy.hip kExpHotRing)"}


def counters(path):
    acc = {}
    for r in csv.DictReader(open(path)):
        if KERNEL in r["Kernel_Name"]:
            acc.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) / T for k, v in acc.items()}


out = {}
for b in sorted(os.listdir(src)):
    d = os.path.join(src, b)
    if not os.path.isdir(d):
        continue
    try:
        durs = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
                for r in csv.DictReader(open(os.path.join(d, "trace", "run_kernel_trace.csv")))
                if KERNEL in r["Kernel_Name"]]
        res = {"launches": len(durs), "avg_ns_per_step": sum(durs[1:]) / max(1, len(durs) - 1) / T}
        for i in (1, 2, 3):
            res.update(counters(os.path.join(d, f"pmc_{i}", "run_counter_collection.csv")))
    except FileNotFoundError as exc:
        res = {"error": str(exc)}
    if "FETCH_SIZE" in res and "WRITE_SIZE" in res:
        res["hbm_bytes_per_step"] = (2 * res["FETCH_SIZE"] + res["WRITE_SIZE"]) * 1024
    out[b] = res
prod = out.get("product", {})
for b, r in out.items():
    if b == "product" or "hbm_bytes_per_step" not in r or "hbm_bytes_per_step" not in prod:
        continue
    r["compiled_out"] = WHAT.get(b, b)
    r["saves_ns_per_step"] = prod["avg_ns_per_step"] - r["avg_ns_per_step"]
    r["saves_bytes_per_step"] = prod["hbm_bytes_per_step"] - r["hbm_bytes_per_step"]
    for k in ("TCC_MISS_sum", "TCC_HIT_sum", "TCC_EA0_RDREQ_sum", "TCC_EA0_RDREQ_DRAM_sum"):
        if k in r and k in prod:
            r["saves_" + k] = prod[k] - r[k]
res = {"kernel": KERNEL, "T": T, "E": E, "units": "per step of the launch (all E envs)", "builds": out,
       "source": os.path.basename(src)}
json.dump(res, open(os.path.join(root, "profiles", f"{rnd}_env_attrib.json"), "w"), indent=1)
print(json.dumps(res, indent=1))
