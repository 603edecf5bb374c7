"""gpurun_out/prof_env_<tag> (scripts/profile_env_counters.sh) -> profiles/<tag>_env_counters.json:
per env kernel, the average duration (kernel trace), HBM bytes per launch from the separate
FETCH_SIZE / WRITE_SIZE passes (KB; FETCH doubled per MI355X_MICROARCH.md's gfx950 note) and the
VALU side:
  fp64_flop      64 x (ADD_F64 + MUL_F64 + TRANS_F64) + 128 x FMA_F64 per launch (every lane of a
                 wave instruction counted: an upper bound where exec masks are partial)
  fp64_frac      fp64_flop / duration / 78.6 TFLOP/s (MI355X fp64 vector peak)
  valu_busy      SQ_ACTIVE_INST_VALU x 4 / (SIMDs x GRBM_GUI_ACTIVE / XCDs): the share of SIMD cycles
                 issuing VALU (rocprof-compute's VALUBusy; GRBM_GUI_ACTIVE summed over the 8 XCDs)
  valu_insts / salu_insts  wave instructions per launch
Usage: python scripts/summarize_env_counters.py gpurun_out/prof_env_r02 profiles/r02_env_counters.json"""
import collections
import csv
import glob
import json
import os
import sys

SIMDS, XCDS, FP64_PEAK = 1024, 8, 78.6e12


def main(src, dst):
    # keyed by kernel name AND grid size ("name@grid"): one template instance serves several of the
    # probe's shapes (k_env_replay<64> runs both the 1024- and the 4096-env legs since round 4), and
    # averaging them together would price neither
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(src, "pmc_*", "run_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            key = r["Kernel_Name"].split("(")[0].replace("void ", "") + "@" + r["Grid_Size"]
            agg[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
    durs = collections.defaultdict(list)
    for r in csv.DictReader(open(os.path.join(src, "trace", "run_kernel_trace.csv"))):
        key = r["Kernel_Name"].split("(")[0].replace("void ", "") + "@" + r["Grid_Size_X"]
        durs[key].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    trace = {k: sum(v) / len(v) for k, v in durs.items()}
    out = {}
    for k, d in agg.items():
        if not any(x in k for x in ("score_pairs", "env_step", "env_replay")) or k not in trace:
            continue
        m = {c: sum(v) / len(v) for c, v in d.items()}
        ns = trace[k]
        flop = 64 * (m["SQ_INSTS_VALU_ADD_F64"] + m["SQ_INSTS_VALU_MUL_F64"] + m["SQ_INSTS_VALU_TRANS_F64"]) + \
            128 * m["SQ_INSTS_VALU_FMA_F64"]
        out[k] = {"avg_ns": ns, "hbm_bytes_per_launch": (2 * m["FETCH_SIZE"] + m["WRITE_SIZE"]) * 1024,
                  "fetch_bytes": 2 * m["FETCH_SIZE"] * 1024, "write_bytes": m["WRITE_SIZE"] * 1024,
                  "fp64_flop": flop, "fp64_tflops": flop / ns * 1e-3, "fp64_frac": flop / (ns * 1e-9) / FP64_PEAK,
                  "valu_busy": m["SQ_ACTIVE_INST_VALU"] * 4 / (SIMDS * m["GRBM_GUI_ACTIVE"] / XCDS),
                  "valu_insts": m["SQ_INSTS_VALU"], "salu_insts": m["SQ_INSTS_SALU"], "lds_insts": m["SQ_INSTS_LDS"],
                  "waves": m["SQ_WAVES"]}
    json.dump({"source": "scripts/profile_env_counters.sh on MI355X (rocprofv3 kernel trace + 4 PMC passes)",
               "kernels": out}, open(dst, "w"), indent=1)
    for k, v in out.items():
        print(k, {a: round(b, 4) if isinstance(b, float) else b for a, b in v.items()})


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
