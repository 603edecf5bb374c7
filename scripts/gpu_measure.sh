# One measurement call (round 5 on): the -m gpu suite and smoke (unless SKIP_TESTS), then the
# profiles FIRST -- profile.sh (k_rollout_steps kernel stats + FETCH / WRITE PMC) and
# profile_env_share.sh (product vs NOENV build), summarised into this tree's profiles/ -- and the full
# bench line LAST, so the line's roofline.profiled / traffic / env traffic come from this same lease.
# The summaries are copied to gpurun_out/profiles_$TAG/ to be committed. Every GPU step under its own
# time limit; the call stops at the first crash.
#   TAG=r05a bash scripts/gpu_measure.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${TAG:-r05a}
if [ -z "$SKIP_TESTS" ]; then
  # assertion failures (rc 1) are read afterwards and the measurements still run; a crash, abort or
  # time limit (any other rc) ends the call
  timeout -k 10 600 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
  rc=$?
  grep -E "^(FAILED|ERROR)|passed|failed" gpurun_out/pytest_$TAG.log | tail -12
  [ $rc -le 1 ] || { tail -40 gpurun_out/pytest_$TAG.log; exit $rc; }
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { tail -20 gpurun_out/smoke_$TAG.log; exit 1; }
  echo smoke ok
fi
if [ -z "$SKIP_PROFILES" ]; then
  TAG=$TAG bash scripts/profile.sh || exit 1
  cd $GRAFT_REPO_ROOT
  python scripts/summarize_profile.py gpurun_out/prof_$TAG $TAG > /dev/null || exit 1
  echo profile ok
  TAG=$TAG bash scripts/profile_env_share.sh || exit 1
  cd $GRAFT_REPO_ROOT
  python scripts/summarize_env_share.py gpurun_out/envshare_$TAG $TAG > /dev/null || exit 1
  echo env share ok
  mkdir -p gpurun_out/profiles_$TAG
  cp profiles/${TAG}_* gpurun_out/profiles_$TAG/
fi
timeout -k 10 900 python bench.py $BENCH_ARGS > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -20 gpurun_out/bench_$TAG.err; exit 1; }
echo bench ok
python - "$TAG" <<'EOF'
import json, sys
d = json.loads(open(f"gpurun_out/bench_{sys.argv[1]}.json").read().strip().splitlines()[-1])
r = d["roofline"]
print("value", d["value"], "ms_per_step", d["ms_per_step"], "kernel ms/step", r["avg_launch_ms"], "frac", r["frac"])
print("profiled", r.get("profiled"))
e = d.get("env_roofline") or {}
print("env", e.get("avg_launch_ms"), (e.get("differential") or {}).get("product_vs_headline"), e.get("frac"))
for k in ("ppo_samples_per_s", "ppo_samples_per_s_mb64"):
    print(k, (d.get(k) or {}).get("value"))
for x in d.get("dropin_loop") or []:
    print("dropin", x.get("workload"), x.get("value"), x.get("rollout_env_steps_per_s"), x.get("update_samples_per_s"),
          (x.get("cpu_baseline") or {}).get("value"))
EOF
