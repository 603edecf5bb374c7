set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_full.log 2>&1 || { tail -30 gpurun_out/pytest_full.log; exit 1; }
tail -1 gpurun_out/pytest_full.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -2 gpurun_out/smoke.log
timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
TAG=r02 timeout -k 10 900 bash scripts/profile_env_counters.sh || exit 1
python scripts/summarize_env_counters.py gpurun_out/prof_env_r02 gpurun_out/r02_env_counters.json
