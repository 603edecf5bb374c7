# Multi-GPU path checks on the one-GPU box: the -m gpu dist tests (world-2 gloo iteration, world-1
# RCCL epoch graph), then bench.py's N = 2 rehearsal with 2 ranks on one GPU over gloo (the
# per-iteration rollout / exchange timeline lands in gpurun_out/bench_gloo2.json).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_dist.py -m gpu -v --timeout 600 --timeout-method thread > gpurun_out/pytest_dist.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed|^E  " gpurun_out/pytest_dist.log | tail -30
[ $rc -eq 0 ] || exit $rc
BENCH_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 2 \
  > gpurun_out/bench_gloo2.json 2> gpurun_out/bench_gloo2.err || { tail -30 gpurun_out/bench_gloo2.err; exit 1; }
python -c "
import json; d=json.loads(open('gpurun_out/bench_gloo2.json').read().strip().splitlines()[-1])
print('value %.3e ms/step %.3f' % (d['value'], d['ms_per_step'])); print(d.get('iteration_timeline')); p=d.get('ppo_samples_per_s'); print(p and {k: p.get(k) for k in ('value','impl','error')})
"
