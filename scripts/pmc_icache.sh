# Instruction-cache counters (SQC block) of the training probe and a short rollout bench, if the
# device lists them (rocprofv3 -L first).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $R/gpurun_out/pmc_list.txt 2>&1 || true
grep -o "SQC_ICACHE[A-Z_]*\|SQ_IFETCH[A-Z_]*\|SQ_INSTS_[A-Z_]*" $R/gpurun_out/pmc_list.txt | sort -u | head -30
grep -q "SQC_ICACHE_MISSES" $R/gpurun_out/pmc_list.txt || exit 0
BS=4096 N=65536 MAXSTEPS=16 timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS --output-format csv -d $R/gpurun_out/ic_train -o run -- python3 $R/scripts/train_probe.py > $R/gpurun_out/ic_train.log 2>&1 || { tail -3 $R/gpurun_out/ic_train.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS --output-format csv -d $R/gpurun_out/ic_roll -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-ppo --no-env-fused > $R/gpurun_out/ic_roll.log 2>&1 || { tail -3 $R/gpurun_out/ic_roll.log; exit 1; }
echo ok
