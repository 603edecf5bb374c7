# One SQ counter pass (8 counters) over the training probe (minibatch 4096) and over a short bench
# rollout; per-kernel sums into gpurun_out/sq_*.csv. Each pass under its own kill timer.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES"
BS=4096 N=65536 MAXSTEPS=16 timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d $R/gpurun_out/sq_train -o run -- python3 $R/scripts/train_probe.py > $R/gpurun_out/sq_train.log 2>&1 || { tail -5 $R/gpurun_out/sq_train.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $R/gpurun_out/sq_roll -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-ppo --no-env-fused --no-env-diff --no-dropin --no-e2e > $R/gpurun_out/sq_roll.log 2>&1 || { tail -5 $R/gpurun_out/sq_roll.log; exit 1; }
echo ok
