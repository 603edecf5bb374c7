# Round-4 call n: trunk-order mix in the training forward (TrainIO::mix) and K6 (BwdIO::mix) --
# parity, then kernel times and step times over the four settings, alternating.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py -m gpu -v -s --timeout 200 --timeout-method thread -k "trunk_order or chunked or per_element or replays_reference or deterministic or trunk_split" > gpurun_out/pytest_r04n.log 2>&1
rc=$?; grep -E "passed|failed" gpurun_out/pytest_r04n.log | tail -2; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do for m in 00 11 10 01; do echo -n "fwd,bwd mix=$m: "; UAVHIP_FWD_MIX=${m:0:1} UAVHIP_BWD_MIX=${m:1:1} KERNELS="k_policy_backward k_policy_forward<true" TAG=r04n_${m}_$r bash scripts/ab_kernel_time.sh base || exit 1; done; done
for r in 1 2; do for m in 00 11; do echo -n "fwd,bwd mix=$m: "; UAVHIP_FWD_MIX=${m:0:1} UAVHIP_BWD_MIX=${m:1:1} BS=4096 EPOCHS=3 timeout -k 10 150 python scripts/train_probe.py 2>&1 | grep bs= || exit 1; done; done
echo all done
