# Round-4 call j: chunked (XCD-aware) weight-gradient mode against stream-K at minibatch 4096 --
# the parity tests, a same-box alternating timing A/B and the k_wgrad trace + FETCH/WRITE passes per mode.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py -m gpu -v -s --timeout 200 --timeout-method thread -k "chunked or per_element or direct_mode or replays_reference or deterministic" > gpurun_out/pytest_r04j.log 2>&1
rc=$?; grep -E "passed|failed" gpurun_out/pytest_r04j.log | tail -2; [ $rc -eq 0 ] || exit $rc
for m in 0 1 0 1; do echo -n "chunk=$m: " >> gpurun_out/probe4096_chunk.log; UAVHIP_WGRAD_CHUNK=$m BS=4096 EPOCHS=3 timeout -k 10 150 python scripts/train_probe.py >> gpurun_out/probe4096_chunk.log 2>&1 || exit 1; done
cat gpurun_out/probe4096_chunk.log
for m in 0 1; do UAVHIP_WGRAD_CHUNK=$m TAG=r04j_c$m bash scripts/profile_train.sh || exit 1; done
echo all done
