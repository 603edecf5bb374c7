#!/bin/bash
# Phase timelines (TRACE=1 build: make -C target-allocation-ppo-transformer_amd/csrc TRACE=1
# BUILD=build_trace OUT=$PWD/scripts/trace_lib/libuavhip.so): rollout forward (full window and
# ring), training forward + backward. GPU box: bash scripts/trace_all.sh
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
export UAVHIP_LIB=$PWD/scripts/trace_lib/libuavhip.so
timeout -k 10 120 python scripts/policy_trace.py > gpurun_out/trace_fwd.log 2>&1 &&
ROWS=1 timeout -k 10 120 python scripts/policy_trace.py > gpurun_out/trace_rows.log 2>&1 &&
timeout -k 10 120 python scripts/train_trace.py > gpurun_out/trace_train.log 2>&1
