#!/bin/bash
# B=32 path check: the batched parity tests (bf16 vs the reference, fp32 batched == single), the
# frame probe and the per-block phase stamps.  Usage: bash scripts/b32_quick.sh tag [knob=value...]
set -o pipefail
TAG=$1
shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_00_timed_configs.py tests/test_gpu_llm.py tests/test_gpu_int8.py -x -v \
    --timeout 180 --timeout-method thread -m gpu -k "ragged or batched or wide or int8" > gpurun_out/b32q_tests_$TAG.log 2>&1 &&
tail -2 gpurun_out/b32q_tests_$TAG.log &&
timeout -k 10 200 python -u scripts/probe_llm.py 64 32 "$@" > gpurun_out/b32q_probe_$TAG.log 2>&1 &&
head -2 gpurun_out/b32q_probe_$TAG.log && sed -n 4,9p gpurun_out/b32q_probe_$TAG.log &&
timeout -k 10 120 python -u scripts/b32_ts.py 2 "$@" > gpurun_out/b32q_ts_$TAG.log 2>&1 && cat gpurun_out/b32q_ts_$TAG.log
