#!/bin/bash
# B=32 batched-linear experiment: knob parity, frame time with the knob off/on, and an eager-mode
# kernel trace with it on.  Usage: bash scripts/b32_check.sh tag knob=value [knob=value...]
set -o pipefail
TAG=$1
shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_llm.py -x -v --timeout 120 --timeout-method thread -m gpu \
    -k "batched_wide_split_k or batched_32_slots or batched_slots_past" > gpurun_out/b32_tests_$TAG.log 2>&1 &&
tail -2 gpurun_out/b32_tests_$TAG.log &&
timeout -k 10 200 python -u scripts/probe_llm.py 64 32 > gpurun_out/b32_probe0_$TAG.log 2>&1 &&
timeout -k 10 200 python -u scripts/probe_llm.py 64 32 "$@" > gpurun_out/b32_probe1_$TAG.log 2>&1 &&
cat gpurun_out/b32_probe0_$TAG.log gpurun_out/b32_probe1_$TAG.log &&
export FISHMI_GRAPH=0 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/pb_$TAG -o run -- python3 scripts/probe_llm.py 8 32 "$@" \
    > gpurun_out/b32_prof_$TAG.log 2>&1 &&
python3 scripts/rocprof_summary.py "$(find /tmp/pb_$TAG -name '*results.db' -print -quit)" gpurun_out/b32_prof_$TAG \
    >> gpurun_out/b32_prof_$TAG.log 2>&1 && echo B32_DONE
