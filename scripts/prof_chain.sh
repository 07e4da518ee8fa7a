#!/bin/bash
# Kernel trace of B=1 S2-Pro frames with the GEMV chain on (knob_sweep, graph replay), summarised,
# plus the frame sequence with gaps.  Usage: bash scripts/prof_chain.sh TAG [knob=value ...]
set -o pipefail
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/pc_$TAG -o run -- \
    python3 scripts/knob_sweep.py "$@" > gpurun_out/pc_$TAG.log 2>&1 &&
python3 scripts/rocprof_summary.py "$(find /tmp/pc_$TAG -name '*results.db' -print -quit)" gpurun_out/pc_$TAG > /dev/null 2>&1 &&
echo PC_DONE
