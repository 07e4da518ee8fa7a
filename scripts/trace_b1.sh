#!/bin/bash
# Kernel sequence of one B=1 decode frame (graph replay) at S2-Pro shapes, plus per-name totals.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${1:-b1}
timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/tr_$TAG -o run -- \
    python3 bench.py --steps 1 --warmup 0 --batch 0 --encode-seconds 0 --no-cpu-baseline --no-pmc \
    > gpurun_out/trace_$TAG.log 2>&1 &&
python3 scripts/frame_trace.py "$(find /tmp/tr_$TAG -name '*results.db' -print -quit)" ${2:-140} > gpurun_out/frame_$TAG.txt 2>&1 &&
echo TRACE_DONE
