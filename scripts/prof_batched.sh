#!/bin/bash
# rocprofv3 kernel trace of the batched (BASELINE config 3) leg only; summarised on the box so the
# raw trace does not travel back.  Usage: bash scripts/prof_batched.sh [tag] [batch]
set -o pipefail
TAG=${1:-b32}
B=${2:-32}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_$TAG -o run -- \
    python3 bench.py --steps 1 --warmup 0 --frames 24 --no-cpu-baseline --batch $B --batch-frames 48 \
    > gpurun_out/prof_$TAG.log 2>&1 &&
python3 scripts/rocprof_summary.py $(find /tmp/prof_$TAG -name '*results.db' -print -quit) gpurun_out/prof_$TAG \
    >> gpurun_out/prof_$TAG.log 2>&1 && echo PROF_DONE
