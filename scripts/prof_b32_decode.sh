#!/bin/bash
# rocprofv3 kernel trace of B=32 decode frames only (scripts/probe_llm.py), summarised on the box.
# Usage: bash scripts/prof_b32_decode.sh [tag]
set -o pipefail
TAG=${1:-b32dec}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_$TAG -o run -- \
    python3 scripts/probe_llm.py 64 32 > gpurun_out/prof_$TAG.log 2>&1 &&
python3 scripts/rocprof_summary.py $(find /tmp/prof_$TAG -name '*results.db' -print -quit) gpurun_out/prof_$TAG \
    >> gpurun_out/prof_$TAG.log 2>&1 && echo PROF_DONE
