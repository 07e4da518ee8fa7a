#!/bin/bash
# Quick kernel-time summary of a short bench run (no tests): rocprofv3 --kernel-trace --stats over
# `bench.py --steps 1 --warmup 0` plus the bench line itself.  Usage: bash scripts/prof_quick.sh TAG [bench args]
set -o pipefail
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/pq_$TAG -o run -- \
    python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-pmc --encode-seconds 0 "$@" > gpurun_out/pq_$TAG.log 2>&1 &&
python3 scripts/rocprof_summary.py "$(find /tmp/pq_$TAG -name '*results.db' -print -quit)" gpurun_out/pq_$TAG \
    --bench gpurun_out/pq_$TAG.log > /dev/null 2>&1 &&
tail -1 gpurun_out/pq_$TAG.log | cut -c1-200 && echo PQ_DONE
