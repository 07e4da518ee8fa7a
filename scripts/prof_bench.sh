#!/bin/bash
# rocprofv3 kernel trace + stats of a short bench run, summarised on the box (the raw trace stays
# in /tmp so the results fit the gpurun_out/ return).  Usage: bash scripts/prof_bench.sh [tag]
set -o pipefail
TAG=${1:-r04}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_$TAG -o run -- \
    python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-pmc > gpurun_out/prof_bench_$TAG.log 2>&1 &&
python3 scripts/rocprof_summary.py "$(find /tmp/prof_$TAG -name '*results.db' -print -quit)" \
    gpurun_out/prof_$TAG --bench gpurun_out/prof_bench_$TAG.log >> gpurun_out/prof_bench_$TAG.log 2>&1 &&
echo PROF_DONE
