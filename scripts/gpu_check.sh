#!/bin/bash
# One GPU-box pass: gpu parity tests, smoke(), the default bench line, and a rocprofv3 kernel-trace
# of a short bench, summarised on the box (the raw trace stays in /tmp so the results fit the
# gpurun_out/ return).  Every GPU step has its own time limit; steps are chained with && so the
# first failure ends the call.  Usage: bash scripts/gpu_check.sh [tag] [extra pytest args...]
set -o pipefail
TAG=${1:-r03}
shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 720 python -u -m pytest tests -x -v --timeout 180 --timeout-method thread -m gpu "$@" \
    > gpurun_out/gpu_tests_$TAG.log 2>&1 && tail -3 gpurun_out/gpu_tests_$TAG.log &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 &&
tail -1 gpurun_out/smoke_$TAG.log &&
timeout -k 10 420 python -u bench.py > gpurun_out/bench_$TAG.log 2>&1 && tail -1 gpurun_out/bench_$TAG.log &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_$TAG -o run -- \
    python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-pmc > gpurun_out/prof_bench_$TAG.log 2>&1 &&
python3 scripts/rocprof_summary.py "$(find /tmp/prof_$TAG -name '*results.db' -print -quit)" \
    gpurun_out/prof_$TAG --bench gpurun_out/prof_bench_$TAG.log >> gpurun_out/prof_bench_$TAG.log 2>&1 &&
echo GPU_CHECK_DONE
