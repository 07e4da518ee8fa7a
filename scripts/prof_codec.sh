#!/bin/bash
# rocprofv3 kernel trace of one config-2 codec decode (scripts/codec_prof.py), per-shape summary.
set -o pipefail
TAG=${1:-codec}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 200 rocprofv3 --kernel-trace -d /tmp/prof_$TAG -o run -- python3 scripts/codec_prof.py \
    > gpurun_out/prof_$TAG.log 2>&1 &&
python3 scripts/codec_prof.py $(find /tmp/prof_$TAG -name '*results.db' -print -quit) >> gpurun_out/prof_$TAG.log 2>&1 &&
python3 scripts/codec_prof.py $(find /tmp/prof_$TAG -name "*results.db" -print -quit) 32 > gpurun_out/seq_$TAG.log 2>&1 &&
echo PROF_DONE
