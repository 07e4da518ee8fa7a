#!/bin/bash
# Skinny prompt GEMM grid sweep (fm_tune prompt_skinny_blocks: K slices until the 64-row blocks reach it).
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for b in 256 384 512 768 1024 1536; do
    echo "== prompt_skinny_blocks=$b"
    timeout -k 10 120 python -u scripts/prefill_probe.py prompt_skinny_blocks=$b 2>&1 | grep "T=   64\|T=  136\|T=  256" || exit 1
done
