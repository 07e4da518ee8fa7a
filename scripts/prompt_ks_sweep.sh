#!/bin/bash
# Prompt-GEMM split-K sweep (fm_tune prompt_ks_tiles / prompt_ks_max) on the prefill probe.
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for kv in "prompt_ks_max=8" "prompt_ks_max=1" "prompt_ks_max=2" "prompt_ks_max=4" "prompt_ks_tiles=192" "prompt_ks_tiles=256" "prompt_ks_tiles=768"; do
    echo "== $kv"
    timeout -k 10 120 python -u scripts/prefill_probe.py $kv 2>&1 | grep -v amdgpu || exit 1
done
