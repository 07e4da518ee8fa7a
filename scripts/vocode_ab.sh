#!/bin/bash
# A/B of the overlapped vocoder (scheduler.StreamVocoder) against the serial one on configs 2, 3 and 5:
# the codec stream test, then two reduced bench runs (no int8 / cpu baseline / pmc / encode legs).
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
FAST="--no-int8 --no-cpu-baseline --no-pmc --encode-seconds 0"
timeout -k 10 300 python -u -m pytest tests/test_gpu_codec_stream.py -x -v --timeout 180 --timeout-method thread -m gpu \
    > gpurun_out/voc_tests.log 2>&1 && tail -2 gpurun_out/voc_tests.log &&
timeout -k 10 400 python -u bench.py $FAST --overlap-vocode "$@" > gpurun_out/bench_voc_ov.log 2>&1 &&
timeout -k 10 400 python -u bench.py $FAST --vocode-chunk 0 "$@" > gpurun_out/bench_voc_se.log 2>&1 &&
python3 - <<'PY'
import json
for tag in ("ov", "se"):
    d = json.loads(open(f"gpurun_out/bench_voc_{tag}.log").read().strip().splitlines()[-1])
    t, l = d["throughput"], d["longform"]
    print(tag, "c2", d["value"], d["breakdown_ms"], "p50 first", d["p50_first_sample_ms"],
          "| c3", t["value"], t["phase_s_rank0"], t.get("codec_busy_s_rank0"), "| c5", l["value"], l["first_sample_ms"],
          l["turn_first_chunk_ms_p50"])
PY
