#!/bin/bash
# Overlapped vocoder under the stream knobs of fm_stream_create (fm_runtime.h): dispatch priority
# (LLM high, codec low) and codec CU masks; reduced bench runs, the config 2 / 3 / 5 values printed.
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
FAST="--no-int8 --no-cpu-baseline --no-pmc --encode-seconds 0"
run() {  # tag env...
    local tag=$1; shift
    env "$@" timeout -k 10 300 python -u bench.py $FAST $EXTRA > gpurun_out/bench_vs_$tag.log 2>&1 || return 1
    python3 -c "
import json
d = json.loads(open('gpurun_out/bench_vs_$tag.log').read().strip().splitlines()[-1])
t, l = d['throughput'], d['longform']
print('$tag', 'c2', d['value'], 'dec', d['breakdown_ms']['decode'], 'codec', d['breakdown_ms']['codec'],
      '| c3', t['value'], t['phase_s_rank0'], t.get('codec_busy_s_rank0'), '| c5', l['value'])"
}
run prio FISHMI_STREAM_PRIO=1 && run cu8 FISHMI_CODEC_CU_STRIDE=8 && run cu4 FISHMI_CODEC_CU_STRIDE=4 &&
run cu2 FISHMI_CODEC_CU_STRIDE=2 && run base X=0 && EXTRA="--serial-vocode --vocode-chunk 0" run serprio FISHMI_STREAM_PRIO=1
