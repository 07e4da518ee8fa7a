"""attn_fd at batch 1, S2-Pro shapes: in-kernel span (first block start .. last block end, from the
fm_tune debug_ts stamps) per launch, to set beside the same launches' rocprofv3 --kernel-trace
durations.  Usage: rocprofv3 --kernel-trace -d DIR -o run -- python scripts/attn_span_probe.py [frames]
then python scripts/attn_span_probe.py --db DIR/.../run_results.db"""
import os
import sqlite3
import sys

import numpy as np
if os.environ.get("WITH_TORCH"):
    import torch  # noqa: F401

if len(sys.argv) > 2 and sys.argv[1] == "--db":
    c = sqlite3.connect(sys.argv[2])
    rows = c.execute("select name, start, end from kernels order by start").fetchall()
    for tag in ("attn_fd_kernel", "fast_attn2_kernel", "sample_fast_kernel", "gemv_kernel"):
        d = np.array([(e - s) / 1e3 for n, s, e in rows if tag in n])
        if len(d):
            print(f"trace {tag}: n {len(d)} mean {d.mean():.2f} us  p10 {np.percentile(d, 10):.2f}  p90 {np.percentile(d, 90):.2f}")
    d = np.array([(e - s) / 1e3 for n, s, e in rows if "attn_fd_kernel" in n])
    print("attn_fd per frame (36 launches) means:", " ".join(f"{x:.1f}" for x in d[: len(d) // 36 * 36].reshape(-1, 36).mean(1)))
    sys.exit(0)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fish-speech_amd"))
from fishmi import native  # noqa: E402
from fishmi.config import S2_PRO_CONFIG, S2_PRO_IM_END_ID, DualARConfig  # noqa: E402
from fishmi.llm import DualARModel  # noqa: E402

frames = int(sys.argv[1]) if len(sys.argv) > 1 else 4
cfg = DualARConfig._from_fish_qwen3_omni(S2_PRO_CONFIG)
cfg.im_end_id = S2_PRO_IM_END_ID
cfg.max_seq_len = 1024
m = DualARModel.synthetic(cfg, seed=0, log2_half=5, device=0, precision="bf16", max_slots=1)
p = np.zeros((cfg.num_codebooks + 1, 64), np.int32)
p[0] = np.random.default_rng(1).integers(16, cfg.semantic_begin_id, 64)
m.prefill(0, p, DualARModel.sampling(mask_im_end=True))
m.decode_frames([0], 8)
import time  # noqa: E402
# graph mode, no stamps: frame time per knob setting (KNOBS="k=v,k=v;k=v" variants)
variants = [dict(kv.split("=") for kv in v.split(",") if kv) for v in os.environ.get("KNOBS", "").split(";")]
for rep in range(2):
    for v in variants:
        for k, x in v.items():
            if k != "graph":
                native.tune(k, int(x))
        m.use_graph(v.get("graph", "1") != "0")  # drops captured frames: the next capture sees the knobs
        m.prefill(0, p, DualARModel.sampling(mask_im_end=True))  # same positions for every variant
        m.decode_frames([0], 60)
        t0 = time.perf_counter()
        m.decode_frames([0], 100)  # positions 124 .. 224 (config 2 averages ~172)
        t1 = time.perf_counter()
        us, n, b = m.kernel_bench("attn", 20)
        ul, nl, bl = m.kernel_bench("linear", 20)
        print(f"rep {rep} {v}: graph frame {(t1 - t0) / 100 * 1e3:.3f} ms; attn replay {us:.2f} us x {n}; "
              f"linear replay {ul:.2f} us x {nl} ({bl / nl / ul / 1e3:.1f} GB/s)")
for cls in ("attn", "linear"):
    us, n, b = m.kernel_bench(cls, 20)
    print(f"kernel_bench {cls}: {us:.2f} us per launch, {n} launches per frame, {us * n / 1e3:.3f} ms per frame")
native.tune("debug_ts", 1)
m.use_graph(False)
m.decode_frames([0], frames)
rec = native.debug_ts_read().astype(np.int64)
native.tune("debug_ts", 0)
fd = rec[(rec[:, 0] >> 32) == 0xFFFC]
fd = fd[np.argsort(fd[:, 1])]
st, en = fd[:, 1], fd[:, 5]
cut = np.where(np.diff(st) > 500)[0]  # launches are > 5 us apart
groups = np.split(np.arange(len(st)), cut + 1)
spans = [(en[g].max() - st[g].min()) / 100 for g in groups]
starts = [(st[g].max() - st[g].min()) / 100 for g in groups]
blk = (en - st) / 100
print(f"attn_fd eager: {len(groups)} launches, blocks/launch {np.mean([len(g) for g in groups]):.1f}, "
      f"in-kernel span mean {np.mean(spans):.2f} us, block start spread {np.mean(starts):.2f} us, "
      f"block time mean {blk.mean():.2f} us")
if os.environ.get("RECAPTURE"):  # graph dropped by use_graph(False), then captured again
    m.use_graph(True)
    m.decode_frames([0], 4)
    print("recapture ok")
