"""Sweep the decode-GEMV knobs (fm_tune) at S2-Pro shapes: per-launch replay timing of one
frame's GEMVs (fm_llm_kernel_bench) and graph-replayed frame time."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fish-speech_amd"))
from fishmi import native  # noqa: E402
from fishmi.config import S2_PRO_CONFIG, S2_PRO_IM_END_ID, DualARConfig  # noqa: E402
from fishmi.llm import DualARModel  # noqa: E402

cfg = DualARConfig._from_fish_qwen3_omni(S2_PRO_CONFIG)
cfg.im_end_id = S2_PRO_IM_END_ID
cfg.max_seq_len = 1024
m = DualARModel.synthetic(cfg, seed=0, log2_half=5, device=0, precision="bf16", max_slots=1)
p = np.zeros((cfg.num_codebooks + 1, 64), np.int32)
p[0] = np.random.default_rng(1).integers(16, cfg.semantic_begin_id, 64)
sp = DualARModel.sampling(mask_im_end=True)
configs = [dict(gemv_u=u, gemv_wpb=w) for u in (4, 8) for w in (4, 8)]
for c in configs:
    for k, v in c.items():
        native.tune(k, v)
    m.use_graph(True)
    m.prefill(0, p, sp)
    m.decode_frames([0], 40)
    us, n, b = m.kernel_bench("linear", 20)
    t0 = time.perf_counter()
    m.decode_frames([0], 100)
    dt = (time.perf_counter() - t0) / 100
    print(f"{c}: gemv {us:7.3f} us/launch x{n} -> {b / n / us / 1e3:7.1f} GB/s | frame {dt * 1e3:.3f} ms",
          flush=True)
