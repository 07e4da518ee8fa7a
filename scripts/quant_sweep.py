"""Weight-only int8 / int4 decode: frame time and per-launch GEMV time at S2-Pro shapes for each
ring depth (fm_tune q_u).  Usage: python scripts/quant_sweep.py [int8|int4 ...]"""
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
quants = sys.argv[1:] or ["int8", "int4"]
us_list = [int(x) for x in os.environ.get("QU", "4,8,16").split(",")]
p = np.zeros((cfg.num_codebooks + 1, 64), np.int32)
p[0] = np.random.default_rng(1).integers(16, cfg.semantic_begin_id, 64)
sp = DualARModel.sampling(mask_im_end=True)
for q in quants:
    m = DualARModel.synthetic(cfg, seed=0, log2_half=5, device=0, precision="bf16", max_slots=1, quant=q)
    for u in us_list:
        native.tune("q_u", u)
        m.use_graph(True)
        m.prefill(0, p, sp)
        m.decode_frames([0], 30)
        us, n, b = m.kernel_bench("linear", 10)
        t0 = time.perf_counter()
        m.decode_frames([0], 100)
        dt = (time.perf_counter() - t0) / 100
        print(f"{q} q_u={u}: gemv {us:7.3f} us/launch x{n} -> {b / n / us / 1e3:7.1f} GB/s | frame {dt * 1e3:.3f} ms",
              flush=True)
    native.tune("q_u", 4)
    del m
