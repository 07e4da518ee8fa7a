"""Prompt prefill at S2-Pro shapes (synthetic bf16 weights): wall time per prompt length and the
eager per-class split (linear / attn / rope / norm / other).
Usage: python scripts/prefill_probe.py [key=value fm_tune knobs ...]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fish-speech_amd"))
from fishmi import native  # noqa: E402
from fishmi.config import S2_PRO_CONFIG, S2_PRO_IM_END_ID, DualARConfig  # noqa: E402
from fishmi.llm import DualARModel  # noqa: E402

for kv in sys.argv[1:]:
    k, v = kv.split("=")
    native.tune(k, int(v))
cfg = DualARConfig._from_fish_qwen3_omni(S2_PRO_CONFIG)
cfg.im_end_id = S2_PRO_IM_END_ID
cfg.max_seq_len = 2048
m = DualARModel.synthetic(cfg, seed=0, log2_half=5, device=0, precision="bf16", max_slots=1)
rng = np.random.default_rng(3)
sp = DualARModel.sampling(mask_im_end=True)
for T in (64, 136, 256, 700, 1400):
    p = np.zeros((cfg.num_codebooks + 1, T), np.int32)
    p[0] = rng.integers(16, cfg.semantic_begin_id, T)
    m.prefill(0, p, sp)
    ts = []
    for _ in range(3):
        t0 = time.perf_counter()
        m.prefill(0, p, sp)
        ts.append(time.perf_counter() - t0)
    m.profile(True)
    m.prefill(0, p, sp)
    cl = {c: m.profile_read(c)[0] for c in ("linear", "attn", "rope", "norm", "other")}
    m.profile(False)
    print(f"T={T:5d}: prefill {min(ts) * 1e3:8.2f} ms  eager classes (ms): " +
          " ".join(f"{k} {v:.2f}" for k, v in cl.items()), flush=True)
