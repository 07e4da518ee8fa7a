"""Decode attention probe at S2-Pro shapes: one frame's "attn" launches (slow decode attention +
fast-model attention) replayed back to back (fm_llm_kernel_bench) at several context lengths and
batch sizes, per fm_tune setting.  Usage: python scripts/attn_probe.py [key=value ...]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fish-speech_amd"))
from fishmi import native  # noqa: E402
from fishmi.config import S2_PRO_CONFIG, S2_PRO_IM_END_ID, DualARConfig  # noqa: E402
from fishmi.llm import DualARModel  # noqa: E402

SETTINGS = [
    {"attn_fd": 0, "attn3": 1},
    {"attn_fd": 1, "fd_min": 32, "fd_min_batched": 256},
    {"attn_fd": 1, "fd_min": 64, "fd_min_batched": 256},
    {"attn_fd": 1, "fd_min": 64, "fd_min_batched": 512},
]
cfg = DualARConfig._from_fish_qwen3_omni(S2_PRO_CONFIG)
cfg.im_end_id = S2_PRO_IM_END_ID
cfg.max_seq_len = 4096
rng = np.random.default_rng(1)
sp = DualARModel.sampling(temperature=0.7, top_p=0.9, top_k=30, seed=0, mask_im_end=True)
for B, lens in ((1, (170, 1000, 3000)), (32, (170, 600))):
    t0 = time.time()
    m = DualARModel.synthetic(cfg, seed=0, log2_half=5, device=0, precision="bf16", max_slots=B)
    print(f"B={B} load+synth {time.time() - t0:.1f}s", flush=True)
    for T in lens:
        for b in range(B):
            p = np.zeros((cfg.num_codebooks + 1, T), np.int32)
            p[0] = rng.integers(16, 151000, T)
            m.prefill(b, p, sp)
        slots = list(range(B))
        for st in SETTINGS:
            for k, v in st.items():
                native.tune(k, int(v))
            m.decode(slots)
            m.decode(slots)
            us, n, _ = m.kernel_bench("attn", reps=20)
            print(f"B={B:2d} ctx~{T:5d} {st}: attn {us:7.2f} us/launch x {n} = {us * n / 1e3:.3f} ms/frame", flush=True)
    m.close()
