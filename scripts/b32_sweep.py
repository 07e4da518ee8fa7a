"""Batched (config 3, B=32) frame-time sweep of fm_tune knobs at S2-Pro shapes: 32 slots prefilled
with ragged prompts, graph-replayed batched frames.
Usage: python scripts/b32_sweep.py 'k1=v1,k2=v2' 'k1=v3' ...   (knobs of a config reset to 0 after)"""
import sys
import time

import numpy as np

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0] + "/fish-speech_amd")
from fishmi import native  # noqa: E402
from fishmi.config import S2_PRO_CONFIG, S2_PRO_IM_END_ID, DualARConfig  # noqa: E402
from fishmi.llm import DualARModel  # noqa: E402

B = 32
cfg = DualARConfig._from_fish_qwen3_omni(S2_PRO_CONFIG)
cfg.im_end_id = S2_PRO_IM_END_ID
cfg.max_seq_len = 1024
m = DualARModel.synthetic(cfg, seed=0, log2_half=5, device=0, precision="bf16", max_slots=B)
rng = np.random.default_rng(2)
prompts = []
for T in rng.integers(16, 257, B):
    p = np.zeros((cfg.num_codebooks + 1, int(T)), np.int32)
    p[0] = rng.integers(16, cfg.semantic_begin_id, int(T))
    prompts.append(p)
sp = DualARModel.sampling(temperature=0.8, top_p=0.8, top_k=30, mask_im_end=True)
confs = [dict(kv.split("=") for kv in a.split(",") if kv) for a in sys.argv[1:]] or [{}]
for rep in range(2):
    for c in confs:
        for k, v in c.items():
            native.tune(k, int(v))
        m.use_graph(True)
        m.prefill_batch(list(range(B)), prompts, [sp] * B)
        m.decode_frames(list(range(B)), 20)
        t0 = time.perf_counter()
        m.decode_frames(list(range(B)), 60)
        dt = (time.perf_counter() - t0) / 60
        print(f"rep {rep} {c}: B={B} frame {dt * 1e3:.3f} ms -> {B / dt / 21.533:.1f} audio-s/s", flush=True)
        for k in c:
            native.tune(k, 0)
