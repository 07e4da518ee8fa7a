"""pass_kernel variants (fm_tune pass_cfg) at S2-Pro shapes: us per persistent fast pass (kernel
replay) and ms per frame.  Usage: python scripts/pass_cfg_sweep.py [cfg ...]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fish-speech_amd"))
from fishmi import native  # noqa: E402
from fishmi.config import S2_PRO_CONFIG, S2_PRO_IM_END_ID, DualARConfig  # noqa: E402
from fishmi.llm import DualARModel  # noqa: E402

cfgs = [int(x) for x in sys.argv[1:]] or [0, 1, 2, 3]
cfg = DualARConfig._from_fish_qwen3_omni(S2_PRO_CONFIG)
cfg.im_end_id = S2_PRO_IM_END_ID
cfg.max_seq_len = 512
m = DualARModel.synthetic(cfg, seed=0, log2_half=5, device=0, precision="bf16", max_slots=1)
rng = np.random.default_rng(1)
prompt = np.zeros((cfg.num_codebooks + 1, 64), np.int32)
prompt[0] = rng.integers(16, 151000, 64)
sp = DualARModel.sampling(temperature=0.7, top_p=0.9, top_k=30, seed=0, mask_im_end=True)
for c in cfgs + cfgs:
    native.tune("pass_cfg", c)
    m.use_graph(True)
    m.prefill(0, prompt, sp)
    m.decode_frames([0], 3)
    t0 = time.time()
    m.decode_frames([0], 24)
    dt = (time.time() - t0) / 24
    us, n, b = m.kernel_bench("pass", 20)
    print(f"pass_cfg={c}: {us:.1f} us/pass ({b / n / (us * 1e-6) / 1e12:.2f} TB/s), {dt * 1e3:.3f} ms/frame", flush=True)
m.close()
