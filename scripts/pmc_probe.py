"""Small S2-Pro decode run for rocprofv3 --pmc passes (FETCH_SIZE / WRITE_SIZE of the decode
GEMVs): prefill 64 tokens + 4 frames, eager launches.  Run with FISHMI_GRAPH=0."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fish-speech_amd"))
from fishmi.config import S2_PRO_CONFIG, S2_PRO_IM_END_ID, DualARConfig  # noqa: E402
from fishmi.llm import DualARModel  # noqa: E402

cfg = DualARConfig._from_fish_qwen3_omni(S2_PRO_CONFIG)
cfg.im_end_id = S2_PRO_IM_END_ID
cfg.max_seq_len = 1024
m = DualARModel.synthetic(cfg, seed=0, log2_half=5, device=0, precision="bf16", max_slots=1)
p = np.zeros((cfg.num_codebooks + 1, 64), np.int32)
p[0] = np.random.default_rng(1).integers(16, cfg.semantic_begin_id, 64)
m.prefill(0, p, DualARModel.sampling(mask_im_end=True))
m.decode_frames([0], 4)
print("frame bytes", m.frame_bytes(1, 68))
