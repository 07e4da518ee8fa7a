"""Four 64-token prefills at S2-Pro shapes (for rocprofv3 --kernel-trace: the prompt-path kernels)."""
import os, sys
import numpy as np
ROOT = "/root/repo" if os.path.exists("/root/repo/fish-speech_amd") else os.getcwd()
sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT", ROOT), "fish-speech_amd"))
from fishmi.config import S2_PRO_CONFIG, S2_PRO_IM_END_ID, DualARConfig
from fishmi.llm import DualARModel
cfg = DualARConfig._from_fish_qwen3_omni(S2_PRO_CONFIG); cfg.im_end_id = S2_PRO_IM_END_ID; cfg.max_seq_len = 1024
m = DualARModel.synthetic(cfg, seed=0, log2_half=5, device=0, precision="bf16", max_slots=1)
p = np.zeros((cfg.num_codebooks + 1, 64), np.int32); p[0] = np.random.default_rng(3).integers(16, cfg.semantic_begin_id, 64)
sp = DualARModel.sampling(mask_im_end=True)
for _ in range(4): m.prefill(0, p, sp)
print("ok")
