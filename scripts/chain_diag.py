"""Persistent GEMV chain vs one kernel per GEMV at full S2-Pro depth (36 + 4 layers, bf16, B=1):
free-running greedy tokens and teacher-forced logits of the same prompt, and the first frame where
the two paths diverge.  Diagnostic for the gemv_chain_kernel hand-offs."""
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
quant = sys.argv[1] if len(sys.argv) > 1 and sys.argv[1] != "bf16" else None
m = DualARModel.synthetic(cfg, seed=0, log2_half=5, device=0, precision="bf16", max_slots=1, quant=quant)
rng = np.random.default_rng(1)
p = np.zeros((cfg.num_codebooks + 1, 64), np.int32)
p[0] = rng.integers(16, cfg.semantic_begin_id, 64)
out = {}
for chain in (0, 1):
    native.tune("gemv_chain", chain)
    t0 = time.perf_counter()
    toks = m.generate(p, 48, top_k=1, mask_im_end=True)
    dt = time.perf_counter() - t0
    slow, fast = m.teacher_decode(p, toks[:, :6])
    out[chain] = (toks, slow, fast)
    print(f"chain={chain}: {toks.shape[1]} frames in {dt * 1e3:.1f} ms", flush=True)
a, b = out[0][0], out[1][0]
bad = np.where((a != b).any(axis=0))[0]
print("tokens identical" if bad.size == 0 else f"first divergent frame {bad[0]} of {a.shape[1]}")
fin = np.isfinite(out[0][1])
print("teacher slow max|diff|", float(np.abs(np.where(fin, out[0][1] - out[1][1], 0)).max()),
      "fast max|diff|", float(np.abs(out[0][2] - out[1][2]).max()),
      "nan in chain logits", bool(np.isnan(out[1][1][fin]).any() or np.isnan(out[1][2]).any()))
