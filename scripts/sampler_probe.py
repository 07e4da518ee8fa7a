"""Where a batch-1 sampler launch spends its time: sample_fast_kernel's phase
stamps (fm_tune debug_ts; s_memrealtime, 100 MHz) over eager S2-Pro frames -- values loaded, wave
maxima, top-K threshold, candidates, exact ranks, end (after the draw and the column store) -- and,
for the codebook samplers, the gap from the end of the head GEMV blocks that wrote the logits
(rowgemv_kernel records) to the sampler's start.

    python scripts/sampler_probe.py [frames]
"""
import os
import sys

import numpy as np

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
# armed once, before the frame graph is captured (the graph keeps the buffer's address: never
# re-arm or free it while the model lives), so graph replays record too
native.tune("debug_ts", 1)
m.prefill(0, p, DualARModel.sampling(mask_im_end=True))
m.decode_frames([0], 2 + frames)
rec = native.debug_ts_read().astype(np.int64)
m.close()
native.tune("debug_ts", 0)
tag = rec[:, 0] >> 32
smp = rec[tag == 0xFFFF]
row = rec[tag == 0xFFFA]  # rowgemv_kernel blocks: {tag | blk, start, streamed, end, ...}
print(f"{len(smp)} sampler launches, {len(row)} row-GEMV block records")
names = ["values in", "wave max", "threshold", "candidates", "ranks", "draw + store"]
ph = np.diff(smp[:, 1:8], axis=1) / 100.0  # us
slow = (smp[:, 0] >> 17) & 1
for which, sel in (("slow head (RAS: two draws)", slow == 1), ("codebook heads", slow == 0)):
    if sel.any():
        med = np.median(ph[sel], axis=0)
        tot = np.median((smp[sel, 7] - smp[sel, 1]) / 100.0)
        print(f"{which}: {sel.sum()} launches, start->end median {tot:.2f} us; " +
              ", ".join(f"{n} {v:.2f}" for n, v in zip(names, med)))
# gap: the latest row-GEMV block end before each sampler start
ends = np.sort(row[:, 3])
gaps = []
for s0 in smp[:, 1]:
    i = np.searchsorted(ends, s0) - 1
    if i >= 0:
        gaps.append((s0 - ends[i]) / 100.0)
if gaps:
    print(f"head-GEMV end -> sampler start: median {np.median(gaps):.2f} us (graph replays)")
