"""Timeline of the fused fast attention + wo launch (fm_rowgemv.hip fattn_wo_kernel) from its
debug_ts records: attention waves (0xFFF9: start, K/V staged, stored) and sampled wo blocks
(0xFFF8: start, weights issued, cheap poll done, full x read, end; aux = polls), per launch,
relative to the launch's first block start (us)."""
import os
import sys

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
m.prefill(0, p, DualARModel.sampling(mask_im_end=True))
m.decode_frames([0], 8)
m.use_graph(False)
native.tune("debug_ts", 1)
m.decode_frames([0], 2)
rec = native.debug_ts_read().astype(np.int64)
native.tune("debug_ts", 0)
att = rec[(rec[:, 0] >> 32) == 0xFFF9]
wo = rec[(rec[:, 0] >> 32) == 0xFFF8]
# launches: attention records sorted by start, split at gaps > 3 us
att = att[np.argsort(att[:, 1])]
cut = np.where(np.diff(att[:, 1]) > 300)[0] + 1
rows = []
for g in np.split(att, cut):
    t0 = g[:, 1].min()
    w = wo[(wo[:, 1] >= t0 - 100) & (wo[:, 1] < t0 + 3000)]
    if not len(w):
        continue
    T = lambda x: (x - t0) / 100.0
    rows.append([T(g[:, 2].max()), T(g[:, 3].max()), T(w[:, 1].max()), T(w[:, 2]).mean(), T(w[:, 3]).mean(),
                 T(w[:, 4]).mean(), T(w[:, 5]).mean(), T(w[:, 5]).max(), np.mean(w[:, 0] & 0xFFFFFFFF)])
r = np.array(rows)
print(f"{len(r)} launches; means (us from the launch's first block start):")
names = ["att staged(max)", "att stored(max)", "wo last start", "wo weights issued", "wo poll ok",
         "wo x read", "wo end(mean)", "wo end(max)", "polls"]
for n, v in zip(names, r.mean(axis=0)):
    print(f"  {n:18s} {v:7.2f}")
