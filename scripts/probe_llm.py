"""Decode-step probe at S2-Pro shapes (synthetic weights): ms/frame, per-kernel-class split,
achieved bytes/s vs frame bytes.  Usage: python scripts/probe_llm.py [frames] [batch]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fish-speech_amd"))
from fishmi.config import S2_PRO_CONFIG, S2_PRO_IM_END_ID, DualARConfig  # noqa: E402
from fishmi.llm import DualARModel  # noqa: E402

args = [x for x in sys.argv[1:] if "=" not in x]
frames = int(args[0]) if len(args) > 0 else 64
B = int(args[1]) if len(args) > 1 else 1
from fishmi import native  # noqa: E402
for kv in (x for x in sys.argv[1:] if "=" in x):  # developer knobs: key=value (fm_tune)
    k, v = kv.split("=")
    native.tune(k, int(v))
cfg = DualARConfig._from_fish_qwen3_omni(S2_PRO_CONFIG)
cfg.im_end_id = S2_PRO_IM_END_ID
cfg.max_seq_len = 1024
t0 = time.time()
m = DualARModel.synthetic(cfg, seed=0, log2_half=5, device=0, precision="bf16", max_slots=B)
print(f"load+synth {time.time() - t0:.1f}s", flush=True)
rng = np.random.default_rng(1)
T = 64
prompts = []
for b in range(B):
    p = np.zeros((cfg.num_codebooks + 1, T), np.int32)
    p[0] = rng.integers(16, 151000, T)
    prompts.append(p)
sp = DualARModel.sampling(temperature=0.7, top_p=0.9, top_k=30, seed=0, mask_im_end=True)
for b in range(B):
    m.prefill(b, prompts[b], sp)
slots = list(range(B))
for _ in range(3):
    m.decode(slots)
t0 = time.time()
for _ in range(frames):
    m.decode(slots)
dt = (time.time() - t0) / frames
fb = m.frame_bytes(B, T + frames)
print(f"B={B}: {dt*1e3:.3f} ms/frame  -> {B/dt:.1f} frames/s = {B/dt/21.533:.2f}x RT aggregate; "
      f"frame bytes {fb/1e9:.3f} GB -> {fb/dt/1e12:.3f} TB/s", flush=True)
# pipelined generate
t0 = time.time()
out = m.generate(prompts[0], frames + 1, top_k=30, seed=3, mask_im_end=True)
dt2 = (time.time() - t0)
print(f"generate(prefill+{frames}) {dt2*1e3:.1f} ms -> {out.shape[1]/dt2:.1f} frames/s", flush=True)
m.profile(True)
for _ in range(4):
    m.decode(slots)
tot = 0
for cls in ["linear", "attn", "rope", "norm", "sample", "other"]:
    ms, n, b = m.profile_read(cls)
    tot += ms
    extra = f" {b/ (ms*1e-3) /1e12:.2f} TB/s" if b else ""
    print(f"  {cls:7s} {ms/4:8.3f} ms/frame  {n//4:5d} launches/frame{extra}")
print(f"  total {tot/4:.3f} ms/frame (eager, event-bracketed)")
