"""Persistent fast pass (fm_pass.hip) against the launch-per-op path at S2-Pro shapes (synthetic
weights): teacher-forced logits of two slots fed the same columns, one decoded with fm_tune
pass_fast 0 and one with 1, then ms/frame of each.
Usage: python scripts/pass_probe.py [frames] [key=value ...]  (fm_tune knobs, e.g. pass_cfg=1)"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fish-speech_amd"))
from fishmi import native  # noqa: E402
from fishmi.config import S2_PRO_CONFIG, S2_PRO_IM_END_ID, DualARConfig  # noqa: E402
from fishmi.llm import DualARModel  # noqa: E402

args = [x for x in sys.argv[1:] if "=" not in x]
frames = int(args[0]) if args else 32
native.tune("pass_prepare", 1)  # the pass weights are built at finalize only when asked for
for kv in (x for x in sys.argv[1:] if "=" in x):
    k, v = kv.split("=")
    native.tune(k, int(v))
cfg = DualARConfig._from_fish_qwen3_omni(S2_PRO_CONFIG)
cfg.im_end_id = S2_PRO_IM_END_ID
cfg.max_seq_len = 512
t0 = time.time()
m = DualARModel.synthetic(cfg, seed=0, log2_half=5, device=0, precision="bf16", max_slots=2)
print(f"load+synth {time.time() - t0:.1f}s", flush=True)
rng = np.random.default_rng(1)
T = 64
prompt = np.zeros((cfg.num_codebooks + 1, T), np.int32)
prompt[0] = rng.integers(16, 151000, T)
nchk = 6
cols = np.zeros((cfg.num_codebooks + 1, nchk), np.int32)
cols[0] = rng.integers(cfg.semantic_begin_id, cfg.semantic_end_id + 1, nchk)
cols[1:] = rng.integers(0, cfg.codebook_size, (cfg.num_codebooks, nchk))
sp = DualARModel.sampling(top_k=1)


def step(slot, on, k):
    native.tune("pass_fast", on)
    m.use_graph(True)  # drop captured frames: the next capture picks up the knob
    m.force(slot, cols[:, k])
    if k == 0:
        m.prefill(slot, prompt, sp)
    else:
        m.decode([slot])
    return m.read_logits(slot)


worst = 0.0
for k in range(nchk):
    s0, f0 = step(0, 0, k)
    s1, f1 = step(1, 1, k)
    fin = np.isfinite(s0)
    ds = float(np.max(np.abs(s0[fin] - s1[fin])))
    df = float(np.max(np.abs(f0 - f1)))
    rf = float(np.sqrt(np.mean((f0 - f1) ** 2)) / np.sqrt(np.mean(f0 ** 2)))
    agree = float(np.mean(np.argmax(f0, -1) == np.argmax(f1, -1)))
    worst = max(worst, rf)
    print(f"frame {k}: slow max|d| {ds:.4g}  fast max|d| {df:.4g} rel-rms {rf:.3e} top1 agree {agree:.2f}", flush=True)
for s in (0, 1):
    m.force(s, None)
sps = DualARModel.sampling(temperature=0.7, top_p=0.9, top_k=30, seed=0, mask_im_end=True)
res = {}
for on in (0, 1, 0, 1):
    native.tune("pass_fast", on)
    m.use_graph(True)
    m.prefill(0, prompt, sps)
    m.decode_frames([0], 3)
    t0 = time.time()
    m.decode_frames([0], frames)
    dt = (time.time() - t0) / frames
    res.setdefault(on, []).append(dt)
    print(f"pass_fast={on}: {dt * 1e3:.3f} ms/frame", flush=True)
print(f"RESULT off {min(res[0]) * 1e3:.3f} ms/frame  on {min(res[1]) * 1e3:.3f} ms/frame  worst fast rel-rms {worst:.3e}")
native.tune("pass_fast", 1)
m.use_graph(True)
m.prefill(0, prompt, sps)
m.decode_frames([0], 2)
us, n, b = m.kernel_bench("pass", 20)
print(f"pass kernel: {us:.2f} us/launch, {n} launches/frame, {b / max(n, 1) / 1e6:.1f} MB/launch -> "
      f"{b / max(n, 1) / (us * 1e-6) / 1e12:.3f} TB/s")
m.close()

if os.environ.get("STAMPS"):
    # per-(workgroup, op) phases of one eager frame's passes (fm_tune debug_ts), in microseconds
    m2 = DualARModel.synthetic(cfg, seed=0, log2_half=5, device=0, precision="bf16", max_slots=1)
    m2.prefill(0, prompt, sps)
    m2.use_graph(False)
    m2.decode([0])
    native.tune("debug_ts", 1)
    m2.decode([0])
    rec = native.debug_ts_read().astype(np.int64)
    native.tune("debug_ts", 0)
    rec_all = rec.copy()
    tag = (rec[:, 0] >> 32) & 0xFFFFFFFF
    rec = rec[(tag >> 24) == 0xFA]
    wg = (rec[:, 0] >> 40) & 0xFF
    op = (rec[:, 0] >> 32) & 0xFF
    gen = rec[:, 0] & 0xFFFFFFFF
    print(f"{len(rec)} pass records, {len(np.unique(gen))} launches")
    g1 = np.unique(gen)[len(np.unique(gen)) // 2]  # one mid-frame pass (cc >= 1)
    r = rec[gen == g1]
    o = op[gen == g1]
    t0 = r[:, 1:7].min()
    us = lambda x: (x - t0) / 100.0  # noqa: E731
    # stamps: 0 previous seam end, 1 consumers all arrived, 2 published, 3 swept, 4 exchange sync,
    # 5 next input row ready; 6 >> 32: spread of the consumer waves' arrival times
    print("op  wait-A med/max | publish | sweep | sync | build (attention) | seam 1->5 med/max | A spread | consumer spread")
    for k in sorted(set(o.tolist())):
        q = r[o == k]
        d = lambda i, j: (q[:, j] - q[:, i]) / 100.0  # noqa: E731
        wa, seam = d(1, 2), d(2, 6)
        print(f"{k:2d}  {np.median(wa):7.2f} {wa.max():7.2f} | {np.median(d(2, 3)):5.2f} | {np.median(d(3, 4)):5.2f} | "
              f"{np.median(d(4, 5)):5.2f} | {np.median(d(5, 6)):5.2f} ({np.median(q[:, 7] & 0xFFFFFFFF) / 100.0:5.2f}) | {np.median(seam):6.2f} {seam.max():6.2f} | "
              f"{(q[:, 2].max() - q[:, 2].min()) / 100.0:5.2f} | {np.median(q[:, 7] >> 32) / 100.0:5.2f}")
    print(f"pass span {(r[:, 6].max() - r[:, 1].min()) / 100.0:.1f} us")
    # stream waves (pass_cfg >= 6): per op, input seen -> 32 fragments consumed -> arrived
    sr = rec_all[((rec_all[:, 0] >> 56) & 0xFF) == 0xFB] if rec_all is not None else np.zeros((0, 8), np.int64)
    if len(sr):
        sg = sr[:, 0] & 0xFFFFFFFF
        sr = sr[sg == g1]
        so = (sr[:, 0] >> 32) & 0xFF
        print("op  stream: open->32 frags med/max | open->arrive med/max (us)")
        for k in sorted(set(so.tolist())):
            q = sr[so == k]
            mid = q[:, 2] > 0
            d1 = (q[mid, 2] - q[mid, 1]) / 100.0
            d2 = (q[:, 3] - q[:, 1]) / 100.0
            print(f"{k:2d}  {np.median(d1) if len(d1) else float('nan'):7.2f} {d1.max() if len(d1) else float('nan'):7.2f} | "
                  f"{np.median(d2):7.2f} {d2.max():7.2f}")
    q = r[o == 0][:, 7] & 0xFFFFFFFF
    print(f"attention (exchange waves' share) {np.median(q) / 100.0:.2f} us")
    m2.close()
