"""Slow-model decode attention alone at S2-Pro shapes: one frame's attn_fd launches replayed back to
back (fm_llm_kernel_bench "attn_slow"), at several context lengths and batch sizes, per fm_tune
setting (SETTINGS="k=v,k=v;k=v").  Usage: python scripts/attn_slow_probe.py"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fish-speech_amd"))
from fishmi import native  # noqa: E402
from fishmi.config import S2_PRO_CONFIG, S2_PRO_IM_END_ID, DualARConfig  # noqa: E402
from fishmi.llm import DualARModel  # noqa: E402

settings = [dict(kv.split("=") for kv in v.split(",") if kv) for v in os.environ.get("SETTINGS", "").split(";")]
base = {}
for st in settings:
    for k in st:
        base.setdefault(k, None)
cfg = DualARConfig._from_fish_qwen3_omni(S2_PRO_CONFIG)
cfg.im_end_id = S2_PRO_IM_END_ID
cfg.max_seq_len = 4096
rng = np.random.default_rng(1)
sp = DualARModel.sampling(temperature=0.7, top_p=0.9, top_k=30, seed=0, mask_im_end=True)
cases = [(1, (60, 120, 180, 250, 500, 1000, 3000)), (32, (150, 400))]
if os.environ.get("CASES"):
    cases = [(int(c.split(":")[0]), tuple(int(x) for x in c.split(":")[1].split("/"))) for c in os.environ["CASES"].split(";")]
for B, lens in cases:
    t0 = time.time()
    m = DualARModel.synthetic(cfg, seed=0, log2_half=5, device=0, precision="bf16", max_slots=B)
    print(f"B={B} load+synth {time.time() - t0:.1f}s", flush=True)
    for T in lens:
        for b in range(B):
            p = np.zeros((cfg.num_codebooks + 1, T), np.int32)
            p[0] = rng.integers(16, 151000, T)
            m.prefill(b, p, sp)
        slots = list(range(B))
        for st in settings:
            for k, v in st.items():
                native.tune(k, int(v))
            m.use_graph(True)
            m.decode(slots)
            m.decode(slots)
            us, n, _ = m.kernel_bench("attn_slow", reps=20)
            print(f"B={B:2d} ctx~{T:5d} {st}: attn_slow {us:7.2f} us/launch x {n}", flush=True)
            if os.environ.get("STAMPS"):  # per-block phases of one eager frame (fm_tune debug_ts)
                native.tune("debug_ts", 1)
                m.use_graph(False)
                m.decode(slots)
                rec = native.debug_ts_read().astype(np.int64)
                native.tune("debug_ts", 0)
                fd = rec[(rec[:, 0] >> 32) == 0xFFFC].astype(np.float64)
                if len(fd):
                    d = (fd[:, 2:6] - fd[:, 1:5]) / 100.0
                    ln = (fd[:, 0].astype(np.int64) & 0xFFFF)
                    ns = (fd[:, 0].astype(np.int64) >> 16) & 0xFFFF
                    print(f"    stamps: {len(fd)} blocks, positions/block {ln.mean():.0f}, splits {ns.mean():.1f}; "
                          f"rt1+qprep {d[:, 0].mean():.2f} passes {d[:, 1].mean():.2f} fold {d[:, 2].mean():.2f} "
                          f"store {d[:, 3].mean():.2f} us; block {(fd[:, 5] - fd[:, 1]).mean() / 100:.2f} us; "
                          f"fold pre-barrier {(fd[:, 6] - fd[:, 3]).mean() / 100:.2f} us", flush=True)
                cmb = rec[(rec[:, 0] >> 32) == 0xFFFB].astype(np.float64)
                if len(cmb):
                    print(f"    combiner: stored->ticket {np.mean(cmb[:, 6] - cmb[:, 5]) / 100:.2f} us, "
                          f"combine {np.mean(cmb[:, 7] - cmb[:, 6]) / 100:.2f} us", flush=True)
    m.close()
