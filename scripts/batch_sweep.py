"""Batched-frame sweep (BASELINE config 3 shape) of fm_tune knobs at S2-Pro shapes.
Usage: python scripts/batch_sweep.py B 'k1=v1,k2=v2' 'k1=v3' ...  (each arg after B is one config)."""
import sys
import time

import numpy as np

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0] + "/fish-speech_amd")
from fishmi import native  # noqa: E402
from fishmi.config import S2_PRO_CONFIG, S2_PRO_IM_END_ID, DualARConfig  # noqa: E402
from fishmi.llm import DualARModel  # noqa: E402

B = int(sys.argv[1])
cfg = DualARConfig._from_fish_qwen3_omni(S2_PRO_CONFIG)
cfg.im_end_id = S2_PRO_IM_END_ID
cfg.max_seq_len = 1024
m = DualARModel.synthetic(cfg, seed=0, log2_half=5, device=0, precision="bf16", max_slots=B)
rng = np.random.default_rng(2)
sp = DualARModel.sampling(mask_im_end=True)
m.use_graph(True)
confs = [dict(kv.split("=") for kv in a.split(",") if kv) for a in sys.argv[2:]] or [{}]
for rep in range(2):
    for c in confs:
        for k, v in c.items():
            native.tune(k, int(v))
        m.use_graph(True)  # drops captured frames: the next capture sees the knobs
        for s in range(B):
            T = int(rng.integers(16, 257))
            p = np.zeros((cfg.num_codebooks + 1, T), np.int32)
            p[0] = rng.integers(16, cfg.semantic_begin_id, T)
            m.prefill(s, p, sp)
        m.decode_frames(list(range(B)), 4)
        t0 = time.perf_counter()
        m.decode_frames(list(range(B)), 40)
        dt = (time.perf_counter() - t0) / 40
        print(f"rep {rep} B={B} {c}: frame {dt * 1e3:.3f} ms  ({B / dt / 21.533:.1f} audio-s/s)", flush=True)

# eager per-class breakdown of one batched frame (HIP events per launch class) + the linear
# class replayed back to back (average launch, algorithmic bytes)
m.use_graph(False)
m.profile(True)
m.decode_frames(list(range(B)), 2)
for cls in ("linear", "attn", "rope", "norm", "sample", "other"):
    ms, n, b = m.profile_read(cls)
    print(f"class {cls}: {ms / 2:.3f} ms/frame, {n // 2} launches/frame, {b / 2e9:.2f} GB/frame", flush=True)
m.profile(False)
us, n, b = m.kernel_bench("linear", 10)
print(f"linear replay: {us:.2f} us/launch x {n} = {us * n / 1e3:.3f} ms/frame, {b / (us * n * 1e-6) / 1e9:.0f} GB/s", flush=True)
