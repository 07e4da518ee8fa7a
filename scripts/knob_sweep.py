"""Frame-time sweep of fm_tune knobs at S2-Pro shapes (B=1, graph-replayed frames).
QUANT=int8|int4 quantizes the linears; each config also reports the decode GEMVs' average launch.
Usage: python scripts/knob_sweep.py 'k1=v1,k2=v2' 'k1=v3' ...   (each arg is one config; the
knobs of a config are reset to the first config's values before the next one is applied)."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0] + "/fish-speech_amd")
from fishmi import native  # noqa: E402
from fishmi.config import S2_PRO_CONFIG, S2_PRO_IM_END_ID, DualARConfig  # noqa: E402
from fishmi.llm import DualARModel  # noqa: E402

cfg = DualARConfig._from_fish_qwen3_omni(S2_PRO_CONFIG)
cfg.im_end_id = S2_PRO_IM_END_ID
cfg.max_seq_len = 1024
m = DualARModel.synthetic(cfg, seed=0, log2_half=5, device=0, precision="bf16", max_slots=1,
                          quant=os.environ.get("QUANT") or None)
p = np.zeros((cfg.num_codebooks + 1, 64), np.int32)
p[0] = np.random.default_rng(1).integers(16, cfg.semantic_begin_id, 64)
sp = DualARModel.sampling(mask_im_end=True)
confs = [dict(kv.split("=") for kv in a.split(",") if kv) for a in sys.argv[1:]] or [{}]
base = {}
for rep in range(2):
    for c in confs:
        for k, v in c.items():
            base.setdefault(k, None)
            native.tune(k, int(v))
        m.use_graph(True)
        m.prefill(0, p, sp)
        ref = m.decode_frames([0], 40)
        t0 = time.perf_counter()
        m.decode_frames([0], 150)
        dt = (time.perf_counter() - t0) / 150
        us, n, b = m.kernel_bench("linear", reps=10)
        print(f"rep {rep} {c}: frame {dt * 1e3:.3f} ms  ({1 / dt / 21.533:.2f}x RT)  tok0 {int(ref[-1, 0, 0])}  "
              f"linear {us:.2f} us x {n}, {b / n / (us * 1e-6) / 1e12:.2f} TB/s", flush=True)
