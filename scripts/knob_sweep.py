"""Frame-time sweep of fm_tune knobs at S2-Pro shapes (B=1, graph-replayed frames).
QUANT=int8|int4 quantizes the linears; each config also reports the decode GEMVs' average launch.
Usage: python scripts/knob_sweep.py 'k1=v1,k2=v2' 'k1=v3' ...   (each arg is one config; every
knob any config touches is reset before each config to the first config's value, or to its
FmTuning default when the first config leaves it out)."""
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
# FmTuning's defaults (fm_kernels.h) for the knobs sweeps touch; a knob the first config sets takes
# that value as its baseline instead
DEFAULTS = {"attn3": 1, "attn_fd": 1, "fd_min": 32, "fd_nw": 8, "fd_min16": 256, "kv_prefetch": 1, "gemv_u": 8,
            "gemv_wpb": 4, "fin_ksb": 0, "gemv_dummy": 2, "rowgemv": 27, "rowgemv_q4": 31, "sampler_kth": 1,
            "row_qkv_rp": 8, "fattn_wo": 1, "fw_cheap": 0, "fw_delay": 0, "fw_prio": 0, "fast_tail": 1,
            "fkv_prefetch": 0, "q_u": 4}
base = {k: int(v) for k, v in confs[0].items()}
touched = {k for c in confs for k in c}
missing = sorted(k for k in touched if k not in base and k not in DEFAULTS)
if missing:
    sys.exit(f"no baseline for {missing}: give them in the first config")
for rep in range(2):
    for c in confs:
        for k in touched:  # every config starts from the baseline
            native.tune(k, base.get(k, DEFAULTS.get(k)))
        for k, v in c.items():
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
