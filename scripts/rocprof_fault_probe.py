"""Developer probe for the rocprofv3 host fault on /opt/rocm's HIP runtime: a
model decodes a few frames, eagerly (GRAPH=0) or through the captured frame graph (GRAPH=1), with
torch never imported (FISHMI_NO_TORCH_FIRST=1 keeps fishmi.native from mapping torch's runtime).
MODEL=tiny uses tests/golden/llm_a, MODEL=s2 the S2-Pro shapes.  KNOBS="k=v,k=v" sets fm_tune
knobs first.  Run under: rocprofv3 --kernel-trace -d DIR -o run -- python3 scripts/rocprof_fault_probe.py"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fish-speech_amd"))
from fishmi import native  # noqa: E402
from fishmi.config import S2_PRO_CONFIG, S2_PRO_IM_END_ID, DualARConfig  # noqa: E402
from fishmi.llm import DualARModel  # noqa: E402

for kv in (x for x in os.environ.get("KNOBS", "").split(",") if x):
    k, v = kv.split("=")
    native.tune(k, int(v))
if os.environ.get("MODEL", "tiny") == "tiny":
    cfg = DualARConfig.from_pretrained(os.path.join(ROOT, "tests", "golden", "llm_b"))
    cfg.im_end_id = 4
    T = 16
else:
    cfg = DualARConfig._from_fish_qwen3_omni(S2_PRO_CONFIG)
    cfg.im_end_id = S2_PRO_IM_END_ID
    cfg.max_seq_len = int(os.environ.get("SEQ", "256"))
    T = 64
m = DualARModel.synthetic(cfg, seed=0, log2_half=5, device=0, precision="bf16", max_slots=1)
m.use_graph(os.environ.get("GRAPH", "1") != "0")
p = np.zeros((cfg.num_codebooks + 1, T), np.int32)
p[0] = np.random.default_rng(1).integers(16, cfg.semantic_begin_id, T)
m.prefill(0, p, DualARModel.sampling(mask_im_end=True))
print("prefill ok", flush=True)
out = m.decode_frames([0], int(os.environ.get("FRAMES", "4")))
print("decode ok", out.shape, "torch imported:", "torch" in sys.modules, flush=True)
m.close()
