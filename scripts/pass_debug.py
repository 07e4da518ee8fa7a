"""Op-by-op comparison of the persistent fast pass (fm_pass.hip exchange granules) with the
launch-per-op path's activation buffers, on a 2 + 1-layer model at S2-Pro widths: both slots get
the same forced columns; after each frame the LAST fast pass's q|k|v, h, SwiGLU row and output x
are compared.  Usage: python scripts/pass_debug.py [key=value ...]"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fish-speech_amd"))
from fishmi import native  # noqa: E402
from fishmi.config import S2_PRO_CONFIG, S2_PRO_IM_END_ID, DualARConfig  # noqa: E402
from fishmi.llm import DualARModel  # noqa: E402

for kv in (x for x in sys.argv[1:] if "=" in x):
    k, v = kv.split("=")
    native.tune(k, int(v))
spec = {**S2_PRO_CONFIG, "text_config": {**S2_PRO_CONFIG["text_config"], "n_layer": 2},
        "audio_decoder_config": {**S2_PRO_CONFIG["audio_decoder_config"], "n_layer": 1}}
cfg = DualARConfig._from_fish_qwen3_omni(spec)
cfg.im_end_id = S2_PRO_IM_END_ID
cfg.max_seq_len = 256
m = DualARModel.synthetic(cfg, seed=0, log2_half=5, device=0, precision="bf16", max_slots=2)
L = native.lib()


def vec(name, n, index=0):
    out = np.zeros(n, np.float32)
    native.check(L.fm_llm_debug_vec(m.h, name.encode(), index, out.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), n))
    return out


rng = np.random.default_rng(1)
T = 16
prompt = np.zeros((cfg.num_codebooks + 1, T), np.int32)
prompt[0] = rng.integers(16, 151000, T)
cols = np.zeros((cfg.num_codebooks + 1, 3), np.int32)
cols[0] = rng.integers(cfg.semantic_begin_id, cfg.semantic_end_id + 1, 3)
cols[1:] = rng.integers(0, cfg.codebook_size, (cfg.num_codebooks, 3))
sp = DualARModel.sampling(top_k=1)
d, nqkv, inter = cfg.fast_dim, (cfg.fast_n_head + 2 * cfg.fast_n_local_heads) * cfg.fast_head_dim, cfg.fast_intermediate_size
nq = cfg.fast_n_head * cfg.fast_head_dim
for k in range(3):
    res = {}
    for slot, on in ((0, 0), (1, 1)):
        native.tune("pass_fast", on)
        m.use_graph(False)
        m.force(slot, cols[:, k])
        if k == 0:
            m.prefill(slot, prompt, sp)
        else:
            m.decode([slot])
        if on:
            res[on] = dict(qkv=vec("gran", nqkv, 0), fh=vec("gran", d, 1), act=vec("gran", inter, 2),
                           fx=vec("gran", d, 3))
        else:
            res[on] = dict(qkv=vec("qkv", nqkv), att=vec("att", nq), fh=vec("fh", d), act=vec("act", inter),
                           fx=vec("fx", d))
        res[on]["logits"] = m.read_logits(slot)[1]
    for key in ("qkv", "fh", "act", "fx", "logits"):
        a, b = res[0][key], res[1][key]
        diff = np.abs(a - b)
        rel = float(np.sqrt(np.mean(diff ** 2)) / (np.sqrt(np.mean(a.astype(np.float64) ** 2)) + 1e-30))
        print(f"frame {k} {key:6s}: rel-rms {rel:.3e} max|d| {diff.max():.4g} |a| {np.abs(a).max():.4g} "
              f"first bad {int(np.argmax(diff > 1e-2 * (np.abs(a).max() + 1e-6))) if (diff > 1e-2 * (np.abs(a).max() + 1e-6)).any() else -1}",
              flush=True)
    a, b = res[0]["logits"], res[1]["logits"]
    for cb_i in (0, 8):
        aa, bb = a[cb_i], b[cb_i]
        blk = np.abs(aa - bb).reshape(-1, 16).max(1)
        s_fit = float(np.dot(aa, bb) / np.dot(aa, aa))
        print(f"  codebook {cb_i + 1}: blocks with max|d|>0.05: {int((blk > 0.05).sum())}/{blk.size}, "
              f"fit scale {s_fit:.4f}, corr {np.corrcoef(aa, bb)[0, 1]:.4f}; in-block pattern",
              np.round(np.abs(aa - bb).reshape(-1, 16).mean(0), 3))
    if k == 0:
        a, b = res[0]["qkv"], res[1]["qkv"]
        print("qkv head0 launch", a[:8], "\n         pass  ", b[:8])
m.close()
