"""Per-block phase timing of the batched (B=32) decode linears (bsacc_kernel, fm_tune "debug_ts"):
per shape, kernel span, dispatch spread, and per-block first-data / stream / barrier / epilogue
times (us), split by the block's tile count.  Usage: python scripts/b32_ts.py [frames] [knob=value...]"""
import os
import sys
from collections import defaultdict

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fish-speech_amd"))
from fishmi import native  # noqa: E402
from fishmi.config import S2_PRO_CONFIG, S2_PRO_IM_END_ID, DualARConfig  # noqa: E402
from fishmi.llm import DualARModel  # noqa: E402

args = [x for x in sys.argv[1:] if "=" not in x]
frames = int(args[0]) if args else 2
native.tune("bstream_acc", 1)
for kv in (x for x in sys.argv[1:] if "=" in x):
    k, v = kv.split("=")
    native.tune(k, int(v))
cfg = DualARConfig._from_fish_qwen3_omni(S2_PRO_CONFIG)
cfg.im_end_id = S2_PRO_IM_END_ID
cfg.max_seq_len = 1024
B = 32
m = DualARModel.synthetic(cfg, seed=0, log2_half=5, device=0, precision="bf16", max_slots=B)
rng = np.random.default_rng(1)
for b in range(B):
    p = np.zeros((cfg.num_codebooks + 1, 64), np.int32)
    p[0] = rng.integers(16, 151000, 64)
    m.prefill(b, p, DualARModel.sampling(mask_im_end=True))
m.decode_frames(list(range(B)), 4)
native.tune("debug_ts", 1)
m.use_graph(False)
m.decode_frames(list(range(B)), frames)
rec = native.debug_ts_read().astype(np.int64)
native.tune("debug_ts", 0)
hi = rec[:, 0] >> 32
rec = rec[hi >= (1 << 16)]  # bsacc records: K << 16 | N >> 4 (GEMV and attention tags are < 2^16)
rec = rec[np.argsort(rec[:, 1])]
launches = []
cur = None
for r in rec:
    tag = int(r[0]) >> 32
    if cur is None or tag != cur["tag"] or r[1] > cur["end"]:
        cur = {"tag": tag, "rows": [], "end": 0}
        launches.append(cur)
    cur["rows"].append(r)
    cur["end"] = max(cur["end"], int(r[4]))
by = defaultdict(list)
for L in launches:
    by[L["tag"]].append(np.array(L["rows"], dtype=np.float64))
print(f"{'K':>6s} {'N':>6s} {'launch':>6s} {'blocks':>6s} {'span':>7s} {'disp':>6s} {'first':>6s} {'stream':>6s} "
      f"{'barr':>6s} {'epi':>6s}  per ntl: blocks, end-from-launch (us)")
for tag, Ls in sorted(by.items()):
    K, N = tag >> 16, (tag & 0xFFFF) * 16
    sp, di, fi, stv, ba, ep, xr = [], [], [], [], [], [], []
    byn = defaultdict(list)
    for a in Ls:
        t0 = a[:, 1].min()
        sp.append(a[:, 4].max() - t0)
        di.append(a[:, 1].max() - t0)
        fi.append(np.mean(a[:, 2] - a[:, 1]))
        stv.append(np.mean(a[:, 3] - a[:, 2]))
        ba.append(np.mean(a[:, 5] - a[:, 3]))
        ep.append(np.mean(a[:, 4] - a[:, 5]))
        xr.append(np.mean(a[:, 7] - a[:, 1]) if a[:, 7].min() > 0 else 0.0)
        for n in np.unique(a[:, 6]):
            sel = a[:, 6] == n
            byn[int(n)].append((int(sel.sum()), np.mean(a[sel, 4] - t0), np.max(a[sel, 4] - t0)))
    f = lambda v: np.mean(v) / 100.0
    extra = "  ".join(f"ntl{n}: {np.mean([x[0] for x in v]):.0f} blk end {np.mean([x[1] for x in v]) / 100:.2f}/"
                      f"{np.mean([x[2] for x in v]) / 100:.2f}" for n, v in sorted(byn.items()))
    print(f"{K:6d} {N:6d} {len(Ls):6d} {len(Ls[0]):6d} {f(sp):7.2f} {f(di):6.2f} {f(fi):6.2f} {f(stv):6.2f} "
          f"{f(ba):6.2f} {f(ep):6.2f}  xready {f(xr):5.2f}  {extra}")
