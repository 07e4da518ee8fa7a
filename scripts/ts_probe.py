"""Per-block phase timing of the decode GEMVs at S2-Pro shapes (fm_tune "debug_ts").
For each GEMV shape: kernel span, dispatch spread, and per-block prologue / stream / epilogue
times (us).  Usage: python scripts/ts_probe.py [frames]"""
import os
import sys
from collections import defaultdict

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fish-speech_amd"))
from fishmi import native  # noqa: E402
from fishmi.config import S2_PRO_CONFIG, S2_PRO_IM_END_ID, DualARConfig  # noqa: E402
from fishmi.llm import DualARModel  # noqa: E402

frames = int(sys.argv[1]) if len(sys.argv) > 1 else 2
for kv in sys.argv[2:]:
    k, v = kv.split("=")
    native.tune(k, int(v))
cfg = DualARConfig._from_fish_qwen3_omni(S2_PRO_CONFIG)
cfg.im_end_id = S2_PRO_IM_END_ID
cfg.max_seq_len = 1024
quant = os.environ.get("TS_QUANT") or None  # int8 / int4 weight-only linears
m = DualARModel.synthetic(cfg, seed=0, log2_half=5, device=0, precision="bf16", max_slots=1, quant=quant)
p = np.zeros((cfg.num_codebooks + 1, 64), np.int32)
p[0] = np.random.default_rng(1).integers(16, cfg.semantic_begin_id, 64)
m.prefill(0, p, DualARModel.sampling(mask_im_end=True))
m.decode_frames([0], 8)
native.tune("debug_ts", 1)
m.use_graph(False)
m.decode_frames([0], frames)
rec = native.debug_ts_read().astype(np.int64)
native.tune("debug_ts", 0)
rec = rec[np.argsort(rec[:, 1])]
smp = rec[(rec[:, 0] >> 32) == 0xFFFF].astype(np.float64)
if len(smp):
    d = np.diff(smp[:, 1:8], axis=1).mean(axis=0) / 100.0
    print("sampler phases (us): load", round(d[0], 2), "max", round(d[1], 2), "kth", round(d[2], 2),
          "bar1+cand+bar2", round(d[3], 2), "rank", round(d[4], 2), "-", round(d[5], 2))
    lo = (smp[:, 0].astype(np.int64) & 0xFFFF)
    print("sampler candidates: mean", round(lo.mean(), 1), "max", lo.max(), "overflow", int(((smp[:, 0].astype(np.int64) >> 16) & 1).sum()))
for tag, name, labels in ((0xFFFE, "fast_attn2", ("load", "prep", "scores", "pv+store")),
                          (0xFFFC, "attn_fd", ("rt1+qprep", "passes", "fold", "store")),
                          (0xFFFD, "attn_decode2", ("kv load", "q prep", "scores", "softmax", "pv", "rec"))):
    a = rec[(rec[:, 0] >> 32) == tag].astype(np.float64)
    if len(a):
        nz = [i for i in range(1, 8) if a[:, i].max() > 0]
        d = np.diff(a[:, nz], axis=1).mean(axis=0) / 100.0
        aux = a[:, 0].astype(np.int64) & 0xFFFFFFFF
        print(f"{name} phases (us):", " ".join(f"{l} {v:.2f}" for l, v in zip(labels, d)),
              "| blocks", len(a), "aux mean", round(float(aux.mean()), 1))
rg = rec[(rec[:, 0] >> 32) == 0xFFFA].astype(np.float64)
if len(rg):
    # row-pair GEMV (fm_rowgemv.hip): launches split at gaps > 5 us between block starts
    st = rg[np.argsort(rg[:, 1])]
    cut = np.where(np.diff(st[:, 1]) > 500)[0] + 1
    spans, blk, strm = [], [], []
    for g in np.split(st, cut):
        spans.append((g[:, 3].max() - g[:, 1].min()) / 100)
        blk.append(np.mean(g[:, 3] - g[:, 1]) / 100)
        strm.append(np.mean(g[:, 2] - g[:, 1]) / 100)
    n = np.array([len(g) for g in np.split(st, cut)])
    for nb in sorted(set(n.tolist())):
        sel = n == nb
        print(f"rowgemv {nb} blocks x {sel.sum()} launches: span {np.mean(np.array(spans)[sel]):.2f} us, "
              f"block {np.mean(np.array(blk)[sel]):.2f} us (loads+dots {np.mean(np.array(strm)[sel]):.2f})")
cmb = rec[(rec[:, 0] >> 32) == 0xFFFB].astype(np.float64)
fd = rec[(rec[:, 0] >> 32) == 0xFFFC].astype(np.float64)
if len(cmb) and len(fd):
    # per launch: first block start .. combiner end, and the combiner's drain+ticket / combine times
    print(f"attn_fd combiner: stored->ticket {np.mean(cmb[:, 6] - cmb[:, 5]) / 100:.2f} us, "
          f"combine {np.mean(cmb[:, 7] - cmb[:, 6]) / 100:.2f} us, block start->end {np.mean(cmb[:, 7] - cmb[:, 1]) / 100:.2f} us, "
          f"splits {np.mean(cmb[:, 0].astype(np.int64) & 0xFFFF):.1f}")
    st = np.sort(fd[:, 1])
    ends = np.sort(cmb[:, 7])
    # launches: cluster block starts with gaps > 20 us
    cut = np.where(np.diff(st) > 2000)[0]
    firsts = np.concatenate([[st[0]], st[cut + 1]])
    n = min(len(firsts), len(ends) // 8)
    spans = [(ends[8 * i + 7] - firsts[i]) / 100 for i in range(n)]
    print(f"attn_fd in-kernel span (first block start .. last combiner end): mean {np.mean(spans):.2f} us over {n} launches")
if os.environ.get("TS_SK"):
    for tag in sorted(set((rec[:, 0] >> 32).tolist())):
        a = rec[(rec[:, 0] >> 32) == tag].astype(np.float64)
        a = a[a[:, 5] > 0]
        if len(a):
            d = lambda i, j: np.mean(a[:, j] - a[:, i]) / 100.0
            print(f"sk N={tag}: issue {d(1, 5):.2f}  rms {d(5, 6):.2f}  stage {d(6, 7):.2f}  barrier {d(7, 2):.2f}  stream {d(2, 3):.2f} us")
launches = []
cur = None
for r in rec:
    tag = int(r[0]) >> 32
    if tag >= 0xFFF0:
        continue
    if cur is None or tag != cur["tag"] or r[1] > cur["end"]:
        cur = {"tag": tag, "rows": [], "end": 0}
        launches.append(cur)
    cur["rows"].append(r)
    cur["end"] = max(cur["end"], int(r[4]))
by = defaultdict(list)
for L in launches:
    a = np.array(L["rows"])
    t0, t1, t2, t3 = (a[:, i] for i in (1, 2, 3, 4))
    by[L["tag"]].append(((t3.max() - t0.min()), (t0.max() - t0.min()), np.mean(t1 - t0), np.mean(t2 - t1),
                         np.mean(t3 - t2), len(a), np.mean(t3 - t0)))
print(f"{'N':>7s} {'launch':>6s} {'blocks':>6s} {'span':>7s} {'disp':>6s} {'pro':>6s} {'stream':>6s} {'epi':>6s} {'blk':>6s}  (us)")
for tag, v in sorted(by.items(), key=lambda kv: -sum(x[0] for x in kv[1])):
    a = np.array(v, dtype=np.float64) / 100.0  # 100 MHz ticks -> us
    print(f"{tag:7d} {len(v):6d} {v[0][5]:6d} {a[:, 0].mean():7.2f} {a[:, 1].mean():6.2f} {a[:, 2].mean():6.2f} "
          f"{a[:, 3].mean():6.2f} {a[:, 4].mean():6.2f} {a[:, 6].mean():6.2f}")
for L in launches[:0]:
    pass
pre = defaultdict(list)
for L in launches:
    a = np.array(L["rows"]).astype(np.float64)
    if a[:, 5].min() > 0:
        pre[L["tag"]].append(np.mean(a[:, [5, 6, 2]] - a[:, [1, 5, 6]], axis=0) / 100.0)
for tag, v in pre.items():
    v = np.mean(v, axis=0)
    print(f"PRENORM N={tag}: loads+ss staged {v[0]:.2f}  rms+X' {v[1]:.2f}  barrier {v[2]:.2f} us")
if os.environ.get("TS_DETAIL"):
    tag = int(os.environ["TS_DETAIL"])
    L = [x for x in launches if x["tag"] == tag][3]
    a = np.array(L["rows"])
    t0 = (a[:, 1] - a[:, 1].min()) / 100.0
    t3 = (a[:, 4] - a[:, 1].min()) / 100.0
    order = np.argsort(t0)
    print("start-time percentiles (us):", np.percentile(t0, [0, 10, 25, 40, 50, 60, 75, 90, 100]).round(2))
    print("end-time percentiles (us):  ", np.percentile(t3, [0, 10, 25, 50, 75, 90, 100]).round(2))
    bx = (a[:, 0] & 0xffff)[order]
    print("first 40 started blocks:", bx[:40].tolist())
    print("last 40 started blocks:", bx[-40:].tolist())
    hist = np.histogram(t0, bins=20)
    print("start histogram:", hist[0].tolist(), "edges", hist[1].round(1).tolist())
