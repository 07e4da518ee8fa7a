"""Are the K / V rows the decode path writes bit-identical to the ones the prompt pass writes for the
same positions?  (the bf16 prefix-reuse divergence.)

generate_long with reuse_prefix keeps the slot's KV of the previous batch: its prompt rows (written by
the prompt pass, fm_llm_prefill) and its fed columns (written by the decode frames).  The re-prefill
flow (the reference's, inference.py:620-724) recomputes all of them with the prompt pass.  The two
flows give the same codes only if those rows agree bit for bit.

A: prefill(prompt) + n-1 teacher-forced decode frames (the columns of the llm_a bf16 golden);
B: one prefill of prompt ++ the same n-1 columns.
Then the slow caches of slot 0 are read (fm_llm_debug_vec "kc" / "vc") and compared per layer over
the decode-written positions [T, T+n-1).  Repeated under knob settings that swap the decode kernels
(row-block GEMV off, tile GEMV variants, attention kernel) to name the op whose bits differ.

    python scripts/kv_identity_probe.py [precision]
"""
import os
import shutil
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.environ.get("FISHMI_PKG", os.path.join(ROOT, "fish-speech_amd")))
GOLD = os.path.join(ROOT, "tests", "golden")

from fishmi import native  # noqa: E402
from fishmi.llm import DualARModel  # noqa: E402


def ckpt():
    d = tempfile.mkdtemp()
    shutil.copytree(os.path.join(GOLD, "llm_a"), os.path.join(d, "c"))
    return os.path.join(d, "c")


def read_cache(m, name, layer, n):
    out = np.zeros(n, np.float32)
    native.check(native.lib().fm_llm_debug_vec(m.h, name.encode(), layer, native.f32p(out), n))
    return out


def caches(m):
    d = m.cfg
    S = d.max_seq_len
    n = d.n_local_heads * S * d.head_dim
    res = []
    for l in range(d.n_layer):
        k = read_cache(m, "kc", l, n).reshape(d.n_local_heads, S, d.head_dim)
        v = read_cache(m, "vc", l, n).reshape(d.n_local_heads, S, d.head_dim)
        res.append((k, v))
    return res


def ulps(a, b):
    ia = a.view(np.uint32).astype(np.int64)
    ib = b.view(np.uint32).astype(np.int64)
    return np.abs(ia - ib) >> 16


def run(m, prompt, cols, label):
    T, n = prompt.shape[1], cols.shape[1]
    sp = m.sampling(top_k=1)
    m.force(0, cols[:, 0])
    m.prefill(0, prompt, sp)
    for i in range(1, n):
        m.force(0, cols[:, i])
        m.decode([0])
    m.force(0, None)
    a = caches(m)
    # the same decode again from a fresh prefill: run-to-run determinism of the decode-written rows
    m.force(0, cols[:, 0])
    m.prefill(0, prompt, sp)
    for i in range(1, n):
        m.force(0, cols[:, i])
        m.decode([0])
    m.force(0, None)
    a2 = caches(m)
    rep = sum(int((x[0][:, T:T + n - 1] != y[0][:, T:T + n - 1]).sum() + (x[1][:, T:T + n - 1] != y[1][:, T:T + n - 1]).sum())
              for x, y in zip(a, a2))
    print(f"[{label}] decode rows differing between two identical runs: {rep}")
    full = np.concatenate([prompt, cols[:, : n - 1]], axis=1)
    m.force(0, cols[:, n - 1])
    m.prefill(0, full, sp)
    m.force(0, None)
    b = caches(m)
    first = None
    lines = []
    for l, ((ka, va), (kb, vb)) in enumerate(zip(a, b)):
        pr = slice(0, T)
        dr = slice(T, T + n - 1)
        kp = int((ka[:, pr] != kb[:, pr]).sum())
        kd = (ka[:, dr] != kb[:, dr])
        vd = (va[:, dr] != vb[:, dr])
        mk = int(ulps(ka[:, dr], kb[:, dr]).max()) if kd.any() else 0
        mv = int(ulps(va[:, dr], vb[:, dr]).max()) if vd.any() else 0
        pos_k = sorted(set((np.nonzero(kd)[1] + T).tolist()))[:6]
        lines.append(f"    layer {l}: prompt rows differ {kp}; decode rows K {int(kd.sum())} (max {mk} ulp, "
                     f"positions {pos_k}) V {int(vd.sum())} (max {mv} ulp)")
        if first is None and (kd.any() or vd.any()):
            first = l
    print(f"[{label}] first layer with differing decode-written rows: {first}")
    print("\n".join(lines))
    return first


def engine_flows(prec):
    """generate_long with reuse_prefix vs whole-conversation re-prefill on the engine golden's request
    (tests/test_gpu_engine.py::test_prefix_reuse_equals_reprefill): codes per batch."""
    from fishmi import engine

    g = np.load(os.path.join(GOLD, "engine.npz"))
    d = ckpt()
    for f in ("tokenizer.json", "tokenizer_config.json"):
        shutil.copy(os.path.join(GOLD, "tok_tiny", f), os.path.join(d, f))
    m = DualARModel.from_pretrained(d, device=0, precision=prec, max_length=2560)
    req = dict(device="cuda", max_new_tokens=7, text=str(g["text"]), top_p=0.9, repetition_penalty=1.1,
               temperature=0.7, compile=False, iterative_prompt=True, chunk_length=30,
               prompt_tokens=[g["ptok0"], g["ptok1"]], prompt_text=["ref a", "<|speaker:1|>ref b"], top_k=1)
    for order in (("reuse", "full", "reuse"),):
        res = {}
        for i, mode in enumerate(order):
            res[f"{mode}{i}"] = [o.codes for o in engine.generate_long(model=m, reuse_prefix=(mode == "reuse"), **req)
                                 if o.action == "sample"]
        keys = list(res)
        for b in range(len(res[keys[0]])):
            same = [bool(np.array_equal(res[keys[0]][b], res[k][b])) for k in keys[1:]]
            print(f"  batch {b}: {keys[0]} == {keys[1:]}: {same}; first column row0 "
                  + " ".join(str(res[k][b][0, :6].tolist()) for k in keys))
    m.close()


def main():
    if os.environ.get("ENGINE"):
        engine_flows(sys.argv[1] if len(sys.argv) > 1 else "bf16")
        return
    prec = sys.argv[1] if len(sys.argv) > 1 else "bf16"
    g = np.load(os.path.join(GOLD, "llm_a_bf16.npz"))
    prompt = g["prompt"]
    T = prompt.shape[1]
    cols = g["seq"][:, T:T + 12]
    m = DualARModel.from_pretrained(ckpt(), device=0, precision=prec, max_length=1024, im_end_id=4)
    L = int(os.environ.get("PROMPT_LEN", T))
    if L > T:  # a longer prompt (decode attention then runs split over blocks): the prompt repeated
        prompt = np.concatenate([prompt] * (L // T + 1), axis=1)[:, :L]
        T = L
    print(f"llm_a {prec}: dim {m.cfg.dim}, layers {m.cfg.n_layer}, T {T}, {cols.shape[1]} columns")
    variants = [
        ("defaults", {}),
        ("no graph", {"__graph": 0}),
        ("rowgemv 0 (tile GEMV for wo / w2 / wqkv / heads)", {"rowgemv": 0}),
        ("rowgemv 0, kv_prefetch 0", {"rowgemv": 0, "kv_prefetch": 0}),
        ("rowgemv 0, attn_fd 0", {"rowgemv": 0, "attn_fd": 0}),
        ("rowgemv 0, fin8 0", {"rowgemv": 0, "fin8": 0}),
        ("rowgemv 0, prompt_gemm 0", {"rowgemv": 0, "prompt_gemm": 0}),
        ("prompt_gemm 0", {"prompt_gemm": 0}),
    ]
    defaults = {"rowgemv": 27, "kv_prefetch": 1, "attn_fd": 1, "fin8": 1, "prompt_gemm": 1}
    for label, knobs in variants:
        for k, v in defaults.items():
            native.tune(k, v)
        m.use_graph(True)
        for k, v in knobs.items():
            if k == "__graph":
                m.use_graph(bool(v))
            else:
                native.tune(k, v)
        try:
            run(m, prompt, cols, label)
        except Exception as e:  # a knob this model cannot take
            print(f"[{label}] error: {e}")


if __name__ == "__main__":
    main()
