"""Shared parity checks for the bf16 decode path (imported by the GPU test modules).

The bf16 bound: the build's bf16 error against the reference's fp32 logits (same weights, same
teacher-forced stream) may be at most BF16_RATIO x the reference's OWN bf16-vs-fp32 error, in RMS
and in max, over the whole stream; top-1 must agree wherever the fp32 top-1/top-2 margin exceeds
twice the larger of the bf16 errors (both builds' argmax are then pinned)."""
import numpy as np

BF16_RATIO = 1.5


def bits_to_f32(b):
    return (np.asarray(b, dtype=np.uint16).astype(np.uint32) << 16).view(np.float32)


def margin(v):
    s = np.sort(v[np.isfinite(v)])[::-1]
    return s[0] - s[1]


def error_stats(ours, ref, tru):
    e_o, e_r = np.abs(ours - tru), np.abs(ref - tru)
    return dict(rms=float(np.sqrt((e_o ** 2).mean())), rms_ref=float(np.sqrt((e_r ** 2).mean())),
                max=float(e_o.max()), max_ref=float(e_r.max()))


def assert_within(stats: dict):
    for tag, d in stats.items():
        assert d["rms"] <= BF16_RATIO * d["rms_ref"] + 1e-6, (tag, d)
        assert d["max"] <= BF16_RATIO * d["max_ref"] + 1e-6, (tag, d)


def bf16_vs_reference(slow, fast, rs, rf, ts, tf, rows=None):
    """slow (n, V or len(rows)) and fast (n, C', cb) logits from the build; rs/rf the reference's
    bf16 logits, ts/tf its fp32 logits of the same teacher-forced stream (slow restricted to `rows`
    when given).  Asserts the bound above and returns the error statistics."""
    n = slow.shape[0]
    rs, rf, ts, tf = rs[:n], rf[:n], ts[:n], tf[:n]
    if rows is not None:
        slow = slow[:, rows]
    fin = np.isfinite(ts)
    assert np.array_equal(np.isfinite(slow), fin) and np.array_equal(np.isfinite(rs), fin)
    out = {"slow": error_stats(slow[fin], rs[fin], ts[fin]),
           "fast": error_stats(fast.ravel(), rf.ravel(), tf.ravel())}
    print("bf16 error vs the reference's fp32 logits (build | reference's own bf16):", out)
    assert_within(out)
    tol = 2 * max(out["slow"]["max"], out["slow"]["max_ref"], out["fast"]["max"], out["fast"]["max_ref"])
    checked = 0
    for i in range(n):
        t = np.where(fin[i], ts[i], -np.inf)
        if margin(t) > tol:
            checked += 1
            assert np.argmax(np.where(fin[i], slow[i], -np.inf)) == np.argmax(t), i
        for c in range(tf.shape[1]):
            if margin(tf[i, c]) > tol:
                checked += 1
                assert np.argmax(fast[i, c]) == np.argmax(tf[i, c]), (i, c)
    out["top1_checked"] = checked
    return out


def bf16_vs_golden(slow, fast, g, rows=None):
    """bf16_vs_reference against a golden holding slow_logits / fast_logits (the reference's bf16,
    as fp32 arrays or as *_bits bf16 patterns) and slow_logits_f32 / fast_logits_f32."""
    rs = bits_to_f32(g["slow_logits_bits"]) if "slow_logits_bits" in g else g["slow_logits"]
    rf = bits_to_f32(g["fast_logits_bits"]) if "fast_logits_bits" in g else g["fast_logits"]
    return bf16_vs_reference(slow, fast, rs, rf, g["slow_logits_f32"], g["fast_logits_f32"], rows)
