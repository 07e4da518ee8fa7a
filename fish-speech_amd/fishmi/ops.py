"""Per-op parity hooks of libfishmi (include/fishmi.h, fm_op_*): one production kernel of the decode
path on caller operands, used by tests/test_gpu_ops.py against the reference's per-op goldens.

Reference semantics pinned (file:line in PoTaTo-Mika/fish-speech):
  rmsnorm   RMSNorm.forward            llama.py:989-1000   (fp32 normalise, round, * weight, round)
  qk_rope   nn.RMSNorm(head_dim) +     llama.py:861-863, 900-902 (one rounding incl. the weight)
            apply_rotary_emb           llama.py:1025-1037 (bf16 cos/sin table, fp32 rotate, round)
  embed     forward_generate embedding llama.py:399-420
  rope_table precompute_freqs_cis      llama.py:1003-1022
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import native

MODES = {"prologue_norm": 0, "prologue_prenorm": 1, "row_kernel": 2}


def _prec(precision: str) -> int:
    return native.FM_PREC_BF16 if precision == "bf16" else native.FM_PREC_FP32


def rmsnorm(x, w, eps, precision="bf16", mode="prologue_prenorm", device=0):
    x = np.ascontiguousarray(x, np.float32)
    R, d = x.reshape(-1, x.shape[-1]).shape
    w = np.ascontiguousarray(w, np.float32)
    y = np.zeros((R, d), np.float32)
    native.check(native.lib().fm_op_rmsnorm(device, _prec(precision), MODES[mode], native.f32p(x),
                                            native.f32p(w), R, d, float(eps), native.f32p(y)))
    return y.reshape(x.shape)


def qk_rope(qkv_row, nh, nkv, hd, pos, rope_base, qn=None, kn=None, eps=1e-6, precision="bf16",
            kernel="slow", device=0):
    """q (nh, hd) and k (nkv, hd) after qk-norm (if weights given) and RoPE at `pos`, as computed
    inside a decode attention kernel: "fd" attn_fd (the slow model's production kernel), "slow"
    attn_decode2, "slow3" attn_dec3, "fast" fast_attn2."""
    raw = np.ascontiguousarray(qkv_row, np.float32).reshape(-1)
    assert raw.size == (nh + 2 * nkv) * hd
    qk = qn is not None
    qn_ = np.ascontiguousarray(qn if qk else np.ones(hd), np.float32)
    kn_ = np.ascontiguousarray(kn if qk else np.ones(hd), np.float32)
    q = np.zeros(nh * hd, np.float32)
    k = np.zeros(nkv * hd, np.float32)
    kid = {"slow": 0, "fast": 1, "slow3": 2, "fd": 3}[kernel]  # attn_decode2 / fast_attn2 / attn_dec3 / attn_fd
    native.check(native.lib().fm_op_qk_rope(device, _prec(precision), kid,
                                            native.f32p(raw), nh, nkv, hd, native.f32p(qn_), native.f32p(kn_),
                                            int(qk), float(eps), float(rope_base), int(pos), native.f32p(q),
                                            native.f32p(k)))
    return q.reshape(nh, hd), k.reshape(nkv, hd)


ATTN_KERNELS = {"slow": 0, "slow3": 2, "fd": 3}  # attn_decode2 / attn_dec3 / attn_fd


def decode_attn(qkv, nh, nkv, hd, pos, kcache, vcache, rope_base, qn=None, kn=None, eps=1e-6,
                precision="bf16", kernel="fd", min_split=32, device=0):
    """The slow decode attention (llama.py:883-945) on R rows: qkv (R, (nh+2nkv)*hd) raw projections,
    pos (R,), kcache / vcache (R, nkv, S, hd) holding rows < pos[r].  Returns (out (R, nh, hd),
    kcache, vcache after the kernel's write of row pos[r])."""
    raw = np.ascontiguousarray(qkv, np.float32)
    R = raw.shape[0]
    assert raw.shape[1] == (nh + 2 * nkv) * hd
    kc = np.ascontiguousarray(kcache, np.float32)
    vc = np.ascontiguousarray(vcache, np.float32)
    S = kc.shape[2]
    assert kc.shape == (R, nkv, S, hd) and vc.shape == kc.shape
    p = np.ascontiguousarray(pos, np.int32)
    qk = qn is not None
    qn_ = np.ascontiguousarray(qn if qk else np.ones(hd), np.float32)
    kn_ = np.ascontiguousarray(kn if qk else np.ones(hd), np.float32)
    out = np.zeros((R, nh, hd), np.float32)
    kco = np.zeros_like(kc)
    vco = np.zeros_like(vc)
    native.check(native.lib().fm_op_decode_attn(device, _prec(precision), ATTN_KERNELS[kernel], native.f32p(raw), R,
                                                nh, nkv, hd, native.f32p(qn_), native.f32p(kn_), int(qk), float(eps),
                                                float(rope_base), native.i32p(p), native.f32p(kc), native.f32p(vc), S,
                                                int(min_split), native.f32p(out), native.f32p(kco), native.f32p(vco)))
    return out, kco, vco


def prompt_attn(q, nh, nkv, hd, pos0, kcache, vcache, precision="bf16", kernel="flash", device=0):
    """Causal attention of R prompt rows (positions pos0 .. pos0+R-1, one slot) over caches
    kcache / vcache (nkv, S, hd): q (R, nh*hd).  kernel "flash" (attn_prefill_kernel) or "split"."""
    qq = np.ascontiguousarray(q, np.float32)
    R = qq.shape[0]
    kc = np.ascontiguousarray(kcache, np.float32)
    vc = np.ascontiguousarray(vcache, np.float32)
    S = kc.shape[1]
    assert qq.shape[1] == nh * hd and kc.shape == (nkv, S, hd) and vc.shape == kc.shape
    out = np.zeros((R, nh, hd), np.float32)
    native.check(native.lib().fm_op_prompt_attn(device, _prec(precision), {"split": 0, "flash": 1}[kernel],
                                                native.f32p(qq), R, nh, nkv, hd, int(pos0), native.f32p(kc),
                                                native.f32p(vc), S, native.f32p(out)))
    return out


def embed(tok, emb, cbemb, num_codebooks, codebook_size, semantic_begin_id, semantic_end_id, scale,
          precision="bf16", device=0):
    """tok: (R, C+1) rows (row r = one position's [text/semantic token, codes...])."""
    t = np.ascontiguousarray(tok, np.int32)
    emb = np.ascontiguousarray(emb, np.float32)
    cbemb = np.ascontiguousarray(cbemb, np.float32)
    R, d = t.shape[0], emb.shape[1]
    x = np.zeros((R, d), np.float32)
    native.check(native.lib().fm_op_embed(device, _prec(precision), native.i32p(t), R, native.f32p(emb),
                                          emb.shape[0], native.f32p(cbemb), d, num_codebooks, codebook_size,
                                          semantic_begin_id, semantic_end_id, int(scale), native.f32p(x)))
    return x


def rope_table(seq_len, head_dim, base):
    out = np.zeros((seq_len, head_dim // 2, 2), np.float32)
    native.check(native.lib().fm_rope_table(seq_len, head_dim, float(base), native.f32p(out)))
    return out


def quant4(w, gs, x=None, device=0):
    """fm_op_quant4: (q [N][K] uint8, scale [N][K/gs], zero [N][K/gs], dequantised w [N][K]) from the
    device int4 quantizer, and with x ([R][K]) the decode GEMV on the dequantised bf16 weights and on
    the streamed 4-bit codes: (..., y_bf16 [R][N], y_q4 [R][N] or None)."""
    w = np.ascontiguousarray(w, np.float32)
    N, K = w.shape
    q = np.zeros((N, K), np.uint8)
    sc = np.zeros((N, K // gs), np.float32)
    zr = np.zeros((N, K // gs), np.float32)
    wd = np.zeros((N, K), np.float32)
    if x is None:
        native.check(native.lib().fm_op_quant4(device, native.f32p(w), N, K, gs,
                                               q.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)),
                                               native.f32p(sc), native.f32p(zr), native.f32p(wd), None, 0, None, None))
        return q, sc, zr, wd
    x = np.ascontiguousarray(x, np.float32).reshape(-1, K)
    R = x.shape[0]
    yb = np.zeros((R, N), np.float32)
    y4 = np.zeros((R, N), np.float32) if (gs % 128 == 0 and K % 128 == 0) else None
    native.check(native.lib().fm_op_quant4(device, native.f32p(w), N, K, gs,
                                           q.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), native.f32p(sc),
                                           native.f32p(zr), native.f32p(wd), native.f32p(x), R,
                                           native.f32p(y4) if y4 is not None else None, native.f32p(yb)))
    return q, sc, zr, wd, yb, y4
