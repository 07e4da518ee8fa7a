"""ctypes wrapper of the CPU restatement (oracle/fishmi_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg -- as the checker or the timed CPU baseline, never by the product path.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "fish-speech_amd"))

from fishmi.checkpoint import (ENCODER_WINDOW, codec_encoder_tensor_shapes,  # noqa: E402
                               codec_tensor_shapes, llm_tensor_shapes)
from fishmi.config import CodecConfig, CodecConfigC, DualARConfig  # noqa: E402
from fishmi.synth import codec_rule, llm_rule  # noqa: E402

LIB_PATH = os.path.join(HERE, "_build", "liboracle.so")
_lib = None


class SamplingC(ctypes.Structure):
    _fields_ = [("temperature", ctypes.c_float), ("top_p", ctypes.c_float),
                ("top_k", ctypes.c_int), ("seed", ctypes.c_uint64), ("mask_im_end", ctypes.c_int)]


def build() -> str:
    src = os.path.join(HERE, "fishmi_oracle.c")
    if not os.path.exists(LIB_PATH) or os.path.getmtime(LIB_PATH) < os.path.getmtime(src):
        subprocess.check_call(["make", "-s", "-C", HERE])
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        build()
        L = ctypes.CDLL(LIB_PATH)
        vp, i64, f32p, i32p = ctypes.c_void_p, ctypes.c_int64, ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_int32)
        L.orc_last_error.restype = ctypes.c_char_p
        L.orc_threads.restype = ctypes.c_int
        L.orc_llm_create.restype = vp
        L.orc_llm_create.argtypes = [vp, ctypes.c_int]
        L.orc_llm_set_tensor.argtypes = [vp, ctypes.c_char_p, f32p, i64]
        L.orc_llm_synth_tensor.argtypes = [vp, ctypes.c_char_p, i64, ctypes.c_uint64, ctypes.c_float, ctypes.c_int]
        L.orc_llm_reset.argtypes = [vp]
        L.orc_llm_forward.argtypes = [vp, i32p, ctypes.c_int, ctypes.c_int, f32p, f32p]
        L.orc_llm_fast.argtypes = [vp, f32p, ctypes.c_int, ctypes.c_int, f32p]
        L.orc_llm_generate.argtypes = [vp, i32p, ctypes.c_int, ctypes.c_int, ctypes.POINTER(SamplingC), i32p]
        L.orc_llm_free.argtypes = [vp]
        L.orc_logits_to_probs.argtypes = [f32p, ctypes.c_int, ctypes.c_float, ctypes.c_float, ctypes.c_int, ctypes.c_int, f32p]
        L.orc_sample.argtypes = [f32p, ctypes.c_int, ctypes.c_float, ctypes.c_float, ctypes.c_int, ctypes.c_int,
                                 ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32]
        L.orc_codec_create.restype = vp
        L.orc_codec_create.argtypes = [vp]
        L.orc_codec_set_tensor.argtypes = [vp, ctypes.c_char_p, f32p, i64]
        L.orc_codec_synth_tensor.argtypes = [vp, ctypes.c_char_p, i64, ctypes.c_uint64, ctypes.c_float, ctypes.c_int]
        L.orc_codec_decode.argtypes = [vp, i32p, ctypes.c_int, f32p, f32p]
        L.orc_codec_free.argtypes = [vp]
        L.orc_codec_encode.argtypes = [vp, f32p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, i32p,
                                       f32p, f32p]
        _lib = L
    return _lib


def _f32p(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))


def _i32p(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))


def _check(rc):
    if rc < 0:
        raise RuntimeError(lib().orc_last_error().decode())
    return rc


def threads() -> int:
    return lib().orc_threads()


class OracleLLM:
    def __init__(self, cfg: DualARConfig, bf16: bool):
        self.cfg, self.bf16 = cfg, bf16
        self._c = cfg.to_c()
        self.h = lib().orc_llm_create(ctypes.byref(self._c), int(bf16))

    def __del__(self):
        if getattr(self, "h", None):
            lib().orc_llm_free(self.h)
            self.h = None

    def load(self, weights):
        for name, t in weights.items():
            a = np.ascontiguousarray(t.as_f32().reshape(-1))
            _check(lib().orc_llm_set_tensor(self.h, name.encode(), _f32p(a), a.size))

    def synth(self, seed: int, log2_half: int = 5):
        for name, shape in llm_tensor_shapes(self.cfg).items():
            c, e = llm_rule(name, log2_half)
            _check(lib().orc_llm_synth_tensor(self.h, name.encode(), int(np.prod(shape)), seed, c, e))

    def reset(self):
        _check(lib().orc_llm_reset(self.h))

    def forward(self, tokens: np.ndarray, pos0: int):
        tok = np.ascontiguousarray(tokens, dtype=np.int32)
        S = tok.shape[1]
        lg = np.zeros(self.cfg.vocab_size, np.float32)
        hid = np.zeros(self.cfg.fast_dim, np.float32)
        _check(lib().orc_llm_forward(self.h, _i32p(tok), S, pos0, _f32p(lg), _f32p(hid)))
        return lg, hid

    def fast(self, hidden=None, code: int = -1, pos: int = 0, logits=True):
        out = np.zeros(self.cfg.codebook_size, np.float32)
        hp = _f32p(np.ascontiguousarray(hidden, np.float32)) if hidden is not None else None
        if hidden is not None:
            keep = np.ascontiguousarray(hidden, np.float32)
            hp = _f32p(keep)
        _check(lib().orc_llm_fast(self.h, hp, code, pos, _f32p(out) if logits else None))
        return out if logits else None

    def generate(self, prompt: np.ndarray, max_new: int, temperature=0.7, top_p=0.9, top_k=1,
                 seed=0, mask_im_end=False):
        p = np.ascontiguousarray(prompt, dtype=np.int32)
        C1, T = p.shape
        mx = max_new if (max_new and T + max_new <= self.cfg.max_seq_len) else self.cfg.max_seq_len - T
        out = np.zeros((C1, mx), np.int32)
        sp = SamplingC(temperature, top_p, top_k, seed, int(bool(mask_im_end)))
        n = _check(lib().orc_llm_generate(self.h, _i32p(p), T, max_new, ctypes.byref(sp), _i32p(out)))
        return out[:, :n]

    @staticmethod
    def last_generate_timing():
        """(prompt pass + first frame seconds, remaining frames seconds) of the last generate."""
        a, b = ctypes.c_double(), ctypes.c_double()
        lib().orc_llm_gen_timing(ctypes.byref(a), ctypes.byref(b))
        return a.value, b.value


def logits_to_probs(logits, temperature, top_p, top_k, bf16=True):
    lg = np.ascontiguousarray(logits, np.float32)
    out = np.zeros_like(lg)
    lib().orc_logits_to_probs(_f32p(lg), lg.size, temperature, top_p, top_k, int(bf16), _f32p(out))
    return out


def sample(logits, temperature, top_p, top_k, seed, step, draw, bf16=True):
    lg = np.ascontiguousarray(logits, np.float32)
    return lib().orc_sample(_f32p(lg), lg.size, temperature, top_p, top_k, int(bf16), seed, step, draw)


class OracleCodec:
    def __init__(self, cfg: CodecConfig):
        self.cfg = cfg
        self._c = cfg.to_c()
        self.h = lib().orc_codec_create(ctypes.byref(self._c))

    def __del__(self):
        if getattr(self, "h", None):
            lib().orc_codec_free(self.h)
            self.h = None

    def load(self, weights):
        for name, t in weights.items():
            a = np.ascontiguousarray(t.as_f32().reshape(-1))
            _check(lib().orc_codec_set_tensor(self.h, name.encode(), _f32p(a), a.size))

    def synth(self, seed: int):
        for name, shape in codec_tensor_shapes(self.cfg).items():
            c, e = codec_rule(name)
            _check(lib().orc_codec_synth_tensor(self.h, name.encode(), int(np.prod(shape)), seed, c, e))

    def synth_encoder(self, seed: int, encoder_dim: int, enc_layers):
        for name, shape in codec_encoder_tensor_shapes(self.cfg, encoder_dim, enc_layers).items():
            c, e = codec_rule(name)
            _check(lib().orc_codec_synth_tensor(self.h, name.encode(), int(np.prod(shape)), seed, c, e))

    def encode(self, audio: np.ndarray, encoder_dim: int, enc_layers: int, taps=False):
        """DAC.encode (modded_dac.py:874-923): -> codes (nq+1, T) [, z_enc (D, 4T), z_pre (D, T)]."""
        a = np.ascontiguousarray(audio, np.float32).reshape(-1)
        T = (a.size + self.cfg.hop - 1) // self.cfg.hop
        codes = np.zeros((self.cfg.n_codebooks + 1, T), np.int32)
        ze = np.zeros((self.cfg.latent, 4 * T), np.float32) if taps else None
        zp = np.zeros((self.cfg.latent, T), np.float32) if taps else None
        n = _check(lib().orc_codec_encode(self.h, _f32p(a), a.size, encoder_dim, enc_layers, ENCODER_WINDOW,
                                          _i32p(codes), _f32p(ze) if taps else None, _f32p(zp) if taps else None))
        assert n == T
        return (codes, ze, zp) if taps else codes

    def decode(self, codes: np.ndarray, want_latent=False):
        cd = np.ascontiguousarray(codes, np.int32)
        T = cd.shape[-1]
        wave = np.zeros(self.cfg.hop * T, np.float32)
        lat = np.zeros(self.cfg.latent * 4 * T, np.float32) if want_latent else None
        n = _check(lib().orc_codec_decode(self.h, _i32p(cd), T, _f32p(wave),
                                          _f32p(lat) if want_latent else None))
        assert n == self.cfg.hop * T
        return (wave, lat.reshape(self.cfg.latent, 4 * T)) if want_latent else wave


def _bind_ops():
    L = lib()
    f32p = ctypes.POINTER(ctypes.c_float)
    L.orc_op_rmsnorm.argtypes = [f32p, f32p, ctypes.c_int, ctypes.c_int, ctypes.c_float, ctypes.c_int, f32p]
    L.orc_op_headnorm.argtypes = [f32p, f32p, ctypes.c_int, ctypes.c_int, ctypes.c_float, ctypes.c_int, f32p]
    L.orc_op_rope_table.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_float, f32p]
    L.orc_op_rope.argtypes = [f32p, f32p, ctypes.c_int, ctypes.c_int, ctypes.c_int, f32p]
    return L


def op_rmsnorm(x, w, eps, bf16=True, head=False):
    L = _bind_ops()
    x = np.ascontiguousarray(x, np.float32)
    w = np.ascontiguousarray(w, np.float32)
    n = x.shape[-1]
    y = np.zeros_like(x)
    fn = L.orc_op_headnorm if head else L.orc_op_rmsnorm
    fn(_f32p(x), _f32p(w), x.size // n, n, eps, int(bf16), _f32p(y))
    return y


def op_rope_table(S, hd, base):
    L = _bind_ops()
    t = np.zeros((S, hd // 2, 2), np.float32)
    L.orc_op_rope_table(S, hd, base, _f32p(t))
    return t


def op_rope(x, tab_rows, bf16=True):
    """x [..., rows, hd]; tab_rows [rows, hd] broadcast over leading dims."""
    L = _bind_ops()
    x = np.ascontiguousarray(x, np.float32)
    hd = x.shape[-1]
    rows = x.size // hd
    tabs = np.ascontiguousarray(np.broadcast_to(tab_rows.reshape(-1, hd), (rows, hd)) if tab_rows.size // hd == rows
                                else tab_rows, np.float32)
    y = np.zeros_like(x)
    L.orc_op_rope(_f32p(x), _f32p(tabs), rows, hd, int(bf16), _f32p(y))
    return y


# ---- weight-only int4 (tools/llama/quantize.py:57-160), numpy restatement -------------------
def _bf16r(x):
    """round-to-nearest-even to bf16, as float32 values (torch's bf16 op results)."""
    b = np.ascontiguousarray(x, np.float32).view(np.uint32)
    r = ((b + 0x7FFF + ((b >> 16) & 1)) & 0xFFFF0000).astype(np.uint32)
    return r.view(np.float32)


def int4_group_quantize(w, gs):
    """get_group_qparams + group_quantize_tensor_from_qparams (quantize.py:57-127) on bf16-valued w
    [N][K], in torch's bf16 arithmetic (fp32 op, bf16 result): (q [N][K] uint8, scale, zero [N][K/gs]
    as float32 of bf16 values), and the affine dequantisation (q - 8) * scale + zero in fp32
    (group_dequantize_tensor_from_qparams, quantize.py:130-152 with float scales)."""
    w = np.ascontiguousarray(w, np.float32)
    N, K = w.shape
    g = w.reshape(N, K // gs, gs)
    mx, mn = g.max(-1), g.min(-1)
    d = np.maximum(_bf16r(mx - mn), _bf16r(np.float32(1e-6)))
    sc = _bf16r(d / np.float32(15))
    s8 = _bf16r(sc * np.float32(8))
    zr = _bf16r(mn + s8)
    lo = _bf16r(zr - s8)
    x = _bf16r(_bf16r(g - lo[..., None]) / sc[..., None])
    q = np.clip(np.rint(x), 0, 15).astype(np.uint8)
    dq = ((q.astype(np.float64) - 8) * sc[..., None].astype(np.float64) + zr[..., None]).astype(np.float32)
    return q.reshape(N, K), sc, zr, dq.reshape(N, K)
