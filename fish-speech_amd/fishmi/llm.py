"""Dual-AR model on libfishmi: the drop-in for DualARTransformer + decode_one_token_ar.

Mirrors the reference's seams (fish_speech/models/text2semantic/llama.py and inference.py):
  * ``DualARModel.from_pretrained(path)``  <- BaseTransformer.from_pretrained (llama.py:479-593)
  * ``model.generate(prompt, ...)``         <- inference.generate (inference.py:241-359)
  * ``model.decode_frames(slots, n)``       <- decode_n_tokens over decode_one_token_ar
                                               (inference.py:96-238), batched over slots
  * ``DecodeOneToken(model)``               <- the injected ``decode_one_token`` operator itself
                                               (inference.py:96-107, injected at :195 and :250)
  * ``model.teacher_step(...)``             <- forward_generate + forward_generate_fast
"""
from __future__ import annotations

import ctypes
import json
import os
from pathlib import Path
from typing import Optional

import numpy as np

from . import native
from .checkpoint import Tensor, llm_tensor_shapes, load_llm_weights
from .config import DualARConfig
from .synth import llm_rule

IM_END_TOKEN = "<|im_end|>"


def resolve_im_end_id(path) -> Optional[int]:
    """FishTokenizer.get_token_id(IM_END_TOKEN) (tokenizer.py) from tokenizer.json, offline."""
    p = Path(path)
    tj = p / "tokenizer.json"
    if tj.exists():
        with open(tj, encoding="utf-8") as f:
            data = json.load(f)
        for t in data.get("added_tokens", []):
            if t.get("content") == IM_END_TOKEN:
                return int(t["id"])
        vocab = data.get("model", {}).get("vocab", {})
        if isinstance(vocab, dict) and IM_END_TOKEN in vocab:
            return int(vocab[IM_END_TOKEN])
    return None


class DualARModel:
    def __init__(self, cfg: DualARConfig, device: int = 0, precision: str = "bf16",
                 max_slots: int = 1, quant: Optional[str] = None, groupsize: int = 128):
        if cfg.im_end_id < 0:
            raise ValueError("config.im_end_id must be set (tokenizer's <|im_end|> id)")
        self.cfg = cfg
        self.device = device
        self.precision = precision
        self.max_slots = max_slots
        self.C1 = cfg.num_codebooks + 1
        L = native.lib()
        if native.device_count() < 1:
            raise native.FishMIError("no HIP device visible; libfishmi has no CPU fallback")
        self._c = cfg.to_c()
        h = ctypes.c_void_p()
        prec = native.FM_PREC_BF16 if precision == "bf16" else native.FM_PREC_FP32
        native.check(L.fm_llm_open(ctypes.byref(self._c), device, prec, max_slots, ctypes.byref(h)))
        self.h = h
        if quant not in (None, "int8", "int4"):
            raise ValueError(f"quant must be None, 'int8' or 'int4', got {quant!r}")
        self.quant = quant
        if quant == "int8":  # WeightOnlyInt8QuantHandler.convert_for_runtime (llama.py:528-535)
            native.check(L.fm_llm_set_quant(h, native.FM_QUANT_INT8))
        elif quant == "int4":  # WeightOnlyInt4QuantHandler(model, groupsize) (llama.py:537-543), bf16 weights
            native.check(L.fm_llm_set_quant_int4(h, int(groupsize)))
        self._finalized = False
        self.tokenizer = None  # FishTokenizer when loaded from a checkpoint with tokenizer.json

    # ---- construction --------------------------------------------------------------
    @classmethod
    def from_pretrained(cls, path, device: int = 0, precision: str = "bf16", max_slots: int = 1,
                        max_length: Optional[int] = None, im_end_id: Optional[int] = None,
                        quant: Optional[str] = None, groupsize: int = 128):
        """quant="int4": quantize the bf16 checkpoint's linears at load (the reference's quantize.py
        --mode int4 --groupsize g, then its int4 runtime); int8 checkpoints are detected."""
        cfg = DualARConfig.from_pretrained(path)
        if max_length is not None:
            cfg.max_seq_len = max_length
        tok = None
        if (Path(path) / "tokenizer.json").exists():
            # llama.py:499-509: the tokenizer's <|semantic:i|> range overrides the config's
            from .prompt import FishTokenizer

            tok = FishTokenizer(str(path))
            if tok.semantic_end_id > 0:
                cfg.semantic_begin_id, cfg.semantic_end_id = tok.semantic_begin_id, tok.semantic_end_id
        im = im_end_id if im_end_id is not None else resolve_im_end_id(path)
        if im is None:
            raise ValueError(f"cannot resolve <|im_end|> id: no tokenizer.json in {path}; pass im_end_id")
        cfg.im_end_id = im
        weights = load_llm_weights(path)
        if any(k.endswith("scales_and_zeros") for k in weights):
            raise ValueError("int4 checkpoints hold torch's _convert_weight_to_int4pack tiles (quantize.py:239-247), "
                             "which this build does not read: load the bf16 checkpoint with quant='int4'")
        if any(t.int8 for t in weights.values()):
            if quant == "int4":
                raise ValueError("int4 quantization needs a float checkpoint, this one is int8")
            quant = "int8"
        m = cls(cfg, device, precision, max_slots, quant, groupsize)
        m.load_weights(weights)
        m.finalize()
        m.tokenizer = tok
        return m

    @classmethod
    def synthetic(cls, cfg: DualARConfig, seed: int, log2_half: int = 5, device: int = 0,
                  precision: str = "bf16", max_slots: int = 1, quant: Optional[str] = None,
                  groupsize: int = 128):
        """Seeded weights at cfg's shapes; quant="int8" quantizes the linears at finalize with
        quantize.py's per-channel rule, quant="int4" with its groupwise rule (groupsize)."""
        m = cls(cfg, device, precision, max_slots, quant, groupsize)
        m.synth(seed, log2_half)
        m.finalize()
        return m

    def load_weights(self, weights: "dict[str, Tensor]"):
        L = native.lib()
        shapes = llm_tensor_shapes(self.cfg)
        missing = [k for k in shapes if k not in weights]
        if missing:
            raise KeyError(f"checkpoint lacks {len(missing)} tensors, e.g. {missing[:3]}")
        names = list(shapes)
        if self.quant == "int8":  # int8 checkpoints carry "<module>.scales" beside the int8 weights
            names += [k for k in weights if k.endswith(".scales")]
        elif any(weights[k].int8 for k in names):
            raise ValueError("int8 weights need DualARModel(..., quant='int8')")
        for name in names:
            t = weights[name]
            a = np.ascontiguousarray(t.data)
            if t.int8:
                dt = native.FM_DT_I8
            else:
                dt = native.FM_DT_BF16 if t.bf16 else native.FM_DT_F32
                if not t.bf16:
                    a = np.ascontiguousarray(a, dtype=np.float32)
            native.check(L.fm_llm_set_tensor(self.h, name.encode(), a.ctypes.data_as(ctypes.c_void_p),
                                             dt, a.size))

    def synth(self, seed: int, log2_half: int = 5):
        L = native.lib()
        for name, shape in llm_tensor_shapes(self.cfg).items():
            c, e = llm_rule(name, log2_half)
            native.check(L.fm_llm_synth_tensor(self.h, name.encode(), int(np.prod(shape)), seed, c, e))

    def finalize(self):
        native.check(native.lib().fm_llm_finalize(self.h))
        self._finalized = True

    def close(self):
        if getattr(self, "h", None):
            native.lib().fm_llm_close(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- decode ----------------------------------------------------------------------
    @staticmethod
    def sampling(temperature=0.7, top_p=0.9, top_k=30, seed=0, mask_im_end=False):
        return native.SamplingC(float(temperature), float(top_p), int(top_k), int(seed) & (2**64 - 1),
                                int(bool(mask_im_end)))

    def prefill(self, slot: int, prompt: np.ndarray, sampling, pos0: int = 0) -> np.ndarray:
        """Prefill `prompt` into `slot` (pos0 > 0: after the slot's cached positions [0, pos0),
        fm_llm_prefill_at); returns the first emitted column (C+1,)."""
        p = np.ascontiguousarray(prompt, dtype=np.int32)
        assert p.shape[0] == self.C1
        col = np.zeros(self.C1, np.int32)
        if pos0:
            native.check(native.lib().fm_llm_prefill_at(self.h, slot, native.i32p(p), p.shape[1], int(pos0),
                                                        ctypes.byref(sampling), native.i32p(col)))
        else:
            native.check(native.lib().fm_llm_prefill(self.h, slot, native.i32p(p), p.shape[1],
                                                     ctypes.byref(sampling), native.i32p(col)))
        return col

    def prefill_batch(self, slots, prompts, samplings) -> np.ndarray:
        """Prefill several requests together (fm_llm_prefill_batch): slots distinct, prompts (C+1, T_i),
        one sampling record each; returns the first columns (n, C+1), as n prefill() calls would."""
        n = len(slots)
        assert n == len(prompts) == len(samplings) and n >= 1
        s = np.ascontiguousarray(slots, dtype=np.int32)
        ps = [np.ascontiguousarray(p, dtype=np.int32) for p in prompts]
        assert all(p.shape[0] == self.C1 for p in ps)
        T = np.array([p.shape[1] for p in ps], np.int32)
        tok = np.ascontiguousarray(np.concatenate([p.ravel() for p in ps]))
        sp = (native.SamplingC * n)(*samplings)
        out = np.zeros((n, self.C1), np.int32)
        native.check(native.lib().fm_llm_prefill_batch(self.h, n, native.i32p(s), native.i32p(tok), native.i32p(T),
                                                       sp, native.i32p(out)))
        return out

    def decode(self, slots) -> np.ndarray:
        s = np.ascontiguousarray(slots, dtype=np.int32)
        out = np.zeros((s.size, self.C1), np.int32)
        native.check(native.lib().fm_llm_decode(self.h, native.i32p(s), s.size, native.i32p(out)))
        return out

    def decode_frames(self, slots, nframes: int) -> np.ndarray:
        """decode_n_tokens without the per-frame host sync: (nframes, n, C+1) columns."""
        s = np.ascontiguousarray(slots, dtype=np.int32)
        out = np.zeros((nframes, s.size, self.C1), np.int32)
        native.check(native.lib().fm_llm_decode_frames(self.h, native.i32p(s), s.size, nframes,
                                                       native.i32p(out)))
        return out

    def generate(self, prompt: np.ndarray, max_new_tokens: int, temperature=0.7, top_p=0.9,
                 top_k=30, seed=0, slot=0, mask_im_end=False) -> np.ndarray:
        """inference.generate: returns the emitted columns (C+1, n) (seq[:, T:])."""
        p = np.ascontiguousarray(prompt, dtype=np.int32)
        T = p.shape[1]
        mx = max_new_tokens if (max_new_tokens and T + max_new_tokens <= self.cfg.max_seq_len) \
            else self.cfg.max_seq_len - T
        out = np.zeros((self.C1, mx), np.int32)
        n = ctypes.c_int(0)
        sp = self.sampling(temperature, top_p, top_k, seed, mask_im_end)
        native.check(native.lib().fm_llm_generate(self.h, slot, native.i32p(p), T, mx,
                                                  ctypes.byref(sp), native.i32p(out), ctypes.byref(n)))
        return out[:, : n.value]

    def generate_at(self, suffix: np.ndarray, pos0: int, max_new_tokens: int, temperature=0.7, top_p=0.9,
                    top_k=30, seed=0, slot=0, mask_im_end=False) -> np.ndarray:
        """generate() whose prompt = the slot's cached positions [0, pos0) + `suffix`
        (fm_llm_generate_at: only the suffix is prefilled).  Returns the emitted columns."""
        p = np.ascontiguousarray(suffix, dtype=np.int32)
        T = p.shape[1]
        mx = max_new_tokens if (max_new_tokens and pos0 + T + max_new_tokens <= self.cfg.max_seq_len) \
            else self.cfg.max_seq_len - pos0 - T
        out = np.zeros((self.C1, mx), np.int32)
        n = ctypes.c_int(0)
        sp = self.sampling(temperature, top_p, top_k, seed, mask_im_end)
        native.check(native.lib().fm_llm_generate_at(self.h, slot, native.i32p(p), T, int(pos0), mx,
                                                     ctypes.byref(sp), native.i32p(out), ctypes.byref(n)))
        return out[:, : n.value]

    def slot_pos(self, slot: int = 0) -> int:
        """Positions of `slot` whose KV is written (its prompt + the columns fed back so far)."""
        v = ctypes.c_int(0)
        native.check(native.lib().fm_llm_slot_pos(self.h, slot, ctypes.byref(v)))
        return v.value

    def teacher_step(self, x: np.ndarray, pos0: int, next_col=None, slot: int = 0):
        xx = np.ascontiguousarray(x, dtype=np.int32)
        lg = np.zeros(self.cfg.vocab_size, np.float32)
        hid = np.zeros(self.cfg.fast_dim, np.float32)
        fl = np.zeros((self.cfg.num_codebooks - 1, self.cfg.codebook_size), np.float32)
        nc = np.ascontiguousarray(next_col, dtype=np.int32) if next_col is not None else None
        native.check(native.lib().fm_llm_teacher_step(
            self.h, slot, native.i32p(xx), xx.shape[1], pos0,
            native.i32p(nc) if nc is not None else None, native.f32p(lg), native.f32p(hid),
            native.f32p(fl) if nc is not None else None))
        return lg, hid, (fl if nc is not None else None)

    # ---- teacher forcing on the production decode path ------------------------------------
    def force(self, slot: int, col) -> None:
        """While forced, the slot's samplers emit `col` (C+1 tokens) and tap their logits
        (fm_llm_force); col=None stops forcing."""
        if col is None:
            native.check(native.lib().fm_llm_force(self.h, slot, None))
            return
        c = np.ascontiguousarray(col, dtype=np.int32).reshape(-1)
        assert c.size == self.C1
        native.check(native.lib().fm_llm_force(self.h, slot, native.i32p(c)))

    def read_logits(self, slot: int = 0):
        """(slow logits [V], fast logits [(C-1), cb]) the last forced frame's samplers were handed."""
        lg = np.zeros(self.cfg.vocab_size, np.float32)
        fl = np.zeros((max(self.cfg.num_codebooks - 1, 1), self.cfg.codebook_size), np.float32)
        native.check(native.lib().fm_llm_read_logits(self.h, slot, native.f32p(lg), native.f32p(fl)))
        return lg, fl[: self.cfg.num_codebooks - 1]

    def teacher_decode(self, prompt: np.ndarray, cols: np.ndarray, slot: int = 0):
        """The reference's teacher-forced loop (oracle/gen_goldens.py teacher_forced: prefill, then
        one forward_generate per emitted column) on the production path: the prefill, then
        n-1 single-frame decodes through the captured frame graph, each sampler forced to emit the
        given column.  cols: (C+1, n).  Returns slow logits (n, V) and fast logits (n, C-1, cb)."""
        cols = np.ascontiguousarray(cols, dtype=np.int32)
        n = cols.shape[1]
        slow = np.zeros((n, self.cfg.vocab_size), np.float32)
        fast = np.zeros((n, self.cfg.num_codebooks - 1, self.cfg.codebook_size), np.float32)
        sp = self.sampling(top_k=1)
        try:
            for i in range(n):
                self.force(slot, cols[:, i])
                if i == 0:
                    self.prefill(slot, prompt, sp)
                else:
                    self.decode([slot])
                slow[i], fast[i] = self.read_logits(slot)
        finally:
            self.force(slot, None)
        return slow, fast

    def read_cache(self, layer: int):
        """Slot 0's slow-layer KV cache rows (developer hook fm_llm_debug_vec "kc" / "vc"):
        k, v as float arrays (n_local_heads, max_seq_len, head_dim) of the stored values."""
        c = self.cfg
        n = c.n_local_heads * c.max_seq_len * c.head_dim
        out = []
        for name in (b"kc", b"vc"):
            a = np.zeros(n, np.float32)
            native.check(native.lib().fm_llm_debug_vec(self.h, name, int(layer), native.f32p(a), n))
            out.append(a.reshape(c.n_local_heads, c.max_seq_len, c.head_dim))
        return out[0], out[1]

    # ---- accounting / profiling --------------------------------------------------------
    def frame_bytes(self, n: int, pos: int) -> int:
        return int(native.lib().fm_llm_frame_bytes(self.h, n, pos))

    def profile(self, enable: bool):
        native.check(native.lib().fm_llm_profile(self.h, int(enable)))

    def profile_read(self, cls: str):
        ms, n, b = ctypes.c_double(), ctypes.c_int64(), ctypes.c_int64()
        native.check(native.lib().fm_llm_profile_read(self.h, cls.encode(), ctypes.byref(ms),
                                                      ctypes.byref(n), ctypes.byref(b)))
        return ms.value, n.value, b.value

    def kernel_bench(self, kernel_class: str = "linear", reps: int = 20):
        """(avg us per launch, launches per frame, algorithmic bytes per frame) of one decode
        frame's launches of kernel_class, replayed back to back (fm_llm_kernel_bench)."""
        us, n, b = ctypes.c_double(), ctypes.c_int64(), ctypes.c_int64()
        native.check(native.lib().fm_llm_kernel_bench(self.h, kernel_class.encode(), reps, ctypes.byref(us),
                                                      ctypes.byref(n), ctypes.byref(b)))
        return us.value, n.value, b.value

    def use_graph(self, enable: bool):
        native.check(native.lib().fm_llm_use_graph(self.h, int(enable)))


class DecodeOneToken:
    """The reference's injected per-step operator, ``decode_one_token_ar(model, x, input_pos,
    temperature, top_p, top_k, semantic_logit_bias, audio_masks, audio_parts, previous_tokens)``
    (inference.py:96-181), on one slot of a DualARModel.  Pass it as ``generate(...,
    decode_one_token=op)`` / ``decode_n_tokens(..., decode_one_token=op)`` (inference.py:195, 250),
    or call it for the prefill step as generate() does (inference.py:323-333).

    The slot owns the KV cache and the RAS window, so the call checks that the caller's state is
    the one the slot holds rather than re-deriving it:
      * x (1, C+1, T), T > 1: a prefill at positions input_pos = [p0, p0 + T); p0 must be 0 or a
        position the slot has already cached (prefix reuse, fm_llm_prefill_at);
      * x (1, C+1, 1): one frame at input_pos == the slot's next position, x == the column this
        operator returned last (decode_n_tokens feeds back exactly that);
      * temperature / top_p / top_k are fixed by the prefill (the reference keeps them for the
        whole generate); semantic_logit_bias must be the reference's (0 on the semantic range and
        <|im_end|>, -inf elsewhere, inference.py:308-320) -- the compact head is exact only there;
      * audio_parts must be None (the prompt side encodes text and VQ codes only).
    Returns a (C+1, 1) int64 tensor on x's device, like the reference."""

    def __init__(self, model: DualARModel, slot: int = 0, seed: int = 0):
        self.m = model
        self.slot = slot
        self.seed = seed
        self._last = None
        self._params = None
        self._bias_ok = set()

    def _check_bias(self, bias):
        if bias is None or id(bias) in self._bias_ok:
            return
        cfg = self.m.cfg
        b = bias.detach().float().reshape(-1).cpu().numpy()
        want = np.full(cfg.vocab_size, -np.inf, np.float32)
        want[cfg.semantic_begin_id: cfg.semantic_end_id + 1] = 0.0
        want[cfg.im_end_id] = 0.0
        if b.shape != want.shape or not np.array_equal(b, want):
            raise ValueError("semantic_logit_bias differs from generate()'s (inference.py:308-320)")
        self._bias_ok.add(id(bias))

    def __call__(self, model, x, input_pos, temperature, top_p, top_k, semantic_logit_bias,
                 audio_masks=None, audio_parts=None, previous_tokens=None):
        import torch

        if audio_parts is not None:
            raise NotImplementedError("audio_parts (continuous audio embeddings) are not on this path")
        self._check_bias(semantic_logit_bias)
        xx = x.detach().reshape(self.m.C1, -1).to("cpu", torch.int32).numpy()
        ip = np.asarray(input_pos.detach().reshape(-1).cpu().numpy(), np.int64)
        params = (float(temperature), float(top_p), int(top_k))
        T = xx.shape[1]
        if T > 1 or ip[0] == 0:
            p0 = int(ip[0])
            if p0 and p0 > self.m.slot_pos(self.slot):
                raise ValueError(f"prefill at {p0} past the slot's cached positions")
            sp = DualARModel.sampling(*params, seed=self.seed)
            col = self.m.prefill(self.slot, xx, sp, pos0=p0)
            self._params = params
        else:
            if self._last is None:
                raise ValueError("decode step before a prefill on this slot")
            if params != self._params:
                raise ValueError("temperature / top_p / top_k changed after the prefill")
            if int(ip[0]) != self.m.slot_pos(self.slot):
                raise ValueError(f"input_pos {int(ip[0])} != the slot's next position {self.m.slot_pos(self.slot)}")
            if not np.array_equal(xx[:, 0], self._last):
                raise ValueError("x is not the column this operator emitted last")
            col = self.m.decode([self.slot])[0]
        self._last = np.asarray(col, np.int32).copy()
        return torch.from_numpy(self._last.astype(np.int64)).reshape(self.m.C1, 1).to(x.device)
