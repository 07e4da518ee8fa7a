"""Checkpoint discovery and loading, mirroring ``BaseTransformer.from_pretrained``
(reference fish_speech/models/text2semantic/llama.py:479-593) without torch on the hot path.

* weight files, in precedence order: ``model.safetensors.index.json`` shards ->
  ``model.safetensors`` -> ``model.pth`` (llama.py:545-584);
* the ``fish_qwen3_omni`` key remap (llama.py:229-246);
* separate ``wq/wk/wv`` concatenated into ``wqkv`` (Attention.load_hook, llama.py:876-881);
* ``model.pth``: optional ``state_dict`` unwrap, ``model.`` prefix strip, ``audio_*`` keys
  dropped (llama.py:567-582) -- loaded with ``torch.load(weights_only=True)`` only.

Tensors come back as numpy arrays: bf16 as uint16 bit patterns (``Tensor.bf16=True``), int8
(the weights of a tools/llama/quantize.py int8 checkpoint) as int8, everything else as float32.  The safetensors reader is a plain header parse + mmap.
"""
from __future__ import annotations

import json
import os
import struct
from collections import OrderedDict
from dataclasses import dataclass
from pathlib import Path
from typing import Iterator

import numpy as np

from .config import CodecConfig, DualARConfig
from .synth import bf16_bits_to_f32, f32_to_bf16_bits

_ST_DTYPES = {
    "F32": (np.float32, False), "F16": (np.float16, False), "BF16": (np.uint16, True),
    "F64": (np.float64, False), "I64": (np.int64, False), "I32": (np.int32, False),
    "I8": (np.int8, False),
}


@dataclass
class Tensor:
    data: np.ndarray   # uint16 bits when bf16, int8 for int8 weights, else float32
    bf16: bool

    @property
    def int8(self) -> bool:
        return self.data.dtype == np.int8

    @property
    def shape(self):
        return self.data.shape

    def as_f32(self) -> np.ndarray:
        if self.bf16:
            return bf16_bits_to_f32(self.data).reshape(self.data.shape)
        return np.asarray(self.data, dtype=np.float32)

    def as_bf16_bits(self) -> np.ndarray:
        return self.data if self.bf16 else f32_to_bf16_bits(self.as_f32()).reshape(self.data.shape)


def read_safetensors(path) -> "OrderedDict[str, Tensor]":
    out = OrderedDict()
    with open(path, "rb") as f:
        (hlen,) = struct.unpack("<Q", f.read(8))
        header = json.loads(f.read(hlen))
    mm = np.memmap(path, dtype=np.uint8, mode="r")
    base = 8 + hlen
    for name, meta in header.items():
        if name == "__metadata__":
            continue
        dt, is_bf16 = _ST_DTYPES[meta["dtype"]]
        a, b = meta["data_offsets"]
        arr = np.frombuffer(mm[base + a: base + b], dtype=dt).reshape(meta["shape"])
        if not is_bf16 and dt not in (np.float32, np.int8):
            arr = arr.astype(np.float32)
        out[name] = Tensor(arr, is_bf16)
    return out


def remap_fish_qwen3_omni_keys(weights: "OrderedDict[str, Tensor]"):
    """llama.py:229-246."""
    if not any(k.startswith(("text_model.", "audio_decoder.")) for k in weights):
        return weights
    new = OrderedDict()
    for k, v in weights.items():
        if k.startswith("text_model.model."):
            nk = k[len("text_model.model."):]
        elif k.startswith("audio_decoder."):
            suf = k[len("audio_decoder."):]
            nk = suf if suf.startswith("codebook_embeddings.") else "fast_" + suf
        else:
            nk = k
        new[nk] = v
    return new


def merge_qkv(weights: "OrderedDict[str, Tensor]"):
    """Attention.load_hook (llama.py:876-881): wq/wk/wv -> wqkv (rows concatenated)."""
    for k in [k for k in weights if k.endswith("attention.wq.weight")]:
        p = k[: -len("wq.weight")]
        q, kk, v = weights.pop(p + "wq.weight"), weights.pop(p + "wk.weight"), weights.pop(p + "wv.weight")
        bf = q.bf16 and kk.bf16 and v.bf16
        if q.int8 and kk.int8 and v.int8:
            data, bf = np.concatenate([q.data, kk.data, v.data], axis=0), False
        elif bf:
            data = np.concatenate([q.data, kk.data, v.data], axis=0)
        else:
            data = np.concatenate([q.as_f32(), kk.as_f32(), v.as_f32()], axis=0)
        weights[p + "wqkv.weight"] = Tensor(data, bf)
    return weights


def load_llm_weights(path) -> "OrderedDict[str, Tensor]":
    """llama.py:545-584.  One deliberate difference: a directory named like a quantize.py int8 output
    ("int8" in the path, llama.py:528) with a model.pth loads that file first.  quantize.py copies
    the source checkpoint's files beside its model.pth (quantize.py:458-466), and the reference's
    precedence would load the copied float shards into the int8 modules instead."""
    p = Path(path)
    index_json, single, pth = p / "model.safetensors.index.json", p / "model.safetensors", p / "model.pth"
    if "int8" in str(p) and pth.exists():
        index_json = single = p / "__none__"
    if index_json.exists():
        with open(index_json) as f:
            idx = json.load(f)
        weights = OrderedDict()
        for shard in sorted(set(idx["weight_map"].values())):
            weights.update(read_safetensors(p / shard))
        weights = remap_fish_qwen3_omni_keys(weights)
    elif single.exists():
        weights = remap_fish_qwen3_omni_keys(read_safetensors(single))
    elif pth.exists():
        import torch  # only for the .pth container format; weights_only=True (no pickle code)

        sd = torch.load(pth, map_location="cpu", mmap=True, weights_only=True)
        if "state_dict" in sd:
            sd = sd["state_dict"]
        if sd and next(iter(sd.keys())).startswith("model."):
            sd = OrderedDict((k.replace("model.", ""), v) for k, v in sd.items())
        weights = OrderedDict()
        for k, v in sd.items():
            if "audio_" in k:
                continue
            if v.dtype == torch.bfloat16:
                weights[k] = Tensor(v.contiguous().view(torch.int16).numpy().view(np.uint16), True)
            elif v.dtype == torch.int8:
                weights[k] = Tensor(v.contiguous().numpy(), False)
            else:
                weights[k] = Tensor(v.float().numpy(), False)
    else:
        raise FileNotFoundError(f"No model weights found in {p}")
    return merge_qkv(weights)


# ----------------------------------------------------------------------------------------
# Expected tensor inventory (names = reference state_dict keys after remap)
# ----------------------------------------------------------------------------------------
def llm_tensor_shapes(cfg: DualARConfig) -> "OrderedDict[str, tuple]":
    s = OrderedDict()
    d, C, cb = cfg.dim, cfg.num_codebooks, cfg.codebook_size
    s["embeddings.weight"] = (cfg.vocab_size, d)
    s["codebook_embeddings.weight"] = (cb * C, d)

    def stack(prefix, n, dim, nh, nkv, hd, inter, qb, ob, qkn):
        for i in range(n):
            p = f"{prefix}{i}."
            s[p + "attention.wqkv.weight"] = ((nh + 2 * nkv) * hd, dim)
            if qb:
                s[p + "attention.wqkv.bias"] = ((nh + 2 * nkv) * hd,)
            s[p + "attention.wo.weight"] = (dim, nh * hd)
            if ob:
                s[p + "attention.wo.bias"] = (dim,)
            if qkn:
                s[p + "attention.q_norm.weight"] = (hd,)
                s[p + "attention.k_norm.weight"] = (hd,)
            s[p + "feed_forward.w1.weight"] = (inter, dim)
            s[p + "feed_forward.w3.weight"] = (inter, dim)
            s[p + "feed_forward.w2.weight"] = (dim, inter)
            s[p + "ffn_norm.weight"] = (dim,)
            s[p + "attention_norm.weight"] = (dim,)

    stack("layers.", cfg.n_layer, d, cfg.n_head, cfg.n_local_heads, cfg.head_dim,
          cfg.intermediate_size, cfg.attention_qkv_bias, cfg.attention_o_bias,
          cfg.attention_qk_norm)
    s["norm.weight"] = (d,)
    if not cfg.tie_word_embeddings:
        s["output.weight"] = (cfg.vocab_size, d)
    if cfg.fast_dim != cfg.dim:
        s["fast_project_in.weight"] = (cfg.fast_dim, d)
        s["fast_project_in.bias"] = (cfg.fast_dim,)
    s["fast_embeddings.weight"] = (cb, cfg.fast_dim)
    stack("fast_layers.", cfg.n_fast_layer, cfg.fast_dim, cfg.fast_n_head,
          cfg.fast_n_local_heads, cfg.fast_head_dim, cfg.fast_intermediate_size,
          cfg.fast_attention_qkv_bias, cfg.fast_attention_o_bias, cfg.fast_attention_qk_norm)
    s["fast_norm.weight"] = (cfg.fast_dim,)
    s["fast_output.weight"] = (cb, cfg.fast_dim)
    return s


def codec_tensor_shapes(c: CodecConfig) -> "OrderedDict[str, tuple]":
    """Decode-side keys of the modded DAC state dict (modded_dac.py / rvq.py / descript)."""
    s = OrderedDict()
    D, cd = c.latent, c.codebook_dim
    for q in range(c.n_codebooks + 1):
        p = ("quantizer.semantic_quantizer.quantizers.0." if q == 0
             else f"quantizer.quantizer.quantizers.{q - 1}.")
        n = c.semantic_codebook_size if q == 0 else c.codebook_size
        s[p + "codebook.weight"] = (n, cd)
        s[p + "out_proj.weight_g"] = (D, 1, 1)
        s[p + "out_proj.weight_v"] = (D, cd, 1)
        s[p + "out_proj.bias"] = (D,)
    H, hd, I = c.t_heads, c.t_head_dim, c.t_inter
    for l in range(c.t_layers):
        p = f"quantizer.post_module.layers.{l}."
        s[p + "attention.wqkv.weight"] = (3 * H * hd, D)
        s[p + "attention.wo.weight"] = (D, H * hd)
        s[p + "feed_forward.w1.weight"] = (I, D)
        s[p + "feed_forward.w3.weight"] = (I, D)
        s[p + "feed_forward.w2.weight"] = (D, I)
        s[p + "ffn_norm.weight"] = (D,)
        s[p + "attention_norm.weight"] = (D,)
        s[p + "attention_layer_scale.gamma"] = (D,)
        s[p + "ffn_layer_scale.gamma"] = (D,)
    s["quantizer.post_module.norm.weight"] = (D,)
    for u in range(2):
        p = f"quantizer.upsample.{u}."
        s[p + "0.conv.weight"] = (D, D, 2)
        s[p + "0.conv.bias"] = (D,)
        s[p + "1.dwconv.conv.weight"] = (D, 1, 7)
        s[p + "1.dwconv.conv.bias"] = (D,)
        s[p + "1.norm.weight"] = (D,)
        s[p + "1.norm.bias"] = (D,)
        s[p + "1.pwconv1.weight"] = (4 * D, D)
        s[p + "1.pwconv1.bias"] = (4 * D,)
        s[p + "1.pwconv2.weight"] = (D, 4 * D)
        s[p + "1.pwconv2.bias"] = (D,)
        s[p + "1.gamma"] = (D,)

    def wn(p, co, ci, k, transposed=False):
        s[p + "conv.parametrizations.weight.original0"] = (ci if transposed else co, 1, 1)
        s[p + "conv.parametrizations.weight.original1"] = (ci, co, k) if transposed else (co, ci, k)
        s[p + "conv.bias"] = (co,)

    ch = c.decoder_dim
    wn("decoder.model.0.", ch, D, 7)
    cin = ch
    for b, st in enumerate([8, 8, 4, 2]):
        cout = cin // 2
        p = f"decoder.model.{b + 1}.block."
        s[p + "0.alpha"] = (1, cin, 1)
        wn(p + "1.", cout, cin, 2 * st, transposed=True)
        for r in range(3):
            rp = f"{p}{r + 2}.block."
            s[rp + "0.alpha"] = (1, cout, 1)
            wn(rp + "1.", cout, cout, 7)
            s[rp + "2.alpha"] = (1, cout, 1)
            wn(rp + "3.", cout, cout, 1)
        cin = cout
    s["decoder.model.5.alpha"] = (1, cin, 1)
    wn("decoder.model.6.", 1, cin, 7)
    return s


def load_codec_weights(path) -> "OrderedDict[str, Tensor]":
    """codec.pth loader (fish_speech/models/dac/inference.py:23-47): optional state_dict
    unwrap, keep/strip the ``generator.`` prefix; weights_only=True."""
    import torch

    sd = torch.load(path, map_location="cpu", mmap=True, weights_only=True)
    if "state_dict" in sd:
        sd = sd["state_dict"]
    if any("generator" in k for k in sd):
        sd = {k.replace("generator.", ""): v for k, v in sd.items() if "generator." in k}
    out = OrderedDict()
    for k, v in sd.items():
        if v.dtype == torch.bfloat16:
            out[k] = Tensor(v.contiguous().view(torch.int16).numpy().view(np.uint16), True)
        else:
            out[k] = Tensor(v.float().numpy(), False)
    return out


def iter_synth(shapes, seed: int, rule) -> Iterator[tuple]:
    """(name, shape, center, log2_half) for synthetic generation (fishmi/synth.py)."""
    for name, shape in shapes.items():
        c, e = rule(name)
        yield name, shape, c, e


def env_bool(name: str, default: bool = False) -> bool:
    v = os.environ.get(name)
    return default if v is None else v not in ("0", "", "false", "False")


ENCODER_RATES = (2, 4, 8, 8)   # DAC encoder_rates (modded_dac_vq.yaml)
ENCODER_WINDOW = 512           # EncoderBlock transformer window: getattr(partial, "window_size", 512)


def codec_encoder_tensor_shapes(c: CodecConfig, encoder_dim: int = 64,
                                enc_layers=(0, 0, 0, 4)) -> "OrderedDict[str, tuple]":
    """Encode-side keys of the modded DAC state dict: Encoder (modded_dac.py:623-709), the
    quantizer's downsample + pre_module (rvq.py:193-276) and the VQ in_proj (descript)."""
    s = OrderedDict()
    D, cd = c.latent, c.codebook_dim

    def wn(p, co, ci, k):
        s[p + "conv.parametrizations.weight.original0"] = (co, 1, 1)
        s[p + "conv.parametrizations.weight.original1"] = (co, ci, k)
        s[p + "conv.bias"] = (co,)

    def transformer(p, dim, layers, heads, hd, inter):
        for l in range(layers):
            q = f"{p}layers.{l}."
            s[q + "attention.wqkv.weight"] = (3 * heads * hd, dim)
            s[q + "attention.wo.weight"] = (dim, heads * hd)
            s[q + "feed_forward.w1.weight"] = (inter, dim)
            s[q + "feed_forward.w3.weight"] = (inter, dim)
            s[q + "feed_forward.w2.weight"] = (dim, inter)
            s[q + "ffn_norm.weight"] = (dim,)
            s[q + "attention_norm.weight"] = (dim,)
            s[q + "attention_layer_scale.gamma"] = (dim,)
            s[q + "ffn_layer_scale.gamma"] = (dim,)
        if layers:
            s[p + "norm.weight"] = (dim,)

    wn("encoder.block.0.", encoder_dim, 1, 7)
    d = encoder_dim
    for b, (st, nl) in enumerate(zip(ENCODER_RATES, enc_layers)):
        h, d = d, d * 2
        p = f"encoder.block.{b + 1}.block."
        for r in range(3):
            rp = f"{p}{r}.block."
            s[rp + "0.alpha"] = (1, h, 1)
            wn(rp + "1.", h, h, 7)
            s[rp + "2.alpha"] = (1, h, 1)
            wn(rp + "3.", h, h, 1)
        s[p + "3.alpha"] = (1, h, 1)
        wn(p + "4.", d, h, 2 * st)
        transformer(p + "5.", d, nl, d // 64, 64, 3 * d)
    s["encoder.block.5.alpha"] = (1, d, 1)
    wn("encoder.block.6.", D, d, 3)
    for i in range(2):
        p = f"quantizer.downsample.{i}."
        s[p + "0.conv.weight"] = (D, D, 2)
        s[p + "0.conv.bias"] = (D,)
        s[p + "1.dwconv.conv.weight"] = (D, 1, 7)
        s[p + "1.dwconv.conv.bias"] = (D,)
        s[p + "1.norm.weight"] = (D,)
        s[p + "1.norm.bias"] = (D,)
        s[p + "1.pwconv1.weight"] = (4 * D, D)
        s[p + "1.pwconv1.bias"] = (4 * D,)
        s[p + "1.pwconv2.weight"] = (D, 4 * D)
        s[p + "1.pwconv2.bias"] = (D,)
        s[p + "1.gamma"] = (D,)
    transformer("quantizer.pre_module.", D, c.t_layers, c.t_heads, c.t_head_dim, c.t_inter)
    for q in range(c.n_codebooks + 1):
        p = ("quantizer.semantic_quantizer.quantizers.0." if q == 0
             else f"quantizer.quantizer.quantizers.{q - 1}.")
        s[p + "in_proj.weight_g"] = (cd, 1, 1)
        s[p + "in_proj.weight_v"] = (cd, D, 1)
        s[p + "in_proj.bias"] = (cd,)
    return s
