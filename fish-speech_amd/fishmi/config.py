"""Model configuration, mirroring the reference's config resolution.

``DualARConfig.from_pretrained`` follows ``BaseModelArgs.from_pretrained`` /
``_from_fish_qwen3_omni`` / ``DualARModelArgs.__post_init__`` (reference
fish_speech/models/text2semantic/llama.py:27-193): the same keys, the same fall-backs of the
fast-model fields to the slow-model fields, and the two flags forced for ``fish_qwen3_omni``
(``scale_codebook_embeddings``, ``norm_fastlayer_input``).  The ctypes structure mirrors
``fm_model_config`` in include/fishmi.h (same field order as the oracle's config).
"""
from __future__ import annotations

import ctypes
import dataclasses
import json
from dataclasses import dataclass
from pathlib import Path
from typing import Optional


def find_multiple(n: int, k: int) -> int:
    return n if n % k == 0 else n + k - (n % k)


@dataclass
class DualARConfig:
    model_type: str = "dual_ar"
    vocab_size: int = 32000
    n_layer: int = 32
    n_head: int = 32
    dim: int = 4096
    intermediate_size: Optional[int] = None
    n_local_heads: int = -1
    head_dim: Optional[int] = 64
    rope_base: float = 10000
    norm_eps: float = 1e-5
    max_seq_len: int = 2048
    tie_word_embeddings: bool = True
    attention_qkv_bias: bool = False
    attention_o_bias: bool = False
    attention_qk_norm: bool = False
    codebook_size: int = 160
    num_codebooks: int = 4
    semantic_begin_id: int = 0
    semantic_end_id: int = 0
    initializer_range: float = 0.02
    scale_codebook_embeddings: bool = False
    n_fast_layer: int = 4
    fast_dim: Optional[int] = None
    fast_n_head: Optional[int] = None
    fast_n_local_heads: Optional[int] = None
    fast_head_dim: Optional[int] = None
    fast_intermediate_size: Optional[int] = None
    fast_attention_qkv_bias: Optional[bool] = None
    fast_attention_qk_norm: Optional[bool] = None
    fast_attention_o_bias: Optional[bool] = None
    norm_fastlayer_input: bool = False
    im_end_id: int = -1  # resolved from the tokenizer (inference.py:207, 320)

    def __post_init__(self):
        if self.n_local_heads == -1:
            self.n_local_heads = self.n_head
        if self.intermediate_size is None:
            self.intermediate_size = find_multiple(int(2 * 4 * self.dim / 3), 256)
        if self.head_dim is None:
            self.head_dim = self.dim // self.n_head
        self.fast_dim = self.fast_dim or self.dim
        self.fast_n_head = self.fast_n_head or self.n_head
        self.fast_n_local_heads = self.fast_n_local_heads or self.n_local_heads
        self.fast_head_dim = self.fast_head_dim or self.head_dim
        self.fast_intermediate_size = self.fast_intermediate_size or self.intermediate_size
        if self.fast_attention_qkv_bias is None:
            self.fast_attention_qkv_bias = self.attention_qkv_bias
        if self.fast_attention_qk_norm is None:
            self.fast_attention_qk_norm = self.attention_qk_norm
        if self.fast_attention_o_bias is None:
            self.fast_attention_o_bias = self.attention_o_bias

    # ---- llama.py:75-99 ------------------------------------------------------------
    @staticmethod
    def from_pretrained(path) -> "DualARConfig":
        path = Path(path)
        if path.is_dir():
            path = path / "config.json"
        with open(path, "r", encoding="utf-8") as f:
            data = json.load(f)
        mt = data["model_type"]
        if mt == "fish_qwen3_omni":
            return DualARConfig._from_fish_qwen3_omni(data)
        if mt not in ("dual_ar", "naive"):
            raise ValueError(f"Unknown model type: {mt}")
        if mt == "naive":
            raise ValueError("naive (single-AR) models are outside the Dual-AR hot path")
        valid = {f.name for f in dataclasses.fields(DualARConfig)}
        return DualARConfig(**{k: v for k, v in data.items() if k in valid})

    # ---- llama.py:101-143 ----------------------------------------------------------
    @staticmethod
    def _from_fish_qwen3_omni(data: dict) -> "DualARConfig":
        tc, adc = data["text_config"], data["audio_decoder_config"]
        flat = dict(
            model_type="dual_ar", vocab_size=tc["vocab_size"], n_layer=tc["n_layer"],
            n_head=tc["n_head"], n_local_heads=tc.get("n_local_heads", -1),
            head_dim=tc.get("head_dim"), dim=tc["dim"],
            intermediate_size=tc.get("intermediate_size"), rope_base=tc.get("rope_base", 10000),
            norm_eps=tc.get("norm_eps", 1e-5), max_seq_len=tc.get("max_seq_len", 2048),
            tie_word_embeddings=tc.get("tie_word_embeddings", True),
            attention_qkv_bias=tc.get("attention_qkv_bias", False),
            attention_o_bias=tc.get("attention_o_bias", False),
            attention_qk_norm=tc.get("attention_qk_norm", False),
            initializer_range=tc.get("initializer_range", 0.02),
            semantic_begin_id=data.get("semantic_start_token_id", 0),
            semantic_end_id=data.get("semantic_end_token_id", 0),
            scale_codebook_embeddings=True, norm_fastlayer_input=True,
            codebook_size=adc["vocab_size"], num_codebooks=adc["num_codebooks"],
            n_fast_layer=adc["n_layer"], fast_dim=adc.get("dim"), fast_n_head=adc.get("n_head"),
            fast_n_local_heads=adc.get("n_local_heads"), fast_head_dim=adc.get("head_dim"),
            fast_intermediate_size=adc.get("intermediate_size"),
            fast_attention_qkv_bias=adc.get("attention_qkv_bias"),
            fast_attention_qk_norm=adc.get("attention_qk_norm"),
            fast_attention_o_bias=adc.get("attention_o_bias"),
        )
        valid = {f.name for f in dataclasses.fields(DualARConfig)}
        return DualARConfig(**{k: v for k, v in flat.items() if k in valid and v is not None})

    @property
    def cache_len(self) -> int:
        """setup_caches rounds max_seq_len up to a multiple of 8 (llama.py:313)."""
        return find_multiple(self.max_seq_len, 8)

    def to_c(self) -> "LLMConfigC":
        c = LLMConfigC()
        for name, _ in LLMConfigC._fields_:
            src = _C_FIELD_MAP.get(name, name)
            setattr(c, name, type(getattr(c, name))(getattr(self, src)))
        return c


class LLMConfigC(ctypes.Structure):
    """== fm_model_config (include/fishmi.h) == orc_llm_config (oracle/fishmi_oracle.c)."""
    _fields_ = [
        ("vocab_size", ctypes.c_int), ("dim", ctypes.c_int), ("n_layer", ctypes.c_int),
        ("n_head", ctypes.c_int), ("n_local_heads", ctypes.c_int), ("head_dim", ctypes.c_int),
        ("intermediate_size", ctypes.c_int),
        ("rope_base", ctypes.c_float), ("norm_eps", ctypes.c_float),
        ("max_seq_len", ctypes.c_int),
        ("qkv_bias", ctypes.c_int), ("o_bias", ctypes.c_int), ("qk_norm", ctypes.c_int),
        ("tie_word_embeddings", ctypes.c_int),
        ("codebook_size", ctypes.c_int), ("num_codebooks", ctypes.c_int),
        ("semantic_begin_id", ctypes.c_int), ("semantic_end_id", ctypes.c_int),
        ("im_end_id", ctypes.c_int),
        ("scale_codebook_embeddings", ctypes.c_int), ("norm_fastlayer_input", ctypes.c_int),
        ("n_fast_layer", ctypes.c_int), ("fast_dim", ctypes.c_int), ("fast_n_head", ctypes.c_int),
        ("fast_n_local_heads", ctypes.c_int), ("fast_head_dim", ctypes.c_int),
        ("fast_intermediate_size", ctypes.c_int),
        ("fast_qkv_bias", ctypes.c_int), ("fast_o_bias", ctypes.c_int),
        ("fast_qk_norm", ctypes.c_int),
    ]


_C_FIELD_MAP = {
    "qkv_bias": "attention_qkv_bias", "o_bias": "attention_o_bias",
    "qk_norm": "attention_qk_norm", "fast_qkv_bias": "fast_attention_qkv_bias",
    "fast_o_bias": "fast_attention_o_bias", "fast_qk_norm": "fast_attention_qk_norm",
}


# ----------------------------------------------------------------------------------------
# Codec (modded DAC decode side); shapes from fish_speech/configs/modded_dac_vq.yaml
# ----------------------------------------------------------------------------------------
@dataclass
class CodecConfig:
    latent: int = 1024               # quantizer.input_dim == encoder_dim * 2**4
    decoder_dim: int = 1536
    n_codebooks: int = 9             # residual codebooks (semantic one is extra)
    codebook_size: int = 1024
    semantic_codebook_size: int = 4096
    codebook_dim: int = 8
    t_layers: int = 8                # post_module WindowLimitedTransformer
    t_heads: int = 16
    t_head_dim: int = 64
    t_inter: int = 3072
    window: int = 128
    rope_base: float = 10000.0
    norm_eps: float = 1e-5
    sample_rate: int = 44100
    hop: int = 2048                  # samples per code frame (modded_dac.py:833, 861)

    @staticmethod
    def from_spec(spec: dict) -> "CodecConfig":
        return CodecConfig(latent=spec["latent"], decoder_dim=spec["decoder_dim"],
                           n_codebooks=spec["n_codebooks"], codebook_size=spec["codebook_size"],
                           semantic_codebook_size=spec["semantic_codebook_size"],
                           codebook_dim=spec["codebook_dim"], t_layers=spec["t_layers"],
                           t_heads=spec["t_heads"], t_head_dim=spec["t_head_dim"],
                           t_inter=spec["t_inter"], window=spec["window"])

    def to_c(self) -> "CodecConfigC":
        c = CodecConfigC()
        for name, _ in CodecConfigC._fields_:
            setattr(c, name, type(getattr(c, name))(getattr(self, name)))
        return c


class CodecConfigC(ctypes.Structure):
    """== fm_codec_config (include/fishmi.h) == orc_codec_config (oracle)."""
    _fields_ = [
        ("latent", ctypes.c_int), ("decoder_dim", ctypes.c_int), ("n_codebooks", ctypes.c_int),
        ("codebook_size", ctypes.c_int), ("semantic_codebook_size", ctypes.c_int),
        ("codebook_dim", ctypes.c_int), ("t_layers", ctypes.c_int), ("t_heads", ctypes.c_int),
        ("t_head_dim", ctypes.c_int), ("t_inter", ctypes.c_int), ("window", ctypes.c_int),
        ("rope_base", ctypes.c_float), ("norm_eps", ctypes.c_float),
    ]


# S2-Pro shapes assumed in SURVEY.md §2.3 (Qwen3-4B-shaped slow model, "400M" fast model).
S2_PRO_CONFIG = {
    "model_type": "fish_qwen3_omni",
    "text_config": {
        "vocab_size": 155776, "n_layer": 36, "n_head": 32, "n_local_heads": 8,
        "head_dim": 128, "dim": 2560, "intermediate_size": 9728, "rope_base": 1000000,
        "norm_eps": 1e-6, "max_seq_len": 4096, "tie_word_embeddings": True,
        "attention_qkv_bias": False, "attention_o_bias": False, "attention_qk_norm": True,
    },
    "audio_decoder_config": {
        "vocab_size": 4096, "num_codebooks": 10, "n_layer": 4, "dim": 2560, "n_head": 32,
        "n_local_heads": 8, "head_dim": 128, "intermediate_size": 9728,
    },
    "semantic_start_token_id": 151678,
    "semantic_end_token_id": 155773,
}
S2_PRO_IM_END_ID = 151645
