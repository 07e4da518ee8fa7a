"""Deterministic synthetic weights shared bit-for-bit by numpy, the C oracle and the HIP library.

There are no real checkpoints on this machine or on the GPU box, so every full-shape run
uses random weights at the real shapes (SURVEY.md §7 "Hard parts", §8d).  To let the
GPU path, the CPU oracle and the imported reference all see *identical* tensors without
shipping gigabytes, each tensor element is a pure function of (seed, tensor name, index):

    key  = seed * K1 + fnv1a32(name) * K2 + index           (uint64, wrapping)
    m    = splitmix64(key) >> 40                            (24 random bits)
    w    = center + (2m - 2**24) * 2**(-24 - log2_half)     (fp32: the product is exact,
                                                             one rounding in the add)
    w    -> bf16 (round-to-nearest-even) when the tensor is stored bf16

The same formula lives in ``oracle/fishmi_oracle.c`` (``orc_synth``) and
``fish-speech_amd/csrc/fm_common.hip`` (``synth_kernel``).
"""
from __future__ import annotations

import numpy as np

K1 = np.uint64(0xD1B54A32D192ED03)
K2 = np.uint64(0x9E3779B97F4A7C15)


def fnv1a32(name: str) -> int:
    h = 0x811C9DC5
    for b in name.encode("utf-8"):
        h ^= b
        h = (h * 0x01000193) & 0xFFFFFFFF
    return h


def _splitmix64(z: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return z


def _synth_range(out: np.ndarray, base: np.uint64, lo: int, hi: int, center: float, log2_half: int) -> None:
    idx = np.arange(lo, hi, dtype=np.uint64)
    with np.errstate(over="ignore"):
        key = base + idx
    m = (_splitmix64(key) >> np.uint64(40)).astype(np.int64)
    r = ((2 * m - (1 << 24)).astype(np.float32)) * np.float32(2.0 ** (-24 - log2_half))
    out[lo:hi] = np.float32(center) + r


_CHUNK = 1 << 23


def synth_f32(seed: int, name: str, n: int, center: float, log2_half: int) -> np.ndarray:
    """fp32 values in [center - 2**-log2_half, center + 2**-log2_half).  Large tensors are made in
    8M-element chunks on a thread pool (numpy ufuncs release the GIL); every element is the same
    pure function of (seed, name, index) either way."""
    with np.errstate(over="ignore"):
        base = np.uint64(seed) * K1 + np.uint64(fnv1a32(name)) * K2
    out = np.empty(n, dtype=np.float32)
    spans = [(lo, min(n, lo + _CHUNK)) for lo in range(0, n, _CHUNK)]
    if len(spans) <= 1:
        for lo, hi in spans:
            _synth_range(out, base, lo, hi, center, log2_half)
        return out
    import os
    from concurrent.futures import ThreadPoolExecutor

    with ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 1)) as ex:
        list(ex.map(lambda s: _synth_range(out, base, s[0], s[1], center, log2_half), spans))
    return out


def f32_to_bf16_bits(x: np.ndarray) -> np.ndarray:
    """Round-to-nearest-even fp32 -> bf16, returned as uint16 bit patterns (NaN-safe)."""
    u = np.ascontiguousarray(x, dtype=np.float32).view(np.uint32)
    nan = (u & 0x7FFFFFFF) > 0x7F800000
    r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint16)
    r[nan] = ((u[nan] >> 16) | 0x40).astype(np.uint16)
    return r


def bf16_bits_to_f32(b: np.ndarray) -> np.ndarray:
    return (np.asarray(b, dtype=np.uint16).astype(np.uint32) << 16).view(np.float32)


def round_bf16(x: np.ndarray) -> np.ndarray:
    return bf16_bits_to_f32(f32_to_bf16_bits(x))


# ---------------------------------------------------------------------------------------
# Per-tensor synthetic distributions.  One rule table for every model family so that the
# Python side (goldens, tests) and the native sides receive the same (center, log2_half).
# ---------------------------------------------------------------------------------------

def llm_rule(name: str, log2_half_linear: int = 5) -> tuple[float, int]:
    """(center, log2_half) for a Dual-AR tensor name (reference key names, llama.py)."""
    if name.endswith("norm.weight"):
        return 1.0, 3          # RMSNorm weights around 1 (+-0.125)
    if name.endswith(".bias"):
        return 0.0, 6
    return 0.0, log2_half_linear  # linears / embeddings: half-range 2**-5 -> std ~0.018


def codec_rule(name: str) -> tuple[float, int]:
    """(center, log2_half) for a modded-DAC decode-side tensor (modded_dac.py / rvq.py keys)."""
    if name.endswith(".alpha"):
        return 1.0, 1          # snake alpha in [0.5, 1.5)
    if name == "decoder.model.6.conv.parametrizations.weight.original0":
        return 0.0625, 6       # output conv gain: keeps the random-weight waveform off tanh's rails
                               # (with g ~ 1 most samples sit at +-1 and parity only tests signs)
    if name.endswith("original0") or name.endswith("weight_g"):
        return 1.0, 2          # weight-norm gain g in [0.75, 1.25)
    if name.endswith("gamma"):
        return 0.0, 3          # LayerScale / ConvNeXt gamma
    if name.endswith("norm.weight"):
        return 1.0, 3
    if name.endswith(".bias"):
        return 0.0, 6
    if "codebook.weight" in name:
        return 0.0, 0          # codebook vectors in [-1, 1)
    return 0.0, 5


def write_synthetic_tokenizer(path: str, vocab_size: int, im_end_id: int, semantic_begin_id: int,
                              n_semantic: int = 4096) -> str:
    """A tokenizer.json for synthetic-weight runs at a real model's vocabulary layout (there is no
    checkpoint tokenizer on the box): single characters at low ids, <|im_end|> and the other chat
    specials just below the semantic range (Qwen-style), <|semantic:i|> at semantic_begin_id + i, the
    rest reserved.  Returns the directory (FishTokenizer(path) loads it)."""
    import json
    import os

    from tokenizers import AddedToken, Regex, Tokenizer, models, pre_tokenizers

    specials = {"<|endoftext|>": im_end_id - 2, "<|im_start|>": im_end_id - 1, "<|im_end|>": im_end_id,
                "<|text|>": im_end_id + 1, "<|voice|>": im_end_id + 2, "<|interleave|>": im_end_id + 3,
                "<|audio_start|>": im_end_id + 4, "<|audio_end|>": im_end_id + 5, "<|audio_pad|>": im_end_id + 6}
    for i in range(5):
        specials[f"<|speaker:{i}|>"] = im_end_id + 10 + i
    assert max(specials.values()) < semantic_begin_id and semantic_begin_id + n_semantic <= vocab_size
    chars = [chr(c) for c in range(32, 127)] + ["\n"]
    vocab = {ch: 16 + i for i, ch in enumerate(chars)}
    vocab["[UNK]"] = 15
    vocab.update(specials)
    sem = [f"<|semantic:{i}|>" for i in range(n_semantic)]
    for i, t in enumerate(sem):
        vocab[t] = semantic_begin_id + i
    used = set(vocab.values())
    for i in range(vocab_size):
        if i not in used:
            vocab[f"<|reserved_{i}|>"] = i
    tk = Tokenizer(models.WordLevel(vocab=vocab, unk_token="[UNK]"))
    tk.pre_tokenizer = pre_tokenizers.Split(Regex("."), behavior="isolated")
    tk.add_special_tokens([AddedToken(t, special=True, normalized=False) for t in list(specials) + sem])
    os.makedirs(path, exist_ok=True)
    tk.save(os.path.join(path, "tokenizer.json"))
    with open(os.path.join(path, "tokenizer_config.json"), "w") as f:
        json.dump({"tokenizer_class": "PreTrainedTokenizerFast", "eos_token": "<|endoftext|>"}, f)
    return path
