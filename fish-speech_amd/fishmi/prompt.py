"""Prompt side of the decode path: tokenizer, conversation encoding and speaker batching.

Mirrors, for inference, the reference's
  * FishTokenizer                          fish_speech/tokenizer.py:55-129
  * Message / Conversation                 fish_speech/conversation.py:20-103
  * ContentSequence.encode(_for_inference) fish_speech/content_sequence.py:154-324
  * split_text_by_speaker,
    group_turns_into_batches               fish_speech/models/text2semantic/inference.py:454-520
with host-side numpy instead of torch (the token matrix is handed to libfishmi as int32).
Parity: tests/test_prompt.py against tests/golden/prompt.npz, produced by running the
reference's own classes (oracle/gen_goldens.py prompt).
"""
from __future__ import annotations

import copy
import os
import re
from dataclasses import dataclass, field
from typing import List, Literal, Optional, Sequence, Union

import numpy as np

EOS_TOKEN = "<|endoftext|>"
PAD_TOKEN = "<|pad|>"
IM_START_TOKEN = "<|im_start|>"
IM_END_TOKEN = "<|im_end|>"
MODALITY_TOKENS = {"text": "<|text|>", "voice": "<|voice|>", "interleave": "<|interleave|>"}
SEMANTIC_TOKEN_TEMPLATE = "<|semantic:{i}|>"


class FishTokenizer:
    """tokenizer.json of a checkpoint via the `tokenizers` library (the reference wraps the same
    file in transformers' PreTrainedTokenizerFast).  Semantic ids: the vocab's <|semantic:i|>."""

    def __init__(self, model_path: str):
        from tokenizers import Tokenizer

        path = model_path if model_path.endswith(".json") else os.path.join(model_path, "tokenizer.json")
        self._tk = Tokenizer.from_file(path)
        vocab = self._tk.get_vocab(with_added_tokens=True)
        ids = [vocab[t] for t in (SEMANTIC_TOKEN_TEMPLATE.format(i=i) for i in range(4096)) if t in vocab]
        self.semantic_begin_id = min(ids) if ids else 0
        self.semantic_end_id = max(ids) if ids else 0
        self._vocab = vocab

    @classmethod
    def from_pretrained(cls, path: str) -> "FishTokenizer":
        return cls(path)

    @property
    def vocab_size(self) -> int:
        return self._tk.get_vocab_size(with_added_tokens=False)

    def get_token_id(self, token: str) -> Optional[int]:
        return self._vocab.get(token)

    def encode(self, text: str, add_special_tokens: bool = False) -> List[int]:
        return self._tk.encode(text, add_special_tokens=add_special_tokens).ids

    def decode(self, tokens) -> str:
        return self._tk.decode(list(np.atleast_1d(tokens).tolist()))


@dataclass
class TextPart:
    text: Optional[str] = None
    tokens: Optional[List[int]] = None
    cal_loss: bool = False

    def __post_init__(self):
        if self.text is None and self.tokens is None:
            raise ValueError("Either text or tokens must be provided")


@dataclass
class VQPart:
    codes: np.ndarray  # (num_codebooks, T) codebook indices
    cal_loss: bool = False

    def __post_init__(self):
        self.codes = np.asarray(self.codes)


@dataclass
class Message:
    role: Literal["system", "user", "assistant"]
    parts: list = field(default_factory=list)
    add_im_start: bool = True
    add_im_end: bool = True
    cal_loss: bool = False
    modality: Optional[Literal["text", "voice", "interleave"]] = None


class Conversation:
    def __init__(self, messages: Optional[List[Message]] = None):
        self.messages = messages or []

    def append(self, message: Message):
        self.messages.append(message)

    def parts(self) -> list:
        """conversation.py:39-77: im_start header (role + modality token), parts, im_end."""
        out = []
        for m in self.messages:
            if m.add_im_start:
                mod = MODALITY_TOKENS[m.modality] if m.modality else ""
                out.append(TextPart(text=f"{IM_START_TOKEN}{m.role}\n{mod}"))
            out.extend(m.parts)
            if m.add_im_end:
                out.append(TextPart(text=IM_END_TOKEN + "\n"))
        return out

    def encode_for_inference(self, tokenizer: FishTokenizer, num_codebooks: int):
        """content_sequence.py:282-324: (num_codebooks+1, T) int64; row 0 the token ids (a VQ
        position holds semantic_begin + code 0), rows 1.. the codes at VQ positions, else 0.
        Returns (values, audio_masks=None, audio_parts=None) like the reference for text/VQ."""
        rows0, vq_cols, vq_codes = [], [], []
        n = 0
        for p in self.parts():
            if isinstance(p, TextPart):
                toks = p.tokens if p.tokens is not None else tokenizer.encode(p.text, add_special_tokens=False)
                toks = np.asarray(toks, dtype=np.int64)
            elif isinstance(p, VQPart):
                codes = p.codes.astype(np.int64)
                toks = codes[0] + tokenizer.semantic_begin_id
                vq_cols.append(np.arange(n, n + codes.shape[1]))
                vq_codes.append(codes)
            else:
                raise ValueError(f"Unsupported part type: {type(p)}")
            rows0.append(toks)
            n += len(toks)
        values = np.zeros((num_codebooks + 1, n), np.int64)
        if rows0:
            values[0] = np.concatenate(rows0)
        if vq_codes:
            values[1:, np.concatenate(vq_cols)] = np.concatenate(vq_codes, axis=1)
        return values, None, None


def split_text_by_speaker(text: str) -> List[str]:
    """inference.py:454-484: turns starting with <|speaker:N|> (text before the first tag and
    empty tags' trailing whitespace follow the reference's rules)."""
    pattern = r"(<\|speaker:\d+\|>)"
    parts = re.split(pattern, text)
    turns, i = [], 0
    while i < len(parts):
        part = parts[i].strip()
        if re.match(pattern, part):
            if i + 1 < len(parts):
                turns.append((part + parts[i + 1]).strip())
                i += 2
            else:
                turns.append(part)
                i += 1
        else:
            i += 1
    return turns


def group_turns_into_batches(turns: Sequence[str], max_speakers: int = 3, max_bytes: int = 300) -> List[str]:
    """inference.py:487-520: greedy batches of at most max_speakers turns / max_bytes UTF-8."""
    batches, cur, cur_bytes = [], [], 0
    for turn in turns:
        tb = len(turn.encode("utf-8"))
        if len(cur) >= max_speakers or (cur_bytes + tb > max_bytes and cur):
            batches.append("\n".join(cur))
            cur, cur_bytes = [turn], tb
        else:
            cur.append(turn)
            cur_bytes += tb
    if cur:
        batches.append("\n".join(cur))
    return batches


def base_conversation(prompt_text: Optional[Union[str, List[str]]] = None,
                      prompt_tokens: Optional[Union[np.ndarray, List[np.ndarray]]] = None) -> Conversation:
    """The system message generate_long starts from (inference.py:558-600): reference texts are
    speaker-tagged and their codes appended as one VQ part."""
    use_prompt = bool(prompt_text) and prompt_tokens is not None and len(prompt_tokens) > 0
    if use_prompt and isinstance(prompt_text, str):
        prompt_text, prompt_tokens = [prompt_text], [prompt_tokens]
    if use_prompt:
        if len(prompt_text) != len(prompt_tokens):
            raise ValueError("Prompt text and tokens must have the same length")
        tagged = [t if re.search(r"<\|speaker:\d+\|>", t) else f"<|speaker:{i}|>{t}"
                  for i, t in enumerate(prompt_text)]
        parts = [TextPart(text="convert the provided text to speech reference to the following:\n\nText:\n"),
                 TextPart(text="\n".join(tagged)),
                 TextPart(text="\n\nSpeech:\n"),
                 VQPart(codes=np.concatenate([np.asarray(c) for c in prompt_tokens], axis=1))]
    else:
        parts = [TextPart(text="convert the provided text to speech")]
    conv = Conversation()
    conv.append(Message(role="system", parts=parts, add_im_start=True, add_im_end=True))
    return conv


def with_user_turn(conv: Conversation, text: str) -> Conversation:
    """A copy of conv with the user batch and an open voice-assistant header (inference.py:618-642)."""
    gen = copy.deepcopy(conv)
    gen.append(Message(role="user", parts=[TextPart(text=text)], add_im_start=True, add_im_end=True))
    gen.append(Message(role="assistant", parts=[], modality="voice", add_im_start=True, add_im_end=False))
    return gen
