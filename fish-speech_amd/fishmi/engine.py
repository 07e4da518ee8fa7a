"""LLM worker seam: the drop-in for the reference's
  * GenerateResponse / WrappedGenerateResponse / GenerateRequest  inference.py:447-451, 736-745
  * generate_long                                                  inference.py:523-733
  * launch_thread_safe_queue                                       inference.py:748-799
backed by libfishmi (fishmi.llm.DualARModel).  Same request keys, same response stream
(one "sample" per text batch with codes = y[1:, T:-1], then "next"), same error contract (an
exception becomes status="error" carrying the exception; the worker keeps serving), one daemon
worker thread owning the model, FIFO requests, `None` stops the worker.

Differences, by design: codes are host int32 numpy arrays (C, N) rather than device tensors
(the vocoder handle takes host codes); sampling uses the counter-based RNG of the HIP sampler,
seeded by the request's `seed` (a fresh random seed when absent), since torch's global RNG
stream is not reproducible across implementations anyway.
"""
from __future__ import annotations

import copy
import logging
import os
import queue
import threading
import time
import traceback
from dataclasses import dataclass
from typing import Iterator, List, Literal, Optional, Union

import numpy as np

from . import prompt as P

log = logging.getLogger("fishmi.engine")


@dataclass
class GenerateResponse:
    action: Literal["sample", "next"]
    codes: Optional[np.ndarray] = None
    text: Optional[str] = None
    # streaming (generate_long(stream_frames=K) only): index of this chunk within its text batch.
    # The chunks of one batch are consecutive code columns of one causal stream: vocode them with
    # the codec's carried state (FishMICodec.stream_reset at chunk 0, then decode_chunk).
    stream: Optional[int] = None
    # multi-GPU serving (fishmi.dist_serving with a vocoder): the float32 PCM of these codes, vocoded
    # on the rank that decoded them; the TTS engine then only forwards it
    audio: Optional[np.ndarray] = None


@dataclass
class WrappedGenerateResponse:
    status: Literal["success", "error"]
    response: Optional[Union[GenerateResponse, Exception]] = None


@dataclass
class GenerateRequest:
    request: dict
    response_queue: queue.Queue


def _codes(x) -> np.ndarray:
    try:  # torch tensors from callers of the reference API
        import torch

        if isinstance(x, torch.Tensor):
            return x.detach().cpu().numpy()
    except ImportError:  # pragma: no cover
        pass
    return np.asarray(x)


@dataclass
class BatchPlan:
    """One generate() of generate_long: the full prompt, how much of it the slot already holds."""
    enc: np.ndarray      # (C+1, T) int32: the whole conversation prompt of this batch
    L: int               # positions [0, L) reused from the slot's KV (prefill enc[:, L:] at pos0 = L)
    sp: object           # the slot's sampling record (model.sampling(...))
    max_new: int         # most columns to emit, the prefill's included (inference.py:262-271)
    text: str


class ConversationJob:
    """generate_long's host side (inference.py:523-733) as a state machine, so that one request's
    text batches can be driven by the serial worker (generate_long) or interleaved with other
    requests' on batched KV slots (fishmi.batching.BatchedWorker) with the same prompts, seeds and
    prefix-reuse decisions.  next_batch() -> BatchPlan | "next" (a sample's batches are done) |
    None (the request is done); finish_batch(y, fed_cols) -> the batch's codes."""

    def __init__(self, model, *, text: str, tokenizer=None, device=None, decode_one_token=None, num_samples: int = 1,
                 max_new_tokens: int = 0, top_p: float = 0.9, top_k: int = 30, repetition_penalty: float = 1.1,
                 temperature: float = 1.0, compile: bool = False, iterative_prompt: bool = True,
                 chunk_length: int = 512, prompt_text=None, prompt_tokens=None, seed: Optional[int] = None,
                 reuse_prefix: bool = False, stream_frames: int = 0, mask_im_end: bool = False):
        if not (0 < top_p <= 1):
            raise AssertionError("top_p must be in (0, 1]")
        if not (0 < temperature < 2):
            raise AssertionError("temperature must be in (0, 2)")
        self.tok = tokenizer if tokenizer is not None else getattr(model, "tokenizer", None)
        if self.tok is None:
            raise ValueError("generate_long needs the checkpoint tokenizer (tokenizer.json)")
        self.model = model
        self.C = model.cfg.num_codebooks
        if isinstance(prompt_tokens, (list, tuple)):
            ptoks = [_codes(t) for t in prompt_tokens]
        elif prompt_tokens is not None:
            # one (C, T) array: base_conversation wraps it together with a str prompt_text, as the
            # reference does (inference.py:544-547)
            ptoks = _codes(prompt_tokens)
        else:
            ptoks = None
        self.base = P.base_conversation(prompt_text, ptoks)
        turns = P.split_text_by_speaker(text)
        self.batches = P.group_turns_into_batches(turns, max_speakers=5, max_bytes=chunk_length) if turns else [text]
        log.info("Split into %d turns, grouped into %d batches", len(turns), len(self.batches))
        self.num_samples, self.max_new_tokens = num_samples, max_new_tokens
        self.top_p, self.top_k, self.temperature = top_p, top_k, temperature
        self.seed, self.reuse_prefix, self.stream_frames = seed, reuse_prefix, stream_frames
        self.mask_im_end = mask_im_end
        self.rng = np.random.default_rng(seed)
        self.sample_idx, self.batch_idx = 0, 0
        self.conv = copy.deepcopy(self.base)
        self.cached = None  # (C+1, P) tokens whose KV the slot holds at positions [0, P)
        self.plan: Optional[BatchPlan] = None
        self.t0 = time.perf_counter()

    def next_batch(self):
        if self.sample_idx >= self.num_samples:
            return None
        if self.batch_idx >= len(self.batches):
            self.sample_idx += 1
            self.batch_idx = 0
            self.conv = copy.deepcopy(self.base)
            self.cached = None
            self.t0 = time.perf_counter()
            return "next"
        batch_text = self.batches[self.batch_idx]
        self.conv.append(P.Message(role="user", parts=[P.TextPart(text=batch_text)]))
        gen = copy.deepcopy(self.conv)
        gen.append(P.Message(role="assistant", parts=[], modality="voice", add_im_end=False))
        encoded, _, _ = gen.encode_for_inference(self.tok, num_codebooks=self.C)
        max_len = self.model.cfg.max_seq_len
        if encoded.shape[1] > max_len - 2048:
            raise ValueError(f"Prompt is too long: {encoded.shape[1]} > {max_len - 2048}")
        s = int(self.rng.integers(0, 2**63 - 1)) if self.seed is None \
            else self.seed + 1000003 * self.sample_idx + self.batch_idx
        enc = encoded.astype(np.int32)
        L = 0
        if self.reuse_prefix and self.cached is not None:
            n = min(self.cached.shape[1], enc.shape[1] - 1)  # at least one new position to prefill
            same = np.all(self.cached[:, :n] == enc[:, :n], axis=0)
            L = int(n if same.all() else np.argmin(same))
        T = enc.shape[1]
        mx = self.max_new_tokens if (self.max_new_tokens and T + self.max_new_tokens <= max_len) else max_len - T
        self.plan = BatchPlan(enc, L, self.model.sampling(self.temperature, self.top_p, self.top_k, s,
                                                          self.mask_im_end), mx, batch_text)
        return self.plan

    def finish_batch(self, y: np.ndarray, fed_cols: np.ndarray) -> np.ndarray:
        """y: (C+1, n) the emitted columns (generate()'s seq[:, T:]); fed_cols: the columns the slot
        consumed while decoding (its KV past the prompt)."""
        plan = self.plan
        if self.reuse_prefix:
            self.cached = np.concatenate([plan.enc, fed_cols], axis=1)
        codes = np.ascontiguousarray(y[1:, :-1])  # y[1:, prompt_length:-1] of the reference
        if (codes < 0).any():
            raise AssertionError(f"Negative code found: {codes}")
        log.info("Batch %d: generated %d frames in %.2fs", self.batch_idx, y.shape[1], time.perf_counter() - self.t0)
        self.conv.append(P.Message(role="assistant", parts=[P.VQPart(codes=codes)], modality="voice"))
        self.batch_idx += 1
        self.plan = None
        return codes


def generate_long(*, model, text: str, tokenizer: Optional[P.FishTokenizer] = None, device=None,
                  decode_one_token=None, num_samples: int = 1, max_new_tokens: int = 0,
                  top_p: float = 0.9, top_k: int = 30, repetition_penalty: float = 1.1,
                  temperature: float = 1.0, compile: bool = False, iterative_prompt: bool = True,
                  chunk_length: int = 512, prompt_text: Optional[Union[str, List[str]]] = None,
                  prompt_tokens=None, seed: Optional[int] = None,
                  reuse_prefix: bool = False, stream_frames: int = 0, stream_growth: int = 1,
                  stream_max: int = 0, mask_im_end: bool = False) -> Iterator[GenerateResponse]:
    """inference.py:523-733 on the native model (slot 0).  `device`, `decode_one_token`, `compile`,
    `iterative_prompt` and `repetition_penalty` are accepted for signature compatibility; like
    the reference, repetition_penalty is not applied (RAS is, inside the sampler).

    The reference re-prefills the whole growing conversation for every text batch
    (inference.py:620-724).  With reuse_prefix, each batch after the first keeps the slot's KV for
    the longest prefix its new prompt shares with what the slot already ran (the previous prompt
    plus the columns fed back while generating), and prefills only the rest (fm_llm_generate_at).
    The prompt tokens are the same, so the codes are the same up to the fp32 accumulation order of
    the reused positions: the decode GEMVs and the prompt GEMM sum K in different orders, so a
    reused K / V row can differ from the re-prefilled one by an ulp (bf16).  The tests hold both
    flows to the reference's own bf16 generate_long (tests/test_gpu_engine.py).  It is opt-in: the
    default is the reference's own re-prefill flow.

    stream_frames > 0 (BASELINE config 5's streamed vocoder): each batch's codes are yielded as they
    are decoded, `stream_frames` columns at a time (GenerateResponse.stream = chunk index), instead of
    once per batch; their concatenation equals the batch's codes.  stream_growth > 1: each chunk is
    that many times the previous one (up to stream_max frames when > 0) -- a first chunk of one
    frame reaches the vocoder right after the prompt, and a chunk of k frames always takes less
    time to generate than the audio already streamed takes to play.  mask_im_end: fixed-length
    generation for benchmarks (the semantic bias keeps <|im_end|> at -inf)."""
    job = ConversationJob(model, text=text, tokenizer=tokenizer, num_samples=num_samples,
                          max_new_tokens=max_new_tokens, top_p=top_p, top_k=top_k, temperature=temperature,
                          chunk_length=chunk_length, prompt_text=prompt_text, prompt_tokens=prompt_tokens,
                          seed=seed, reuse_prefix=reuse_prefix, stream_frames=stream_frames,
                          mask_im_end=mask_im_end)
    while True:
        plan = job.next_batch()
        if plan is None:
            return
        if plan == "next":
            yield GenerateResponse(action="next")
            continue
        enc, L = plan.enc, plan.L
        if stream_frames > 0:
            y, fed_cols = yield from _stream_batch(model, enc, L, max_new_tokens, stream_frames, plan.text, plan.sp,
                                                   stream_growth, stream_max)
        else:
            if L > 0:
                y = model.generate_at(enc[:, L:], L, max_new_tokens, temperature=temperature, top_p=top_p,
                                      top_k=top_k, seed=plan.sp.seed, mask_im_end=mask_im_end)
            else:
                y = model.generate(enc, max_new_tokens, temperature=temperature, top_p=top_p, top_k=top_k,
                                   seed=plan.sp.seed, mask_im_end=mask_im_end)
            fed = model.slot_pos() - enc.shape[1] if reuse_prefix else 0  # columns fed back while decoding
            fed_cols = y[:, :fed]
        codes = job.finish_batch(y, fed_cols)
        if stream_frames <= 0:
            yield GenerateResponse(action="sample", codes=codes, text=plan.text)


def _stream_batch(model, enc, L, max_new_tokens, stream_frames, text, sp, growth=1, cap=0):
    """One generate() of generate_long, decoded `stream_frames` frames at a time (prefill, then
    decode_frames chunks on slot 0; with growth > 1 the chunks grow geometrically up to cap): yields
    the confirmed code columns of each chunk, returns (y (C+1, n) as generate() would, every column
    fed back to the model)."""
    T = enc.shape[1]
    mx = max_new_tokens if (max_new_tokens and T + max_new_tokens <= model.cfg.max_seq_len) \
        else model.cfg.max_seq_len - T
    im_end = model.cfg.im_end_id
    cols = [model.prefill(0, enc[:, L:], sp, pos0=L)]
    fed = []
    done = cols[0][0] == im_end or mx <= 1
    emitted, chunk, step = 0, 0, stream_frames
    while not done:
        k = min(step, mx - len(cols))
        step = step * max(1, growth)
        if cap > 0:
            step = min(step, cap)
        out = model.decode_frames([0], k)[:, 0, :]
        fed.extend([cols[-1]] + list(out[:-1]))  # frame j feeds the column sampled before it
        for c in out:
            cols.append(c)
            if c[0] == im_end or len(cols) >= mx:
                done = True
                break
        # every column but the newest is final (the newest may be the batch's dropped last column)
        if len(cols) - 1 > emitted:
            part = np.stack(cols[emitted:len(cols) - 1], axis=1)[1:]
            yield GenerateResponse(action="sample", codes=np.ascontiguousarray(part), text=text, stream=chunk)
            emitted, chunk = len(cols) - 1, chunk + 1
    y = np.stack(cols, axis=1)
    fed_cols = np.stack(fed, axis=1) if fed else y[:, :0]
    return y, fed_cols


def _device_index(device) -> int:
    if device is None:
        return 0
    if isinstance(device, int):
        return device
    if not isinstance(device, str):  # torch.device
        idx = getattr(device, "index", None)
        return int(idx) if isinstance(idx, int) else 0
    return int(device.split(":")[1]) if ":" in device else 0


def _precision(precision) -> str:
    s = str(precision).lower()
    if "float32" in s or s in ("fp32", "f32", "float"):
        return "fp32"
    return "bf16"  # torch.bfloat16 / torch.half / "bf16": the bf16 path


def load_model(checkpoint_path: str, device=0, precision="bf16", max_slots: int = 1):
    """init_model (inference.py:362-392): the native Dual-AR model with its tokenizer attached."""
    from .llm import DualARModel

    model = DualARModel.from_pretrained(checkpoint_path, device=_device_index(device),
                                       precision=_precision(precision), max_slots=max_slots)
    if model.tokenizer is None:
        raise ValueError(f"{checkpoint_path} has no tokenizer.json")
    return model


def launch_thread_safe_queue(checkpoint_path, device, precision, compile: bool = False,
                             model=None, max_slots: int = 1, tick_frames: int = 8) -> "queue.Queue":
    """inference.py:748-799: a daemon worker owning the model; returns its input queue once the
    model is loaded.  `model` (optional) hands in an already-built DualARModel (tests).

    max_slots == 1: the reference's worker, one request at a time (generate_long on slot 0).
    max_slots > 1: fishmi.batching.BatchedWorker -- up to max_slots requests decode together on
    their own KV slots (batched hipGraph frames), same queue contract (BASELINE config 3)."""
    ready = threading.Event()
    failure: List[BaseException] = []
    holder: dict = {}

    def worker():
        try:
            m = model if model is not None else load_model(checkpoint_path, device, precision, max_slots)
        except BaseException as e:  # surface load failures to the caller instead of hanging
            failure.append(e)
            ready.set()
            return
        if max_slots > 1:
            from .batching import BatchedWorker

            w = BatchedWorker(m, max_slots, tick_frames)
            holder["q"] = w.input
            ready.set()
            w.run()
            return
        input_queue: "queue.Queue" = queue.Queue()
        holder["q"] = input_queue
        ready.set()
        while True:
            item = input_queue.get()
            if item is None:
                break
            try:
                for chunk in generate_long(model=m, **item.request):
                    item.response_queue.put(WrappedGenerateResponse(status="success", response=chunk))
            except Exception as e:
                log.error(traceback.format_exc())
                item.response_queue.put(WrappedGenerateResponse(status="error", response=e))

    threading.Thread(target=worker, daemon=True).start()
    ready.wait()
    if failure:
        raise failure[0]
    return holder["q"]
