"""Batched LLM worker: concurrent generate_long requests on the KV slots of one GPU (BASELINE config 3
through the reference's own seam).

The reference's worker (inference.py:748-799) serves one request at a time at batch 1.  This worker
keeps the same queue contract -- GenerateRequest(request, response_queue) in, WrappedGenerateResponse
("sample" per text batch, or streamed chunks, then "next"; "error" carrying the exception) out, `None`
stops it -- but gives every request a KV slot of its own and advances all of them together:

  * each request is a fishmi.engine.ConversationJob (the same prompts, seeds and prefix-reuse
    decisions as the serial generate_long);
  * a tick prefills the text batches that are starting (together, fm_llm_prefill_batch, when none
    reuses a cached prefix), then decodes `k` batched frames for every slot that is decoding
    (fm_llm_decode_frames: one hipGraph-captured frame per step), k = min(tick_frames, the fewest
    columns any of them may still emit);
  * a slot whose batch has ended (<|im_end|> or max_new_tokens) is answered and moves to its next
    text batch; frames a slot decodes past its <|im_end|> within a tick are discarded (its next
    batch re-prefills those positions, as every batch does);
  * requests wait in FIFO order for a free slot.

In the fp32 validation mode a batched frame computes every slot's row exactly as a batch-1 frame
does, so each request's codes equal its serial generate_long codes (tests/test_batching.py on CPU
with a scripted model, tests/test_gpu_engine.py on the GPU).  In bf16 the batched linears sum in a
different order (bsacc_kernel), within the bf16 parity bound of tests/test_gpu_00_timed_configs.py.
"""
from __future__ import annotations

import collections
import logging
import queue
import traceback
from dataclasses import dataclass, field
from typing import Deque, Dict, List, Optional

import numpy as np

from .engine import ConversationJob, GenerateRequest, GenerateResponse, WrappedGenerateResponse

log = logging.getLogger("fishmi.batching")


@dataclass
class _Slot:
    item: GenerateRequest
    job: ConversationJob
    plan: object = None
    cols: List[np.ndarray] = field(default_factory=list)  # every column the batch produced (overshoot too)
    n_valid: int = 0       # columns of the batch's y (up to <|im_end|> / max_new)
    frames: int = 0        # decode frames run for the batch (= columns fed back)
    emitted: int = 0       # streamed: columns already sent
    chunk: int = 0         # streamed: next chunk index
    done: bool = False     # the batch has ended


class BatchedWorker:
    def __init__(self, model, max_slots: Optional[int] = None, tick_frames: int = 8):
        self.m = model
        self.max_slots = max_slots or model.max_slots
        if self.max_slots > model.max_slots:
            raise ValueError(f"max_slots {self.max_slots} > the model's {model.max_slots}")
        self.tick_frames = max(1, tick_frames)
        self.im_end = model.cfg.im_end_id
        self.input: "queue.Queue" = queue.Queue()
        self.pending: Deque[GenerateRequest] = collections.deque()
        self.active: Dict[int, _Slot] = {}
        self.free = list(range(self.max_slots))[::-1]
        self.stopping = False
        self.stats = {"ticks": 0, "frames": 0, "slot_frames": 0, "requests": 0}
        self.on_done = None  # optional callback(item): the request has sent its last response

    # ---- responses ---------------------------------------------------------------------------
    @staticmethod
    def _put(item: GenerateRequest, resp):
        if isinstance(resp, Exception):
            item.response_queue.put(WrappedGenerateResponse(status="error", response=resp))
        else:
            item.response_queue.put(WrappedGenerateResponse(status="success", response=resp))

    def _fail(self, slot: int, e: Exception, item: Optional[GenerateRequest] = None):
        st = self.active.pop(slot, None)
        log.error("request failed: %s", traceback.format_exc())
        item = st.item if st is not None else item
        self._put(item, e)
        self.free.append(slot)
        if self.on_done is not None:
            self.on_done(item)

    # ---- per-slot state machine -----------------------------------------------------------------
    def _advance(self, slot: int) -> bool:
        """Move the slot to its request's next text batch; True if it needs a prefill."""
        st = self.active[slot]
        while True:
            plan = st.job.next_batch()
            if plan is None:
                self.active.pop(slot)
                self.free.append(slot)
                self.stats["requests"] += 1
                if self.on_done is not None:
                    self.on_done(st.item)
                return False
            if plan == "next":
                self._put(st.item, GenerateResponse(action="next"))
                continue
            st.plan, st.cols, st.n_valid, st.frames = plan, [], 0, 0
            st.emitted, st.chunk, st.done = 0, 0, False
            return True

    def _take(self, st: _Slot, col: np.ndarray):
        """One column the slot's batch produced; the batch ends at <|im_end|> or max_new columns."""
        st.cols.append(col)
        if st.done:
            return
        st.n_valid += 1
        if col[0] == self.im_end or st.n_valid >= st.plan.max_new:
            st.done = True

    def _stream(self, slot: int):
        st = self.active[slot]
        if st.job.stream_frames <= 0:
            return
        final = st.n_valid - 1  # every valid column but the newest is a code column for sure
        if final > st.emitted and (st.done or final - st.emitted >= st.job.stream_frames):
            part = np.stack(st.cols[st.emitted:final], axis=1)[1:]
            self._put(st.item, GenerateResponse(action="sample", codes=np.ascontiguousarray(part),
                                                text=st.plan.text, stream=st.chunk))
            st.emitted, st.chunk = final, st.chunk + 1

    def _finish(self, slot: int) -> bool:
        """The slot's batch ended: answer it and plan the next one (True: needs a prefill)."""
        st = self.active[slot]
        self._stream(slot)
        y = np.stack(st.cols[: st.n_valid], axis=1)
        nf = min(st.frames, st.n_valid)  # fed columns the prefix-reuse bookkeeping may rely on
        fed = np.stack(st.cols[:nf], axis=1) if nf else y[:, :0]
        codes = st.job.finish_batch(y, fed)
        if st.job.stream_frames <= 0:
            self._put(st.item, GenerateResponse(action="sample", codes=codes, text=st.plan.text))
        return self._advance(slot)

    # ---- device work ------------------------------------------------------------------------------
    def _prefill(self, slots: List[int]):
        fresh = [s for s in slots if self.active[s].plan.L == 0]
        if len(fresh) > 1:
            firsts = self.m.prefill_batch(fresh, [self.active[s].plan.enc for s in fresh],
                                          [self.active[s].plan.sp for s in fresh])
            for s, col in zip(fresh, firsts):
                self._take(self.active[s], col)
        else:
            fresh = []
        for s in slots:
            if s in fresh:
                continue
            p = self.active[s].plan
            self._take(self.active[s], self.m.prefill(s, p.enc[:, p.L:], p.sp, pos0=p.L))

    def tick(self, block: Optional[bool] = None) -> bool:
        """One scheduling step; False once stopped and idle.  block (default: when idle) waits for
        the next request on the input queue."""
        if block is None:
            block = not self.active and not self.pending and not self.stopping
        while True:
            try:
                item = self.input.get(block=block)
            except queue.Empty:
                break
            block = False
            if item is None:
                self.stopping = True
            elif not self.stopping:
                self.pending.append(item)
            else:  # after the stop sentinel: answered, never silently dropped
                self._put(item, RuntimeError("the LLM worker is stopping"))
        starting: List[int] = []
        while self.pending and self.free:
            item = self.pending.popleft()
            slot = self.free.pop()
            try:
                self.active[slot] = _Slot(item, ConversationJob(self.m, **item.request))
                if self._advance(slot):
                    starting.append(slot)
            except Exception as e:
                self._fail(slot, e, item)
        # prefill the batches that start, answering (and replanning) those that end at once
        while starting:
            try:
                self._prefill(starting)
            except Exception:
                # one bad request must not take down the cohort: the slots that have no first column
                # yet are prefilled again one at a time, and only those that fail get the error
                ok = []
                for s in starting:
                    if self.active[s].cols:
                        ok.append(s)
                        continue
                    try:
                        self._prefill([s])
                        ok.append(s)
                    except Exception as e:
                        self._fail(s, e)
                starting = ok
            nxt = []
            for s in starting:
                if self.active[s].done:
                    try:
                        if self._finish(s):
                            nxt.append(s)
                    except Exception as e:
                        self._fail(s, e)
            starting = nxt
        live = [s for s, st in self.active.items() if not st.done]
        if live:
            k = min(self.tick_frames, min(self.active[s].plan.max_new - self.active[s].n_valid for s in live))
            try:
                out = self.m.decode_frames(live, k)
            except Exception as e:
                for s in live:
                    self._fail(s, e)
                return True
            self.stats["ticks"] += 1
            self.stats["frames"] += k
            self.stats["slot_frames"] += k * len(live)
            for j, s in enumerate(live):
                st = self.active[s]
                for f in range(k):
                    self._take(st, out[f, j])
                st.frames += k
                try:  # a response queue that raises fails its own request only
                    self._stream(s)
                except Exception as e:
                    self._fail(s, e)
            for s in live:
                if s in self.active and self.active[s].done:
                    try:
                        if self._finish(s):
                            self._prefill_later(s)
                    except Exception as e:
                        self._fail(s, e)
        return not (self.stopping and not self.active and not self.pending)

    def _prefill_later(self, slot: int):
        # a slot moving to its next text batch is prefilled right away (same tick), alone
        try:
            self._prefill([slot])
            if self.active[slot].done and self._finish(slot):
                self._prefill_later(slot)
        except Exception as e:
            self._fail(slot, e)

    def fail_all(self, e: Exception):
        """Answer every active and waiting request with `e` and free their slots (a failure outside the
        per-request guards: the requests are lost, the callers are not left waiting)."""
        for s in list(self.active):
            self._fail(s, e)
        while self.pending:
            item = self.pending.popleft()
            self._put(item, e)
            if self.on_done is not None:
                self.on_done(item)

    def run(self):
        while True:
            try:
                if not self.tick():
                    return
            except Exception as e:  # keep serving: the requests in flight get the error
                log.error("worker tick failed: %s", traceback.format_exc())
                self.fail_all(e)
