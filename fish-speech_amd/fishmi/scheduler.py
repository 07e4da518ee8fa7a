"""Dynamic data-parallel request queue for batched serving (BASELINE configs 3 and 4).

Rank 0 owns the request list. Each rank decodes up to `max_concurrent` streams in its own KV
slots, as one batched Dual-AR frame per step (the hipGraph-captured decode frame). Ranks pull work
at synchronous *ticks*:

  1. all_gather of (free slots, active streams, finished results) from every rank, as int64;
  2. rank 0 hands out the next requests one at a time, round-robin over the ranks that still
     have free slots. This is a pure function of the gathered counts, so every rank computes the
     same assignment without another message;
  3. rank 0 scatters the assigned request descriptors: id, prompt length, frames and seed, then
     the prompt token matrix;
  4. results of the streams that finished since the last tick are gathered to rank 0: int16 PCM
     (the wire format of tools/server/inference.py:18-39) or the codes.

A rank that frees slots early gets new work at the next tick, and lengths may differ per request.
The loop ends when the queue is empty and no rank has an active stream. A tick is every
`tick_frames` decode frames: three small collectives against about 11 ms of decode per frame
at B=32.

Collectives run on the default process group: RCCL with device tensors on the GPU box, gloo with
host tensors in the CPU tests. There is no exchange on the decode path itself.

The reference's precedent is a static `files[RANK::WORLD_SIZE]` split
(tools/vqgan/extract_vq.py:150-197). A static split idles ranks whose requests finish early; the
tick queue does not.
"""
from __future__ import annotations

import dataclasses
import queue as _queue
import threading
import time
from typing import Callable, Dict, List, Optional, Sequence

import numpy as np


@dataclasses.dataclass
class Request:
    id: int
    prompt: np.ndarray   # (C+1, T) int32
    frames: int          # frames to decode (max_new_tokens; <|im_end|> may end it earlier)
    seed: int = 0


@dataclasses.dataclass
class Result:
    id: int
    rank: int
    data: np.ndarray     # int16 PCM or int32 codes, 1-D


def _dist():
    import torch.distributed as dist

    return dist


def _device():
    import torch

    if _dist().get_backend() == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def assign(free: Sequence[int], remaining: int) -> List[int]:
    """How many new requests each rank gets: one at a time, round-robin over ranks with free slots,
    until the queue or the free slots run out. Every rank evaluates this identically."""
    take = [0] * len(free)
    left = list(free)
    while remaining > 0 and any(left):
        for r in range(len(left)):
            if remaining and left[r]:
                take[r] += 1
                left[r] -= 1
                remaining -= 1
    return take


class TickQueue:
    """The rank-0-owned request queue, pulled at synchronous ticks (module docstring)."""

    HDR = 4  # id, T, frames, seed (int64 words per descriptor)

    def __init__(self, requests: Optional[Sequence[Request]], rows: int):
        dist = _dist()
        self.world, self.rank = dist.get_world_size(), dist.get_rank()
        self.rows = rows
        self.dev = _device()
        self.pending = list(requests or []) if self.rank == 0 else []
        import torch

        n = torch.tensor([len(self.pending)], dtype=torch.int64, device=self.dev)
        dist.broadcast(n, src=0)
        self.remaining = int(n.item())
        self.ticks = 0
        self.results: List[Result] = []   # rank 0: gathered results, in arrival order

    def tick(self, free: int, active: int, finished: Sequence[Result] = ()) -> Optional[List[Request]]:
        """One synchronous tick. Returns this rank's new requests, or None once the queue is empty
        and no rank has active streams (the caller stops)."""
        import torch

        dist = _dist()
        self.ticks += 1
        mine = torch.tensor([free, active, len(finished)], dtype=torch.int64, device=self.dev)
        allv = [torch.zeros_like(mine) for _ in range(self.world)]
        dist.all_gather(allv, mine)
        st = np.stack([a.cpu().numpy() for a in allv])
        if st[:, 2].any():
            self._gather_results(finished, st[:, 2])
        take = assign(st[:, 0].tolist(), self.remaining)
        total = sum(take)
        if total == 0:
            return None if (self.remaining == 0 and st[:, 1].sum() == 0) else []
        out = self._scatter(take)
        self.remaining -= total
        return out

    def _scatter(self, take: List[int]) -> List[Request]:
        import torch

        dist = _dist()
        # header pass: per-rank payload lengths (int32 words) so one padded scatter follows
        lens = torch.zeros(self.world, dtype=torch.int64, device=self.dev)
        chunks = None
        if self.rank == 0:
            bufs = []
            for r in range(self.world):
                reqs, self.pending = self.pending[: take[r]], self.pending[take[r]:]
                words: List[np.ndarray] = []
                for q in reqs:
                    p = np.ascontiguousarray(q.prompt, dtype=np.int32)
                    if p.ndim != 2 or p.shape[0] != self.rows:
                        raise ValueError(f"request {q.id}: prompt shape {p.shape}, expected ({self.rows}, T)")
                    hdr = np.array([q.id, p.shape[1], q.frames, q.seed], np.int64)
                    words += [hdr.view(np.int32), p.reshape(-1)]
                b = np.concatenate(words) if words else np.zeros(0, np.int32)
                bufs.append(b)
                lens[r] = b.size
        dist.broadcast(lens, src=0)
        nmax = max(int(lens.max().item()), 1)
        mine = torch.zeros(nmax, dtype=torch.int32, device=self.dev)
        if self.rank == 0:
            chunks = []
            for b in bufs:
                pad = np.zeros(nmax, np.int32)
                pad[: b.size] = b
                chunks.append(torch.from_numpy(pad).to(self.dev))
        dist.scatter(mine, chunks, src=0)
        buf = mine.cpu().numpy()[: int(lens[self.rank].item())]
        out, o = [], 0
        for _ in range(take[self.rank]):
            rid, T, frames, seed = buf[o: o + 2 * self.HDR].view(np.int64).tolist()
            o += 2 * self.HDR
            prompt = buf[o: o + self.rows * T].reshape(self.rows, T).copy()
            o += self.rows * T
            out.append(Request(int(rid), prompt, int(frames), int(seed)))
        return out

    def _gather_results(self, finished: Sequence[Result], counts: np.ndarray):
        """Finished streams' payloads to rank 0: (id, n, payload) records, one padded gather."""
        import torch

        dist = _dist()
        words: List[np.ndarray] = []
        for res in finished:
            d = np.ascontiguousarray(res.data)
            raw = d.view(np.uint8)
            pad = (-raw.size) % 4
            raw = np.concatenate([raw, np.zeros(pad, np.uint8)]) if pad else raw
            code = {np.dtype(np.int16): 1, np.dtype(np.int32): 2}[d.dtype]
            words += [np.array([res.id, d.size, code], np.int64).view(np.int32), raw.view(np.int32)]
        b = np.concatenate(words) if words else np.zeros(0, np.int32)
        n = torch.tensor([b.size], dtype=torch.int64, device=self.dev)
        ns = [torch.zeros_like(n) for _ in range(self.world)]
        dist.all_gather(ns, n)
        ns = [int(x.item()) for x in ns]
        nmax = max(max(ns), 1)
        pad = np.zeros(nmax, np.int32)
        pad[: b.size] = b
        t = torch.from_numpy(pad).to(self.dev)
        outs = [torch.empty_like(t) for _ in range(self.world)] if self.rank == 0 else None
        dist.gather(t, outs, dst=0)
        if self.rank != 0:
            return
        for r in range(self.world):
            buf = outs[r].cpu().numpy()[: ns[r]]
            o = 0
            for _ in range(int(counts[r])):
                rid, size, code = buf[o: o + 6].view(np.int64).tolist()
                o += 6
                dt = np.int16 if code == 1 else np.int32
                nb = size * np.dtype(dt).itemsize
                nw = (nb + 3) // 4
                self.results.append(Result(int(rid), r, buf[o: o + nw].view(np.uint8)[:nb].view(dt).copy()))
                o += nw


@dataclasses.dataclass
class _Stream:
    req: Request
    cols: List[np.ndarray]
    done: int = 0


def serve(queue: TickQueue, max_concurrent: int, start: Callable[[int, Request], np.ndarray],
          step: Callable[[List[int], int], np.ndarray], finish: Callable[[int, Request, np.ndarray], np.ndarray],
          tick_frames: int = 16, im_end: Optional[int] = None,
          start_batch: Optional[Callable[[List[tuple]], np.ndarray]] = None,
          progress: Optional[Callable[[int, Request, List[np.ndarray]], None]] = None) -> Dict[str, int]:
    """Per-rank serving loop over the tick queue.

    start(slot, req) prefills the request into its KV slot and returns the first column (C+1,);
    start_batch([(slot, req), ...]), when given, prefills a tick's new requests together and returns
    their first columns (n, C+1) (fm_llm_prefill_batch).
    step(slots, n) decodes n batched frames for the slots and returns (n, len(slots), C+1).
    finish(slot, req, cols (C+1, N)) turns the stream into its result payload (PCM or codes).
    progress(slot, req, cols), when given, sees every live stream's columns so far after each
    tick's decode (a consumer may start on all but the newest, which may be the dropped last one).
    A stream ends after req.frames columns, or at the column whose main token is `im_end`. The
    last column is dropped either way, like `codes = y[1:, T:-1]` in generate_long
    (inference.py:683-688).
    Returns counters: frames decoded, streams served, ticks."""
    free_slots = list(range(max_concurrent))[::-1]
    active: Dict[int, _Stream] = {}
    finished: List[Result] = []
    frames = served = 0
    while True:
        new = queue.tick(len(free_slots), len(active), finished)
        finished = []
        if new is None:
            break
        if start_batch is not None and new:
            pairs = [(free_slots.pop(), req) for req in new]
            firsts = start_batch(pairs)
            for (slot, req), col in zip(pairs, firsts):
                active[slot] = _Stream(req, [col], 1)
        else:
            for req in new:
                slot = free_slots.pop()
                active[slot] = _Stream(req, [start(slot, req)], 1)
        done_now = []
        for slot, s in active.items():  # a stream can end on its first column
            if s.done >= s.req.frames or (im_end is not None and s.cols[-1][0] == im_end):
                done_now.append(slot)
        if active and len(done_now) < len(active):
            live = [s for s in active if s not in done_now]
            n = min(tick_frames, min(active[s].req.frames - active[s].done for s in live))
            out = step(live, n)
            frames += n * len(live)
            for j, slot in enumerate(live):
                st = active[slot]
                for k in range(n):
                    if st.done >= st.req.frames or (im_end is not None and st.cols[-1][0] == im_end):
                        break
                    st.cols.append(out[k, j])
                    st.done += 1
                if st.done >= st.req.frames or (im_end is not None and st.cols[-1][0] == im_end):
                    done_now.append(slot)
                elif progress is not None:
                    progress(slot, st.req, st.cols)
        for slot in done_now:
            st = active.pop(slot)
            cols = np.stack(st.cols, 1)[:, :-1]  # codes = y[1:, T:-1]: the last column is dropped
            finished.append(Result(st.req.id, queue.rank, finish(slot, st.req, cols)))
            free_slots.append(slot)
            served += 1
    return {"frames": frames, "served": served, "ticks": queue.ticks}


class _VocState:
    __slots__ = ("ctx", "sent", "pcm", "err")

    def __init__(self):
        self.ctx, self.sent, self.pcm, self.err = None, 0, [], None


class StreamVocoder:
    """serve()'s vocoder off the decode's critical path.  The codec runs on a host thread of its
    own, on the codec handle's HIP stream (separate from the LLM's), so a tick's vocoding overlaps
    the next tick's decode frames on the GPU (ctypes calls release the GIL).  `progress` streams
    each live request's finished columns (all but the newest) in chunks of `chunk` frames through a
    causal codec stream context of that request (fm_codec_stream_decode: the chunks' PCM is the
    one-shot decode's, bit for bit); `finish` vocodes the rest and returns the request's float32
    PCM.  Contexts are pooled and rewound (fm_codec_stream_rewind) instead of freed per request.
    Every codec call runs on the one thread, in submission order (the handle is single-threaded).
    busy_s: the thread's time inside codec calls."""

    def __init__(self, codec, chunk: int = 128):
        self.codec = codec
        self.chunk = max(1, min(int(chunk), codec.max_frames))
        self.fifo: "_queue.Queue" = _queue.Queue()
        self.live: Dict[int, _VocState] = {}
        self.pool: list = []   # rewound contexts (vocoder thread only)
        self.ctxs: list = []   # every context opened (closed by close())
        self.busy_s = 0.0
        self.th = threading.Thread(target=self._run, daemon=True)
        self.th.start()

    def submit(self, fn):
        """Run fn() on the vocoder thread after everything submitted before; returns (event,
        box): box holds fn's result, or the exception it raised, once the event is set."""
        ev, box = threading.Event(), []
        self.fifo.put((fn, ev, box))
        return ev, box

    def _run(self):
        while True:
            it = self.fifo.get()
            if it is None:
                return
            fn, ev, box = it
            t = time.perf_counter()
            try:
                box.append(fn())
            except BaseException as e:  # handed to the waiter, the thread lives on
                box.append(e)
            self.busy_s += time.perf_counter() - t
            ev.set()

    def _chunk(self, v: _VocState, codes: np.ndarray):
        if v.err is not None:
            return None
        try:
            if v.ctx is None:
                if self.pool:
                    v.ctx = self.pool.pop()
                else:
                    v.ctx = self.codec.open_stream()
                    self.ctxs.append(v.ctx)
            v.pcm.append(v.ctx.decode_chunk(codes))
        except BaseException as e:
            v.err = e
        return None

    def _release(self, v: _VocState):
        if v.ctx is not None:
            ctx, v.ctx = v.ctx, None
            ctx.rewind()
            self.pool.append(ctx)

    def progress(self, slot: int, req: Request, cols: List[np.ndarray]):
        v = self.live.setdefault(req.id, _VocState())
        ready = len(cols) - 1  # the newest column may be the dropped last one
        while ready - v.sent >= self.chunk:
            codes = np.ascontiguousarray(np.stack(cols[v.sent: v.sent + self.chunk], 1)[1:])
            self.submit(lambda v=v, c=codes: self._chunk(v, c))
            v.sent += self.chunk

    def finish(self, slot: int, req: Request, cols: np.ndarray) -> np.ndarray:
        """cols (C+1, N), the last column already dropped -> float32 PCM (2048 N,)."""
        v = self.live.pop(req.id, None) or _VocState()
        mx = self.codec.max_frames
        for t in range(v.sent, cols.shape[1], mx):
            codes = np.ascontiguousarray(cols[1:, t: t + mx])
            self.submit(lambda v=v, c=codes: self._chunk(v, c))
        ev, box = self.submit(lambda v=v: self._release(v))
        ev.wait()
        if v.err is not None:
            raise v.err
        if box and isinstance(box[0], BaseException):
            raise box[0]
        return np.concatenate(v.pcm) if v.pcm else np.zeros(0, np.float32)

    def close(self):
        self.fifo.put(None)
        self.th.join()
        for ctx in self.ctxs:
            ctx.close()
        self.ctxs, self.pool = [], []
