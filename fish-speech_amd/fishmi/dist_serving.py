"""Multi-GPU serving behind the reference's worker seam (BASELINE config 4).

One process per GPU (torchrun), every rank a fishmi.batching.BatchedWorker on its own KV slots.
Rank 0 keeps the reference's queue contract (inference.py:748-799): GenerateRequest(request,
response_queue) in, WrappedGenerateResponse out, `None` stops -- so the TTS engine and the HTTP
server above it are unchanged.  The ranks meet at synchronous ticks:

  1. all_gather of (free slots, busy, outbox bytes, rank 0's queued requests, rank 0's stop flag);
  2. the responses each rank produced since the last tick are gathered to rank 0 and put on their
     requests' response queues (rank 0's own go straight there);
  3. rank 0 hands its queued requests out round-robin over the ranks with free slots
     (fishmi.scheduler.assign, a pure function of the gathered counts) and scatters them;
  4. every rank runs one BatchedWorker tick (prefills, then up to tick_frames batched frames).

The loop ends when rank 0 has seen `None` and no rank has queued, active or unsent work.  While
idle, rank 0 waits at most `idle_wait` seconds for a request before the next tick, so the other
ranks never sit in a collective past its timeout.

Wire format: msgpack (numpy arrays as {shape, dtype, bytes}), over uint8 tensors on the default
process group (RCCL with device tensors on the GPU box, gloo with host tensors in the CPU tests).
Requests carry their prompt tokens.  With a `vocoder` (a FishMICodec per rank), every "sample"
response is vocoded on the rank that decoded it -- one-shot, or the request's own causal codec
stream for streamed chunks -- and travels with its float32 PCM (GenerateResponse.audio) beside the
codes, so rank 0 vocodes only its own share (the return direction carries audio;
the TTS engine forwards the PCM).  float32 rather than int16 keeps every byte the single-process
engine would produce (the int16 conversions happen where they do there); at config-4 rates that is
~0.2 MB per audio second over xGMI.  There is no collective on the decode path.

Stragglers: the ticks are synchronous, so a rank's long step delays everyone's next tick.  A tick's
work per rank is bounded: at most `tick_frames` batched frames, and the prefills of the text batches
starting on that rank (the prompt linears run as one GEMM over all of them, ~10-45 ms for
256-1400-token prompts); requests are dealt one at a time round-robin over the ranks with free
slots (scheduler.assign), so prompt work spreads over the ranks instead of queueing behind one.

Failures: an exception that escapes a tick (a collective error, a wire decode error, a bug) fails
every request this rank holds -- routed, queued, active -- with that error, then tears the process
group down so the other ranks' next collective fails too and they do the same; rank 0 keeps
answering later requests with the error instead of leaving their callers blocked.
"""
from __future__ import annotations

import builtins
import collections
import dataclasses
import logging
import queue
import threading
import time
from typing import Deque, Dict, List, Optional, Tuple

import numpy as np

from .batching import BatchedWorker
from .engine import GenerateRequest, GenerateResponse, WrappedGenerateResponse
from .scheduler import _device, _dist, assign

log = logging.getLogger("fishmi.dist_serving")


# ---- wire format ----------------------------------------------------------------------------------
def _enc(o):
    try:
        import torch

        if isinstance(o, torch.Tensor):
            o = o.detach().cpu().numpy()
        elif isinstance(o, torch.device):
            return str(o)
    except ImportError:  # pragma: no cover
        pass
    if isinstance(o, np.ndarray):
        a = np.ascontiguousarray(o)
        return {"__nd__": True, "s": list(a.shape), "d": a.dtype.str, "b": a.tobytes()}
    if isinstance(o, np.generic):
        return o.item()
    raise TypeError(f"cannot send {type(o).__name__} to another rank")


def _dec(d):
    if d.get("__nd__"):
        return np.frombuffer(d["b"], dtype=np.dtype(d["d"])).reshape(d["s"]).copy()
    return d


def pack(obj) -> bytes:
    import msgpack

    return msgpack.packb(obj, default=_enc, use_bin_type=True)


def unpack(b: bytes):
    import msgpack

    return msgpack.unpackb(b, object_hook=_dec, raw=False, strict_map_key=False)


def _exc_to_wire(e: BaseException) -> dict:
    return {"type": type(e).__name__, "msg": str(e)}


def _exc_from_wire(d: dict) -> Exception:
    t = getattr(builtins, d["type"], None)
    if isinstance(t, type) and issubclass(t, Exception):
        return t(d["msg"])
    return RuntimeError(f"{d['type']}: {d['msg']}")


def response_to_wire(w: Optional[WrappedGenerateResponse]) -> dict:
    """None marks "the request is done" (no more responses follow)."""
    if w is None:
        return {"done": True}
    if w.status == "error":
        return {"status": "error", "exc": _exc_to_wire(w.response)}
    r = w.response
    return {"status": "success", "action": r.action, "codes": r.codes, "text": r.text, "stream": r.stream,
            "audio": getattr(r, "audio", None)}


def response_from_wire(d: dict) -> Optional[WrappedGenerateResponse]:
    if d.get("done"):
        return None
    if d["status"] == "error":
        return WrappedGenerateResponse(status="error", response=_exc_from_wire(d["exc"]))
    return WrappedGenerateResponse(status="success", response=GenerateResponse(
        action=d["action"], codes=d["codes"], text=d["text"], stream=d["stream"], audio=d.get("audio")))


class _Outbox:
    """A remote request's response_queue on the rank decoding it: responses wait for the next tick."""

    def __init__(self, rid: int, sink: list):
        self.rid, self.sink = rid, sink

    def put(self, w):
        self.sink.append((self.rid, w))


class _Vocoder:
    """This rank's vocoder, off the tick's critical path: one FIFO of (request queue, response) items
    served by a thread of its own, so a rank that finishes a long request does not hold every rank's
    next all_gather while it vocodes (tools/vqgan/extract_vq.py:150-197 runs its codec beside the
    loader the same way).  One FIFO keeps each request's responses in order; results go back to the
    tick thread through `ready`, which the tick drains into its outbox (the outbox stays
    single-threaded).  A codec call that raises answers its request with the error and drops that
    request's later samples; every other request keeps being served."""

    def __init__(self, codec, device=None):
        self.codec, self.device = codec, device
        self.fifo: "queue.Queue" = queue.Queue()
        self.ready: "queue.Queue" = queue.Queue()
        self.backlog = 0  # items put and not yet drained back (read by the tick thread)
        self._lock = threading.Lock()
        self.th = threading.Thread(target=self._run, daemon=True)
        self.th.start()

    def submit(self, v: "_Vocoding", w, done: bool = False):
        with self._lock:
            self.backlog += 1
        self.fifo.put((v, w, done))

    def drain(self, deliver) -> int:
        """Hand every finished item to deliver(v, w) (tick thread); returns how many are still in
        flight."""
        n = 0
        while True:
            try:
                v, w = self.ready.get_nowait()
            except queue.Empty:
                break
            deliver(v, w)
            n += 1
        with self._lock:
            self.backlog -= n
            return self.backlog

    def close(self):
        self.fifo.put(None)

    def _run(self):
        if self.device is not None and getattr(self.device, "type", None) == "cuda":
            import torch

            torch.cuda.set_device(self.device)  # the current device is per thread
        while True:
            it = self.fifo.get()
            if it is None:
                return
            v, w, done = it
            # every item goes back on `ready` whatever happens, so the backlog drains and the
            # request's done marker is delivered (a dead thread would leave this rank busy forever)
            if done:
                try:
                    v.close()
                except Exception as e:  # the stream's close failing ends nothing but its own context
                    log.error("closing a vocoder stream failed: %r", e)
                self.ready.put((v, None))
                continue
            try:
                out = v.vocode(self.codec, w)
            except Exception as e:
                log.error("vocoder item failed: %r", e)
                v.failed = True
                out = WrappedGenerateResponse(status="error", response=e)
            self.ready.put((v, out))


class _Vocoding:
    """A request's response queue on the rank that decodes it, with a vocoder: each "sample"
    response gets its PCM (VQManager.decode_vq_tokens, vq_manager.py:16-21, or the request's own
    causal stream for latency="balanced" chunks) on this rank's vocoder thread before it moves on."""

    def __init__(self, inner, vocoder: _Vocoder, item=None):
        self.inner, self.voc, self.ctx, self.item = inner, vocoder, None, item
        self.failed = False

    def put(self, w):
        self.voc.submit(self, w)

    def vocode(self, codec, w):
        """(vocoder thread) the response with its PCM; after a codec error, the error once and the
        request's later samples dropped (its caller has its answer)"""
        if self.failed:  # the caller has its error: nothing more of this request reaches it
            return _DROP
        if w is None or w.status != "success" or not isinstance(w.response, GenerateResponse) \
                or w.response.action != "sample" or w.response.codes is None:
            return w
        r = w.response
        try:
            codes = np.asarray(r.codes)
            if r.stream is not None:  # chunk k of one text batch's stream: this request's codec state
                if r.stream == 0 or self.ctx is None:
                    self.close()
                    self.ctx = codec.open_stream()
                pcm = self.ctx.decode_chunk(codes)
            else:
                pcm = codec.decode_codes(codes)
        except Exception as e:
            log.error("vocoding failed: %r", e)
            self.failed = True
            try:
                self.close()
            except Exception as e2:
                log.error("closing the failed request's codec stream failed: %r", e2)
            return WrappedGenerateResponse(status="error", response=e)
        return WrappedGenerateResponse(status="success", response=dataclasses.replace(
            r, audio=np.ascontiguousarray(pcm, dtype=np.float32)))

    def close(self):
        if self.ctx is not None:
            try:
                self.ctx.close()
            finally:
                self.ctx = None


class _Drop:
    """Marks a response the vocoder dropped (a sample after its request's codec error)."""


_DROP = _Drop()


# ---- the worker ---------------------------------------------------------------------------------
class DistributedWorker:
    STAT = 5  # free, busy, outbox bytes, queued (rank 0), stopping (rank 0)

    def __init__(self, model, max_slots: Optional[int] = None, tick_frames: int = 8, idle_wait: float = 0.02,
                 vocoder=None, device=None):
        dist = _dist()
        self.world, self.rank = dist.get_world_size(), dist.get_rank()
        # the collectives' device: explicit (the caller's GPU), never this thread's current device
        self.dev = device if device is not None else _device()
        # a FishMICodec on this rank's GPU: vocode where the codes are decoded, on a thread of its own
        self.vocoder = _Vocoder(vocoder, self.dev) if vocoder is not None else None
        self.w = BatchedWorker(model, max_slots, tick_frames)
        self.w.on_done = self._done
        self.idle_wait = idle_wait
        self.input: "queue.Queue" = queue.Queue()          # rank 0: the seam's queue
        self.queued: Deque[Tuple[int, GenerateRequest]] = collections.deque()
        self.routes: Dict[int, GenerateRequest] = {}         # rank 0: rid -> the caller's request
        self.outbox: List[Tuple[int, Optional[WrappedGenerateResponse]]] = []
        self._blob = b""  # packed outbox, sent at this tick's gather
        self.next_id = 0
        self.stopping = False
        self.failed: Optional[BaseException] = None
        self.stats = {"ticks": 0, "served": 0, "sent_to": [0] * self.world}

    def _wrap(self, item: GenerateRequest) -> GenerateRequest:
        if self.vocoder is None:
            return item
        v = _Vocoding(item.response_queue, self.vocoder)
        w = GenerateRequest(request=item.request, response_queue=v)
        if hasattr(item, "_rid"):
            w._rid = item._rid
        v.item = w
        return w

    def _deliver(self, v: _Vocoding, w):
        """(tick thread) a vocoded response, or the request's done marker, in the request's order"""
        if w is _DROP:
            return
        if w is None:
            self._finished(v.item, v.inner)
        else:
            v.inner.put(w)

    def _done(self, item: GenerateRequest):
        q = item.response_queue
        if isinstance(q, _Vocoding):  # behind the request's samples still being vocoded
            q.voc.submit(q, None, done=True)
            self.stats["served"] += 1
            return
        self._finished(item, q)

    def _finished(self, item: GenerateRequest, q):
        if isinstance(q, _Outbox):
            q.put(None)
        else:
            self.routes.pop(getattr(item, "_rid", None), None)
        if not isinstance(item.response_queue, _Vocoding):
            self.stats["served"] += 1

    # ---- collectives ----------------------------------------------------------------------------
    def _tensor(self, b: bytes, n: int):
        import torch

        t = torch.zeros(max(n, 1), dtype=torch.uint8)
        if b:
            t[: len(b)] = torch.frombuffer(bytearray(b), dtype=torch.uint8)
        return t.to(self.dev)

    def _gather_outboxes(self, sizes: List[int]):
        import torch

        dist = _dist()
        blob, self._blob = self._blob, b""
        n = max(max(sizes), 1)
        t = self._tensor(blob, n)
        outs = [torch.empty_like(t) for _ in range(self.world)] if self.rank == 0 else None
        dist.gather(t, outs, dst=0)
        if self.rank != 0:
            return
        for r in range(1, self.world):
            if sizes[r]:
                for rid, d in unpack(outs[r][: sizes[r]].cpu().numpy().tobytes()):
                    self._route(rid, response_from_wire(d))

    def _route(self, rid: int, w: Optional[WrappedGenerateResponse]):
        item = self.routes.get(rid)
        if item is None:
            log.error("response for unknown request %d", rid)
            return
        if w is None:
            del self.routes[rid]
        else:
            item.response_queue.put(w)

    def _scatter(self, take: List[int]) -> List[GenerateRequest]:
        import torch

        dist = _dist()
        lens = torch.zeros(self.world, dtype=torch.int64, device=self.dev)
        blobs = []
        mine: List[GenerateRequest] = []
        if self.rank == 0:
            for r in range(self.world):
                items = [self.queued.popleft() for _ in range(take[r])]
                self.stats["sent_to"][r] += len(items)
                if r == 0:
                    mine = [it for _, it in items]
                    blobs.append(b"")
                else:
                    blobs.append(pack([[rid, it.request] for rid, it in items]))
                lens[r] = len(blobs[-1])
        dist.broadcast(lens, src=0)
        ln = lens.cpu().tolist()
        n = max(max(ln), 1)
        t = self._tensor(b"", n)
        chunks = [self._tensor(b, n) for b in blobs] if self.rank == 0 else None
        dist.scatter(t, chunks, src=0)
        if self.rank == 0:
            return mine
        out = []
        for rid, req in unpack(t[: ln[self.rank]].cpu().numpy().tobytes()):
            out.append(GenerateRequest(request=req, response_queue=_Outbox(int(rid), self.outbox)))
        return out

    # ---- one tick -------------------------------------------------------------------------------
    def _intake(self):
        block = not self.routes and not self.queued and not self.stopping
        first = True
        while True:
            try:
                item = self.input.get(timeout=self.idle_wait) if (block and first) else self.input.get_nowait()
            except queue.Empty:
                return
            first = False
            if item is None:
                self.stopping = True
            elif not self.stopping:
                rid = self.next_id
                self.next_id += 1
                item._rid = rid
                self.routes[rid] = item
                self.queued.append((rid, item))

    def tick(self) -> bool:
        """One synchronous tick on every rank; False (on every rank alike) once stopped and idle."""
        import torch

        dist = _dist()
        self.stats["ticks"] += 1
        t0 = time.perf_counter()
        try:
            return self._tick(dist)
        finally:  # (straggler check: a tick that waits on another rank's slow step shows here)
            dt = time.perf_counter() - t0
            self.stats["tick_max_s"] = max(self.stats.get("tick_max_s", 0.0), dt)

    def _tick(self, dist) -> bool:
        import torch

        if self.rank == 0:
            self._intake()
        wk = self.w
        free = wk.max_slots - len(wk.active) - len(wk.pending)
        busy = len(wk.active) + len(wk.pending)
        if self.vocoder is not None:  # vocoded since the last tick -> outbox / callers
            busy += self.vocoder.drain(self._deliver)
        if self.rank != 0 and self.outbox:  # this tick ships everything produced so far
            self._blob = pack([[rid, response_to_wire(w)] for rid, w in self.outbox])
            self.outbox.clear()  # _Outbox proxies hold this list: clear it in place
        vec = torch.tensor([free, busy, len(self._blob), len(self.queued), int(self.stopping)], dtype=torch.int64,
                           device=self.dev)
        allv = [torch.zeros_like(vec) for _ in range(self.world)]
        dist.all_gather(allv, vec)
        st = np.stack([a.cpu().numpy() for a in allv])
        if self.rank == 0:  # rank 0's own responses need no collective
            for rid, w in self.outbox:
                self._route(rid, w)
            self.outbox.clear()
        if st[1:, 2].any():
            self._gather_outboxes(st[:, 2].tolist())
        if st[0, 4] and not st[:, 1].any() and not st[1:, 2].any() and st[0, 3] == 0:
            return False
        take = assign(st[:, 0].tolist(), int(st[0, 3]))
        if sum(take):
            for it in self._scatter(take):
                wk.pending.append(self._wrap(it))
        if wk.active or wk.pending:
            wk.tick(block=False)
        return True

    def _fail_everything(self, e: BaseException):
        """A tick raised: every request this rank holds gets the error; then the process group goes
        down so no other rank waits in a collective for this one."""
        err = e if isinstance(e, Exception) else RuntimeError(repr(e))
        log.error("rank %d: serving loop failed: %r", self.rank, e)
        self.w.fail_all(err)  # active + pending (their queues: callers, outboxes)
        if self.vocoder is not None:  # their errors and done markers pass the vocoder's FIFO
            self.vocoder.close()
            self.vocoder.th.join(timeout=60)
            self.vocoder.drain(self._deliver)
        if self.rank == 0:
            for rid, item in list(self.routes.items()):  # queued here or decoding on another rank
                item.response_queue.put(WrappedGenerateResponse(status="error", response=err))
            self.routes.clear()
            self.queued.clear()
        try:
            _dist().destroy_process_group()
        except Exception:  # pragma: no cover - already torn down
            pass

    def run(self):
        try:
            while self.tick():
                if self.vocoder is not None and self.vocoder.backlog and not (self.w.active or self.w.pending):
                    time.sleep(0.001)  # only vocoding left on this rank: let it run, then tick again
            if self.vocoder is not None:
                self.vocoder.close()
        except BaseException as e:
            self._fail_everything(e)
            self.failed = e
            if self.rank == 0:  # later requests are answered, not left blocking their callers
                while True:
                    item = self.input.get()
                    if item is None:
                        break
                    item.response_queue.put(WrappedGenerateResponse(status="error", response=RuntimeError(
                        f"the multi-GPU LLM worker failed: {e!r}")))
            return
        log.info("rank %d: %s", self.rank, self.stats)


def launch_distributed_queue(checkpoint_path, device, precision, max_slots: int = 32, tick_frames: int = 8,
                             model=None, idle_wait: float = 0.02, vocoder=None):
    """launch_thread_safe_queue across the process group: every rank loads the model on its own GPU
    and runs a DistributedWorker in a daemon thread.  Returns (input queue, thread); only rank 0's
    queue is served (requests put on another rank's queue are never read).  Put `None` on rank 0's
    queue to stop every rank; join the thread to wait for it.  vocoder: this rank's codec (or a
    callable building it on the worker thread): responses then carry their PCM."""
    from .engine import _device_index, load_model

    ready = threading.Event()
    failure: List[BaseException] = []
    holder: dict = {}

    def worker():
        try:
            dev = None
            if _dist().get_backend() == "nccl":  # the current device is per thread: set it here
                import torch

                torch.cuda.set_device(_device_index(device))
                dev = torch.device("cuda", _device_index(device))
            m = model if model is not None else load_model(checkpoint_path, device, precision, max_slots)
            voc = vocoder() if callable(vocoder) else vocoder
            w = DistributedWorker(m, max_slots, tick_frames, idle_wait, vocoder=voc, device=dev)
        except BaseException as e:
            failure.append(e)
            ready.set()
            return
        holder["w"] = w
        ready.set()
        w.run()

    th = threading.Thread(target=worker, daemon=True)
    th.start()
    ready.wait()
    if failure:
        raise failure[0]
    holder["w"].thread = th
    th.worker = holder["w"]
    return holder["w"].input, th
