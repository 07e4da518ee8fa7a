"""Batched LLM worker (fishmi.batching.BatchedWorker) on CPU with a scripted model: concurrent
requests on shared KV slots get exactly the responses the serial worker (generate_long, the
reference's one-request-at-a-time flow, inference.py:748-799) gives each of them alone.

The scripted model stands in for libfishmi's slot API (prefill / prefill_batch / decode_frames /
generate / generate_at / slot_pos): every slot's next column is a hash of the slot's whole token
history, its seed and its step, so a column decoded on the wrong slot, at the wrong position or
after the wrong fed-back column changes every later one.  The GPU counterpart (the real model,
fp32) is tests/test_gpu_engine.py::test_batched_worker_matches_serial."""
import os
import queue
import zlib
from types import SimpleNamespace

import numpy as np
import pytest

from conftest import GOLDEN

IM_END, SB, SE, CB, C = 4, 200, 327, 128, 10


class ScriptedModel:
    def __init__(self, max_slots=1, max_seq_len=2560):
        from fishmi.prompt import FishTokenizer

        self.cfg = SimpleNamespace(num_codebooks=C, max_seq_len=max_seq_len, im_end_id=IM_END,
                                   semantic_begin_id=SB, semantic_end_id=SE, codebook_size=CB)
        self.tokenizer = FishTokenizer(os.path.join(GOLDEN, "tok_tiny"))
        self.max_slots = max_slots
        self.hist = [[] for _ in range(max_slots)]
        self.last = [None] * max_slots
        self.sp = [None] * max_slots
        self.step = [0] * max_slots
        self.calls = []

    @staticmethod
    def sampling(temperature=0.7, top_p=0.9, top_k=30, seed=0, mask_im_end=False):
        return SimpleNamespace(temperature=temperature, top_p=top_p, top_k=top_k, seed=int(seed) & (2**64 - 1),
                               mask_im_end=bool(mask_im_end))

    def _next(self, s):
        h = np.asarray(self.hist[s], np.int64).tobytes()
        key = zlib.crc32(h + repr((self.sp[s].seed, self.step[s], self.sp[s].top_k)).encode())
        main = IM_END if (key % 9 == 0 and not self.sp[s].mask_im_end) else SB + key % CB
        col = np.array([main, max(0, min(CB - 1, main - SB))] + [(key >> (3 * q)) % CB for q in range(C - 1)],
                       np.int32)
        self.last[s] = col
        return col

    def prefill(self, slot, prompt, sp, pos0=0):
        assert pos0 <= len(self.hist[slot])
        p = np.asarray(prompt, np.int32)
        self.hist[slot] = self.hist[slot][:pos0] + [tuple(c) for c in p.T]
        self.sp[slot], self.step[slot] = sp, 0
        self.calls.append(("prefill", slot))
        return self._next(slot)

    def prefill_batch(self, slots, prompts, sps):
        self.calls.append(("prefill_batch", tuple(slots)))
        return np.stack([self.prefill(s, p, sp) for s, p, sp in zip(slots, prompts, sps)])

    def decode_frames(self, slots, n):
        assert len(set(slots)) == len(slots)
        for s in slots:
            assert len(self.hist[s]) + n <= self.cfg.max_seq_len
        self.calls.append(("decode", tuple(slots), n))
        out = np.zeros((n, len(slots), C + 1), np.int32)
        for k in range(n):
            for j, s in enumerate(slots):
                self.hist[s].append(tuple(self.last[s]))
                self.step[s] += 1
                out[k, j] = self._next(s)
        return out

    def _gen(self, slot, prompt, pos0, max_new, sp):
        T = pos0 + prompt.shape[1]
        mx = max_new if (max_new and T + max_new <= self.cfg.max_seq_len) else self.cfg.max_seq_len - T
        cols = [self.prefill(slot, prompt, sp, pos0)]
        while len(cols) < mx and cols[-1][0] != IM_END:
            cols.append(self.decode_frames([slot], 1)[0, 0])
        return np.stack(cols, axis=1)

    def generate(self, prompt, max_new, temperature=0.7, top_p=0.9, top_k=30, seed=0, slot=0, mask_im_end=False):
        return self._gen(slot, np.asarray(prompt), 0, max_new, self.sampling(temperature, top_p, top_k, seed,
                                                                              mask_im_end))

    def generate_at(self, suffix, pos0, max_new, temperature=0.7, top_p=0.9, top_k=30, seed=0, slot=0,
                    mask_im_end=False):
        return self._gen(slot, np.asarray(suffix), pos0, max_new, self.sampling(temperature, top_p, top_k, seed,
                                                                                 mask_im_end))

    def slot_pos(self, slot=0):
        return len(self.hist[slot])


def _requests():
    rng = np.random.default_rng(3)
    texts = ["<|speaker:0|>Good morning. <|speaker:1|>Morning! Coffee? <|speaker:0|>Yes please, black.",
             "a plain sentence without any speaker tags",
             "<|speaker:0|>one. <|speaker:1|>two two. <|speaker:0|>three three three. <|speaker:1|>four.",
             "short", "<|speaker:2|>Third voice speaks here for a while, then stops."]
    reqs = []
    for i in range(9):
        r = dict(text=texts[i % len(texts)], max_new_tokens=int(rng.integers(3, 40)), top_p=0.9, top_k=30,
                 temperature=0.7, chunk_length=30, seed=100 + i, device="cuda", compile=False,
                 iterative_prompt=True, repetition_penalty=1.1)
        if i % 3 == 1:
            r["prompt_tokens"] = [rng.integers(0, CB, (C, 5)), rng.integers(0, CB, (C, 3))]
            r["prompt_text"] = ["ref a", "<|speaker:1|>ref b"]
        if i % 4 == 2:
            r["reuse_prefix"] = True
        if i % 5 == 3:
            r["stream_frames"] = 4
        if i == 7:
            r["num_samples"] = 2
        reqs.append(r)
    return reqs


def _summary(resps):
    """(action, codes) per response, streamed chunks of one batch concatenated (chunk sizes may
    differ between the two workers; the codes of each batch may not)."""
    out = []
    for w in resps:
        assert w.status == "success", w.response
        r = w.response
        if r.action == "sample" and r.stream is not None and r.stream > 0:
            out[-1] = ("sample", np.concatenate([out[-1][1], r.codes], axis=1))
        else:
            out.append((r.action, None if r.codes is None else np.asarray(r.codes)))
    return out


@pytest.mark.parametrize("slots,tick", [(3, 8), (4, 1), (16, 5)])
def test_batched_worker_equals_serial(slots, tick):
    from fishmi import engine
    from fishmi.batching import BatchedWorker

    reqs = _requests()
    serial = []
    for r in reqs:
        m1 = ScriptedModel(1)
        serial.append([engine.WrappedGenerateResponse("success", o) for o in engine.generate_long(model=m1, **r)])
    mb = ScriptedModel(slots)
    w = BatchedWorker(mb, slots, tick_frames=tick)
    qs = [queue.Queue() for _ in reqs]
    for r, q in zip(reqs, qs):
        w.input.put(engine.GenerateRequest(request=r, response_queue=q))
    w.input.put(None)
    w.run()
    assert any(c[0] == "decode" and len(c[1]) > 1 for c in mb.calls)  # slots really decoded together
    assert any(c[0] == "prefill_batch" for c in mb.calls)
    for i, (q, ref) in enumerate(zip(qs, serial)):
        got = []
        while not q.empty():
            got.append(q.get())
        a, b = _summary(got), _summary(ref)
        assert [x[0] for x in a] == [x[0] for x in b], i
        for (_, ca), (_, cb) in zip(a, b):
            if ca is not None:
                np.testing.assert_array_equal(ca, cb, err_msg=f"request {i}")
    assert w.stats["requests"] == len(reqs)


def test_batched_worker_errors_are_per_request():
    """A request that fails (temperature outside (0, 2), inference.py:542) answers "error"; the others
    are served."""
    from fishmi import engine
    from fishmi.batching import BatchedWorker

    mb = ScriptedModel(2)
    w = BatchedWorker(mb, 2, tick_frames=4)
    good = dict(text="short", max_new_tokens=6, seed=1)
    bad = dict(text="x", max_new_tokens=6, seed=2, temperature=5.0)
    qs = [queue.Queue() for _ in range(3)]
    for r, q in zip((good, bad, good), qs):
        w.input.put(engine.GenerateRequest(request=r, response_queue=q))
    w.input.put(None)
    w.run()
    assert qs[1].get().status == "error"
    for q in (qs[0], qs[2]):
        rs = [q.get() for _ in range(q.qsize())]
        assert [x.response.action for x in rs] == ["sample", "next"]


def test_launch_thread_safe_queue_batched():
    """The seam: launch_thread_safe_queue(max_slots > 1) serves through the batched worker."""
    from fishmi import engine

    mb = ScriptedModel(4)
    q_in = engine.launch_thread_safe_queue(None, 0, "bf16", model=mb, max_slots=4)
    qs = [queue.Queue() for _ in range(6)]
    for i, q in enumerate(qs):
        q_in.put(engine.GenerateRequest(request=dict(text=f"request {i}", max_new_tokens=12, seed=i), response_queue=q))
    for i, q in enumerate(qs):
        got = [q.get(timeout=60)]
        while got[-1].response.action != "next":
            got.append(q.get(timeout=60))
        ref = list(engine.generate_long(model=ScriptedModel(1), text=f"request {i}", max_new_tokens=12, seed=i))
        assert [g.response.action for g in got] == [o.action for o in ref]
        for g, o in zip(got, ref):
            if o.codes is not None:
                np.testing.assert_array_equal(g.response.codes, o.codes)
    q_in.put(None)


def test_batched_prefill_failure_fails_only_its_request():
    """A batch prefill that raises is retried slot by slot: only the request whose prompt fails gets
    the error, the rest of the cohort is served (one bad request took down the cohort)."""
    from fishmi import engine
    from fishmi.batching import BatchedWorker

    class Flaky(ScriptedModel):
        def prefill(self, slot, prompt, sp, pos0=0):
            if np.asarray(prompt).shape[1] > 0 and getattr(self, "poison", None) == slot:
                raise ValueError("poisoned prompt")
            return super().prefill(slot, prompt, sp, pos0)

    mb = Flaky(3)
    w = BatchedWorker(mb, 3, tick_frames=4)
    qs = [queue.Queue() for _ in range(3)]
    for i, q in enumerate(qs):
        w.input.put(engine.GenerateRequest(request=dict(text=f"r{i}", max_new_tokens=5, seed=i), response_queue=q))
    mb.poison = 1  # the slot the second request lands on (slots are handed out 0, 1, 2)
    w.input.put(None)
    w.run()
    got = [[q.get() for _ in range(q.qsize())] for q in qs]
    assert [g[0].status for g in got] == ["success", "error", "success"]
    assert "poisoned" in str(got[1][0].response)
    for i in (0, 2):
        ref = list(engine.generate_long(model=ScriptedModel(1), text=f"r{i}", max_new_tokens=5, seed=i))
        assert [g.response.action for g in got[i]] == [o.action for o in ref]
        np.testing.assert_array_equal(got[i][0].response.codes, ref[0].codes)


def test_requests_after_stop_are_answered():
    """A request queued behind the `None` sentinel gets an error response instead of being dropped."""
    from fishmi import engine
    from fishmi.batching import BatchedWorker

    w = BatchedWorker(ScriptedModel(2), 2, tick_frames=4)
    q1, q2 = queue.Queue(), queue.Queue()
    w.input.put(engine.GenerateRequest(request=dict(text="a", max_new_tokens=4, seed=1), response_queue=q1))
    w.input.put(None)
    w.input.put(engine.GenerateRequest(request=dict(text="b", max_new_tokens=4, seed=2), response_queue=q2))
    w.run()
    assert q1.get().status == "success"
    late = q2.get(timeout=5)
    assert late.status == "error" and "stopping" in str(late.response)
