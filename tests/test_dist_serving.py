"""Multi-GPU serving through the worker seam (fishmi.dist_serving, BASELINE config 4) on world_size-2
gloo with the scripted model of tests/test_batching.py: requests put on rank 0's queue are decoded
on both ranks' KV slots, and every request gets exactly the responses the serial worker
(generate_long, inference.py:748-799) gives it alone, errors included, in order."""
import os
import queue
import socket
import time
import traceback

import numpy as np


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _serial(reqs):
    from fishmi import engine
    from test_batching import ScriptedModel

    out = []
    for r in reqs:
        try:
            out.append([engine.WrappedGenerateResponse("success", o)
                        for o in engine.generate_long(model=ScriptedModel(1), **r)])
        except Exception as e:
            out.append([engine.WrappedGenerateResponse("error", e)])
    return out


def _check(got, ref, i):
    from test_batching import _summary

    if ref[-1].status == "error":
        assert [g.status for g in got] == ["error"], i
        assert type(got[0].response) is type(ref[0].response), i
        assert str(got[0].response) == str(ref[0].response), i
        return
    a, b = _summary(got), _summary(ref)
    assert [x[0] for x in a] == [x[0] for x in b], i
    for (_, ca), (_, cb) in zip(a, b):
        if ca is not None:
            np.testing.assert_array_equal(ca, cb, err_msg=f"request {i}")


def _collect(q, n_final):
    """Responses until the request's last one ("next" of its last sample, or an error)."""
    got, finals = [], 0
    while finals < n_final:
        w = q.get(timeout=60)
        got.append(w)
        if w.status == "error":
            break
        if w.response.action == "next":
            finals += 1
    return got


class ScriptedVocoder:
    """Stands in for FishMICodec: PCM is a per-column function of the codes (HOP samples a column),
    so a causal stream of chunks vocodes to the one-shot decode of their concatenation.  delay: seconds
    each call takes (a slow vocoder); fail_at: the call that raises (a codec error)."""
    HOP = 4

    def __init__(self, delay=0.0, fail_at=None):
        self.calls = 0
        self.delay, self.fail_at = delay, fail_at

    def decode_codes(self, codes):
        self.calls += 1
        if self.delay:
            time.sleep(self.delay)
        if self.fail_at is not None and self.calls == self.fail_at:
            raise RuntimeError("injected codec failure")
        c = np.asarray(codes, np.int64)
        col = (c * np.arange(1, c.shape[0] + 1)[:, None]).sum(0) % 997
        return np.repeat(col.astype(np.float32) / 997.0, self.HOP)

    def open_stream(self):
        voc = self

        class _S:
            def decode_chunk(self, codes):
                return voc.decode_codes(codes)

            def close(self):
                pass

        return _S()


def _worker(rank, world, port, out_q, slots, tick, mode="plain"):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from fishmi import engine
        from fishmi.dist_serving import DistributedWorker, launch_distributed_queue
        from test_batching import ScriptedModel, _requests

        model = ScriptedModel(slots)
        voc = None
        if mode == "vocode":
            voc = ScriptedVocoder()
        elif mode == "slowvoc":  # rank 1 vocodes slowly: rank 0's ticks must not wait for it
            voc = ScriptedVocoder(delay=0.25 if rank == 1 else 0.0)
        elif mode == "badvoc":  # rank 1's codec raises once: that request fails, the rest are served
            voc = ScriptedVocoder(fail_at=2 if rank == 1 else None)
        if mode == "fail" and rank == 1:  # a tick that raises outside every per-request guard
            orig = DistributedWorker.tick

            def bad_tick(self):
                if self.stats["ticks"] >= 12:
                    raise RuntimeError("injected tick failure")
                return orig(self)

            DistributedWorker.tick = bad_tick
        q_in, th = launch_distributed_queue(None, 0, "bf16", max_slots=slots, tick_frames=tick, model=model,
                                            vocoder=voc)
        if rank == 0:
            reqs = _requests()
            reqs.append(dict(text="bad", max_new_tokens=6, seed=2, temperature=5.0))
            reqs.append(dict(text="<|speaker:0|>long " * 4, max_new_tokens=30, seed=9, prompt_tokens=[
                np.arange(40, dtype=np.int64).reshape(10, 4) % 128], prompt_text=["ref"]))
            ref = _serial(reqs)
            time.sleep(0.2)  # a few idle ticks first
            qs = [queue.Queue() for _ in reqs]
            for r, q in zip(reqs, qs):
                q_in.put(engine.GenerateRequest(request=r, response_queue=q))
            if mode == "fail":
                # every request ends (answered or failed); none leaves its caller blocked
                errs = 0
                for i, (q, rf) in enumerate(zip(qs, ref)):
                    n_final = 0 if rf[-1].status == "error" else sum(w.response.action == "next" for w in rf)
                    got = _collect(q, max(n_final, 1))
                    errs += got[-1].status == "error"
                assert errs >= 2, errs  # the "bad" request + at least one failed by the injected error
                late = queue.Queue()  # a request after the failure is answered too
                q_in.put(engine.GenerateRequest(request=reqs[0], response_queue=late))
                assert late.get(timeout=30).status == "error"
            elif mode == "badvoc":
                failed = 0
                for i, (q, rf) in enumerate(zip(qs, ref)):
                    n_final = 0 if rf[-1].status == "error" else sum(w.response.action == "next" for w in rf)
                    got = _collect(q, max(n_final, 1))
                    if got[-1].status == "error" and rf[-1].status != "error":
                        assert "injected codec failure" in str(got[-1].response), got[-1].response
                        failed += 1
                        continue
                    _check(got, rf, i)
                assert failed == 1, failed  # exactly the request whose samples hit the failing call
            else:
                for i, (q, rf) in enumerate(zip(qs, ref)):
                    n_final = 0 if rf[-1].status == "error" else sum(w.response.action == "next" for w in rf)
                    got = _collect(q, max(n_final, 1))
                    _check(got, rf, i)
                    if voc is not None:  # every sample carries the PCM of its own codes
                        for w in got:
                            if w.status == "success" and w.response.action == "sample":
                                assert w.response.audio is not None, i
                                np.testing.assert_array_equal(w.response.audio,
                                                              ScriptedVocoder().decode_codes(w.response.codes))
            q_in.put(None)
        th.join(timeout=120)
        assert not th.is_alive()
        if mode == "slowvoc" and rank == 0:
            # rank 1 spends 0.25 s per vocoder call on its vocoder thread; rank 0's ticks (each an
            # all_gather with rank 1) never waited for one of them
            assert th.worker.stats["tick_max_s"] < 0.15, th.worker.stats
        decoded = [c for c in model.calls if c[0] in ("prefill", "prefill_batch")]
        if voc is not None:
            assert voc.calls > 0, f"rank {rank} vocoded nothing"
        out_q.put((rank, "ok", len(decoded)))
    except Exception:
        out_q.put((rank, traceback.format_exc(), 0))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def _run(slots, tick, mode="plain"):
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q, slots, tick, mode)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(2):
        rank, msg, n = q.get(timeout=180)
        res[rank] = (msg, n)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(2):
        assert res[r][0] == "ok", res[r][0]
        assert res[r][1] > 0 or mode == "fail", f"rank {r} decoded nothing"


def test_distributed_worker_world2_equals_serial():
    _run(slots=2, tick=3)


def test_distributed_worker_world2_one_slot_per_rank():
    _run(slots=1, tick=8)


def test_distributed_worker_world2_vocodes_per_rank():
    """Each rank vocodes the samples it decoded; every response's PCM equals the one-shot decode of
    its codes (streamed chunks included), and both ranks' vocoders ran."""
    _run(slots=2, tick=3, mode="vocode")


def test_distributed_worker_world2_slow_vocoder_does_not_stall_ticks():
    """Rank 1's vocoder takes 0.25 s a call: it runs on the rank's vocoder thread, so the
    synchronous ticks (all_gather across the ranks) are not held by it -- rank 0's longest tick stays
    under 0.15 s -- and every response still arrives in order with its PCM."""
    _run(slots=2, tick=3, mode="slowvoc")


def test_distributed_worker_world2_codec_error_fails_one_request():
    """Rank 1's codec raises on one call: that request is answered with the error, every other
    request (on both ranks) gets exactly its serial responses, and the ranks keep serving."""
    _run(slots=2, tick=3, mode="badvoc")


def test_distributed_worker_world2_tick_failure_fails_requests():
    """A tick on rank 1 raises outside every per-request guard: rank 0's callers all get an answer
    (the requests in flight fail with the error), later requests are answered with an error, and
    both worker threads end instead of hanging in a collective."""
    _run(slots=2, tick=3, mode="fail")


def test_wire_roundtrip():
    from fishmi import engine
    from fishmi.dist_serving import pack, response_from_wire, response_to_wire, unpack

    req = dict(text="hi", seed=3, prompt_tokens=[np.arange(12, dtype=np.int32).reshape(3, 4)], prompt_text=["a"],
               top_p=np.float32(0.5), device="cuda:0", stream_frames=0)
    back = unpack(pack(req))
    np.testing.assert_array_equal(back["prompt_tokens"][0], req["prompt_tokens"][0])
    assert back["prompt_tokens"][0].dtype == np.int32 and back["top_p"] == 0.5 and back["text"] == "hi"
    w = engine.WrappedGenerateResponse("success", engine.GenerateResponse("sample", np.ones((2, 3), np.int32), "t", 1,
                                                                          np.linspace(-1, 1, 7, dtype=np.float32)))
    w2 = response_from_wire(unpack(pack(response_to_wire(w))))
    assert w2.response.action == "sample" and w2.response.stream == 1 and w2.response.text == "t"
    np.testing.assert_array_equal(w2.response.codes, w.response.codes)
    np.testing.assert_array_equal(w2.response.audio, w.response.audio)
    assert w2.response.audio.dtype == np.float32
    e = response_from_wire(unpack(pack(response_to_wire(engine.WrappedGenerateResponse("error", ValueError("x"))))))
    assert e.status == "error" and isinstance(e.response, ValueError) and str(e.response) == "x"
    assert response_from_wire(unpack(pack(response_to_wire(None)))) is None


def test_vocoder_thread_survives_failing_stream_close():
    """the per-rank vocoder thread must deliver every item even when a codec stream's
    close() raises (on the request's done marker, and again after a decode error): the backlog drains
    to 0, each done marker arrives, the thread stays alive, and after an error nothing more of that
    request reaches its caller."""
    from fishmi import engine
    from fishmi.dist_serving import _DROP, _Vocoder, _Vocoding

    class BadCloseVocoder(ScriptedVocoder):
        def open_stream(self):
            voc = self

            class _S:
                def decode_chunk(self, codes):
                    return voc.decode_codes(codes)

                def close(self):
                    raise RuntimeError("injected close failure")

            return _S()

    def sample(stream, k):
        return engine.WrappedGenerateResponse("success", engine.GenerateResponse(
            "sample", np.full((3, 2), k, np.int32), "t", stream))

    voc = _Vocoder(BadCloseVocoder(fail_at=5))
    got = {}

    class Sink:
        def __init__(self, name):
            self.name = name

        def put(self, w):
            got.setdefault(self.name, []).append(w)

    a, b = _Vocoding(Sink("a"), voc), _Vocoding(Sink("b"), voc)
    for k in range(3):  # a: a 3-chunk stream, then its done marker (its close raises)
        a.put(sample(k, k))
    voc.submit(a, None, done=True)
    for k in range(3):  # b: chunk 1 hits the failing decode (call 5), its later chunks are dropped
        b.put(sample(k, 10 + k))
    b.put(engine.WrappedGenerateResponse("success", engine.GenerateResponse("next")))
    voc.submit(b, None, done=True)
    finished = []

    def deliver(v, w):
        if w is None:
            finished.append(v)
        elif w is not _DROP:
            v.inner.put(w)

    t0 = time.time()
    while voc.drain(deliver) > 0:
        assert time.time() - t0 < 10, "vocoder backlog never drained"
        time.sleep(0.01)
    assert finished == [a, b]
    assert voc.th.is_alive()
    assert [w.status for w in got["a"]] == ["success"] * 3
    assert [w.status for w in got["b"]] == ["success", "error"]
    assert "injected codec failure" in str(got["b"][1].response)
    voc.close()
    voc.th.join(timeout=5)
    assert not voc.th.is_alive()
