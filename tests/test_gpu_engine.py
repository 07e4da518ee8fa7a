"""B1 worker seam on the GPU: fishmi.engine.generate_long / launch_thread_safe_queue against the
reference's own generate_long (tests/golden/engine.npz: greedy, fp32, llm_a weights, tiny
tokenizer, reference prompt + three speaker batches).  Codes must be identical."""
import json
import os
import queue
import shutil

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu


def _ckpt(tmp_path):
    d = tmp_path / "ckpt"
    shutil.copytree(os.path.join(GOLDEN, "llm_a"), d)
    for f in ("tokenizer.json", "tokenizer_config.json"):
        shutil.copy(os.path.join(GOLDEN, "tok_tiny", f), d / f)
    return str(d)


def _request(g, **kw):
    r = dict(device="cuda", max_new_tokens=7, text=str(g["text"]), top_p=0.9, repetition_penalty=1.1,
             temperature=0.7, compile=False, iterative_prompt=True, chunk_length=30,
             prompt_tokens=[g["ptok0"], g["ptok1"]], prompt_text=["ref a", "<|speaker:1|>ref b"], top_k=1)
    r.update(kw)
    return r


def _drain(q):
    out = []
    while True:
        w = q.get(timeout=300)
        out.append(w)
        if w.status == "error" or w.response.action == "next":
            return out


def test_generate_long_matches_reference(golden, tmp_path):
    from fishmi import engine

    g = golden("engine.npz")
    from fishmi.llm import DualARModel

    # generate_long refuses prompts longer than max_seq_len - 2048 (inference.py:651-654), so the
    # reference ran with max_length 2560 as well
    m = DualARModel.from_pretrained(_ckpt(tmp_path), device=0, precision="fp32", max_length=2560)
    assert m.tokenizer is not None and m.cfg.im_end_id == 4
    req = _request(g)
    outs = list(engine.generate_long(model=m, **req))
    assert [o.action for o in outs] == json.loads(str(g["actions"]))
    samples = [o for o in outs if o.action == "sample"]
    assert [o.text for o in samples] == json.loads(str(g["batch_texts"]))
    for i, o in enumerate(samples):
        np.testing.assert_array_equal(o.codes, g[f"codes_{i}"])


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_prefix_reuse_equals_reprefill(golden, tmp_path, precision):
    """generate_long's later batches keep the slot's KV for the prefix they share
    with the previous batch's prompt and fed columns, and prefill only the rest.  The codes equal
    the whole-conversation re-prefill (the reference's own flow, inference.py:620-724) in fp32 and
    bf16, and fewer positions are prefilled."""
    from fishmi import engine
    from fishmi.llm import DualARModel

    g = golden("engine.npz")
    m = DualARModel.from_pretrained(_ckpt(tmp_path), device=0, precision=precision, max_length=2560)
    calls = []
    gen_at = m.generate_at

    def spy(suffix, pos0, *a, **k):
        calls.append((pos0, suffix.shape[1]))
        return gen_at(suffix, pos0, *a, **k)

    m.generate_at = spy
    req = _request(g)
    reused = [o.codes for o in engine.generate_long(model=m, reuse_prefix=True, **req) if o.action == "sample"]
    full = [o.codes for o in engine.generate_long(model=m, reuse_prefix=False, **req) if o.action == "sample"]
    assert len(reused) == len(full) >= 3
    for a, b in zip(reused, full):
        np.testing.assert_array_equal(a, b)
    assert len(calls) == len(full) - 1 and all(p0 > 0 for p0, _ in calls)
    if precision == "fp32":
        for i, c in enumerate(reused):
            np.testing.assert_array_equal(c, g[f"codes_{i}"])


def test_worker_queue_contract(golden, tmp_path):
    """launch_thread_safe_queue: FIFO requests, sample* + next per request, an exception becomes
    status="error" and the worker keeps serving, None stops it (inference.py:748-799)."""
    from fishmi import engine
    from fishmi.llm import DualARModel

    g = golden("engine.npz")
    m = DualARModel.from_pretrained(_ckpt(tmp_path), device=0, precision="fp32", max_length=2560)
    q = engine.launch_thread_safe_queue(None, "cuda:0", "float32", model=m)
    rq = queue.Queue()
    q.put(engine.GenerateRequest(request=_request(g, temperature=5.0), response_queue=rq))  # invalid
    q.put(engine.GenerateRequest(request=_request(g), response_queue=rq))
    bad = _drain(rq)
    assert len(bad) == 1 and bad[0].status == "error" and isinstance(bad[0].response, AssertionError)
    good = _drain(rq)
    assert all(w.status == "success" for w in good)
    codes = [w.response.codes for w in good if w.response.action == "sample"]
    for i, c in enumerate(codes):
        np.testing.assert_array_equal(c, g[f"codes_{i}"])
    # sampled (top_k=30) requests are reproducible with the same seed
    q.put(engine.GenerateRequest(request=_request(g, top_k=30, seed=5), response_queue=rq))
    a = [w.response.codes for w in _drain(rq) if w.response.action == "sample"]
    q.put(engine.GenerateRequest(request=_request(g, top_k=30, seed=5), response_queue=rq))
    b = [w.response.codes for w in _drain(rq) if w.response.action == "sample"]
    for x, y in zip(a, b):
        np.testing.assert_array_equal(x, y)
    q.put(None)


def test_load_model_from_checkpoint_dir(tmp_path):
    """init_model path: config.json + safetensors shards + tokenizer.json in one directory."""
    from fishmi import engine

    m = engine.load_model(_ckpt(tmp_path), "cuda:0", "bfloat16")
    assert m.tokenizer.semantic_begin_id == m.cfg.semantic_begin_id == 200
    assert m.cfg.im_end_id == 4


@pytest.mark.parametrize("slots", [3, 12])
def test_batched_worker_matches_serial(golden, tmp_path, slots):
    """launch_thread_safe_queue(max_slots > 1): concurrent generate_long requests on batched KV slots
    (fishmi.batching.BatchedWorker; 12 slots take the bstream batched linears) answer each request
    with exactly its serial generate_long codes (fp32 validation mode), streamed and reused-prefix
    requests included; the first request is the reference golden's."""
    from fishmi import engine
    from fishmi.llm import DualARModel

    g = golden("engine.npz")
    m = DualARModel.from_pretrained(_ckpt(tmp_path), device=0, precision="fp32", max_length=2560,
                                    max_slots=slots)
    reqs = [_request(g)]
    texts = ["<|speaker:0|>Hello there. <|speaker:1|>Hi! How are you doing today?", "just one sentence",
             "<|speaker:0|>a. <|speaker:1|>bb. <|speaker:0|>ccc dd ee."]
    for i in range(7):
        reqs.append(_request(g, text=texts[i % 3], top_k=30, seed=50 + i, max_new_tokens=9 + 3 * i,
                             reuse_prefix=(i % 2 == 0), stream_frames=(5 if i % 3 == 1 else 0)))
    serial = [list(engine.generate_long(model=m, **r)) for r in reqs]
    q_in = engine.launch_thread_safe_queue(None, 0, "fp32", model=m, max_slots=slots)
    qs = [queue.Queue() for _ in reqs]
    for r, q in zip(reqs, qs):
        q_in.put(engine.GenerateRequest(request=r, response_queue=q))
    for i, (q, ref) in enumerate(zip(qs, serial)):
        got = _drain(q)
        assert all(w.status == "success" for w in got), got[-1].response

        def batches(rs):
            out = []
            for r in rs:
                if r.action == "sample" and r.stream is not None and r.stream > 0:
                    out[-1] = np.concatenate([out[-1], r.codes], axis=1)
                elif r.action == "sample":
                    out.append(np.asarray(r.codes))
            return out

        a, b = batches([w.response for w in got]), batches(ref)
        assert len(a) == len(b) >= 1, i
        for x, y in zip(a, b):
            np.testing.assert_array_equal(x, y, err_msg=f"request {i}")
    np.testing.assert_array_equal(serial[0][0].codes, g["codes_0"])
    q_in.put(None)


def test_distributed_worker_rccl_world1_matches_serial(golden, tmp_path):
    """The multi-GPU serving worker (fishmi.dist_serving) over RCCL with device tensors, one rank:
    requests and responses cross the tick collectives (scatter / gather of msgpack bytes on the
    GPU) and each request still gets its serial generate_long codes (fp32).  The world-2 routing is
    tests/test_dist_serving.py (gloo)."""
    import socket

    import torch
    import torch.distributed as dist

    from fishmi import engine
    from fishmi.dist_serving import launch_distributed_queue
    from fishmi.llm import DualARModel

    g = golden("engine.npz")
    m = DualARModel.from_pretrained(_ckpt(tmp_path), device=0, precision="fp32", max_length=2560, max_slots=4)
    reqs = [_request(g)] + [_request(g, text=t, top_k=30, seed=70 + i, max_new_tokens=10 + 4 * i)
                            for i, t in enumerate(["one two three", "<|speaker:0|>a b. <|speaker:1|>c d e."])]
    serial = [list(engine.generate_long(model=m, **r)) for r in reqs]
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    try:
        q_in, th = launch_distributed_queue(None, 0, "fp32", max_slots=4, tick_frames=4, model=m)
        qs = [queue.Queue() for _ in reqs]
        for r, q in zip(reqs, qs):
            q_in.put(engine.GenerateRequest(request=r, response_queue=q))
        for i, (q, ref) in enumerate(zip(qs, serial)):
            got = _drain(q)
            assert all(w.status == "success" for w in got), got[-1].response
            a = [np.asarray(w.response.codes) for w in got if w.response.action == "sample"]
            b = [np.asarray(r.codes) for r in ref if r.action == "sample"]
            assert len(a) == len(b) >= 1, i
            for x, y in zip(a, b):
                np.testing.assert_array_equal(x, y, err_msg=f"request {i}")
        q_in.put(None)
        th.join(timeout=60)
        assert not th.is_alive()
    finally:
        dist.destroy_process_group()
