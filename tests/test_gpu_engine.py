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


def test_prefix_reuse_equals_reprefill_fp32(golden, tmp_path):
    """generate_long's later batches keep the slot's KV for the prefix they share
    with the previous batch's prompt and fed columns, and prefill only the rest.  In the fp32
    validation mode the codes equal the whole-conversation re-prefill (the reference's own flow,
    inference.py:620-724) and the reference's own generate_long codes; fewer positions are
    prefilled.  (bf16: test_prefix_reuse_bf16_within_reference_error below.)"""
    from fishmi import engine
    from fishmi.llm import DualARModel

    g = golden("engine.npz")
    m = DualARModel.from_pretrained(_ckpt(tmp_path), device=0, precision="fp32", max_length=2560)
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
    for i, c in enumerate(reused):
        np.testing.assert_array_equal(c, g[f"codes_{i}"])


def _teacher_forced_flow(m, g, req, reuse):
    """Drive generate_long's host side (engine.ConversationJob) batch by batch with every sampler
    forced to the reference's bf16 columns (engine_bf16.npz): batch i prefills its conversation
    prompt -- with reuse, only the part past the slot's cached prefix, at pos0 = L -- then decodes
    the rest of its columns.  Returns per batch (slow logits, fast logits, L)."""
    from fishmi import engine

    job = engine.ConversationJob(m, reuse_prefix=reuse, **req)
    out = []
    for i in range(int(g["n_batches"])):
        plan = job.next_batch()
        enc, L = plan.enc, plan.L
        np.testing.assert_array_equal(enc, g[f"prompt_{i}"])  # the reference's encoded conversation
        cols = g[f"cols_{i}"]
        n = cols.shape[1]
        slow = np.zeros((n, m.cfg.vocab_size), np.float32)
        fast = np.zeros((n, m.cfg.num_codebooks - 1, m.cfg.codebook_size), np.float32)
        sp = m.sampling(top_k=1)
        try:
            for j in range(n):
                m.force(0, cols[:, j])
                if j == 0:
                    m.prefill(0, enc[:, L:], sp, pos0=L)
                else:
                    m.decode([0])
                slow[j], fast[j] = m.read_logits(0)
        finally:
            m.force(0, None)
        assert m.slot_pos() == enc.shape[1] + n - 1
        job.finish_batch(cols, cols[:, : n - 1])
        out.append((slow, fast, L))
    assert job.next_batch() == "next"
    return out


def test_prefix_reuse_bf16_within_reference_error(golden, tmp_path):
    """bf16 prefix reuse held to the reference.  The reference ran generate_long
    in bf16 and, per text batch, replayed its whole-conversation prompt and emitted columns
    teacher-forced in bf16 and in fp32 (oracle/gen_goldens.py cmd_engine_bf16).  The native flow
    with reuse_prefix -- later batches prefill only the suffix past the KV the slot already holds,
    part of it written by the previous batch's DECODE frames -- gives logits within 1.5x the
    reference's own bf16-vs-fp32 error over the conversation's stream, as does the native re-prefill
    flow.  The decode-written rows are not required to equal the prompt pass's bit for bit: the
    prompt GEMM accumulates K in another order than the decode GEMVs (test_decode_written_kv_rows
    below)."""
    from fishmi.llm import DualARModel
    from parity_util import bf16_vs_reference

    g = golden("engine_bf16.npz")
    req = _request(golden("engine.npz"))
    m = DualARModel.from_pretrained(_ckpt(tmp_path), device=0, precision="bf16", max_length=2560)
    reused = _teacher_forced_flow(m, g, req, reuse=True)
    full = _teacher_forced_flow(m, g, req, reuse=False)
    assert [L for _, _, L in full] == [0] * len(full)
    assert reused[0][2] == 0 and all(L > 0 for _, _, L in reused[1:])
    nb = len(full)
    ref = [np.concatenate([g[f"{k}_{i}"] for i in range(nb)]) for k in ("slow", "fast", "slow32", "fast32")]
    for flow in (reused, full):  # the bound over the whole conversation's stream, as for every bf16 golden
        bf16_vs_reference(np.concatenate([s for s, _, _ in flow]), np.concatenate([f for _, f, _ in flow]), *ref)
    for i, ((s_r, f_r, L), (s_f, f_f, _)) in enumerate(zip(reused, full)):
        fin = np.isfinite(s_f)
        print(f"batch {i}: reused {L} positions; reuse vs re-prefill max |d logit| "
              f"{np.abs(s_r[fin] - s_f[fin]).max():.3g} slow, {np.abs(f_r - f_f).max():.3g} fast")


def test_decode_written_kv_rows(golden, tmp_path):
    """What prefix reuse relies on, measured directly (scripts/kv_identity_probe.py): after a prompt
    of 300 positions (flash-decode attention then runs in several splits) and 11 teacher-forced
    decode frames, the K / V rows the decode frames wrote are compared with the rows one prompt pass
    over prompt ++ those columns writes.  (1) Two identical decode runs write bit-identical rows --
    the run-to-run race of the reverted fused slow attention (cecda67) broke exactly this, by
    thousands of ulps from layer 1 on.  (2) With the prompt linears on the GEMV-order linear kernel
    (fm_tune prompt_gemm 0) the rows are bit-identical; with the default LDS-tiled prompt GEMM, whose
    K accumulation order differs, at most a few elements differ, by at most 2 bf16 ulps."""
    from fishmi import native
    from fishmi.llm import DualARModel

    gl = golden("llm_a_bf16.npz")
    T0 = gl["prompt"].shape[1]
    cols = gl["seq"][:, T0:T0 + 12]
    prompt = np.concatenate([gl["prompt"]] * 13, axis=1)[:, :300]
    T, n = prompt.shape[1], cols.shape[1]
    m = DualARModel.from_pretrained(_ckpt(tmp_path), device=0, precision="bf16", max_length=1024)
    sp = m.sampling(top_k=1)

    def decode_rows():
        for i in range(n):
            m.force(0, cols[:, i])
            if i == 0:
                m.prefill(0, prompt, sp)
            else:
                m.decode([0])
        m.force(0, None)
        return [m.read_cache(l) for l in range(m.cfg.n_layer)]

    def prompt_rows():
        m.force(0, cols[:, n - 1])
        m.prefill(0, np.concatenate([prompt, cols[:, : n - 1]], axis=1), sp)
        m.force(0, None)
        return [m.read_cache(l) for l in range(m.cfg.n_layer)]

    def diff(a, b):
        d = [(x[:, T:T + n - 1], y[:, T:T + n - 1]) for kv_a, kv_b in zip(a, b) for x, y in zip(kv_a, kv_b)]
        cnt = sum(int((x != y).sum()) for x, y in d)
        ulp = max(int((np.abs(x.view(np.int32).astype(np.int64) - y.view(np.int32).astype(np.int64)) >> 16).max())
                  for x, y in d)
        return cnt, ulp, sum(x.size for x, _ in d)

    try:
        a1 = decode_rows()
        a2 = decode_rows()
        assert diff(a1, a2)[0] == 0, "decode-written K / V rows differ between two identical runs"
        cnt, ulp, tot = diff(a1, prompt_rows())
        print(f"default prompt GEMM: {cnt} of {tot} decode-written elements differ (max {ulp} ulp)")
        assert cnt <= tot // 100 and ulp <= 2
        native.tune("prompt_gemm", 0)
        assert diff(decode_rows(), prompt_rows())[0] == 0
    finally:
        native.tune("prompt_gemm", 1)


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
