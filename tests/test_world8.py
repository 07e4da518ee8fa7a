"""BASELINE config 4 at the world size it names, on CPU (gloo, 8 processes): 256 requests over 8 ranks.

The driver measures config 4 on an 8-GPU node; these tests pin what that run relies on, at world 8:

* the tick queue (fishmi/scheduler.py) with config 4's request list -- 256 prompts of 16-256 tokens
  (bench.py throughput_leg: uniform lengths, seed 2) -- and scripted decoders whose per-frame cost
  differs by rank (rank r: (r + 1) x 0.4 ms a frame, an 8:1 spread): every request is answered exactly
  once with its own codes; the collective cost of a tick stays small; the time rank 0 waits for a
  straggler at a tick stays within one tick of the slowest rank's decoding (tick_frames frames);
  and a rank whose streams end early is refilled at the next tick (the queue balances request
  lengths dynamically, unlike the reference's static files[RANK::WORLD_SIZE] split,
  tools/vqgan/extract_vq.py:150-197);
* the serving worker (fishmi/dist_serving.py) at world 8 with the same skew: each request's
  responses equal its serial generate_long responses, in order.
"""
import os
import socket
import time
import traceback

import numpy as np
import pytest

WORLD = 8
C1 = 11  # S2-Pro: 10 codebooks + the main token
IM_END = 7
FRAME_S = 0.0004  # scripted decode cost per frame on rank 0; rank r pays (r + 1) x this


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _config4_requests():
    """bench.py throughput_leg's list at N=8: batch 32 x world 8 = 256 requests, prompt lengths
    uniform in [16, 256] (seed 2); frames vary here (5-40) so streams end at different ticks."""
    from fishmi.scheduler import Request

    rng = np.random.default_rng(2)
    n = 32 * WORLD
    lens = rng.integers(16, 257, n)
    frames = rng.integers(5, 41, n)
    return [Request(i, (np.arange(C1 * int(lens[i]), dtype=np.int32).reshape(C1, -1) + i) % 997, int(frames[i]),
                    31 * i + 7) for i in range(n)]


def _stop(rid):
    return 3 + rid % 11 if rid % 5 == 0 else None  # every fifth request hits <|im_end|> early


def _col(req, k):
    s = _stop(req.id)
    tok0 = IM_END if (s is not None and k == s) else 50 + k
    return np.array([tok0, req.id % 1024, k, req.seed % 97, req.prompt.shape[1]] + [req.id % 13] * (C1 - 5),
                    np.int32)


def _expected(req):
    cols = []
    for k in range(req.frames):
        cols.append(_col(req, k))
        if cols[-1][0] == IM_END:
            break
    return np.stack(cols, 1)[1:, :-1]


def _queue_worker(rank, port, out_q, conc, tick_frames):
    import torch.distributed as dist

    from fishmi import scheduler as S

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        q = S.TickQueue(_config4_requests() if rank == 0 else None, C1)
        slots = {}
        delay = FRAME_S * (rank + 1)
        ticks = []  # (entered, left) of every tick on this rank, perf_counter seconds
        orig_tick = q.tick

        def timed_tick(*a, **k):
            t0 = time.perf_counter()
            r = orig_tick(*a, **k)
            ticks.append((t0, time.perf_counter()))
            return r

        q.tick = timed_tick

        def start(slot, req):
            assert slot not in slots and len(slots) < conc
            slots[slot] = [req, 1]
            return _col(req, 0)

        def step(live, n):
            time.sleep(n * delay)  # the rank's batched frames
            out = np.zeros((n, len(live), C1), np.int32)
            for j, s in enumerate(live):
                req, k = slots[s]
                for f in range(n):
                    out[f, j] = _col(req, k + f)
                slots[s][1] = k + n
            return out

        def finish(slot, req, cols):
            del slots[slot]
            return np.ascontiguousarray(cols[1:]).reshape(-1).astype(np.int32)

        stats = S.serve(q, conc, start, step, finish, tick_frames=tick_frames, im_end=IM_END)
        res = [(r.id, r.rank, r.data) for r in q.results] if rank == 0 else None
        out_q.put((rank, "ok", stats, ticks, res))
    except Exception:
        out_q.put((rank, traceback.format_exc(), None, None, None))
    finally:
        dist.destroy_process_group()


def _spawn(target, args_of, timeout=240):
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, port, q) + args_of(r)) for r in range(WORLD)]
    for p in procs:
        p.start()
    out = {}
    try:
        for _ in range(WORLD):
            item = q.get(timeout=timeout)
            out[item[0]] = item[1:]
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    for r in range(WORLD):
        assert out[r][0] == "ok", out[r][0]
    return out


@pytest.mark.parametrize("conc,tick_frames", [(32, 8), (8, 6)])
def test_tick_queue_config4_world8_skewed_ranks(conc, tick_frames):
    """conc 32: config 4 as benched (32 slots per rank, every request dealt at the first tick);
    conc 8: four waves of requests, so finished slots are refilled at later ticks."""
    out = _spawn(_queue_worker, lambda r: (conc, tick_frames))
    reqs = {r.id: r for r in _config4_requests()}
    res = out[0][3]
    ids = [rid for rid, _, _ in res]
    assert sorted(ids) == list(range(len(reqs))), "every request answered exactly once"
    for rid, rank, data in res:
        np.testing.assert_array_equal(data.reshape(C1 - 1, -1), _expected(reqs[rid]), err_msg=f"request {rid}")
    served = [out[r][1]["served"] for r in range(WORLD)]
    assert sum(served) == len(reqs)
    ticks = [out[r][2] for r in range(WORLD)]
    n = min(len(t) for t in ticks)
    assert all(len(t) == n for t in ticks), "every rank runs the same ticks"
    # per tick: the collective cost (the last rank to arrive waits for nobody) and rank 0's wait
    overhead = [min(ticks[r][i][1] - ticks[r][i][0] for r in range(WORLD)) for i in range(n)]
    wait0 = [ticks[0][i][1] - ticks[0][i][0] - overhead[i] for i in range(n)]
    straggler_bound = tick_frames * FRAME_S * WORLD + 0.1  # one tick of the slowest rank's frames + slack
    print(f"conc {conc}: {n} ticks, served per rank {served}, tick collective cost median "
          f"{np.median(overhead) * 1e3:.2f} ms (max {max(overhead) * 1e3:.2f}), rank 0 straggler wait max "
          f"{max(wait0) * 1e3:.1f} ms (bound {straggler_bound * 1e3:.0f} ms)")
    assert np.median(overhead) < 0.05 and max(overhead) < 0.5
    assert max(wait0) < straggler_bound
    # the ticks are synchronous (a rank's speed does not buy it more requests: every rank decodes
    # tick_frames frames between all_gathers); what balances is length -- a rank whose streams end
    # early is refilled at the next tick, so with several waves every rank serves more than one
    assert min(served) >= min(conc, len(reqs) // WORLD), served


def _serving_worker(rank, port, out_q):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        import queue

        from fishmi import engine
        from fishmi.dist_serving import launch_distributed_queue
        from test_batching import ScriptedModel, _requests
        from test_dist_serving import _check, _collect, _serial

        class SkewedModel(ScriptedModel):  # rank r decodes (r + 1) x slower
            def decode_frames(self, slots, n):
                time.sleep(n * FRAME_S * (rank + 1))
                return super().decode_frames(slots, n)

        model = SkewedModel(4)
        q_in, th = launch_distributed_queue(None, 0, "bf16", max_slots=4, tick_frames=4, model=model)
        if rank == 0:
            reqs = []
            for k in range(5):  # 45 requests: more than the 32 slots of the group
                for r in _requests():
                    r = dict(r, seed=r["seed"] + 1000 * k)
                    reqs.append(r)
            ref = _serial(reqs)
            qs = [queue.Queue() for _ in reqs]
            for r, q in zip(reqs, qs):
                q_in.put(engine.GenerateRequest(request=r, response_queue=q))
            for i, (q, rf) in enumerate(zip(qs, ref)):
                n_final = 0 if rf[-1].status == "error" else sum(w.response.action == "next" for w in rf)
                _check(_collect(q, max(n_final, 1)), rf, i)  # its serial responses, in order
            q_in.put(None)
        th.join(timeout=180)
        assert not th.is_alive()
        out_q.put((rank, "ok", len([c for c in model.calls if c[0] in ("prefill", "prefill_batch")])))
    except Exception:
        out_q.put((rank, traceback.format_exc(), 0))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def test_distributed_worker_world8_skewed_ranks():
    out = _spawn(_serving_worker, lambda r: ())
    busy = [out[r][1] for r in range(WORLD)]
    assert sum(1 for b in busy if b > 0) >= WORLD // 2, busy  # the requests spread over the group
