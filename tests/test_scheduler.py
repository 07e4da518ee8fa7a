"""Dynamic DP tick queue (fishmi/scheduler.py; BASELINE configs 3/4) on gloo at world_size 2.

A fake engine stands in for the GPU decode: stream `id` emits column k = [tok0, id, k, ...], with
tok0 = IM_END at frame `stop` for requests that stop early. Checks: every request is served exactly
once; results reach rank 0 intact; `<|im_end|>` ends a stream and the last column is dropped, as
in generate_long (inference.py:683-688); no rank exceeds its concurrency; the work spreads over
both ranks."""
import os
import socket

import numpy as np
import pytest

IM_END = 7
C1 = 4


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _requests(n):
    from fishmi.scheduler import Request

    rng = np.random.default_rng(0)
    out = []
    for i in range(n):
        T = int(rng.integers(1, 9))
        out.append(Request(i, (np.arange(C1 * T, dtype=np.int32).reshape(C1, T) + 100 * i),
                           int(rng.integers(1, 40)), seed=1000 + i))
    return out


def _stop(rid):
    return 5 + rid % 7 if rid % 3 == 0 else None  # every third request hits <|im_end|> early


def expected_codes(req):
    n = req.frames
    s = _stop(req.id)
    cols = []
    for k in range(n):
        tok0 = IM_END if (s is not None and k == s) else 50 + k
        cols.append([tok0, req.id, k, req.seed % 97])
        if tok0 == IM_END:
            break
    return np.array(cols, np.int32).T[1:, :-1]


def _worker(rank, world, port, q, n_req, conc, batched=False):
    import torch.distributed as dist

    from fishmi import scheduler as S

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        queue = S.TickQueue(_requests(n_req) if rank == 0 else None, C1)
        slots = {}
        peak = [0]

        def start(slot, req):
            assert slot not in slots
            slots[slot] = [req, 0]
            peak[0] = max(peak[0], len(slots))
            return step_col(slot)

        def step_col(slot):
            req, k = slots[slot]
            s = _stop(req.id)
            slots[slot][1] += 1
            return np.array([IM_END if (s is not None and k == s) else 50 + k, req.id, k, req.seed % 97], np.int32)

        def step(live, n):
            return np.stack([np.stack([step_col(s) for s in live]) for _ in range(n)])

        seen = {}

        def progress(slot, req, cols):  # growing prefixes of the stream, never rewritten
            prev = seen.get(req.id, [])
            assert len(cols) > len(prev) and all(np.array_equal(a, b) for a, b in zip(prev, cols))
            seen[req.id] = [c.copy() for c in cols]

        def finish(slot, req, cols):
            del slots[slot]
            prev = seen.get(req.id)
            if prev:  # all but the newest column a consumer saw are the stream's final columns
                np.testing.assert_array_equal(np.stack(prev[:-1], 1), cols[:, :len(prev) - 1])
            return np.ascontiguousarray(cols[1:]).reshape(-1).astype(np.int32)

        def start_batch(pairs):  # a tick's new requests at once (fm_llm_prefill_batch's seam)
            return np.stack([start(slot, req) for slot, req in pairs])

        stats = S.serve(queue, conc, start, step, finish, tick_frames=6, im_end=IM_END,
                        start_batch=start_batch if batched else None, progress=progress)
        res = [(r.id, r.rank, r.data.tolist()) for r in queue.results] if rank == 0 else None
        q.put((rank, stats, peak[0], res))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("n_req,conc,batched", [(11, 3, False), (2, 4, False), (0, 2, False), (11, 3, True)])
def test_tick_queue_world2(n_req, conc, batched):
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q, n_req, conc, batched)) for r in range(2)]
    for p in procs:
        p.start()
    out = {}
    for _ in range(2):
        rank, stats, peak, res = q.get(timeout=120)
        out[rank] = (stats, peak, res)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res = out[0][2]
    assert sorted(r[0] for r in res) == list(range(n_req))
    reqs = {r.id: r for r in _requests(n_req)}
    for rid, rank, data in res:
        exp = expected_codes(reqs[rid])
        np.testing.assert_array_equal(np.array(data, np.int32).reshape(C1 - 1, -1), exp)
    assert out[0][0]["served"] + out[1][0]["served"] == n_req
    assert out[0][1] <= conc and out[1][1] <= conc
    if n_req >= 2:
        assert out[0][0]["served"] >= 1 and out[1][0]["served"] >= 1


def test_assign_round_robin():
    from fishmi.scheduler import assign

    assert assign([3, 3], 4) == [2, 2]
    assert assign([0, 5, 1], 4) == [0, 3, 1]
    assert assign([2, 2], 0) == [0, 0]
    assert assign([32] * 8, 256) == [32] * 8
