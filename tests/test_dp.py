"""world_size-2 gloo test of the data-parallel request scatter / PCM gather (fishmi/dp.py) that
bench.py and the engine use over RCCL on the GPU box."""
import os
import socket

import numpy as np
import pytest


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    import torch.distributed as dist

    from fishmi import dp

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rows = 11
        prompts = None
        if rank == 0:
            prompts = [np.arange(rows * (5 + 3 * r), dtype=np.int32).reshape(rows, -1) + 1000 * r
                       for r in range(world)]
        mine = dp.scatter_prompts(prompts, rows)
        # each "rank" synthesises a PCM whose length and content depend on its prompt
        pcm = np.sin(np.arange(2048 * mine.shape[1] + rank, dtype=np.float32) * 0.01 + float(mine[0, 0]))
        got = dp.gather_pcm(dp.pcm_to_int16(pcm))
        q.put((rank, mine.tolist(), None if got is None else [g.tolist() for g in got]))
    finally:
        dist.destroy_process_group()


def test_scatter_gather_world2():
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(2):
        rank, mine, got = q.get(timeout=120)
        res[rank] = (np.array(mine, np.int32), got)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    rows = 11
    from fishmi import dp

    for r in range(2):
        exp = np.arange(rows * (5 + 3 * r), dtype=np.int32).reshape(rows, -1) + 1000 * r
        np.testing.assert_array_equal(res[r][0], exp)
    assert res[1][1] is None
    got = res[0][1]
    for r in range(2):
        T = 5 + 3 * r
        first = 1000 * r
        pcm = np.sin(np.arange(2048 * T + r, dtype=np.float32) * 0.01 + float(first))
        np.testing.assert_array_equal(np.array(got[r], np.int16), dp.pcm_to_int16(pcm))


def test_pcm_to_int16_clips():
    from fishmi import dp

    x = np.array([-2.0, -1.0, 0.0, 0.5, 1.0, 3.0], np.float32)
    np.testing.assert_array_equal(dp.pcm_to_int16(x), [-32767, -32767, 0, 16383, 32767, 32767])
