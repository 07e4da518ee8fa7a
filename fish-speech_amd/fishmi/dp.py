"""Data-parallel request scatter / result gather across one process per GPU.

Utterances are independent: every rank holds a full weight replica and decodes its own
requests with no exchange on the data path.  The only collectives are

  * scatter of request descriptors (prompt token matrix (C+1) x T, int32) from rank 0, and
  * gather of the synthesised PCM (int16, the reference's streaming wire format,
    tools/server/inference.py:18-39) back to rank 0,

over RCCL (backend "nccl", device tensors on xGMI) on the GPU box, or gloo (host tensors) in
the CPU tests.  Variable lengths travel as a small length header followed by one padded
collective, so each exchange is two collectives regardless of world size.

The reference's own precedent is a static `files[RANK::WORLD_SIZE]` split
(tools/vqgan/extract_vq.py:197); here rank 0 owns the request list and assigns request i to
rank i % world (round-robin, matching the fixed-size weak-scaling bench).
"""
from __future__ import annotations

from typing import List, Optional, Sequence

import numpy as np


def _dist():
    import torch.distributed as dist

    return dist


def _device():
    import torch

    dist = _dist()
    if dist.get_backend() == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def scatter_prompts(prompts: Optional[Sequence[np.ndarray]], rows: int) -> np.ndarray:
    """Rank 0 passes one (rows x T_r) int32 prompt per rank; every rank returns its own."""
    import torch

    dist = _dist()
    world, rank = dist.get_world_size(), dist.get_rank()
    dev = _device()
    hdr = torch.zeros(world, dtype=torch.int64, device=dev)
    if rank == 0:
        if prompts is None or len(prompts) != world:
            raise ValueError(f"rank 0 must supply exactly {world} prompts")
        for r, p in enumerate(prompts):
            if p.ndim != 2 or p.shape[0] != rows:
                raise ValueError(f"prompt {r} has shape {p.shape}, expected ({rows}, T)")
            hdr[r] = p.shape[1]
    dist.broadcast(hdr, src=0)
    tmax = int(hdr.max().item())
    mine = torch.empty(rows * tmax, dtype=torch.int32, device=dev)
    chunks = None
    if rank == 0:
        chunks = []
        for p in prompts:
            buf = np.zeros((rows, tmax), np.int32)
            buf[:, : p.shape[1]] = p
            chunks.append(torch.from_numpy(buf.reshape(-1)).to(dev))
    dist.scatter(mine, chunks, src=0)
    t = int(hdr[rank].item())
    return np.ascontiguousarray(mine.cpu().numpy().reshape(rows, tmax)[:, :t])


def pcm_to_int16(pcm: np.ndarray) -> np.ndarray:
    """float PCM in [-1, 1] -> int16 (tools/server/inference.py:33, x * 32767)."""
    return (np.clip(pcm, -1.0, 1.0) * 32767.0).astype(np.int16)


def gather_pcm(pcm16: np.ndarray) -> Optional[List[np.ndarray]]:
    """Every rank passes its int16 PCM; rank 0 returns the list ordered by rank, others None."""
    import torch

    dist = _dist()
    world, rank = dist.get_world_size(), dist.get_rank()
    dev = _device()
    n = torch.tensor([pcm16.size], dtype=torch.int64, device=dev)
    lens = [torch.zeros(1, dtype=torch.int64, device=dev) for _ in range(world)]
    dist.all_gather(lens, n)
    lens = [int(x.item()) for x in lens]
    nmax = max(lens)
    buf = np.zeros(nmax, np.int16)
    buf[: pcm16.size] = pcm16.reshape(-1)
    # int16 travels as its raw bytes viewed as int32 pairs (RCCL has no int16 type in torch)
    if nmax % 2:
        buf = np.concatenate([buf, np.zeros(1, np.int16)])
    mine = torch.from_numpy(buf.view(np.int32).copy()).to(dev)
    outs = [torch.empty_like(mine) for _ in range(world)] if rank == 0 else None
    dist.gather(mine, outs, dst=0)
    if rank != 0:
        return None
    return [outs[r].cpu().numpy().view(np.int16)[: lens[r]].copy() for r in range(world)]
