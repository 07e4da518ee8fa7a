"""B2 operator seam (DecodeOneToken, inference.py:96-107) on a scripted model: the state checks
that keep the caller's KV / RAS state and the slot's in step.  CPU only."""
import numpy as np
import pytest
import torch

from fishmi.config import DualARConfig
from fishmi.llm import DecodeOneToken


class _Scripted:
    """Stands in for DualARModel: prefill / decode / slot_pos with a counter for columns."""

    def __init__(self, C1=3, vocab=64):
        self.C1 = C1
        self.cfg = DualARConfig(vocab_size=vocab, num_codebooks=C1 - 1, semantic_begin_id=32,
                                semantic_end_id=63, im_end_id=4)
        self.pos = 0
        self.n = 0
        self.calls = []

    def slot_pos(self, slot=0):
        return self.pos

    def prefill(self, slot, x, sp, pos0=0):
        self.calls.append(("prefill", pos0, x.shape[1], sp.temperature, sp.top_k))
        self.pos = pos0 + x.shape[1]
        return self._col()

    def decode(self, slots):
        self.calls.append(("decode", self.pos))
        self.pos += 1
        return self._col()[None]

    def _col(self):
        self.n += 1
        return np.array([32 + self.n] + [self.n] * (self.C1 - 1), np.int32)


def _bias(cfg):
    b = torch.full((1, 1, cfg.vocab_size), float("-inf"))
    b[0, 0, cfg.semantic_begin_id: cfg.semantic_end_id + 1] = 0.0
    b[0, 0, cfg.im_end_id] = 0.0
    return b


def _args(m):
    return torch.tensor(0.7), torch.tensor(0.9), 30, _bias(m.cfg)


def test_prefill_then_decode_feeds_back():
    m = _Scripted()
    op = DecodeOneToken(m)
    t, p, k, b = _args(m)
    first = op(None, torch.zeros(1, 3, 5, dtype=torch.int32), torch.arange(5), t, p, k, b, None, None)
    assert first.shape == (3, 1) and first.dtype == torch.int64
    nxt = op(None, first.view(1, 3, 1), torch.tensor([5]), t, p, k, b, None, None)
    assert m.calls[0][:3] == ("prefill", 0, 5) and m.calls[1] == ("decode", 5)
    assert int(nxt[0, 0]) == 34


def test_state_mismatches_raise():
    m = _Scripted()
    op = DecodeOneToken(m)
    t, p, k, b = _args(m)
    with pytest.raises(ValueError, match="before a prefill"):
        op(None, torch.zeros(1, 3, 1, dtype=torch.int32), torch.tensor([3]), t, p, k, b)
    first = op(None, torch.zeros(1, 3, 4, dtype=torch.int32), torch.arange(4), t, p, k, b)
    with pytest.raises(ValueError, match="next position"):
        op(None, first.view(1, 3, 1), torch.tensor([7]), t, p, k, b)
    with pytest.raises(ValueError, match="emitted last"):
        op(None, torch.zeros(1, 3, 1, dtype=torch.int32), torch.tensor([4]), t, p, k, b)
    with pytest.raises(ValueError, match="changed after the prefill"):
        op(None, first.view(1, 3, 1), torch.tensor([4]), torch.tensor(0.5), p, k, b)
    with pytest.raises(ValueError, match="semantic_logit_bias"):
        op(None, first.view(1, 3, 1), torch.tensor([4]), t, p, k, torch.zeros(1, 1, m.cfg.vocab_size))
    with pytest.raises(NotImplementedError):
        op(None, first.view(1, 3, 1), torch.tensor([4]), t, p, k, b, torch.ones(1), torch.ones(1))


def test_prefix_prefill_at_cached_position():
    m = _Scripted()
    op = DecodeOneToken(m)
    t, p, k, b = _args(m)
    op(None, torch.zeros(1, 3, 6, dtype=torch.int32), torch.arange(6), t, p, k, b)
    op(None, torch.zeros(1, 3, 3, dtype=torch.int32), torch.arange(4, 7), t, p, k, b)
    assert m.calls[-1][:3] == ("prefill", 4, 3)
    with pytest.raises(ValueError, match="past the slot"):
        op(None, torch.zeros(1, 3, 2, dtype=torch.int32), torch.arange(9, 11), t, p, k, b)
