"""scheduler.StreamVocoder (the serving loop's vocoder on a host thread of its own) with a fake
causal codec on the CPU: each request's chunks, streamed through a pooled context while its later
columns are still arriving, concatenate to the one-shot decode of its codes; contexts are rewound
and reused, never more than the streams live at once; a codec error reaches the request's finish
and leaves the others served.  The real codec's chunk / rewind equality is
tests/test_gpu_codec_stream.py."""
import threading

import numpy as np
import pytest

C1 = 4


class _Ctx:
    """Causal fake: output frame t = running sum of codes[1] up to t (the carried state), plus
    codes[2]."""

    def __init__(self, codec):
        self.codec, self.acc = codec, 0

    def decode_chunk(self, codes):
        assert codes.shape[0] == C1 - 1 and 1 <= codes.shape[1] <= self.codec.max_frames
        assert threading.current_thread() is not threading.main_thread()  # off the decode thread
        if self.codec.fail_on is not None and (codes[0] == self.codec.fail_on).any():
            raise RuntimeError("codec failure")
        s = self.acc + np.cumsum(codes[0].astype(np.int64))
        self.acc = int(s[-1])
        self.codec.calls.append(codes.shape[1])
        return (s + codes[1]).astype(np.float32)

    def rewind(self):
        self.acc = 0
        self.codec.rewinds += 1

    def close(self):
        self.codec.closed += 1


class _Codec:
    def __init__(self, max_frames, fail_on=None):
        self.max_frames, self.fail_on = max_frames, fail_on
        self.opened = self.rewinds = self.closed = 0
        self.calls = []

    def open_stream(self):
        self.opened += 1
        return _Ctx(self)


def _one_shot(cols):
    codes = cols[1:]
    return (np.cumsum(codes[0].astype(np.int64)) + codes[1]).astype(np.float32)


def _streams(n, T, seed):
    rng = np.random.default_rng(seed)
    return [rng.integers(0, 50, (C1, T + 1)).astype(np.int32) for _ in range(n)]


@pytest.mark.parametrize("chunk,max_frames", [(1, 64), (8, 64), (32, 16), (100, 40)])
def test_chunks_equal_one_shot_and_contexts_pooled(chunk, max_frames):
    from fishmi import scheduler as S

    codec = _Codec(max_frames)
    voc = S.StreamVocoder(codec, chunk)
    assert voc.chunk == min(chunk, max_frames)
    T = 70
    for wave in range(3):
        streams = _streams(3, T, wave)
        reqs = [S.Request(10 * wave + i, np.zeros((C1, 1), np.int32), T, 0) for i in range(3)]
        cols = [[] for _ in streams]
        for t in range(0, T + 1, 9):  # ticks of 9 columns, streams interleaved
            for i, c in enumerate(streams):
                cols[i] += [c[:, j] for j in range(t, min(t + 9, T + 1))]
                voc.progress(i, reqs[i], cols[i])
        for i in (2, 0, 1):  # finishing order differs from the start order
            full = np.stack(cols[i], 1)[:, :-1]  # serve() drops the last column
            np.testing.assert_array_equal(voc.finish(i, reqs[i], full), _one_shot(full))
    assert codec.opened == 3 and codec.rewinds == 9  # one context per live stream, reused
    assert max(codec.calls) <= voc.chunk or max(codec.calls) <= max_frames
    voc.close()
    assert codec.closed == 3


def test_stream_without_progress_and_empty_stream():
    from fishmi import scheduler as S

    codec = _Codec(16)
    voc = S.StreamVocoder(codec, 8)
    c = _streams(1, 40, 5)[0][:, :40]
    r = S.Request(1, np.zeros((C1, 1), np.int32), 40, 0)
    np.testing.assert_array_equal(voc.finish(0, r, c), _one_shot(c))  # all of it at the end, split by max_frames
    assert codec.calls == [16, 16, 8]
    e = voc.finish(0, S.Request(2, np.zeros((C1, 1), np.int32), 1, 0), np.zeros((C1, 0), np.int32))
    assert e.dtype == np.float32 and e.size == 0  # a stream that ended on its first column
    voc.close()


def test_codec_error_reaches_its_request_only():
    from fishmi import scheduler as S

    codec = _Codec(64, fail_on=49)
    voc = S.StreamVocoder(codec, 4)
    good = _streams(1, 30, 7)[0] % 40
    bad = good.copy()
    bad[1, 10] = 49
    reqs = [S.Request(i, np.zeros((C1, 1), np.int32), 30, 0) for i in range(2)]
    cols = [[], []]
    for t in range(31):
        for i, c in enumerate((good, bad)):
            cols[i].append(c[:, t])
            voc.progress(i, reqs[i], cols[i])
    with pytest.raises(RuntimeError, match="codec failure"):
        voc.finish(1, reqs[1], np.stack(cols[1], 1)[:, :-1])
    full = np.stack(cols[0], 1)[:, :-1]
    np.testing.assert_array_equal(voc.finish(0, reqs[0], full), _one_shot(full))
    # the failed request's context was rewound and pooled: the next request starts clean
    r2 = S.Request(5, np.zeros((C1, 1), np.int32), 30, 0)
    np.testing.assert_array_equal(voc.finish(0, r2, full), _one_shot(full))
    assert codec.opened == 2
    voc.close()
