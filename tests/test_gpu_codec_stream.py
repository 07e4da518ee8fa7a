"""GPU: streamed codec decode (BASELINE config 5's chunked vocoder) against the one-shot decode.

The codec is causal end to end (causal convs, window-limited causal attention), so decoding a
stream of chunks with each causal reader's previous rows carried (fm_codec_decode_chunk) must
reproduce the one-shot decode of the concatenated codes.  Every output element is computed by the
same kernels with the same operands in the same order, so the bound is bit-for-bit equality.
"""
import json

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _codec(golden, prec, max_frames):
    from fishmi.codec import FishMICodec
    from fishmi.config import CodecConfig

    g = golden("codec_full.npz")
    cfg = CodecConfig.from_spec(json.loads(str(g["spec"])))
    return FishMICodec.synthetic(cfg, int(g["synth_seed"]), 0, prec, max_frames)


@pytest.mark.parametrize("prec", ["fp32", "bf16"])
def test_streamed_chunks_equal_one_shot(prec, golden):
    """300 frames (past the transformer's 128-frame window and every conv's receptive field)
    decoded as ragged chunks give the one-shot waveform; a reset starts an independent stream."""
    m = _codec(golden, prec, 320)
    rng = np.random.default_rng(9)
    C1, T = m.cfg.n_codebooks + 1, 300
    codes = np.zeros((C1, T), np.int32)
    codes[0] = rng.integers(0, m.cfg.semantic_codebook_size, T)
    codes[1:] = rng.integers(0, m.cfg.codebook_size, (C1 - 1, T))
    full = m.decode_codes(codes)
    for sizes in ((1, 7, 22, 22, 100, 148), (22,) * 13 + (14,), (300,)):
        m.stream_reset()
        pcm, t = [], 0
        for n in sizes:
            pcm.append(m.decode_chunk(np.ascontiguousarray(codes[:, t:t + n])))
            t += n
        assert t == T
        np.testing.assert_array_equal(np.concatenate(pcm), full)
    m.close()


def test_stream_rejects_oversized_chunk(golden):
    from fishmi.native import FishMIError

    m = _codec(golden, "bf16", 16)
    m.stream_reset()
    with pytest.raises(FishMIError):
        m.decode_chunk(np.zeros((m.cfg.n_codebooks + 1, 17), np.int32))
    m.close()


def test_interleaved_stream_contexts_equal_one_shot(golden):
    """Two stream contexts (fm_codec_stream_open) plus the handle's own stream, their chunks
    interleaved on one handle: each reproduces the one-shot decode of its own codes bit for bit
    (one context per streamed request in the TTS engine)."""
    m = _codec(golden, "bf16", 160)
    rng = np.random.default_rng(21)
    C1, T = m.cfg.n_codebooks + 1, 150
    streams = []
    for _ in range(3):
        c = np.zeros((C1, T), np.int32)
        c[0] = rng.integers(0, m.cfg.semantic_codebook_size, T)
        c[1:] = rng.integers(0, m.cfg.codebook_size, (C1 - 1, T))
        streams.append(c)
    full = [m.decode_codes(c) for c in streams]
    ctx = [m.open_stream(), m.open_stream(), None]
    m.stream_reset()
    pcm = [[], [], []]
    sizes = [(22,) * 6 + (18,), (7, 30, 50, 63), (1, 49, 50, 50)]
    pos = [0, 0, 0]
    step = 0
    while any(p < T for p in pos):
        for i in range(3):
            if step < len(sizes[i]):
                n = sizes[i][step]
                chunk = np.ascontiguousarray(streams[i][:, pos[i]:pos[i] + n])
                pcm[i].append(ctx[i].decode_chunk(chunk) if ctx[i] is not None else m.decode_chunk(chunk))
                pos[i] += n
        step += 1
    for i in range(3):
        np.testing.assert_array_equal(np.concatenate(pcm[i]), full[i])
    ctx[0].close()
    ctx[1].close()
    m.close()


def test_rewound_context_and_stream_vocoder_equal_one_shot(golden):
    """A rewound context (fm_codec_stream_rewind) starts from zero state like a fresh one, and
    scheduler.StreamVocoder -- chunks on its own host thread, contexts pooled and rewound between
    requests -- gives each request the one-shot waveform bit for bit, whatever the chunk size and
    however the requests' progress calls interleave."""
    from fishmi import scheduler as S

    m = _codec(golden, "bf16", 160)
    rng = np.random.default_rng(33)
    C1, T = m.cfg.n_codebooks + 2, 150  # a frame column: the main token, then the codec's rows
    streams = []
    for _ in range(4):
        c = np.zeros((C1, T + 1), np.int32)  # + the column serve() drops at the end
        c[0] = rng.integers(0, 1000, T + 1)
        c[1] = rng.integers(0, m.cfg.semantic_codebook_size, T + 1)
        c[2:] = rng.integers(0, m.cfg.codebook_size, (C1 - 2, T + 1))
        streams.append(c)
    full = [m.decode_codes(np.ascontiguousarray(c[1:, :T])) for c in streams]
    ctx = m.open_stream()
    ctx.decode_chunk(np.ascontiguousarray(streams[0][1:, :40]))
    ctx.rewind()
    np.testing.assert_array_equal(ctx.decode_chunk(np.ascontiguousarray(streams[1][1:, :T - 60])),
                                  full[1][: (T - 60) * m.frame_length])
    ctx.close()
    for chunk in (1, 32, 96):
        voc = S.StreamVocoder(m, chunk)
        for w0 in (0, 2):  # the second wave reuses the first wave's contexts
            wave = streams[w0:w0 + 2]
            reqs = [S.Request(i, np.zeros((C1, 1), np.int32), T, 0) for i in range(len(wave))]
            cols = [[] for _ in wave]
            for t in range(0, T + 1, 17):  # a tick: 17 new columns per live stream
                for i, c in enumerate(wave):
                    cols[i] += [c[:, j] for j in range(t, min(t + 17, T + 1))]
                    voc.progress(i, reqs[i], cols[i])
            for i, c in enumerate(wave):
                pcm = voc.finish(i, reqs[i], np.stack(cols[i], 1)[:, :-1])
                np.testing.assert_array_equal(pcm, full[w0 + i])
        assert len(voc.ctxs) == 2
        voc.close()
    m.close()
