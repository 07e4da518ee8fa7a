"""GPU parity of the modded-DAC decode path (DAC.from_indices) against reference goldens.

Tolerances (waveform in [-1, 1] after tanh):
  * fp32 mode vs the reference fp32 waveform: max |err| <= 2e-3 (tiny) / RMS <= 1e-3 * signal
    RMS (full shapes) -- accumulation order only;
  * bf16 mode vs the reference fp32 waveform: RMS error <= 1.5x the reference's OWN bf16-vs-fp32
    RMS error on the same codes (the bound the reference itself meets in bf16).
"""
import json

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _codec(name, golden, prec, max_frames=64):
    from fishmi.codec import FishMICodec
    from fishmi.config import CodecConfig

    g = golden(f"{name}.npz")
    cfg = CodecConfig.from_spec(json.loads(str(g["spec"])))
    return FishMICodec.synthetic(cfg, int(g["synth_seed"]), 0, prec, max_frames), g


def _rms(x):
    return float(np.sqrt(np.mean(np.square(x, dtype=np.float64))))


@pytest.mark.parametrize("name", ["codec_tiny", "codec_full"])
def test_fp32_matches_reference(name, golden):
    m, g = _codec(name, golden, "fp32")
    codes = g["codes"][0]
    wave = m.decode_codes(codes)
    ref = g["wave_fp32"].reshape(-1)
    assert wave.shape == ref.shape
    if name == "codec_tiny":
        assert np.abs(wave - ref).max() < 2e-3
    assert _rms(wave - ref) <= 1e-3 * _rms(ref)


@pytest.mark.parametrize("name", ["codec_tiny", "codec_full"])
def test_bf16_within_reference_bf16_error(name, golden):
    m, g = _codec(name, golden, "bf16")
    wave = m.decode_codes(g["codes"][0])
    ref = g["wave_fp32"].reshape(-1)
    ref_bf16_err = _rms(g["wave_bf16"].reshape(-1) - ref)
    assert _rms(wave - ref) <= 1.5 * ref_bf16_err + 1e-4, (_rms(wave - ref), ref_bf16_err)
    assert np.abs(wave).max() <= 1.0


def test_causal_prefix_property(golden):
    """rvq.py:374-398-style known answer: the decode is causal end to end, so decoding a prefix
    of the codes reproduces the prefix of the full decode (the basis of streaming)."""
    m, g = _codec("codec_tiny", golden, "fp32")
    codes = g["codes"][0]
    full = m.decode_codes(codes)
    for h in (1, 5, int(g["prefix_T"])):
        pre = m.decode_codes(np.ascontiguousarray(codes[:, :h]))
        assert np.abs(pre - full[: pre.size]).max() < 1e-4


def test_from_indices_batch_and_no_mutation(golden):
    m, g = _codec("codec_tiny", golden, "fp32")
    idx = np.stack([g["codes"][0], g["codes"][0]])
    before = idx.copy()
    out = m.from_indices(idx)
    assert out.shape == (2, 1, idx.shape[-1] * 2048)
    np.testing.assert_array_equal(idx, before)  # the reference clamps in place; we do not
    np.testing.assert_allclose(out[0], out[1])


def test_intermediate_latents_match_oracle(golden):
    """Localises codec errors: the post-transformer latent and the decoder-input latent (after
    both ConvNeXt upsample stages) agree with the C oracle in fp32 (1e-4 relative)."""
    import ctypes

    import oracle as O
    from fishmi.config import CodecConfig

    m, g = _codec("codec_full", golden, "fp32")
    cfg = CodecConfig.from_spec(json.loads(str(g["spec"])))
    codes = g["codes"][0]
    T = codes.shape[1]
    o = O.OracleCodec(cfg)
    o.synth(int(g["synth_seed"]))
    post = np.zeros((cfg.latent, T), np.float32)
    rvq = np.zeros_like(post)
    O.lib().orc_codec_debug_taps.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    O.lib().orc_codec_debug_taps(rvq.ctypes.data, post.ctypes.data)  # filled by the next decode
    wave_o, lat = o.decode(codes, want_latent=True)
    O.lib().orc_codec_debug_taps(None, None)
    wave = m.decode_codes(codes)
    for stage, ref in ((1, post.T), (3, lat.T)):
        x = m.debug_read(stage, T)
        assert np.abs(x - ref).max() <= 1e-4 * np.abs(ref).max(), stage
    assert np.abs(wave - wave_o).max() < 5e-3


def _segments(g, wave):
    """The fixture keeps frames [0, head) and the last `tail` frames of the 216-frame waveform."""
    head, tail = int(g["head_frames"]), int(g["tail_frames"])
    T = g["codes"].shape[-1]
    w = wave.reshape(-1)
    return np.concatenate([w[: head * 2048], w[(T - tail) * 2048:]]), head * 2048


def test_long_fp32_matches_reference(golden):
    """Config-2 length (216 frames): the post transformer's 128-frame causal window
    (modded_dac.py:380-398) is crossed, so the window mask is checked against the reference."""
    m, g = _codec("codec_long", golden, "fp32", max_frames=216)
    got, _ = _segments(g, m.decode_codes(g["codes"][0]))
    ref = g["wave_fp32"]
    assert _rms(got - ref) <= 1e-3 * _rms(ref), (_rms(got - ref), _rms(ref))
    m.close()


@pytest.mark.parametrize("mode", ["one_shot", "streamed"])
def test_long_bf16_within_reference_bf16_error(mode, golden):
    """bf16 over 216 frames vs the reference fp32 waveform. Bounds are 1.5x the reference's own
    bf16 error in both of its bf16 modes: the CLI's dac.to(bf16) (inference.py:416) and the engine's
    autocast over fp32 weights (vq_manager.py:16-21). Two measures are used: RMS error, and the
    multi-resolution STFT log-magnitude error in dB (oracle/signals.py). The
    streamed decode uses 22-frame chunks, as config 5's vocoder does."""
    import signals

    m, g = _codec("codec_long", golden, "bf16", max_frames=216)
    codes = g["codes"][0]
    if mode == "one_shot":
        wave = m.decode_codes(codes)
    else:
        m.stream_reset()
        wave = np.concatenate([m.decode_chunk(np.ascontiguousarray(codes[:, t:t + 22]))
                               for t in range(0, codes.shape[1], 22)])
    got, head = _segments(g, wave)
    ref = g["wave_fp32"]
    err = _rms(got - ref)
    db = signals.stft_logmag_error_db(got[head:], ref[head:])
    for k in ("wave_bf16", "wave_autocast"):
        assert err <= 1.5 * float(g[k + "_rms_err"]), (k, err, float(g[k + "_rms_err"]))
        assert db <= 1.5 * float(g[k + "_stft_db"]), (k, db, float(g[k + "_stft_db"]))
    assert np.abs(wave).max() <= 1.0
    m.close()
