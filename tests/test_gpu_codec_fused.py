"""GPU: the fused decoder ResidualUnit (resunit_kernel, fm_tune codec_fuse) against the two-launch
form (k7 conv_gemm2 + k1 conv_gemm2).

The fused kernel runs the same k-steps (tap-major, 32 channels each) through the same MFMA into
the same fp32 accumulators, and rounds h, y and both Snakes exactly as the two epilogues do, so
the bound is bit-for-bit equality of the waveform: one-shot at config-2 length (216 frames, the
reference's own codes), streamed in config 2's growing chunks (carried causal context through the
fused units' input prefix), and 300 random frames in ragged chunks.  Stages at 96 and 192
channels are fused; the 768 / 384 stages keep the two launches in both modes.
"""
import json

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _codec(golden, max_frames):
    from fishmi.codec import FishMICodec
    from fishmi.config import CodecConfig

    g = golden("codec_long.npz")
    cfg = CodecConfig.from_spec(json.loads(str(g["spec"])))
    return FishMICodec.synthetic(cfg, int(g["synth_seed"]), 0, "bf16", max_frames), g


def _both(m, f, knob="codec_fuse"):
    from fishmi import native

    native.tune(knob, 0)
    try:
        two = f()
    finally:
        native.tune(knob, 1)
    return f(), two


def _stream(m, codes, sizes):
    m.stream_reset()
    out, t = [], 0
    for n in sizes:
        out.append(m.decode_chunk(np.ascontiguousarray(codes[:, t:t + n])))
        t += n
    assert t == codes.shape[1]
    return np.concatenate(out)


def test_fused_equals_two_launch_one_shot(golden):
    m, g = _codec(golden, 216)
    codes = g["codes"][0]
    fused, two = _both(m, lambda: m.decode_codes(codes))
    assert fused.shape == (codes.shape[1] * 2048,)
    np.testing.assert_array_equal(fused, two)
    m.close()


def test_fused_equals_two_launch_streamed(golden):
    m, g = _codec(golden, 216)
    codes = g["codes"][0]
    fused, two = _both(m, lambda: _stream(m, codes, (1, 4, 16, 64, 131)))
    np.testing.assert_array_equal(fused, two)
    np.testing.assert_array_equal(fused, m.decode_codes(codes))
    m.close()


def test_fused_random_ragged(golden):
    m, _ = _codec(golden, 320)
    rng = np.random.default_rng(11)
    C1, T = m.cfg.n_codebooks + 1, 300
    codes = np.zeros((C1, T), np.int32)
    codes[0] = rng.integers(0, m.cfg.semantic_codebook_size, T)
    codes[1:] = rng.integers(0, m.cfg.codebook_size, (C1 - 1, T))
    fused, two = _both(m, lambda: _stream(m, codes, (3, 9, 22, 100, 166)))
    np.testing.assert_array_equal(fused, two)
    assert np.abs(fused).max() <= 1.0
    m.close()


def test_fused_encoder_units_equal_two_launch(golden):
    """The encoder's ResidualUnits (64 / 128 / 256 / 512 channels at codec_enc_full's widths) run
    the same fused kernel: z_enc and the codes bit-identical to the two-launch form, bf16."""
    from fishmi import native
    from fishmi.codec import FishMICodec
    from fishmi.config import CodecConfig

    g = golden("codec_enc_full.npz")
    spec = json.loads(str(g["spec"]))
    m = FishMICodec(CodecConfig.from_spec(spec), 0, "bf16", max_frames=16)
    m.enable_encoder(spec["encoder_dim"], [int(v) for v in g["enc_layers"]])
    m.synth(int(g["synth_seed"]))
    m.synth_encoder(int(g["synth_seed"]))
    m.finalize()

    def run():
        codes = m.encode_audio(g["audio"])
        return codes, m.debug_read(10, codes.shape[1])

    native.tune("resunit_enc", 0)
    try:
        c0, z0 = run()
    finally:
        native.tune("resunit_enc", 1)
    c1, z1 = run()
    np.testing.assert_array_equal(z1, z0)
    np.testing.assert_array_equal(c1, c0)
    m.close()


def test_feedforward_swiglu_gemm_equals_three_launches(golden):
    """The codec transformer's FeedForward (modded_dac.py:316-317) as one split-K GEMM over
    [W1 | W3] with the SwiGLU epilogue (fm_tune codec_swiglu) equals w1, w3 and silu_mul bit for
    bit, one-shot and streamed."""
    m, g = _codec(golden, 216)
    codes = g["codes"][0]
    fused, three = _both(m, lambda: m.decode_codes(codes), "codec_swiglu")
    np.testing.assert_array_equal(fused, three)
    fused, three = _both(m, lambda: _stream(m, codes, (1, 4, 16, 64, 131)), "codec_swiglu")
    np.testing.assert_array_equal(fused, three)
    m.close()


def test_rope_in_projection_epilogue_equals_rope_kernel(golden):
    """The codec transformer's RoPE applied in the wqkv split-K epilogue (fm_tune codec_rope)
    equals the separate rope_qk_kernel bit for bit, one-shot and streamed (absolute positions)."""
    m, g = _codec(golden, 216)
    codes = g["codes"][0]
    fused, two = _both(m, lambda: m.decode_codes(codes), "codec_rope")
    np.testing.assert_array_equal(fused, two)
    fused, two = _both(m, lambda: _stream(m, codes, (1, 4, 16, 64, 131)), "codec_rope")
    np.testing.assert_array_equal(fused, two)
    m.close()


def test_norm_in_residual_epilogue_equals_rmsnorm_kernel(golden):
    """The codec transformer's ffn_norm / next attention_norm / final norm computed in the wo and
    w2 split-K epilogues (fm_tune codec_norm), with rmsnorm_wave_kernel's sum order, equal the
    separate rmsnorm launches bit for bit, one-shot and streamed."""
    m, g = _codec(golden, 216)
    codes = g["codes"][0]
    fused, two = _both(m, lambda: m.decode_codes(codes), "codec_norm")
    np.testing.assert_array_equal(fused, two)
    fused, two = _both(m, lambda: _stream(m, codes, (1, 4, 16, 64, 131)), "codec_norm")
    np.testing.assert_array_equal(fused, two)
    m.close()


@pytest.mark.parametrize("cfg", [0, 2])
def test_fused_tile_variants_equal_two_launch(cfg, golden):
    """The non-default resunit tile variants (fm_tune resunit_cfg 0: BM 128 / 256 with 8 time tiles
    per wave; 2: BM 128 at both widths) are bit-identical to the two-launch form as well."""
    from fishmi import native

    m, g = _codec(golden, 216)
    codes = g["codes"][0]
    native.tune("resunit_cfg", cfg)
    try:
        fused, two = _both(m, lambda: m.decode_codes(codes))
    finally:
        native.tune("resunit_cfg", 1)
    np.testing.assert_array_equal(fused, two)
    m.close()


def test_fused_then_fallback_stages_equal_two_launch(golden):
    """decoder_dim 384: the 192- and 96-channel stages run fused, the 48- and 24-channel stages fall
    back to two launches after them (the fallback's k7 scratch must not alias the rotated
    activation buffers).  Fused == two-launch bit for bit, one-shot and streamed."""
    import dataclasses

    from fishmi.codec import FishMICodec
    from fishmi.config import CodecConfig

    g = golden("codec_long.npz")
    cfg = dataclasses.replace(CodecConfig.from_spec(json.loads(str(g["spec"]))), decoder_dim=384)
    m = FishMICodec.synthetic(cfg, int(g["synth_seed"]), 0, "bf16", 64)
    try:
        rng = np.random.default_rng(5)
        C1, T = m.cfg.n_codebooks + 1, 48
        codes = np.zeros((C1, T), np.int32)
        codes[0] = rng.integers(0, m.cfg.semantic_codebook_size, T)
        codes[1:] = rng.integers(0, m.cfg.codebook_size, (C1 - 1, T))
        fused, two = _both(m, lambda: m.decode_codes(codes))
        assert np.isfinite(fused).all()
        np.testing.assert_array_equal(fused, two)
        sf, st = _both(m, lambda: _stream(m, codes, (5, 11, 32)))
        np.testing.assert_array_equal(sf, st)
        np.testing.assert_array_equal(sf, fused)
    finally:
        m.close()
