"""Every alternate kernel path behind an fm_tune knob (fm_kernels.h FmTuning) under the same parity
bar as the default path it replaces: the batch-1 decode variants against the reference's fp32
logits (1e-4) and, at S2-Pro widths in bf16, within BF16_RATIO x the reference's own bf16 error;
the prompt-chunk variants (row attention / linear_kernel instead of attn_prefill_kernel / the
LDS-tiled GEMM) likewise; the codec's conv_gemm_kernel and whole-K paths against the reference
waveform.  The batched-decode knobs are covered in test_gpu_llm.py
(test_batched_wide_split_k_matches_single)."""
import json

import numpy as np
import pytest

from test_gpu_llm import _bf16_vs_reference, _cfg, _model

pytestmark = pytest.mark.gpu

# FmTuning's defaults (fm_kernels.h), restored after every test
DEFAULTS = {"attn3": 1, "attn_fd": 1, "fd_min": 32, "fd_nw": 8, "fd_min16": 256, "gemv_chain": 0, "gemv_nt": 1, "gemv_u": 8, "gemv_wpb": 4,
            "ksb_balance": 0, "ksb_blocks": 512, "attn_cap": 32, "prefill_attn": 1, "prompt_gemm": 1,
            "conv2": 1, "conv_splitk": 1, "kv_prefetch": 1, "fin_ksb": 0, "gemv_dummy": 2, "rowgemv": 27, "rowgemv_q4": 31, "sampler_kth": 1, "row_qkv_rp": 8,
            "fattn_wo": 1, "fw_cheap": 0, "fw_delay": 0, "prompt_skinny": 1, "prompt_skinny_blocks": 256, "prompt_swiglu": 1, "prompt_fin": 1, "prompt_qkv_slab": 1, "prompt_unroll": 1}

DECODE_KNOBS = [{"attn3": 0}, {"attn3": 0, "attn_fd": 0}, {"fd_nw": 4}, {"fd_nw": 4, "fd_min": 16}, {"fd_nw": 16},
                {"fd_min16": 16}, {"fd_nw": 16, "fd_min16": 16}, {"gemv_chain": 1}, {"gemv_nt": 0}, {"gemv_u": 4},
                {"gemv_u": 2}, {"gemv_wpb": 8}, {"ksb_balance": 1}, {"ksb_blocks": 64}, {"attn_cap": 0},
                {"kv_prefetch": 0}, {"fin_ksb": 4}, {"gemv_dummy": 0}, {"gemv_dummy": 1}, {"rowgemv": 0},
                {"rowgemv": 1}, {"rowgemv": 2}, {"rowgemv": 3}, {"rowgemv": 7}, {"rowgemv": 31}, {"fattn_wo": 0}, {"fw_cheap": 1}, {"fw_delay": 100},
                {"rowgemv": 0, "fin_ksb": 4}, {"rowgemv": 0, "gemv_u": 4}, {"sampler_kth": 0},
                {"row_qkv_rp": 4}, {"row_qkv_rp": 16}]


@pytest.fixture
def tune():
    from fishmi import native

    touched = []

    def put(knobs):
        for k, v in knobs.items():
            touched.append(k)
            native.tune(k, v)

    yield put
    for k in touched:
        native.tune(k, DEFAULTS[k])


def _ids(knobs):
    return ",".join(f"{k}={v}" for k, v in knobs.items())


@pytest.mark.parametrize("knobs", DECODE_KNOBS, ids=_ids)
def test_fp32_decode_variants(knobs, golden, tune):
    tune(knobs)
    m, g, cfg = _model("llm_a", "fp32", golden)
    T = g["prompt"].shape[1]
    slow, fast = m.teacher_decode(g["prompt"], g["seq"][:, T:])
    ref = g["slow_logits"]
    fin = np.isfinite(ref)
    assert np.array_equal(np.isfinite(slow), fin)
    np.testing.assert_allclose(slow[fin], ref[fin], atol=1e-4, rtol=0)
    np.testing.assert_allclose(fast, g["fast_logits"], atol=1e-4, rtol=0)


@pytest.mark.parametrize("knobs", DECODE_KNOBS + [{"prefill_attn": 0}, {"prompt_gemm": 0}, {"prompt_skinny": 0},
                                                  {"prompt_skinny_blocks": 1}, {"prompt_skinny_blocks": 4096},
                                                  {"prompt_swiglu": 0}, {"prompt_fin": 0}, {"prompt_qkv_slab": 0}],
                         ids=_ids)
def test_wide_bf16_variants_vs_reference(knobs, golden, tune):
    from fishmi.llm import DualARModel

    tune(knobs)
    g = golden("llm_wide_bf16.npz")
    cfg = _cfg("llm_wide")
    m = DualARModel.synthetic(cfg, int(g["synth_seed"]), int(g["log2_half"]), 0, "bf16", 1)
    T = g["prompt"].shape[1]
    slow, fast = m.teacher_decode(g["prompt"], g["seq"][:, T:])
    _bf16_vs_reference(slow, fast, g, rows=g["slow_rows"])
    m.close()


@pytest.mark.parametrize("knobs", [{"conv2": 0}, {"conv_splitk": 0}, {"conv2": 0, "conv_splitk": 0}], ids=_ids)
@pytest.mark.parametrize("prec", ["fp32", "bf16"])
def test_codec_variants_vs_reference(prec, knobs, golden, tune):
    from fishmi.codec import FishMICodec
    from fishmi.config import CodecConfig

    tune(knobs)
    g = golden("codec_full.npz")
    cfg = CodecConfig.from_spec(json.loads(str(g["spec"])))
    m = FishMICodec.synthetic(cfg, int(g["synth_seed"]), 0, prec, 64)
    wave = m.decode_codes(g["codes"][0])
    ref = g["wave_fp32"].reshape(-1)
    rms = lambda x: float(np.sqrt(np.mean(np.square(x, dtype=np.float64))))
    assert wave.shape == ref.shape
    if prec == "fp32":
        assert rms(wave - ref) <= 1e-3 * rms(ref)
    else:
        ref_bf16_err = rms(g["wave_bf16"].reshape(-1) - ref)
        assert rms(wave - ref) <= 1.5 * ref_bf16_err + 1e-4, (rms(wave - ref), ref_bf16_err)


@pytest.mark.parametrize("knob,blocks", [("prompt_swiglu", 1), ("prompt_swiglu", 4096), ("prompt_qkv_slab", 256),
                                          ("prompt_qkv_slab", 4096), ("prompt_unroll", 256), ("prompt_unroll", 1)])
def test_prompt_fusions_bit_identical(golden, tune, knob, blocks):
    """The skinny prompt GEMM's fused epilogues give the teacher-forced logits of the unfused launches
    bit for bit (the same roundings on the same sums): w1 || w3 with the interleaved SwiGLU -- stored
    by the kernel itself when unsliced (blocks 1), in the split-K epilogue (CE_SWIGLU8) when sliced --
    against the stored output + swiglu_i8_kernel; the QKV slices summed + biased + rounded by
    qk_rope_cache_kernel against the split-K epilogue's stored projection."""
    from fishmi.llm import DualARModel

    g = golden("llm_wide_bf16.npz")
    cfg = _cfg("llm_wide")
    out = []
    for v in (1, 0):
        tune({knob: v, "prompt_skinny_blocks": blocks})
        m = DualARModel.synthetic(cfg, int(g["synth_seed"]), int(g["log2_half"]), 0, "bf16", 1)
        T = g["prompt"].shape[1]
        out.append(m.teacher_decode(g["prompt"], g["seq"][:, T:]))
        m.close()
    np.testing.assert_array_equal(out[0][0], out[1][0])
    np.testing.assert_array_equal(out[0][1], out[1][1])
