"""Weight-only int4 (fm_llm_set_quant_int4; tools/llama/quantize.py WeightOnlyInt4QuantHandler,
llama.py:537-543) on the GPU.  The device quantizer is pinned bit-exact to the reference's own
group_quantize_tensor (tests/golden/int4_quant.npz).  The reference's packed matmul
(_weight_int4pack_mm) does not run on this CPU, so the matmul is parity-unpinned: it is held to the
same linear on the dequantised bf16 weights (every other kernel's operand) instead.  Run on the
MI355X box: pytest -m gpu."""
import numpy as np
import pytest

from parity_util import bits_to_f32

pytestmark = pytest.mark.gpu


def _bf16r(x):
    b = np.ascontiguousarray(x, np.float32).view(np.uint32)
    return ((b + 0x7FFF + ((b >> 16) & 1)) & 0xFFFF0000).astype(np.uint32).view(np.float32)


@pytest.mark.parametrize("gs", [32, 64, 128, 256])
def test_device_quantizer_matches_reference(golden, gs):
    """launch_quant4: codes, scales and zeros bit-exact with group_quantize_tensor; the dequantised
    weights are bf16 of group_dequantize_tensor's values."""
    from fishmi import ops

    g = golden("int4_quant.npz")
    w = bits_to_f32(g[f"w_bits_g{gs}"])
    q, sc, zr, wd = ops.quant4(w, gs)
    sz = bits_to_f32(g[f"sz_bits_g{gs}"])
    np.testing.assert_array_equal(q, g[f"q_g{gs}"])
    np.testing.assert_array_equal(sc, sz[..., 0].T)
    np.testing.assert_array_equal(zr, sz[..., 1].T)
    np.testing.assert_array_equal(wd, _bf16r(g[f"dq_g{gs}"]))


@pytest.mark.parametrize("R", [1, 4])
def test_q4_gemv_equals_dequantized_linear(R):
    """The streamed int4 GEMV (4-bit codes as bf16 128 + q, each group's affine map applied to the
    unit sums) against float64 x . ((q - 8) s + z)^T, and the bf16 GEMV on the dequantised bf16
    weights against float64 x . w_deq^T."""
    from fishmi import ops

    rng = np.random.default_rng(3)
    N, K = 1040, 2560
    w = _bf16r(rng.standard_normal((N, K)).astype(np.float32) * 0.03)
    x = _bf16r(rng.standard_normal((R, K)).astype(np.float32))
    q, sc, zr, wd, yb, y4 = ops.quant4(w, 128, x)
    ref = x.astype(np.float64) @ wd.astype(np.float64).T
    # the streamed form applies each group's affine map exactly: x . ((q - 8) s + z)
    ng = K // 128
    wx = ((q.astype(np.float64) - 8).reshape(N, ng, 128) * sc[..., None] + zr[..., None]).reshape(N, K)
    ref4 = x.astype(np.float64) @ wx.T
    # EPI_F32 rounds each output to bf16 (the head's round(x . w) as fp32): one bf16 ulp, plus the
    # fp32 summation slack (the 128 + q form cancels 136 s sum x: a few more bits)
    tol = lambda r: np.abs(r) * 2.0 ** -8 + 4e-6 * np.abs(r).max() * np.sqrt(K)  # noqa: E731
    assert (np.abs(yb - ref) <= tol(ref)).all()
    assert (np.abs(y4 - ref4) <= tol(ref4)).all()
    # the two weight forms (bf16-rounded vs exact dequantisation) agree to bf16 weight rounding
    assert np.sqrt(np.mean((y4 - yb) ** 2)) <= 4e-3 * np.sqrt(np.mean(yb ** 2))


@pytest.mark.parametrize("rowgemv", [31, 0, 3])
def test_int4_model_stream_matches_dequantized_model(golden, rowgemv):
    """S2-Pro widths (llm_wide: 2 slow + 1 fast layers), int4 with group size 128, teacher-forced
    frames through the production decode graph: the streamed 4-bit GEMVs (fm_tune int4_stream 1;
    wo / w2 / wqkv / w1 || w3 on the int4 row-block GEMV, fm_rowgemv.hip QM 2, with rowgemv_q4 31 (also the
    first layers' wqkv and the codebook head), the default, w1 || w3 on the tiles with 3, all on the
    16-row tiles with 0) against the same model on its dequantised bf16 weights
    (int4_stream 0) -- logits equal up to
    the rounding of the dequantised weights (the streamed form applies the affine map exactly, the
    copy holds it rounded to bf16); and the int4 model tracks the bf16 model (quantization error only)."""
    from fishmi import native
    from fishmi.config import DualARConfig
    from fishmi.llm import DualARModel

    import os

    from conftest import GOLDEN

    g = golden("llm_wide_bf16.npz")
    cfg = DualARConfig.from_pretrained(os.path.join(GOLDEN, "llm_wide"))
    cfg.im_end_id = 4
    T = g["prompt"].shape[1]
    cols = g["seq"][:, T:T + 5]
    m = DualARModel.synthetic(cfg, int(g["synth_seed"]), int(g["log2_half"]), 0, "bf16", 1, quant="int4",
                              groupsize=128)
    out = {}
    native.tune("rowgemv_q4", rowgemv)
    try:
        for st in (1, 0):
            native.tune("int4_stream", st)
            m.use_graph(True)
            out[st] = m.teacher_decode(g["prompt"], cols)
    finally:
        native.tune("int4_stream", 1)
        native.tune("rowgemv_q4", 31)
        m.close()
    mb = DualARModel.synthetic(cfg, int(g["synth_seed"]), int(g["log2_half"]), 0, "bf16", 1)
    try:
        sb, fb = mb.teacher_decode(g["prompt"], cols)
    finally:
        mb.close()
    rows = g["slow_rows"]
    for k in (0, 1):  # slow, fast
        a, b = out[1][k], out[0][k]
        if k == 0:
            a, b = a[:, rows], b[:, rows]
        fin = np.isfinite(b)
        rel = np.sqrt(np.mean((a[fin] - b[fin]) ** 2)) / np.sqrt(np.mean(b[fin] ** 2))
        assert rel < 2e-2, (k, rel)  # (exact vs bf16-rounded dequantised weights)
        assert np.array_equal(np.isfinite(a), fin)
    # against the bf16 model: correlated, not equal (the int4 quantisation error)
    f4, fbf = out[1][1].ravel(), fb.ravel()
    assert np.corrcoef(f4, fbf)[0, 1] > 0.8
