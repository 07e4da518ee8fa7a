"""Weight-only int4 quantizer restatement (oracle/oracle.py int4_group_quantize) against the
reference's own group_quantize_tensor / group_dequantize_tensor (tools/llama/quantize.py:57-160)
run on seeded bf16 matrices (tests/golden/int4_quant.npz, oracle/gen_goldens.py int4_quant): codes,
scales and zeros bit-exact, every group size the reference's handler accepts.  The packed matmul
(_weight_int4pack_mm) does not run on this CPU: the int4 path is parity-unpinned at that level."""
import numpy as np
import pytest


@pytest.mark.parametrize("gs", [32, 64, 128, 256])
def test_int4_restatement_matches_reference(golden, gs):
    import oracle as O
    from parity_util import bits_to_f32

    g = golden("int4_quant.npz")
    w = bits_to_f32(g[f"w_bits_g{gs}"])
    q, sc, zr, dq = O.int4_group_quantize(w, gs)
    ref_sz = bits_to_f32(g[f"sz_bits_g{gs}"])  # [K/gs][N][2]
    np.testing.assert_array_equal(q, g[f"q_g{gs}"])
    np.testing.assert_array_equal(sc, ref_sz[..., 0].T)
    np.testing.assert_array_equal(zr, ref_sz[..., 1].T)
    np.testing.assert_array_equal(dq, g[f"dq_g{gs}"])
    # the clamp row (constant weights) and the reconstruction bound of the affine form
    assert np.all(sc[1] == O._bf16r(O._bf16r(np.float32(1e-6)) / np.float32(15)))
    err = np.abs(dq - w).reshape(w.shape[0], -1, gs).max(-1)
    err[1] = 0  # the constant row reconstructs to zero - 8 * scale (the reference's own result)
    assert (err <= 1.5 * sc + 1e-7).all()  # (bf16 rounding of zero and of the scaled offsets)
