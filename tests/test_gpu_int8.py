"""Weight-only int8 decode linears, opt-in: parity against the reference's own
int8 model -- tools/llama/quantize.py WeightOnlyInt8QuantHandler + WeightOnlyInt8Linear, run by
oracle/gen_goldens.py (llm_int8, llm_wide_int8).  Run on the MI355X box: pytest -m gpu."""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN
from test_gpu_llm import IM_END, _bf16_vs_reference, _cfg

pytestmark = pytest.mark.gpu


def _qmodel(prec, max_slots=1):
    from fishmi.llm import DualARModel

    m = DualARModel.from_pretrained(os.path.join(GOLDEN, "llm_q_int8"), 0, prec, max_slots, im_end_id=IM_END)
    assert m.quant == "int8"
    return m


def test_int8_checkpoint_fp32_greedy_tokens_exact(golden):
    """The int8 checkpoint quantize.py writes (model.pth: int8 weights + bf16 scales, biases unused),
    fp32 validation mode: free-running greedy tokens == the reference int8 model's."""
    g = golden("llm_q_int8_fp32.npz")
    m = _qmodel("fp32")
    T = g["prompt"].shape[1]
    ref = g["seq"][:, T:]
    np.testing.assert_array_equal(m.generate(g["prompt"], ref.shape[1], top_k=1), ref)


def test_int8_fp32_production_decode_logits(golden):
    """fp32 mode, production decode path (int8 gemv_kernel stream + prefill on linear_kernel with
    the scale epilogue), teacher-forced: logits within 1e-4 of the reference int8 model's."""
    g = golden("llm_q_int8_fp32.npz")
    m = _qmodel("fp32")
    T = g["prompt"].shape[1]
    slow, fast = m.teacher_decode(g["prompt"], g["seq"][:, T:])
    fin = np.isfinite(g["slow_logits"])
    assert np.array_equal(np.isfinite(slow), fin)
    np.testing.assert_allclose(slow[fin], g["slow_logits"][fin], atol=1e-4, rtol=0)
    np.testing.assert_allclose(fast, g["fast_logits"], atol=1e-4, rtol=0)


def test_int8_bf16_production_decode_vs_reference(golden):
    """bf16 int8 production path vs the reference int8 model: within BF16_RATIO x the reference's
    own bf16-vs-fp32 error (round(round(acc) * scale) in both)."""
    g = golden("llm_q_int8_bf16.npz")
    m = _qmodel("bf16")
    T = g["prompt"].shape[1]
    slow, fast = m.teacher_decode(g["prompt"], g["seq"][:, T:])
    st = _bf16_vs_reference(slow, fast, g)
    assert st["top1_checked"] > 20


def test_int8_quantized_on_device_equals_checkpoint(golden):
    """The same synthetic bf16 weights quantized by finalize (quant_rows_kernel) instead of loaded
    from quantize.py's state_dict: identical greedy tokens (the per-channel rule, bf16 scales)."""
    from fishmi.llm import DualARModel

    g = golden("llm_q_int8_fp32.npz")
    cfg = _cfg("llm_q_int8")
    m = DualARModel.synthetic(cfg, 29, 3, 0, "fp32", 1, quant="int8")
    T = g["prompt"].shape[1]
    ref = g["seq"][:, T:]
    np.testing.assert_array_equal(m.generate(g["prompt"], ref.shape[1], top_k=1), ref)


@pytest.mark.parametrize("bstream", [1, 0])
@pytest.mark.parametrize("n", [4, 12, 20])
def test_int8_batched_slots_match_single(n, bstream, golden):
    """int8 at B <= 8 (gemv_kernel int8 stream), 8 < B <= 32 on bstream_kernel (scales in the
    epilogues and in finalize_norm) or linear_kernel: every slot's stream == its batch-1 stream, and
    slot 0 (the golden prompt) == the reference int8 model's (fp32 mode)."""
    from fishmi import native
    from fishmi.llm import DualARModel

    g = golden("llm_q_int8_fp32.npz")
    m = _qmodel("fp32", max_slots=n)
    cfg = m.cfg
    rng = np.random.default_rng(5)
    prompts = []
    for s in range(n):
        p = g["prompt"].copy()
        if s:
            p[0, 1:5] = rng.integers(16, cfg.semantic_begin_id, 4)
        prompts.append(p)
    n_new = 10
    native.tune("bstream", bstream)
    try:
        single = [m.generate(p, n_new, top_k=1, slot=s, mask_im_end=True) for s, p in enumerate(prompts)]
        sp = DualARModel.sampling(top_k=1, mask_im_end=True)
        firsts = [m.prefill(s, p, sp) for s, p in enumerate(prompts)]
        fr = m.decode_frames(list(range(n)), n_new - 1)
    finally:
        native.tune("bstream", 1)
    T = g["prompt"].shape[1]
    np.testing.assert_array_equal(single[0], g["seq"][:, T:T + n_new])
    for s in range(n):
        got = np.concatenate([firsts[s][:, None], fr[:, s, :].T], axis=1)
        np.testing.assert_array_equal(got, single[s])


@pytest.mark.parametrize("rowgemv", [27, 0, 7])
def test_int8_wide_real_widths_vs_reference(golden, rowgemv):
    """S2-Pro widths (d=2560, I=9728, 32/8x128 heads, V=155776, cb=4096) at reduced depth, int8 from
    the synthetic bf16 weights quantized on the device, bf16 production decode path teacher-forced
    with the reference int8 model's columns: within BF16_RATIO x its own bf16 error -- with wo / w2
    on the int8 row-block GEMV (fm_rowgemv.hip QM 1, the default) and on the 16-row tiles."""
    from fishmi import native
    from fishmi.llm import DualARModel

    native.tune("rowgemv", rowgemv)
    try:
        _int8_wide(golden)
    finally:
        native.tune("rowgemv", 27)


def _int8_wide(golden):
    from fishmi.llm import DualARModel

    path = os.path.join(GOLDEN, "llm_wide_int8_bf16.npz")
    if not os.path.exists(path):
        pytest.skip("llm_wide_int8_bf16.npz not generated")
    g = golden("llm_wide_int8_bf16.npz")
    cfg = _cfg("llm_wide")
    m = DualARModel.synthetic(cfg, int(g["synth_seed"]), int(g["log2_half"]), 0, "bf16", 1, quant="int8")
    T = g["prompt"].shape[1]
    slow, fast = m.teacher_decode(g["prompt"], g["seq"][:, T:])
    _bf16_vs_reference(slow, fast, g, rows=g["slow_rows"])
    assert len(json.loads(str(g["qsums"]))) > 0
    m.close()
