"""Batch-1 GEMV chain (fm_tune gemv_chain; fm_gemv.hip gemv_chain_kernel): a layer's wo -> w1||w3 ->
w2 -> next layer's qkv as one launch with in-launch hand-offs.  The chain changes scheduling only --
every stage runs the same GEMV body, in the same summation order -- so its outputs must be
BIT-identical to the one-launch-per-GEMV path, frame after frame, across graph replays of several
utterances on one model, and within the parity bound against the reference's logits.  The
llama.py references are the same as the decode tests' (test_gpu_00_timed_configs.py)."""
import json

import numpy as np
import pytest

from parity_util import bf16_vs_golden

pytestmark = pytest.mark.gpu

IM_END = 4


def _cfg(g):
    from fishmi.config import DualARConfig

    cfg = DualARConfig._from_fish_qwen3_omni(json.loads(str(g["config"])))
    cfg.im_end_id = IM_END
    return cfg


@pytest.fixture
def chain():
    """gemv_chain on / off against the 16-row tile launch chain it replaces: the row-block GEMVs
    (rowgemv) and the fused fast attention + wo (fattn_wo) are off in both runs."""
    from fishmi import native

    def put(on):
        native.tune("gemv_chain", int(on))

    native.tune("rowgemv", 0)
    native.tune("fattn_wo", 0)
    yield put
    native.tune("gemv_chain", 0)
    native.tune("rowgemv", 27)
    native.tune("fattn_wo", 1)


def _prompt(cfg, T, seed):
    rng = np.random.default_rng(seed)
    p = np.zeros((cfg.num_codebooks + 1, T), np.int32)
    p[0] = rng.integers(16, cfg.semantic_begin_id, T)
    return p


@pytest.mark.parametrize("precision", ["bf16", "fp32"])
def test_chain_bit_identical_to_launch_chain(precision, golden, chain):
    """S2-Pro widths (2 slow + 1 fast layers): three sampled utterances (graph-replayed frames) with
    the chain equal the unchained run token for token and logit for logit."""
    from fishmi.llm import DualARModel

    g = golden("llm_ragged_bf16.npz")
    cfg = _cfg(g)
    cfg.max_seq_len = 256
    m = DualARModel.synthetic(cfg, int(g["synth_seed"]), int(g["log2_half"]), 0, precision, 1)
    try:
        runs = {}
        for on in (0, 1):
            chain(on)
            m.use_graph(True)  # re-capture the frame graph under the knob
            out = []
            for u in range(3):  # utterances: the second and third replay the captured graph
                cols = m.generate(_prompt(cfg, 40 + 7 * u, 10 + u), 24, top_k=30, seed=100 + u, mask_im_end=True)
                out.append((cols, *m.read_logits(0)))
            runs[on] = out
        for u in range(3):
            a, b = runs[0][u], runs[1][u]
            np.testing.assert_array_equal(a[0], b[0], err_msg=f"utterance {u}: tokens")
            np.testing.assert_array_equal(a[1], b[1], err_msg=f"utterance {u}: slow logits")
            np.testing.assert_array_equal(a[2], b[2], err_msg=f"utterance {u}: fast logits")
    finally:
        m.close()


def test_chain_full_depth_bf16_vs_reference(golden, chain):
    """36 + 4 layers through the production decode graph with the chain, twice on one model (the
    second pass replays the captured graph): within the bf16 bound of the reference, and equal."""
    from fishmi.llm import DualARModel

    chain(1)
    g = golden("llm_full_bf16.npz")
    cfg = _cfg(g)
    m = DualARModel.synthetic(cfg, int(g["synth_seed"]), int(g["log2_half"]), 0, "bf16", 1)
    try:
        T = g["prompt"].shape[1]
        s1, f1 = m.teacher_decode(g["prompt"], g["seq"][:, T:])
        s2, f2 = m.teacher_decode(g["prompt"], g["seq"][:, T:])
    finally:
        m.close()
    np.testing.assert_array_equal(s1, s2)
    np.testing.assert_array_equal(f1, f2)
    st = bf16_vs_golden(s1, f1, g, rows=g["slow_rows"])
    assert st["top1_checked"] >= 9
