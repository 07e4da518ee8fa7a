"""The persistent fast pass (fm_pass.hip, fm_tune pass_fast 1: one launch per batch-1 fast-model
pass, LDS-DMA loader ring + consumer waves + granule exchange) against the reference goldens, the
same bound as the launch-per-op path (tests/parity_util.py).  Opt-in (slower than the launch path on
MI355X), kept under these tests.  Run on the MI355X box: pytest -m gpu."""
import json

import numpy as np
import pytest

from parity_util import bf16_vs_golden

pytestmark = pytest.mark.gpu

IM_END = 4


@pytest.fixture
def pass_on():
    from fishmi import native

    native.tune("pass_fast", 1)
    yield
    native.tune("pass_fast", 0)


def _cfg(g):
    from fishmi.config import DualARConfig

    cfg = DualARConfig._from_fish_qwen3_omni(json.loads(str(g["config"])))
    cfg.im_end_id = IM_END
    return cfg


@pytest.mark.parametrize("ring", [0, 1, 4, 5, 6, 7])
def test_pass_full_depth_bf16_vs_reference(golden, pass_on, ring):
    """Config 2 at full depth (4 fast layers per pass, 10 passes per frame), graph-replayed frames,
    every ring configuration (fm_tune pass_cfg): within the bf16 bound of the reference."""
    from fishmi import native
    from fishmi.llm import DualARModel

    native.tune("pass_cfg", ring)
    g = golden("llm_full_bf16.npz")
    m = DualARModel.synthetic(_cfg(g), int(g["synth_seed"]), int(g["log2_half"]), 0, "bf16", 1)
    try:
        T = g["prompt"].shape[1]
        slow, fast = m.teacher_decode(g["prompt"], g["seq"][:, T:])
    finally:
        native.tune("pass_cfg", 0)
        m.close()
    st = bf16_vs_golden(slow, fast, g, rows=g["slow_rows"])
    assert st["top1_checked"] >= 9


def test_pass_matches_launch_path_and_replays(golden, pass_on):
    """The same frames with the persistent pass and with one launch per op: fast logits agree to
    bf16 rounding-order level (relative RMS < 2e-2, argmax equal where the margin is clear), and a
    graph replay of the captured frame gives the eager frame's logits bit for bit."""
    from fishmi import native
    from fishmi.llm import DualARModel

    import os

    from conftest import GOLDEN
    from fishmi.config import DualARConfig

    g = golden("llm_wide_bf16.npz")
    cfg = DualARConfig.from_pretrained(os.path.join(GOLDEN, "llm_wide"))
    cfg.im_end_id = IM_END
    m = DualARModel.synthetic(cfg, int(g["synth_seed"]), int(g["log2_half"]), 0, "bf16", 2)
    T = g["prompt"].shape[1]
    cols = g["seq"][:, T:T + 6]
    sp = DualARModel.sampling(top_k=1)
    try:
        out = {}
        for slot, on, graph in ((0, 0, True), (1, 1, True)):
            native.tune("pass_fast", on)
            m.use_graph(graph)
            fl = []
            for k in range(cols.shape[1]):
                m.force(slot, cols[:, k])
                if k == 0:
                    m.prefill(slot, g["prompt"], sp)
                else:
                    m.decode([slot])
                fl.append(m.read_logits(slot)[1])
            out[on] = np.stack(fl)
        a, b = out[0], out[1]
        rel = np.sqrt(np.mean((a - b) ** 2)) / np.sqrt(np.mean(a ** 2))
        assert rel < 2e-2, rel
        srt = np.sort(a, axis=-1)
        clear = (srt[..., -1] - srt[..., -2]) > 0.1
        assert np.array_equal(np.argmax(a, -1)[clear], np.argmax(b, -1)[clear])
        # eager vs graph replay of the persistent pass: bit-identical
        native.tune("pass_fast", 1)
        res = {}
        for graph in (False, True):
            m.use_graph(graph)
            m.force(0, cols[:, 0])
            m.prefill(0, g["prompt"], sp)
            m.force(0, cols[:, 1])
            m.decode([0])
            res[graph] = m.read_logits(0)[1]
        np.testing.assert_array_equal(res[False], res[True])
    finally:
        for s in (0, 1):
            m.force(s, None)
        m.use_graph(True)
        m.close()
