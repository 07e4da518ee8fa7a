"""GPU parity of the Dual-AR decode path (libfishmi, called through the C ABI) against the
reference goldens and the CPU oracle.  Run on the MI355X box: pytest -m gpu."""
import os

import numpy as np
import pytest

from conftest import GOLDEN
from parity_util import bf16_vs_golden

pytestmark = pytest.mark.gpu

IM_END = 4


def _cfg(name):
    from fishmi.config import DualARConfig

    cfg = DualARConfig.from_pretrained(os.path.join(GOLDEN, name))
    cfg.im_end_id = IM_END
    return cfg


def _model(name, tag, golden, max_slots=1):
    from fishmi.checkpoint import load_llm_weights
    from fishmi.llm import DualARModel

    g = golden(f"{name}_{tag}.npz")
    cfg = _cfg(name)
    prec = "bf16" if tag == "bf16" else "fp32"
    m = DualARModel(cfg, 0, prec, max_slots)
    if name == "llm_a":
        m.load_weights(load_llm_weights(os.path.join(GOLDEN, name)))
    else:
        m.synth(int(g["synth_seed"]), int(g["log2_half"]))
    m.finalize()
    return m, g, cfg


@pytest.mark.parametrize("name", ["llm_a", "llm_b"])
def test_fp32_greedy_tokens_exact(name, golden):
    """fp32 validation mode of the same kernels: free-running greedy == reference tokens."""
    m, g, _ = _model(name, "fp32", golden)
    T = g["prompt"].shape[1]
    ref = g["seq"][:, T:]
    out = m.generate(g["prompt"], ref.shape[1], top_k=1)
    np.testing.assert_array_equal(out, ref)


def _reference_loop(op, prompt, max_new, cfg, top_k):
    """generate() + decode_n_tokens() control flow (inference.py:241-359, 184-238) around an
    injected decode_one_token operator, as the reference drives it."""
    import torch

    C1 = cfg.num_codebooks + 1
    T = prompt.shape[1]
    x = torch.from_numpy(prompt.astype(np.int32)).view(1, C1, T)
    temperature, top_p = torch.tensor(0.7), torch.tensor(0.9)
    bias = torch.full((1, 1, cfg.vocab_size), float("-inf"))
    bias[0, 0, cfg.semantic_begin_id: cfg.semantic_end_id + 1] = 0.0
    bias[0, 0, cfg.im_end_id] = 0.0
    first = op(None, x, torch.arange(0, T), temperature, top_p, top_k, bias, None, None)
    cols = [first]
    cur, pos = first.view(1, C1, -1), torch.tensor([T], dtype=torch.int)
    prev = torch.zeros((C1, 16), dtype=torch.int)
    for _ in range(max_new - 1):
        nxt = op(None, cur, pos, temperature, top_p, top_k, bias, None, None, previous_tokens=prev).clone()
        pos += 1
        cur = nxt.view(1, C1, -1)
        prev = prev.roll(-1, dims=1)
        prev[:, -1] = nxt.view(C1, -1)[:, 0]
        cols.append(nxt)
        if cur[0, 0, -1] == cfg.im_end_id:
            break
    return torch.cat(cols, dim=1).numpy()


@pytest.mark.parametrize("name", ["llm_a", "llm_b"])
def test_decode_one_token_operator_in_reference_loop(name, golden):
    """B2: DecodeOneToken driven by the reference's generate/decode_n_tokens loop (prefill call,
    then one call per frame with the fed-back column) reproduces the reference's greedy tokens."""
    from fishmi.llm import DecodeOneToken

    m, g, cfg = _model(name, "fp32", golden)
    T = g["prompt"].shape[1]
    ref = g["seq"][:, T:]
    out = _reference_loop(DecodeOneToken(m), g["prompt"], ref.shape[1], cfg, top_k=1)
    np.testing.assert_array_equal(out, ref)


@pytest.mark.parametrize("rmsnorm_block", [0, 1])
@pytest.mark.parametrize("name", ["llm_a", "llm_b"])
def test_fp32_teacher_step_prefill_path_logits(name, rmsnorm_block, golden, knob):
    """fm_llm_teacher_step (every step through the PREFILL kernels: linear_kernel, row RMSNorm,
    qk_rope_cache + split attention): logits, hidden states and fast logits within 1e-4 of the
    reference's, with the wave-per-row RMSNorm (default) and the block-per-row one."""
    knob("rmsnorm_block", rmsnorm_block, 0)
    m, g, cfg = _model(name, "fp32", golden)
    T = g["prompt"].shape[1]
    seq = g["seq"]
    x, pos = g["prompt"], 0
    for i in range(seq.shape[1] - T):
        col = seq[:, T + i]
        lg, hid, fl = m.teacher_step(x, pos, next_col=col)
        ref = g["slow_logits"][i]
        fin = np.isfinite(ref)
        assert np.array_equal(np.isfinite(lg), fin)
        np.testing.assert_allclose(lg[fin], ref[fin], atol=1e-4, rtol=0)
        np.testing.assert_allclose(hid, g["hidden"][i], atol=1e-4, rtol=0)
        np.testing.assert_allclose(fl, g["fast_logits"][i], atol=1e-4, rtol=0)
        pos = T + i
        x = col.reshape(-1, 1)


def _bf16_vs_reference(slow, fast, g, rows=None):
    return bf16_vs_golden(slow, fast, g, rows)


@pytest.mark.parametrize("name", ["llm_a", "llm_b"])
def test_bf16_production_decode_vs_reference(name, golden):
    """bf16 PRODUCTION decode path (prefill, then graph-replayed decode_frame_small frames: fused
    GEMV prologue norms / SLABFIN residuals, attn_fd_kernel flash-decode with fused
    QK-norm/RoPE/KV-write, the sampler kernels) teacher-forced with the reference's emitted columns: slow and fast logits
    within BF16_RATIO x the reference's own bf16 error of the fp32 reference."""
    m, g, cfg = _model(name, "bf16", golden)
    T = g["prompt"].shape[1]
    slow, fast = m.teacher_decode(g["prompt"], g["seq"][:, T:])
    st = _bf16_vs_reference(slow, fast, g)
    assert st["top1_checked"] > 20


@pytest.mark.parametrize("name", ["llm_a", "llm_b"])
def test_fp32_production_decode_logits(name, golden):
    """fp32 validation mode of the production decode path (same kernels and graph as bf16):
    teacher-forced slow and fast logits within 1e-4 of the reference's fp32 ones."""
    m, g, cfg = _model(name, "fp32", golden)
    T = g["prompt"].shape[1]
    slow, fast = m.teacher_decode(g["prompt"], g["seq"][:, T:])
    ref = g["slow_logits"]
    fin = np.isfinite(ref)
    assert np.array_equal(np.isfinite(slow), fin)
    np.testing.assert_allclose(slow[fin], ref[fin], atol=1e-4, rtol=0)
    np.testing.assert_allclose(fast, g["fast_logits"], atol=1e-4, rtol=0)


def test_graph_matches_eager(golden):
    m, g, _ = _model("llm_a", "bf16", golden)
    T = g["prompt"].shape[1]
    m.use_graph(False)
    a = m.generate(g["prompt"], 20, top_k=30, seed=7)
    m.use_graph(True)
    b = m.generate(g["prompt"], 20, top_k=30, seed=7)
    np.testing.assert_array_equal(a, b)


def test_sampling_matches_oracle_fp32(golden):
    """top_k=30 / top_p / temperature / RAS with the shared counter-based RNG: the GPU stream
    equals the CPU restatement's (fp32 mode, so logits agree to ~1e-6)."""
    import oracle as O

    m, g, cfg = _model("llm_a", "fp32", golden)
    o = O.OracleLLM(cfg, False)
    from fishmi.checkpoint import load_llm_weights

    o.load(load_llm_weights(os.path.join(GOLDEN, "llm_a")))
    for seed in (1, 2, 3):
        ref = o.generate(g["prompt"], 24, temperature=0.7, top_p=0.9, top_k=30, seed=seed)
        out = m.generate(g["prompt"], 24, temperature=0.7, top_p=0.9, top_k=30, seed=seed)
        np.testing.assert_array_equal(out, ref)


def test_batched_slots_match_single(golden):
    """Config-3 style batching: n slots decoded together give each slot's batch-1 stream."""
    from fishmi.llm import DualARModel

    m, g, cfg = _model("llm_b", "fp32", golden, max_slots=4)
    rng = np.random.default_rng(0)
    prompts = []
    for s in range(4):
        p = g["prompt"].copy()
        p[0, 1:5] = rng.integers(16, cfg.semantic_begin_id, 4)
        prompts.append(p)
    n_new = 12
    single = [m.generate(p, n_new, top_k=1, slot=s, mask_im_end=True) for s, p in enumerate(prompts)]
    sp = DualARModel.sampling(top_k=1, mask_im_end=True)
    cols = [[m.prefill(s, p, sp)] for s, p in enumerate(prompts)]
    for _ in range(n_new - 1):
        out = m.decode([0, 1, 2, 3])
        for s in range(4):
            cols[s].append(out[s])
    for s in range(4):
        np.testing.assert_array_equal(np.stack(cols[s], axis=1), single[s])


def test_wide_real_widths_production_decode_vs_reference(golden):
    """S2-Pro widths (d=2560, 32/8x128 heads, I=9728, V=155776, C=10, cb=4096) at reduced depth,
    bf16, the PRODUCTION decode path the bench times: a 64-token prefill, then 16 graph-replayed
    batch-1 frames (gemv_kernel PRO_NORM/PRO_PRENORM + EPI_SLABFIN/EPI_SWIGLU8, attn_fd_kernel,
    fast_attn2, samplers), teacher-forced with the reference's columns; error within BF16_RATIO x
    the reference's own bf16 error of its fp32 logits."""
    from fishmi.llm import DualARModel

    g = golden("llm_wide_bf16.npz")
    cfg = _cfg("llm_wide")
    m = DualARModel.synthetic(cfg, int(g["synth_seed"]), int(g["log2_half"]), 0, "bf16", 1)
    T = g["prompt"].shape[1]
    assert T >= 64 and g["seq"].shape[1] - T >= 17
    slow, fast = m.teacher_decode(g["prompt"], g["seq"][:, T:])
    _bf16_vs_reference(slow, fast, g, rows=g["slow_rows"])
    m.close()


def test_wide_batched_32_slots_production_decode_vs_reference(golden):
    """BASELINE config 3's batched path at S2-Pro widths: 32 slots decoded together (bstream_kernel
    linears, finalize_norm, attn_fd_kernel, hipGraph per frame), every slot
    teacher-forced with the reference's columns: each slot's logits within BF16_RATIO x the
    reference's own bf16 error, and all 32 slots identical (rows are independent)."""
    from fishmi.llm import DualARModel

    g = golden("llm_wide_bf16.npz")
    cfg = _cfg("llm_wide")
    B = 32
    m = DualARModel.synthetic(cfg, int(g["synth_seed"]), int(g["log2_half"]), 0, "bf16", B)
    T = g["prompt"].shape[1]
    cols = g["seq"][:, T:]
    n = cols.shape[1]
    V, C1 = cfg.vocab_size, cfg.num_codebooks + 1
    slow = np.zeros((B, n, V), np.float32)
    fast = np.zeros((B, n, cfg.num_codebooks - 1, cfg.codebook_size), np.float32)
    sp = DualARModel.sampling(top_k=1)
    try:
        for i in range(n):
            for s in range(B):
                m.force(s, cols[:, i])
            if i == 0:
                for s in range(B):
                    m.prefill(s, g["prompt"], sp)
            else:
                m.decode(list(range(B)))
            for s in range(B):
                slow[s, i], fast[s, i] = m.read_logits(s)
    finally:
        for s in range(B):
            m.force(s, None)
    _bf16_vs_reference(slow[0], fast[0], g, rows=g["slow_rows"])
    for s in range(1, B):
        np.testing.assert_array_equal(slow[s], slow[0])
        np.testing.assert_array_equal(fast[s], fast[0])
    m.close()


def test_batched_32_slots_match_single_fp32(golden):
    """Config 3 at its real batch (32 slots per GPU) through the batched path: every slot's greedy
    stream equals its own batch-1 stream (fp32 validation mode)."""
    from fishmi.llm import DualARModel

    n = 32
    m, g, cfg = _model("llm_b", "fp32", golden, max_slots=n)
    rng = np.random.default_rng(11)
    prompts = []
    for s in range(n):
        p = g["prompt"].copy()
        p[0, 1:5] = rng.integers(16, cfg.semantic_begin_id, 4)
        prompts.append(p)
    n_new = 8
    single = [m.generate(p, n_new, top_k=1, slot=s, mask_im_end=True) for s, p in enumerate(prompts)]
    sp = DualARModel.sampling(top_k=1, mask_im_end=True)
    firsts = [m.prefill(s, p, sp) for s, p in enumerate(prompts)]
    fr = m.decode_frames(list(range(n)), n_new - 1)
    for s in range(n):
        got = np.concatenate([firsts[s][:, None], fr[:, s, :].T], axis=1)
        np.testing.assert_array_equal(got, single[s])


@pytest.mark.parametrize("name", ["llm_a", "llm_b"])
def test_top_k_above_64_matches_oracle_fp32(name, golden):
    """top_k > 64 (the reference's logits_to_probs takes any top_k, inference.py:54-77): the
    samplers' wide path (the row sorted in LDS, the reference's cumsum in rank order) draws the
    same streams as the CPU restatement's full sort, slow head with RAS and fast head, with nuclei
    far wider than 64 tokens (top_p 1.0 / 0.99) and top_k past the row length."""
    import oracle as O
    from fishmi import native

    m, g, cfg = _model(name, "fp32", golden)
    o = O.OracleLLM(cfg, False)
    if name == "llm_a":
        from fishmi.checkpoint import load_llm_weights

        o.load(load_llm_weights(os.path.join(GOLDEN, "llm_a")))
    else:
        o.synth(int(g["synth_seed"]), int(g["log2_half"]))
    for fast in (1, 0):
        native.tune("sampler_fast", fast)
        try:
            for top_k, top_p, temp, seed in ((100, 1.0, 0.9, 5), (1000, 0.99, 1.3, 6), (65, 0.95, 0.7, 7)):
                ref = o.generate(g["prompt"], 16, temperature=temp, top_p=top_p, top_k=top_k, seed=seed)
                m.use_graph(fast == 1)
                out = m.generate(g["prompt"], 16, temperature=temp, top_p=top_p, top_k=top_k, seed=seed)
                np.testing.assert_array_equal(out, ref, err_msg=f"top_k {top_k} sampler_fast {fast}")
        finally:
            native.tune("sampler_fast", 1)
            m.use_graph(True)


def test_top_k_above_64_at_s2_pro_head_width(golden):
    """The samplers' wide path (top_k > 64) at the production head widths (slow head: the 4096
    semantic tokens + <|im_end|> of a 155776-token vocabulary; fast head: 4096 codes), bf16: a free
    slot samples each frame, a twin slot replays that column forced and taps the logits its
    samplers were handed; every emitted token equals the C oracle's draw (logits_to_probs +
    multinomial, inference.py:43-93, with RAS, inference.py:117-144) on those same logits."""
    import oracle as O
    from fishmi import native
    from fishmi.llm import DualARModel

    g = golden("llm_wide_bf16.npz")
    cfg = _cfg("llm_wide")
    m = DualARModel.synthetic(cfg, int(g["synth_seed"]), int(g["log2_half"]), 0, "bf16", 2)
    C, cb, sb = cfg.num_codebooks, cfg.codebook_size, cfg.semantic_begin_id
    allowed = np.zeros(cfg.vocab_size, bool)
    allowed[sb: cfg.semantic_end_id + 1] = True
    n_new = 8
    try:
        for fast in (1, 0):
            native.tune("sampler_fast", fast)
            m.use_graph(fast == 1)
            for top_k, top_p, temp, seed in ((100, 1.0, 0.9, 5), (1000, 0.99, 1.3, 6), (4096, 0.95, 0.7, 7)):
                sp = DualARModel.sampling(temperature=temp, top_p=top_p, top_k=top_k, seed=seed, mask_im_end=True)
                prev = np.zeros((C + 1, 10), np.int64)
                for i in range(n_new):
                    col = m.prefill(1, g["prompt"], sp) if i == 0 else m.decode([1])[0]
                    m.force(0, col)
                    if i == 0:
                        m.prefill(0, g["prompt"], sp)
                    else:
                        m.decode([0])
                    slow, fl = m.read_logits(0)
                    m.force(0, None)
                    lg = np.where(allowed, slow, -np.inf).astype(np.float32)
                    tok = O.sample(lg, temp, top_p, top_k, seed, i, 0)
                    if i > 0:
                        hi = O.sample(lg, 1.0, 0.9, top_k, seed, i, 1)
                        if (prev[0] == tok).any() and sb <= tok <= cfg.semantic_end_id:
                            tok = hi
                    want = [tok, min(max(tok - sb, 0), cb - 1)]
                    for q in range(1, C):
                        want.append(O.sample(fl[q - 1], temp, top_p, top_k, seed, i, 1 + q))
                    np.testing.assert_array_equal(col, want, err_msg=f"frame {i} top_k {top_k} sampler_fast {fast}")
                    if i > 0:
                        prev = np.roll(prev, -1, axis=1)
                        prev[:, -1] = col
    finally:
        native.tune("sampler_fast", 1)
        m.use_graph(True)
        m.close()


def test_im_end_stops_and_masking(golden):
    """generate() stops after emitting <|im_end|> (inference.py:233); mask_im_end forbids it."""
    m, g, cfg = _model("llm_a", "fp32", golden)
    out = m.generate(g["prompt"], 40, top_k=30, seed=11, mask_im_end=True)
    assert out.shape[1] == 40 and not (out[0] == IM_END).any()
    assert ((out[0] >= cfg.semantic_begin_id) & (out[0] <= cfg.semantic_end_id)).all()
    assert (out[1] == out[0] - cfg.semantic_begin_id).all()


def test_profile_counters(golden):
    m, g, cfg = _model("llm_a", "bf16", golden)
    m.profile(True)
    m.generate(g["prompt"], 4, top_k=1)
    ms, n, b = m.profile_read("linear")
    assert n > 0 and ms > 0 and b > 0
    m.profile(False)
    assert m.frame_bytes(1, 30) > 0
    # replay hook used by bench.py's roofline: does not disturb the stream of the slot
    sp = m.sampling(top_k=1, mask_im_end=True)
    m.prefill(0, g["prompt"], sp)
    a = m.decode_frames([0], 3)
    us, n, b = m.kernel_bench("linear", reps=3)
    assert us > 0 and n > 0 and b > 0
    rest = m.decode_frames([0], 3)
    ref = m.generate(g["prompt"], 8, top_k=1, mask_im_end=True)
    np.testing.assert_array_equal(a[:, 0].T, ref[:, 1:4])
    np.testing.assert_array_equal(rest[:, 0].T, ref[:, 5:8])  # frame 4 ran inside the hook


def test_decode_frames_matches_generate(golden):
    """decode_n_tokens without host sync: prefill + decode_frames over 3 slots (2 slots sampled,
    one greedy) reproduces each slot's own generate() stream."""
    from fishmi.llm import DualARModel

    m, g, cfg = _model("llm_b", "bf16", golden, max_slots=3)
    rng = np.random.default_rng(5)
    prompts, sps = [], []
    for s in range(3):
        p = g["prompt"].copy()
        p[0, 1:5] = rng.integers(16, cfg.semantic_begin_id, 4)
        prompts.append(p)
        sps.append(dict(top_k=1 if s == 2 else 30, seed=100 + s, mask_im_end=True))
    n_new = 17
    single = [m.generate(p, n_new, slot=s, **sps[s]) for s, p in enumerate(prompts)]
    firsts = [m.prefill(s, p, DualARModel.sampling(**sps[s])) for s, p in enumerate(prompts)]
    fr = m.decode_frames([0, 1, 2], n_new - 1)
    assert fr.shape == (n_new - 1, 3, cfg.num_codebooks + 1)
    for s in range(3):
        got = np.concatenate([firsts[s][:, None], fr[:, s, :].T], axis=1)
        np.testing.assert_array_equal(got, single[s])


@pytest.fixture
def knob():
    """fm_tune knobs set by a test, restored to their defaults afterwards."""
    from fishmi import native

    set_ = {}

    def put(key, value, default):
        set_[key] = default
        native.tune(key, value)

    yield put
    for k, d in set_.items():
        native.tune(k, d)


@pytest.mark.parametrize("bstream", [1, 0])
@pytest.mark.parametrize("n", [12, 20])
def test_batched_slots_past_gemv_match_single(n, bstream, golden, knob):
    """Config-3 batching past the batch-1 GEMV (n > 8 slots) gives each slot its own batch-1
    greedy stream (fp32 mode): the register-resident weight stream bstream_kernel (default) and the
    MFMA linear_kernel (fm_tune bstream=0)."""
    from fishmi.llm import DualARModel

    knob("bstream", bstream, 1)

    m, g, cfg = _model("llm_b", "fp32", golden, max_slots=n)
    rng = np.random.default_rng(7)
    prompts = []
    for s in range(n):
        p = g["prompt"].copy()
        p[0, 1:5] = rng.integers(16, cfg.semantic_begin_id, 4)
        prompts.append(p)
    n_new = 10
    single = [m.generate(p, n_new, top_k=1, slot=s, mask_im_end=True) for s, p in enumerate(prompts)]
    sp = DualARModel.sampling(top_k=1, mask_im_end=True)
    firsts = [m.prefill(s, p, sp) for s, p in enumerate(prompts)]
    fr = m.decode_frames(list(range(n)), n_new - 1)
    for s in range(n):
        got = np.concatenate([firsts[s][:, None], fr[:, s, :].T], axis=1)
        np.testing.assert_array_equal(got, single[s])


@pytest.mark.parametrize("knobs", [{}, {"bstream": 0}, {"bstream": 0, "linear_fill": 1024},
                                   {"bstream_acc": 0, "bstream_nw": 16}, {"bstream_acc": 0, "bstream_kparts": 2},
                                   {"batched_fused_attn": 0}, {"attn_cap_batched": 32},
                                   {"fd_min_batched": 64}, {"bstream": 0, "linear_u32": 8}, {"bstream_acc": 0},
                                   {"fd_nw_batched": 8}, {"fd_nw_batched": 16, "fd_min_batched": 64},
                                   {"bs_qkv_slab": 0}])
def test_batched_wide_split_k_matches_single(knobs, golden, knob):
    """S2-Pro widths, 20 slots: the batched linears (bf16 production: bsacc_kernel; fp32 validation
    mode: bstream_kernel, whose K-part slabs + finalize_norm the default runs), whole-K linear_kernel,
    and linear_kernel's opt-in split K (linear_fill: sc1 partials + ticketed last-slice reduction)
    reproduce every slot's batch-1 greedy stream (fp32 mode)."""
    from fishmi.llm import DualARModel

    defaults = {"bstream": 1, "linear_fill": 0, "bstream_nw": 0, "bstream_kparts": 0, "batched_fused_attn": 1,
                "attn_cap_batched": 128, "fd_min_batched": 512, "linear_u32": 4, "bstream_acc": 1, "fd_nw_batched": 4,
                "bs_qkv_slab": 1}
    for k, v in knobs.items():
        knob(k, v, defaults[k])

    g = golden("llm_wide_bf16.npz")
    cfg = _cfg("llm_wide")
    n = 20
    m = DualARModel.synthetic(cfg, int(g["synth_seed"]), int(g["log2_half"]), 0, "fp32", n)
    rng = np.random.default_rng(9)
    prompts = []
    for s in range(n):
        p = g["prompt"].copy()
        p[0, 1:5] = rng.integers(16, cfg.semantic_begin_id, 4)
        prompts.append(p)
    n_new = 4
    single = [m.generate(p, n_new, top_k=1, slot=s, mask_im_end=True) for s, p in enumerate(prompts)]
    sp = DualARModel.sampling(top_k=1, mask_im_end=True)
    firsts = [m.prefill(s, p, sp) for s, p in enumerate(prompts)]
    fr = m.decode_frames(list(range(n)), n_new - 1)
    for s in range(n):
        got = np.concatenate([firsts[s][:, None], fr[:, s, :].T], axis=1)
        np.testing.assert_array_equal(got, single[s])
    m.close()


def test_long_context_split_attention_matches_oracle(golden):
    """Contexts longer than one attention block's rows (256 here) take the split path of the
    decode attention (per-split partials + last-arriver combine): greedy stream == oracle."""
    import oracle as O
    from fishmi.llm import DualARModel

    cfg = _cfg("llm_b")
    cfg.max_seq_len = 640
    g = golden("llm_b_fp32.npz")
    m = DualARModel.synthetic(cfg, int(g["synth_seed"]), int(g["log2_half"]), 0, "fp32", 1)
    o = O.OracleLLM(cfg, False)
    o.synth(int(g["synth_seed"]), int(g["log2_half"]))
    rng = np.random.default_rng(3)
    T = 300
    p = np.zeros((cfg.num_codebooks + 1, T), np.int32)
    p[0] = rng.integers(16, cfg.semantic_begin_id, T)
    sem = rng.random(T) < 0.5  # semantic positions carry codebook tokens
    p[0, sem] = rng.integers(cfg.semantic_begin_id, cfg.semantic_end_id + 1, int(sem.sum()))
    p[1:, sem] = rng.integers(0, cfg.codebook_size, (cfg.num_codebooks, int(sem.sum())))
    ref = o.generate(p, 12, top_k=1)
    out = m.generate(p, 12, top_k=1)
    np.testing.assert_array_equal(out, ref)


def test_fast_sampler_equals_radix_sampler(golden):
    """The two-stage register top-K sampler and the LDS radix-select sampler draw the same
    streams (same candidates in the same order, same RNG draws), sampled and greedy."""
    from fishmi import native

    m, g, cfg = _model("llm_a", "bf16", golden)
    outs = {}
    for fast in (1, 0):
        native.tune("sampler_fast", fast)
        m.use_graph(False)
        outs[fast] = [m.generate(g["prompt"], 24, top_k=k, seed=s, temperature=0.9, top_p=0.95)
                      for k, s in ((30, 1), (64, 2), (1, 3), (5, 4))]
    native.tune("sampler_fast", 1)
    m.use_graph(True)
    for a, b in zip(outs[1], outs[0]):
        np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("name", ["llm_a", "llm_b"])
def test_fast_attention_in_wo_prologue(name, golden):
    """fm_tune attn_wo=1 (PRO_FATT): the fast model's attention recomputed by every block of the
    Wo GEMV from LDS-staged operands gives the same fp32 greedy stream as the reference."""
    from fishmi import native

    native.tune("attn_wo", 1)
    try:
        m, g, _ = _model(name, "fp32", golden)
        T = g["prompt"].shape[1]
        ref = g["seq"][:, T:]
        out = m.generate(g["prompt"], ref.shape[1], top_k=1)
        np.testing.assert_array_equal(out, ref)
    finally:
        native.tune("attn_wo", 0)


@pytest.mark.parametrize("n", [3, 10])
def test_prefill_batch_matches_single(n, golden):
    """fm_llm_prefill_batch (config 3's tick of new requests prefilled together: one slow-stack pass
    over all prompt rows packed into 256-row chunks, prompts spanning chunks, attention per prompt
    segment, one batched first frame) gives every request the same first column and the same
    greedy continuation as its own fm_llm_prefill (fp32 mode); n = 3 takes the batch-1 GEMV tail,
    n = 10 the batched one."""
    from fishmi.llm import DualARModel

    m, g, cfg = _model("llm_b", "fp32", golden, max_slots=n)
    rng = np.random.default_rng(31 + n)
    lens = rng.integers(5, 150, n)
    prompts = []
    for T in lens:
        p = np.zeros((cfg.num_codebooks + 1, int(T)), np.int32)
        p[0] = rng.integers(16, cfg.semantic_begin_id, int(T))
        p[1:] = rng.integers(0, cfg.codebook_size, (cfg.num_codebooks, int(T)))
        prompts.append(p)
    sps = [DualARModel.sampling(top_k=1, seed=s, mask_im_end=True) for s in range(n)]
    slots = list(range(n))
    single = [m.prefill(s, p, sp) for s, p, sp in zip(slots, prompts, sps)]
    single_fr = m.decode_frames(slots, 6)
    batch = m.prefill_batch(slots[::-1], prompts[::-1], sps[::-1])[::-1]
    batch_fr = m.decode_frames(slots, 6)
    np.testing.assert_array_equal(np.stack(single), batch)
    np.testing.assert_array_equal(single_fr, batch_fr)
    m.close()
