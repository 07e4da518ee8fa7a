"""Parity at the configurations bench.py times.  This module sorts first among the GPU tests, so
under `pytest -x -m gpu` nothing else can hide a failure here.

* Config 2 at FULL S2-Pro depth (36 slow + 4 fast layers, 64-token prompt, prefill + 8 frames),
  bf16, through the production decode graph (teacher forcing with the reference's columns).
* A 3000-token context at S2-Pro widths (config 5's regime): every frame's slow attention spans
  many flash-decode splits.
* Config 3's ragged batch: 32 slots holding 32 different prompts of uniform 16..256 tokens (the
  BASELINE distribution, seed 2), so every slot sits at its own position; decoded together on the
  batched path, each slot's logits against the reference's batch-1 run of its own prompt (bf16),
  and each slot's greedy stream against its own batch-1 stream (fp32 validation mode).

* Round 5: config 2 over all 216 bench frames (positions 64..280) and config 3's ragged batch at
  full depth (36 + 4 layers), the depths and positions the bench actually runs.

Goldens: oracle/gen_goldens.py llm_full / llm_long / llm_ragged / llm_full216 / llm_ragged_full (the
reference run on CPU in the dev container; weights regenerate from the seed on the device).  Bound:
tests/parity_util.py."""
import json

import numpy as np
import pytest

from parity_util import bf16_vs_golden, bf16_vs_reference, bits_to_f32

pytestmark = pytest.mark.gpu

IM_END = 4


def _cfg(g):
    from fishmi.config import DualARConfig

    cfg = DualARConfig._from_fish_qwen3_omni(json.loads(str(g["config"])))
    cfg.im_end_id = IM_END
    return cfg


def _teacher_case(name, golden):
    from fishmi.llm import DualARModel

    g = golden(name)
    cfg = _cfg(g)
    m = DualARModel.synthetic(cfg, int(g["synth_seed"]), int(g["log2_half"]), 0, "bf16", 1)
    try:
        T = g["prompt"].shape[1]
        slow, fast = m.teacher_decode(g["prompt"], g["seq"][:, T:])
    finally:
        m.close()
    return bf16_vs_golden(slow, fast, g, rows=g["slow_rows"])


def test_config2_full_depth_bf16_vs_reference(golden):
    """36 + 4 layers: bf16 error growth over the whole depth against the reference's own."""
    st = _teacher_case("llm_full_bf16.npz", golden)
    assert st["top1_checked"] >= 9


def test_long_context_bf16_vs_reference(golden):
    """3000-token prompt (prefill in chunks, flash-decode over >= 3000 positions per frame)."""
    g = golden("llm_long_bf16.npz")
    assert g["prompt"].shape[1] >= 3000
    _teacher_case("llm_long_bf16.npz", golden)


def _golden_or_skip(golden, name):
    import os

    from conftest import GOLDEN

    if not os.path.exists(os.path.join(GOLDEN, name)):
        pytest.skip(f"{name} not generated (oracle/gen_goldens.py)")
    return golden(name)


def test_config2_full_depth_64_frames_bf16_vs_reference(golden):
    """Config 2 at full depth over 64 decode frames (positions 64..128) through the production
    decode graph, teacher-forced with the reference's columns: every frame's slow logits and the
    last codebook's fast logits within BF16_RATIO x the reference's own bf16 error."""
    from fishmi.llm import DualARModel

    g = _golden_or_skip(golden, "llm_full64_bf16.npz")
    cfg = _cfg(g)
    T = g["prompt"].shape[1]
    assert g["seq"].shape[1] - T >= 65
    m = DualARModel.synthetic(cfg, int(g["synth_seed"]), int(g["log2_half"]), 0, "bf16", 1)
    try:
        slow, fast = m.teacher_decode(g["prompt"], g["seq"][:, T:])
    finally:
        m.close()
    rows = g["slow_rows"]
    st = bf16_vs_reference(slow[:, rows], fast[:, -1:], bits_to_f32(g["slow_logits_bits"]),
                           bits_to_f32(g["fast_last_bits"])[:, None], g["slow_logits_f32"],
                           g["fast_last_f32"][:, None])
    assert st["top1_checked"] >= 30  # (36 of 130 clear margins at this seed)


def test_config2_full_depth_216_frames_bf16_vs_reference(golden):
    """Config 2 exactly as bench.py runs it: full depth, 64-token prompt, prefill + 216 decode frames
    (positions 64..280), teacher-forced through the production decode graph; every frame's slow
    logits and the last codebook's fast logits within BF16_RATIO x the reference's own bf16 error."""
    from fishmi.llm import DualARModel

    g = _golden_or_skip(golden, "llm_full216_bf16.npz")
    cfg = _cfg(g)
    T = g["prompt"].shape[1]
    assert T == 64 and g["seq"].shape[1] - T >= 217 and cfg.n_layer == 36
    m = DualARModel.synthetic(cfg, int(g["synth_seed"]), int(g["log2_half"]), 0, "bf16", 1)
    try:
        slow, fast = m.teacher_decode(g["prompt"], g["seq"][:, T:])
    finally:
        m.close()
    rows = g["slow_rows"]
    st = bf16_vs_reference(slow[:, rows], fast[:, -1:], bits_to_f32(g["slow_logits_bits"]),
                           bits_to_f32(g["fast_last_bits"])[:, None], g["slow_logits_f32"],
                           g["fast_last_f32"][:, None])
    assert st["top1_checked"] >= 60


def test_long_context_4_layers_bf16_vs_reference(golden):
    """3000-token prompt through 4 slow layers: the long-context error growth over depth."""
    g = _golden_or_skip(golden, "llm_long4_bf16.npz")
    assert g["prompt"].shape[1] >= 3000 and _cfg(g).n_layer == 4
    _teacher_case("llm_long4_bf16.npz", golden)


_RAGGED_LOGITS = {}  # (prefill, chain, slab) -> the default forms' logits (the older-forms case compares)


@pytest.fixture
def knob():
    from fishmi import native

    set_ = {}

    def put(key, value, default):
        set_[key] = default
        native.tune(key, value)

    yield put
    for k, d in set_.items():
        native.tune(k, d)


@pytest.mark.parametrize("prefill,chain,slab,older", [("batch", 0, 1, 0), ("single", 0, 1, 0), ("batch", 1, 1, 0),
                                                      ("batch", 0, 0, 0), ("batch", 0, 1, 1)])
def test_config3_ragged_32_slots_bf16_vs_reference(prefill, chain, slab, older, golden, knob):
    """32 distinct prompts (16..256 tokens) in permuted slots: first frame from prefill_batch (the
    serving tick's path) or per-slot prefill, then batched decode frames (bsacc_kernel linears,
    finalize_norm, attn_fd at 32 different positions), every slot teacher-forced with its own
    reference columns.  Pooled over slots, the error is within BF16_RATIO x the reference's.
    chain = 1: the fm_tune bstream_chain variant (bsacc SLABFIN / PRENORM, no finalize_norm);
    slab = 0: the QKV projection's own STORE epilogue instead of K-part slabs summed by the attention
    (fm_tune bs_qkv_slab); older = 1: bsacc's round-5 forms (X loaded after the weight ring, the
    one-output-per-thread epilogue: fm_tune bs_xfirst 0, bs_vec_epi 0), whose logits must equal the
    default's bit for bit (same loads, same fp32 sums in the same order)."""
    from fishmi.llm import DualARModel

    knob("bstream_chain", chain, 0)
    knob("bs_qkv_slab", slab, 1)
    knob("bs_xfirst", 1 - older, 1)
    knob("bs_vec_epi", 1 - older, 1)
    g = golden("llm_ragged_bf16.npz")
    cfg = _cfg(g)
    B = int(g["lens"].size)
    assert B == 32 and g["lens"].min() >= 16 and g["lens"].max() <= 256 and len(set(g["lens"].tolist())) > 16
    cols = g["cols"]  # (B, C+1, n)
    n = cols.shape[2]
    prompts = [g[f"prompt_{i}"] for i in range(B)]
    slot_of = np.random.default_rng(4).permutation(B)  # prompt i lives in slot slot_of[i]
    order = [int(slot_of[i]) for i in np.random.default_rng(5).permutation(B)]  # frame row order
    m = DualARModel.synthetic(cfg, int(g["synth_seed"]), int(g["log2_half"]), 0, "bf16", B)
    slow = np.zeros((B, n, cfg.vocab_size), np.float32)
    fast = np.zeros((B, n, cfg.num_codebooks - 1, cfg.codebook_size), np.float32)
    sp = DualARModel.sampling(top_k=1)
    try:
        for k in range(n):
            for i in range(B):
                m.force(int(slot_of[i]), cols[i, :, k])
            if k == 0:
                if prefill == "batch":
                    m.prefill_batch([int(s) for s in slot_of], prompts, [sp] * B)
                else:
                    for i in range(B):
                        m.prefill(int(slot_of[i]), prompts[i], sp)
            else:
                m.decode(order)
            for i in range(B):
                slow[i, k], fast[i, k] = m.read_logits(int(slot_of[i]))
    finally:
        for s in range(B):
            m.force(s, None)
        m.close()
    rows = g["slow_rows"]
    key = (prefill, chain, slab)
    if older:  # the default forms' logits of the same run, bit for bit
        np.testing.assert_array_equal(slow, _RAGGED_LOGITS[key][0])
        np.testing.assert_array_equal(fast, _RAGGED_LOGITS[key][1])
    else:
        _RAGGED_LOGITS[key] = (slow, fast)
    st = bf16_vs_reference(slow.reshape(B * n, -1)[:, rows], fast[:, :, -1:].reshape(B * n, 1, -1),
                           bits_to_f32(g["slow_logits_bits"]).reshape(B * n, -1),
                           bits_to_f32(g["fast_last_bits"]).reshape(B * n, 1, -1),
                           g["slow_logits_f32"].reshape(B * n, -1), g["fast_last_f32"].reshape(B * n, 1, -1))
    assert st["top1_checked"] >= B


def test_config3_ragged_32_slots_64_frames_bf16_vs_reference(golden):
    """Config 3's ragged batch over 64 decode frames (positions up to 320): 32 prompts in permuted
    slots, prefill_batch then 64 batched frames, all teacher-forced with each prompt's reference
    columns; logits checked at the golden's kept frames (0, 32, 64)."""
    from fishmi.llm import DualARModel

    g = _golden_or_skip(golden, "llm_ragged64_bf16.npz")
    cfg = _cfg(g)
    B = int(g["lens"].size)
    cols = g["cols"]
    n = cols.shape[2]
    kf = [int(k) for k in g["keep_frames"]]
    assert B == 32 and n >= 65 and kf[-1] == n - 1
    prompts = [g[f"prompt_{i}"] for i in range(B)]
    slot_of = np.random.default_rng(6).permutation(B)
    order = [int(slot_of[i]) for i in np.random.default_rng(7).permutation(B)]
    m = DualARModel.synthetic(cfg, int(g["synth_seed"]), int(g["log2_half"]), 0, "bf16", B)
    slow = np.zeros((B, len(kf), len(g["slow_rows"])), np.float32)
    fast = np.zeros((B, len(kf), 1, cfg.codebook_size), np.float32)
    sp = DualARModel.sampling(top_k=1)
    try:
        for k in range(n):
            for i in range(B):
                m.force(int(slot_of[i]), cols[i, :, k])
            if k == 0:
                m.prefill_batch([int(s) for s in slot_of], prompts, [sp] * B)
            else:
                m.decode(order)
            if k in kf:
                for i in range(B):
                    s_, f_ = m.read_logits(int(slot_of[i]))
                    slow[i, kf.index(k)] = s_[g["slow_rows"]]
                    fast[i, kf.index(k), 0] = f_[-1]
    finally:
        for s in range(B):
            m.force(s, None)
        m.close()
    nk = len(kf)
    st = bf16_vs_reference(slow.reshape(B * nk, -1), fast.reshape(B * nk, 1, -1),
                           bits_to_f32(g["slow_logits_bits"]).reshape(B * nk, -1),
                           bits_to_f32(g["fast_last_bits"]).reshape(B * nk, 1, -1),
                           g["slow_logits_f32"].reshape(B * nk, -1), g["fast_last_f32"].reshape(B * nk, 1, -1))
    assert st["top1_checked"] >= B


def test_config3_ragged_32_slots_full_depth_bf16_vs_reference(golden):
    """Config 3's ragged batch at FULL depth (36 + 4 layers): 32 prompts of 16..256 tokens in
    permuted slots, prefill_batch then 8 batched frames (bsacc_kernel, finalize_norm, attn_fd at 32
    positions through 36 layers), teacher-forced; logits at the golden's kept frames (0, 4, 8)
    against each prompt's batch-1 reference run."""
    from fishmi.llm import DualARModel

    g = _golden_or_skip(golden, "llm_ragged_full_bf16.npz")
    cfg = _cfg(g)
    assert cfg.n_layer == 36
    B = int(g["lens"].size)
    cols = g["cols"]
    n = cols.shape[2]
    kf = [int(k) for k in g["keep_frames"]]
    assert B == 32 and n >= 9 and kf[-1] == n - 1
    prompts = [g[f"prompt_{i}"] for i in range(B)]
    slot_of = np.random.default_rng(8).permutation(B)
    order = [int(slot_of[i]) for i in np.random.default_rng(9).permutation(B)]
    m = DualARModel.synthetic(cfg, int(g["synth_seed"]), int(g["log2_half"]), 0, "bf16", B)
    slow = np.zeros((B, len(kf), len(g["slow_rows"])), np.float32)
    fast = np.zeros((B, len(kf), 1, cfg.codebook_size), np.float32)
    sp = DualARModel.sampling(top_k=1)
    try:
        for k in range(n):
            for i in range(B):
                m.force(int(slot_of[i]), cols[i, :, k])
            if k == 0:
                m.prefill_batch([int(s) for s in slot_of], prompts, [sp] * B)
            else:
                m.decode(order)
            if k in kf:
                for i in range(B):
                    s_, f_ = m.read_logits(int(slot_of[i]))
                    slow[i, kf.index(k)] = s_[g["slow_rows"]]
                    fast[i, kf.index(k), 0] = f_[-1]
    finally:
        for s in range(B):
            m.force(s, None)
        m.close()
    nk = len(kf)
    st = bf16_vs_reference(slow.reshape(B * nk, -1), fast.reshape(B * nk, 1, -1),
                           bits_to_f32(g["slow_logits_bits"]).reshape(B * nk, -1),
                           bits_to_f32(g["fast_last_bits"]).reshape(B * nk, 1, -1),
                           g["slow_logits_f32"].reshape(B * nk, -1), g["fast_last_f32"].reshape(B * nk, 1, -1))
    assert st["top1_checked"] >= B


def _ragged_prompts(cfg, B, seed):
    """Config 3's prompt-length distribution (uniform 16..256), random text / semantic tokens."""
    rng = np.random.default_rng(seed)
    lens = rng.integers(16, 257, B)
    prompts = []
    for T in lens:
        p = np.zeros((cfg.num_codebooks + 1, int(T)), np.int32)
        p[0] = rng.integers(16, cfg.semantic_begin_id, int(T))
        sem = rng.random(int(T)) < 0.4
        p[0, sem] = rng.integers(cfg.semantic_begin_id, cfg.semantic_end_id + 1, int(sem.sum()))
        p[1:, sem] = rng.integers(0, cfg.codebook_size, (cfg.num_codebooks, int(sem.sum())))
        prompts.append(p)
    return lens, prompts


def _ragged_fp32(m, cfg, B, n_new, seed):
    lens, prompts = _ragged_prompts(cfg, B, seed)
    from fishmi.llm import DualARModel

    slot_of = [int(s) for s in np.random.default_rng(seed + 1).permutation(B)]
    single = [m.generate(p, n_new, top_k=1, slot=slot_of[i], mask_im_end=True) for i, p in enumerate(prompts)]
    sp = DualARModel.sampling(top_k=1, mask_im_end=True)
    firsts = m.prefill_batch(slot_of, prompts, [sp] * B)
    fr = m.decode_frames(slot_of[::-1], n_new - 1)[:, ::-1]  # rows in reversed slot order
    for i in range(B):
        got = np.concatenate([firsts[i][:, None], fr[:, i, :].T], axis=1)
        np.testing.assert_array_equal(got, single[i], err_msg=f"prompt {i} (T={lens[i]}) in slot {slot_of[i]}")


def test_config3_ragged_32_slots_fp32_match_single(golden):
    """fp32 validation mode, tiny model: 32 ragged prompts batched == each one's batch-1 stream."""
    from fishmi.config import DualARConfig
    from fishmi.llm import DualARModel
    import os
    from conftest import GOLDEN

    cfg = DualARConfig.from_pretrained(os.path.join(GOLDEN, "llm_b"))
    cfg.im_end_id = IM_END
    cfg.max_seq_len = 320
    g = golden("llm_b_fp32.npz")
    m = DualARModel.synthetic(cfg, int(g["synth_seed"]), int(g["log2_half"]), 0, "fp32", 32)
    try:
        _ragged_fp32(m, cfg, 32, 12, seed=2)
    finally:
        m.close()


def test_config3_ragged_32_slots_fp32_wide_match_single(golden):
    """fp32 validation mode at S2-Pro widths (2 + 1 layers): the same property on the batched
    bstream / finalize_norm / attn_fd path with the real head counts and widths."""
    from fishmi.llm import DualARModel

    g = golden("llm_ragged_bf16.npz")
    cfg = _cfg(g)
    cfg.max_seq_len = 272
    m = DualARModel.synthetic(cfg, int(g["synth_seed"]), int(g["log2_half"]), 0, "fp32", 32)
    try:
        _ragged_fp32(m, cfg, 32, 5, seed=12)
    finally:
        m.close()
