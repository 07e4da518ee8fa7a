"""Pin the CPU restatement (oracle/) against fixtures produced by the REAL reference
(oracle/gen_goldens.py imports /root/reference in the dev container; see its header).

CPU-only: these run under ``-m "not gpu"``.
"""
import json
import os

import numpy as np
import pytest

import oracle as O
from fishmi.checkpoint import codec_tensor_shapes, llm_tensor_shapes, load_llm_weights
from fishmi.config import CodecConfig, DualARConfig

from conftest import GOLDEN

IM_END = 4


def _llm(name, tag, golden):
    g = golden(f"{name}_{tag}.npz")
    wdir = os.path.join(GOLDEN, name)
    cfg = DualARConfig.from_pretrained(wdir)
    cfg.im_end_id = IM_END
    o = O.OracleLLM(cfg, tag == "bf16")
    if name == "llm_a":
        o.load(load_llm_weights(wdir))
    else:
        o.synth(int(g["synth_seed"]), int(g["log2_half"]))
    return o, g, cfg


def test_loader_matches_reference_inventory():
    """fish_qwen3_omni config + remap + sharded index + split wq/wk/wv (llama.py:75-143,
    229-246, 545-586, 876-881) yields exactly the reference module's state_dict keys."""
    wdir = os.path.join(GOLDEN, "llm_a")
    cfg = DualARConfig.from_pretrained(wdir)
    assert cfg.scale_codebook_embeddings and cfg.norm_fastlayer_input
    assert (cfg.semantic_begin_id, cfg.semantic_end_id) == (200, 327)
    w = load_llm_weights(wdir)
    shapes = llm_tensor_shapes(cfg)
    assert set(w) == set(shapes)
    for k, s in shapes.items():
        assert tuple(w[k].shape) == tuple(s), k
    cb = DualARConfig.from_pretrained(os.path.join(GOLDEN, "llm_b"))
    assert cb.fast_dim == 96 and cb.fast_n_local_heads == 1 and not cb.scale_codebook_embeddings


@pytest.mark.parametrize("name", ["llm_a", "llm_b"])
def test_fp32_greedy_tokens_exact(name, golden):
    """fp32 validation mode: free-running greedy stream == reference, token for token."""
    o, g, _ = _llm(name, "fp32", golden)
    T = g["prompt"].shape[1]
    ref = g["seq"][:, T:]
    out = o.generate(g["prompt"], ref.shape[1], top_k=1)
    np.testing.assert_array_equal(out, ref)


@pytest.mark.parametrize("name", ["llm_a", "llm_b"])
def test_fp32_teacher_forced_logits(name, golden):
    o, g, cfg = _llm(name, "fp32", golden)
    T = g["prompt"].shape[1]
    seq = g["seq"]
    o.reset()
    x, pos = g["prompt"], 0
    for i in range(seq.shape[1] - T):
        lg, hid = o.forward(x, pos)
        ref = g["slow_logits"][i]
        fin = np.isfinite(ref)
        np.testing.assert_allclose(lg[fin], ref[fin], atol=2e-5, rtol=0)
        np.testing.assert_allclose(hid, g["hidden"][i], atol=2e-5, rtol=0)
        col = seq[:, T + i]
        o.fast(hid, -1, 0, logits=False)
        a = int(np.clip(col[0] - cfg.semantic_begin_id, 0, cfg.codebook_size - 1))
        for c in range(1, cfg.num_codebooks):
            fl = o.fast(None, a, c)
            np.testing.assert_allclose(fl, g["fast_logits"][i, c - 1], atol=2e-5, rtol=0)
            a = int(col[c + 1])
        pos = T + i
        x = col.reshape(-1, 1)


def _margin(v):
    s = np.sort(v[np.isfinite(v)])[::-1]
    return s[0] - s[1]


@pytest.mark.parametrize("name", ["llm_a", "llm_b"])
def test_bf16_teacher_forced_top1(name, golden):
    """bf16: logits within a few bf16 ulps; top-1 agrees wherever the reference's top-1/top-2
    margin exceeds the bf16 noise (accumulation order flips near-ties)."""
    o, g, cfg = _llm(name, "bf16", golden)
    T = g["prompt"].shape[1]
    seq = g["seq"]
    o.reset()
    x, pos = g["prompt"], 0
    n_checked = n_agree = 0
    for i in range(seq.shape[1] - T):
        lg, hid = o.forward(x, pos)
        ref = g["slow_logits"][i]
        fin = np.isfinite(ref)
        err = np.abs(lg[fin] - ref[fin])
        assert err.max() <= 0.08 * max(1.0, np.abs(ref[fin]).max()), (i, err.max())
        rl = np.where(fin, lg, -np.inf)
        if _margin(ref) > 0.07:
            n_checked += 1
            n_agree += int(np.argmax(rl) == np.argmax(ref))
        col = seq[:, T + i]
        o.fast(hid, -1, 0, logits=False)
        a = int(np.clip(col[0] - cfg.semantic_begin_id, 0, cfg.codebook_size - 1))
        for c in range(1, cfg.num_codebooks):
            fl = o.fast(None, a, c)
            rf = g["fast_logits"][i, c - 1]
            if _margin(rf) > 0.07:
                n_checked += 1
                n_agree += int(np.argmax(fl) == np.argmax(rf))
            a = int(col[c + 1])
        pos = T + i
        x = col.reshape(-1, 1)
    assert n_checked > 20
    assert n_agree == n_checked


def test_ops_rmsnorm_bitexact(golden):
    g = golden("ops.npz")
    y = O.op_rmsnorm(g["rms_x"], g["rms_w"], 1e-6, bf16=True)
    np.testing.assert_array_equal(y, g["rms_y"])


def test_ops_qknorm_bitexact(golden):
    g = golden("ops.npz")
    y = O.op_rmsnorm(g["qk_x"], g["qk_w"], 1e-6, bf16=True, head=True)
    np.testing.assert_array_equal(y, g["qk_y"])


def test_ops_rope_table_and_apply(golden):
    g = golden("ops.npz")
    np.testing.assert_array_equal(O.op_rope_table(64, 32, 10000.0), g["rope_table"])
    big = O.op_rope_table(4096, 128, 1000000.0)[::97]
    # table entries may differ by 1 bf16 ulp where cos/sin of the fp32 angle rounds at a tie
    assert np.mean(big != g["rope_table_big"]) < 1e-3
    assert np.abs(big - g["rope_table_big"]).max() <= 2 ** -8
    x, pos = g["rope_x"], g["rope_pos"]  # [1, 5, 4, 32]
    tab = g["rope_table"][pos].reshape(5, 1, 32)
    y = np.stack([O.op_rope(x[0, s], np.broadcast_to(tab[s], (4, 32)).copy()) for s in range(5)])
    np.testing.assert_array_equal(y[None], g["rope_y"])


def test_logits_to_probs(golden):
    """inference.py:54-77 in bf16.  Rows whose top_k boundary falls inside a tie are compared
    as multisets: the CPU reference's unstable introsort orders ties arbitrarily (CUDA's radix
    sort is stable -> lowest index first, which is what the oracle and the GPU use)."""
    g = golden("ops.npz")
    for lg, pr, (t, p, k) in zip(g["lp_logits"], g["lp_probs"], g["lp_params"]):
        out = O.logits_to_probs(lg, t, p, int(k), True)
        if np.array_equal(out, pr):
            continue
        np.testing.assert_array_equal(np.sort(out), np.sort(pr))
        top = lg[np.isfinite(lg)].max()
        assert (lg[out > 0] == top).all() or (lg[pr != out] == top).all()
    assert int(g["tie_idx"].reshape(-1)[0]) == 5  # reference: lowest index among ties here


def test_sampler_deterministic_and_masked():
    rng = np.random.default_rng(0)
    lg = rng.normal(0, 2, 512).astype(np.float32)
    lg = (lg.astype(np.float32).view(np.uint32) & 0xFFFF0000).view(np.float32)
    a = O.sample(lg, 0.7, 0.9, 30, 123, 5, 0)
    b = O.sample(lg, 0.7, 0.9, 30, 123, 5, 0)
    assert a == b
    probs = O.logits_to_probs(lg, 0.7, 0.9, 30)
    assert probs[a] > 0
    seen = {O.sample(lg, 0.7, 0.9, 30, 123, s, 0) for s in range(200)}
    assert seen <= set(np.nonzero(probs)[0]) and len(seen) > 3
    assert O.sample(lg, 0.7, 0.9, 1, 9, 1, 0) == int(np.argmax(lg))


def _codec(name, golden):
    g = golden(f"{name}.npz")
    cfg = CodecConfig.from_spec(json.loads(str(g["spec"])))
    c = O.OracleCodec(cfg)
    c.synth(int(g["synth_seed"]))
    return c, g, cfg


def test_codec_tiny_matches_reference(golden):
    c, g, cfg = _codec("codec_tiny", golden)
    wave, lat = c.decode(g["codes"][0], want_latent=True)
    np.testing.assert_allclose(lat, g["latent_fp32"][0], atol=2e-4, rtol=0)
    ref = g["wave_fp32"].reshape(-1)
    assert np.abs(wave - ref).max() < 2e-4


@pytest.mark.slow
def test_codec_full_shapes_matches_reference(golden):
    """Real modded_dac_vq.yaml shapes (1024 latent, 1536 decoder, 8-layer transformer)."""
    c, g, cfg = _codec("codec_full", golden)
    wave = c.decode(g["codes"][0])
    ref = g["wave_fp32"].reshape(-1)
    rms = np.sqrt(np.mean((wave - ref) ** 2))
    assert rms < 1e-3 * np.sqrt(np.mean(ref ** 2)), rms


def test_codec_causal_prefix(golden):
    """rvq.py:374-398-style known answer: decoding a prefix of the codes reproduces the
    prefix of the full decode (the whole decode path is causal)."""
    c, g, cfg = _codec("codec_tiny", golden)
    codes = g["codes"][0]
    full = c.decode(codes)
    h = int(g["prefix_T"])
    pre = c.decode(np.ascontiguousarray(codes[:, :h]))
    assert np.abs(pre - full[: pre.size]).max() < 1e-4


@pytest.mark.slow
def test_bf16_wide_real_widths(golden):
    """S2-Pro widths (d=2560, 32/8 heads x 128, I=9728, V=155776, C=10, cb=4096), 2 slow + 1
    fast layer, synthetic weights: teacher-forced top-1 and logits tolerance in bf16."""
    g = golden("llm_wide_bf16.npz")
    cfg = DualARConfig.from_pretrained(os.path.join(GOLDEN, "llm_wide"))
    cfg.im_end_id = IM_END
    o = O.OracleLLM(cfg, True)
    o.synth(int(g["synth_seed"]), int(g["log2_half"]))
    o.reset()
    T = g["prompt"].shape[1]
    seq, rows = g["seq"], g["slow_rows"]
    x, pos = g["prompt"], 0
    for i in range(seq.shape[1] - T):
        lg, hid = o.forward(x, pos)
        ref = g["slow_logits"][i]
        assert np.abs(lg[rows] - ref).max() < 0.05 * max(1.0, np.abs(ref).max())
        if _margin(ref) > 0.07:
            assert rows[np.argmax(lg[rows])] == rows[np.argmax(ref)]
        col = seq[:, T + i]
        o.fast(hid, -1, 0, logits=False)
        a = int(np.clip(col[0] - cfg.semantic_begin_id, 0, cfg.codebook_size - 1))
        for c in range(1, cfg.num_codebooks):
            fl = o.fast(None, a, c)
            rf = g["fast_logits"][i, c - 1]
            assert np.abs(fl - rf).max() < 0.05 * max(1.0, np.abs(rf).max())
            if _margin(rf) > 0.07:
                assert np.argmax(fl) == np.argmax(rf)
            a = int(col[c + 1])
        pos = T + i
        x = col.reshape(-1, 1)


def _codec_enc(name, golden):
    g = golden(f"{name}.npz")
    spec = json.loads(str(g["spec"]))
    cfg = CodecConfig.from_spec(spec)
    c = O.OracleCodec(cfg)
    c.synth(int(g["synth_seed"]))
    el = [int(v) for v in g["enc_layers"]]
    c.synth_encoder(int(g["synth_seed"]), spec["encoder_dim"], el)
    return c, g, cfg, spec, el


def _codes_match(codes, g, tol):
    """Codes equal to the reference's wherever its nearest/second-nearest margin exceeds tol
    (an fp32 reassociation can only flip a decision closer than that)."""
    ref, margin = g["codes"][0], g["margin"]
    firm = margin > tol
    assert firm.mean() > 0.9
    np.testing.assert_array_equal(codes[firm], ref[firm])
    assert codes.shape == ref.shape and int(g["lens"][0]) == ref.shape[1]


@pytest.mark.parametrize("name", ["codec_enc_tiny", "codec_enc_full"])
def test_codec_encode_matches_reference(name, golden):
    """DAC.encode (modded_dac.py:874-923): encoder output, quantizer input (after downsample +
    pre_module) and all 10 codebooks' codes vs the reference run on the same audio (right-padded
    to a multiple of 2048 samples)."""
    c, g, cfg, spec, el = _codec_enc(name, golden)
    codes, ze, zp = c.encode(g["audio"], spec["encoder_dim"], el[-1], taps=True)
    for got, ref in ((ze, g["z_enc"][0]), (zp, g["z_pre"][0])):
        err = np.sqrt(np.mean((got - ref) ** 2)) / np.sqrt(np.mean(ref ** 2))
        assert err < 1e-4, err
    _codes_match(codes, g, 1e-5)
