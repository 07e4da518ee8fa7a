#!/usr/bin/env python3
"""Generate golden fixtures by running the REAL reference (/root/reference) on CPU.

TEST INFRASTRUCTURE ONLY.  Runs in the survey/dev container (where /root/reference exists);
the GPU box never runs this.  It imports the reference in place (no source is copied),
with the stand-ins of oracle/ref_stubs.py for packages that are absent here, and writes
small data fixtures (inputs + expected outputs) under tests/golden/.

    python oracle/gen_goldens.py all        # everything below
    python oracle/gen_goldens.py llm ops codec codec_full llm_wide

Reference call sites exercised (file:line in /root/reference):
  * BaseModelArgs.from_pretrained / _from_fish_qwen3_omni     llama.py:75-143
  * _remap_fish_qwen3_omni_keys, Attention.load_hook (wq/wk/wv) llama.py:229-246, 876-881
  * generate / decode_one_token_ar / decode_n_tokens (top_k=1) inference.py:96-359
  * forward_generate / forward_generate_fast (teacher forcing)  llama.py:390-466, 798-827
  * RMSNorm, nn.RMSNorm (qk-norm), precompute_freqs_cis,
    apply_rotary_emb                                            llama.py:989-1037
  * logits_to_probs                                             inference.py:54-77
  * DAC.from_indices -> DownsampleResidualVectorQuantize.decode
    -> WindowLimitedTransformer -> upsample -> Decoder          modded_dac.py:925-927, rvq.py:352-366
  * causal-prefix property of the codec (rvq.py:374-398 style)
  * Conversation.encode_for_inference, split_text_by_speaker, group_turns_into_batches and the
    generate_long conversation flow                             conversation.py:39-103,
                                                                content_sequence.py:154-324,
                                                                inference.py:454-707
"""
from __future__ import annotations

import functools
import json
import os
import sys
import time
from collections import OrderedDict

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
GOLD = os.path.join(REPO, "tests", "golden")
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(REPO, "fish-speech_amd"))

import ref_stubs  # noqa: E402
import signals  # noqa: E402

ref_stubs.install()

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402
from safetensors.torch import save_file  # noqa: E402

from fishmi import synth  # noqa: E402

torch.set_num_threads(8)
IM_END_ID = 4


class StubTokenizer:
    """Only what generate()/decode_n_tokens() call: get_token_id(IM_END_TOKEN)."""

    def get_token_id(self, tok):
        assert tok == "<|im_end|>"
        return IM_END_ID


def bf16_tensor(x_f32: np.ndarray, shape) -> torch.Tensor:
    bits = synth.f32_to_bf16_bits(x_f32.reshape(-1))
    return torch.from_numpy(bits.view(np.int16).copy()).view(torch.bfloat16).reshape(shape)


def synth_state(keys_shapes, seed, rule):
    out = OrderedDict()
    for k, shape in keys_shapes:
        n = int(np.prod(shape))
        c, e = rule(k)
        out[k] = bf16_tensor(synth.synth_f32(seed, k, n, c, e), shape)
    return out


# --------------------------------------------------------------------------------------
# Dual-AR LLM
# --------------------------------------------------------------------------------------
LLM_A_CONFIG = {
    "model_type": "fish_qwen3_omni",
    "text_config": {
        "vocab_size": 512, "n_layer": 4, "n_head": 4, "n_local_heads": 2, "head_dim": 32,
        "dim": 128, "intermediate_size": 256, "rope_base": 1000000, "norm_eps": 1e-6,
        "max_seq_len": 256, "tie_word_embeddings": True, "attention_qkv_bias": False,
        "attention_o_bias": False, "attention_qk_norm": True,
    },
    "audio_decoder_config": {
        "vocab_size": 128, "num_codebooks": 10, "n_layer": 2, "dim": 128, "n_head": 4,
        "n_local_heads": 2, "head_dim": 32, "intermediate_size": 256,
    },
    "semantic_start_token_id": 200,
    "semantic_end_token_id": 327,
}

LLM_B_CONFIG = {
    "model_type": "dual_ar",
    "vocab_size": 400, "n_layer": 3, "n_head": 4, "n_local_heads": 1, "head_dim": 32,
    "dim": 128, "intermediate_size": 320, "rope_base": 10000, "norm_eps": 1e-5,
    "max_seq_len": 192, "tie_word_embeddings": False, "attention_qkv_bias": True,
    "attention_o_bias": True, "attention_qk_norm": False, "codebook_size": 64,
    "num_codebooks": 6, "semantic_begin_id": 300, "semantic_end_id": 363,
    "n_fast_layer": 2, "fast_dim": 96, "fast_n_head": 3, "fast_n_local_heads": 1,
    "fast_head_dim": 32, "fast_intermediate_size": 192, "scale_codebook_embeddings": False,
    "norm_fastlayer_input": False,
}


def to_qwen3_omni_key(k: str) -> str:
    """Inverse of llama.py:229-246 _remap_fish_qwen3_omni_keys (to store fixtures the
    way an S2-Pro checkpoint stores them)."""
    if k.startswith("codebook_embeddings."):
        return "audio_decoder." + k
    if k.startswith("fast_"):
        return "audio_decoder." + k[len("fast_"):]
    return "text_model.model." + k


def build_llm(config: dict, weights_dir: str | None, seed: int, log2_half: int):
    from fish_speech.models.text2semantic import llama

    cfg_path = os.path.join(weights_dir or "/tmp/fishmi_cfg", "config.json")
    os.makedirs(os.path.dirname(cfg_path), exist_ok=True)
    with open(cfg_path, "w") as f:
        json.dump(config, f, indent=1)
    cfg = llama.BaseModelArgs.from_pretrained(cfg_path)
    torch.manual_seed(0)
    model = llama.DualARTransformer(cfg)
    keys = [(k, tuple(v.shape)) for k, v in model.state_dict().items()]
    state = synth_state(keys, seed, functools.partial(synth.llm_rule, log2_half_linear=log2_half))
    if weights_dir is not None:
        # store as an S2-Pro style checkpoint: qwen3-omni key layout, 2 shards + index,
        # and layer 0's attention split into wq/wk/wv (exercises Attention.load_hook).
        stored = OrderedDict()
        for k, v in state.items():
            if k == "layers.0.attention.wqkv.weight":
                qs = cfg.n_head * cfg.head_dim
                ks = cfg.n_local_heads * cfg.head_dim
                stored[to_qwen3_omni_key("layers.0.attention.wq.weight")] = v[:qs].contiguous()
                stored[to_qwen3_omni_key("layers.0.attention.wk.weight")] = v[qs:qs + ks].contiguous()
                stored[to_qwen3_omni_key("layers.0.attention.wv.weight")] = v[qs + ks:].contiguous()
            else:
                stored[to_qwen3_omni_key(k)] = v
        names = list(stored)
        half = len(names) // 2
        shards = {"model-00001-of-00002.safetensors": names[:half],
                  "model-00002-of-00002.safetensors": names[half:]}
        wmap = {}
        for fn, ns in shards.items():
            save_file({n: stored[n] for n in ns}, os.path.join(weights_dir, fn))
            wmap.update({n: fn for n in ns})
        with open(os.path.join(weights_dir, "model.safetensors.index.json"), "w") as f:
            json.dump({"metadata": {}, "weight_map": wmap}, f, indent=1)
        # load back exactly the way from_pretrained does (llama.py:550-586)
        from safetensors.torch import load_file

        loaded = OrderedDict()
        for fn in sorted(set(wmap.values())):
            loaded.update(load_file(os.path.join(weights_dir, fn), device="cpu"))
        loaded = llama._remap_fish_qwen3_omni_keys(loaded)
        err = model.load_state_dict(loaded, strict=False, assign=True)
    else:
        err = model.load_state_dict(state, strict=False, assign=True)
    assert not err.missing_keys and not err.unexpected_keys, err
    model.tokenizer = StubTokenizer()
    return model.eval()


def make_prompt(cfg, T: int, seed: int) -> torch.Tensor:
    """(C+1, T) int64 prompt: text tokens, an im_start, a run of semantic frames with codes,
    and more text (covers the codebook-embedding branch in prefill, llama.py:399-420)."""
    rng = np.random.default_rng(seed)
    C = cfg.num_codebooks
    p = np.zeros((C + 1, T), dtype=np.int64)
    p[0] = rng.integers(16, cfg.semantic_begin_id, size=T)
    p[0, 0] = 1
    s0, s1 = T // 3, T // 3 + max(3, T // 4)
    codes0 = rng.integers(0, cfg.codebook_size, size=s1 - s0)
    p[0, s0:s1] = cfg.semantic_begin_id + codes0
    p[1, s0:s1] = codes0
    p[2:, s0:s1] = rng.integers(0, cfg.codebook_size, size=(C - 1, s1 - s0))
    p[0, s1] = IM_END_ID
    return torch.from_numpy(p)


def teacher_forced(model, seq: torch.Tensor, T: int, nsteps: int, dtype):
    """Per-frame slow logits (+ semantic bias) and fast logits, replaying decode_one_token_ar
    (inference.py:96-181) with the reference's own emitted columns as the sampled tokens."""
    from torch.nn.attention import SDPBackend, sdpa_kernel

    cfg = model.config
    C, V, cb = cfg.num_codebooks, cfg.vocab_size, cfg.codebook_size
    model._cache_setup_done = False
    model.setup_caches(1, cfg.max_seq_len, dtype=dtype)
    with torch.inference_mode():  # zero the caches left by the free-running generate()
        for b in list(model.layers) + list(model.fast_layers):
            b.attention.kv_cache.k_cache.zero_()
            b.attention.kv_cache.v_cache.zero_()
    bias = torch.full((1, 1, V), float("-inf"), dtype=dtype)
    bias[0, 0, cfg.semantic_begin_id: cfg.semantic_end_id + 1] = 0.0
    bias[0, 0, IM_END_ID] = 0.0
    slow_all, fast_all, hid_all = [], [], []
    x = seq[:, :T].view(1, C + 1, T)
    pos = torch.arange(T)
    for i in range(nsteps):
        col = seq[:, T + i]
        ctx = sdpa_kernel(SDPBackend.MATH) if i > 0 else _nullctx()
        with ctx, torch.inference_mode():
            fr = model.forward_generate(x, pos)
            slow = (fr.logits + bias)[0, -1].float().numpy().copy()
            h = fr.hidden_states
            hid_all.append(h.reshape(-1).float().numpy().copy())
            model.forward_generate_fast(h, torch.tensor([0]))
            a = torch.clamp(col[0:1] - cfg.semantic_begin_id, 0, cb - 1)
            hs = model.fast_embeddings(a)
            fl = []
            for c in range(1, C):
                lg = model.forward_generate_fast(hs, torch.tensor([c]))
                fl.append(lg.reshape(-1).float().numpy().copy())
                hs = model.fast_embeddings(col[c + 1: c + 2])
        slow_all.append(slow)
        fast_all.append(np.stack(fl))
        x = col.view(1, C + 1, 1)
        pos = torch.tensor([T + i])
    return np.stack(slow_all), np.stack(fast_all), np.stack(hid_all)


class _nullctx:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


def run_llm_case(name, config, weights_dir, seed, log2_half, T, n_new, dtypes, prompt_seed):
    from fish_speech.models.text2semantic import inference

    for dtype in dtypes:
        model = build_llm(config, weights_dir, seed, log2_half).to(dtype)
        cfg = model.config
        prompt = make_prompt(cfg, T, prompt_seed)
        t0 = time.time()
        seq = inference.generate(model=model, prompt=prompt.clone(), max_new_tokens=n_new,
                                 audio_masks=None, audio_parts=None, temperature=0.7,
                                 top_p=0.9, top_k=1)
        n = seq.shape[1] - T
        slow, fast, hid = teacher_forced(model, seq, T, n, dtype)
        tag = {torch.float32: "fp32", torch.bfloat16: "bf16"}[dtype]
        out = os.path.join(GOLD, f"{name}_{tag}.npz")
        extra = {}
        if dtype == torch.bfloat16:
            # the same teacher-forced stream through the fp32 model: the reference's own bf16 error
            # (slow/fast bf16 - fp32) is the bound a bf16 build is held to (tests/test_gpu_llm.py)
            m32 = build_llm(config, weights_dir, seed, log2_half).to(torch.float32)
            s32, f32, _ = teacher_forced(m32, seq, T, n, torch.float32)
            extra = dict(slow_logits_f32=s32, fast_logits_f32=f32)
        np.savez_compressed(out, prompt=prompt.numpy().astype(np.int32),
                            seq=seq.numpy().astype(np.int32), slow_logits=slow,
                            fast_logits=fast, hidden=hid, synth_seed=seed,
                            log2_half=log2_half, torch_version=torch.__version__,
                            threads=torch.get_num_threads(), **extra)
        print(f"{name} {tag}: T={T} generated {n} frames in {time.time() - t0:.1f}s -> {out}")
        print("  first columns:", seq[:, T:T + 3].T.tolist())


def cmd_llm():
    wdir = os.path.join(GOLD, "llm_a")
    os.makedirs(wdir, exist_ok=True)
    run_llm_case("llm_a", LLM_A_CONFIG, wdir, seed=11, log2_half=3, T=24, n_new=32,
                 dtypes=[torch.float32, torch.bfloat16], prompt_seed=1)
    bdir = os.path.join(GOLD, "llm_b")
    os.makedirs(bdir, exist_ok=True)
    with open(os.path.join(bdir, "config.json"), "w") as f:
        json.dump(LLM_B_CONFIG, f, indent=1)
    run_llm_case("llm_b", LLM_B_CONFIG, None, seed=23, log2_half=3, T=17, n_new=24,
                 dtypes=[torch.float32, torch.bfloat16], prompt_seed=2)


# --------------------------------------------------------------------------------------
# Per-op goldens
# --------------------------------------------------------------------------------------
def cmd_ops():
    from fish_speech.models.text2semantic import inference, llama

    rng = np.random.default_rng(5)
    out = {}
    # RMSNorm (llama.py:989-1000): fp32 normalise, round to bf16, * bf16 weight
    x = torch.from_numpy(rng.normal(0, 3, (6, 256)).astype(np.float32)).bfloat16()
    m = llama.RMSNorm(256, eps=1e-6)
    m.weight.data = torch.from_numpy(rng.normal(1, 0.2, 256).astype(np.float32)).bfloat16()
    with torch.no_grad():
        out["rms_x"], out["rms_w"], out["rms_y"] = x.float(), m.weight.float(), m(x).float()
        out["rms_y32"] = m.float()(x.float()).float()  # the fp32 model on the same values
    # qk-norm nn.RMSNorm(head_dim) on bf16 (llama.py:861-863)
    q = torch.from_numpy(rng.normal(0, 2, (2, 3, 4, 64)).astype(np.float32)).bfloat16()
    qn = torch.nn.RMSNorm(64, 1e-6).bfloat16()
    qn.weight.data = torch.from_numpy(rng.normal(1, 0.2, 64).astype(np.float32)).bfloat16()
    with torch.no_grad():
        out["qk_x"], out["qk_w"], out["qk_y"] = q.float(), qn.weight.float(), qn(q).float()
        out["qk_y32"] = qn.float()(q.float()).float()
    # RoPE (llama.py:1003-1037)
    fc = llama.precompute_freqs_cis(64, 32, 10000)
    out["rope_table"] = fc.float()
    xr = torch.from_numpy(rng.normal(0, 1, (1, 5, 4, 32)).astype(np.float32)).bfloat16()
    pos = torch.tensor([0, 3, 17, 40, 63])
    out["rope_pos"] = pos.to(torch.int32)
    out["rope_x"] = xr.float()
    out["rope_y"] = llama.apply_rotary_emb(xr, fc[pos]).float()
    out["rope_y32"] = llama.apply_rotary_emb(xr.float(), fc[pos]).float()
    # Dual-AR input embedding (llama.py:399-420) captured at the first block's input, llm_a shapes
    # (fish_qwen3_omni: scale_codebook_embeddings) with the synthetic weights of seed 11
    for tag, dt in (("", torch.bfloat16), ("32", torch.float32)):
        em = build_llm(LLM_A_CONFIG, None, seed=11, log2_half=3).to(dt)
        ecfg = em.config
        inp = make_prompt(ecfg, 20, 8).view(1, ecfg.num_codebooks + 1, 20)
        got = {}
        h = em.layers[0].register_forward_pre_hook(lambda mod, args: got.update(x=args[0].clone()))
        with torch.no_grad():
            em.forward_generate(inp)
        h.remove()
        out["emb_tok"] = inp[0].numpy().astype(np.int32)
        out["emb_x" + tag] = got["x"][0].float()
    fc2 = llama.precompute_freqs_cis(4096, 128, 1000000)
    out["rope_table_big"] = fc2[::97].float()
    # logits_to_probs (inference.py:54-77) with bf16 temperature / top_p tensors
    cases = [(0.7, 0.9, 30), (1.0, 0.9, 30), (0.7, 0.5, 5), (0.7, 0.9, 1), (0.3, 0.99, 64),
             (1.0, 0.9, 30)]
    lp_in, lp_out, lp_par = [], [], []
    for ci, (t, p, k) in enumerate(cases):
        lg = rng.normal(0, 2.0, 300).astype(np.float32)
        lg[rng.integers(0, 300, 8)] = lg.max()          # ties at the top
        if ci == 5:
            lg[:100] = -np.inf                           # constrained-bias style row
        lgt = torch.from_numpy(lg).bfloat16()
        probs = inference.logits_to_probs(lgt, torch.tensor(t).bfloat16(),
                                          torch.tensor(p).bfloat16(), k)
        lp_in.append(lgt.float().numpy())
        lp_out.append(probs.float().numpy())
        lp_par.append([t, p, k])
    out["lp_logits"] = np.stack(lp_in)
    out["lp_probs"] = np.stack(lp_out)
    out["lp_params"] = np.array(lp_par, dtype=np.float64)
    # argmax tie order of sample() under top_k=1 (sort order of ties)
    lg = torch.zeros(64).bfloat16()
    lg[[5, 9, 40]] = 3.0
    idx, _ = inference.sample(lg.view(1, 1, -1), torch.tensor(0.7).bfloat16(),
                              torch.tensor(0.9).bfloat16(), 1)
    out["tie_logits"] = lg.float()
    out["tie_idx"] = idx.to(torch.int32)
    np.savez_compressed(os.path.join(GOLD, "ops.npz"),
                        **{k: (v.numpy() if torch.is_tensor(v) else v) for k, v in out.items()},
                        torch_version=torch.__version__)
    print("ops: tie idx", int(idx), "->", os.path.join(GOLD, "ops.npz"))


# --------------------------------------------------------------------------------------
# Codec (modded DAC decode)
# --------------------------------------------------------------------------------------
CODEC_TINY = dict(encoder_dim=8, latent=128, decoder_dim=256, n_codebooks=9, codebook_size=32,
                  semantic_codebook_size=64, codebook_dim=8, t_layers=2, t_heads=2,
                  t_head_dim=64, t_inter=384, window=16)
CODEC_FULL = dict(encoder_dim=64, latent=1024, decoder_dim=1536, n_codebooks=9,
                  codebook_size=1024, semantic_codebook_size=4096, codebook_dim=8,
                  t_layers=8, t_heads=16, t_head_dim=64, t_inter=3072, window=128)


def build_codec(spec: dict, seed: int, enc_layers=None):
    from fish_speech.models.dac.modded_dac import DAC, ModelArgs, WindowLimitedTransformer
    from fish_speech.models.dac.rvq import DownsampleResidualVectorQuantize

    tcfg = ModelArgs(block_size=2048, n_layer=spec["t_layers"], n_head=spec["t_heads"],
                     dim=spec["latent"], intermediate_size=spec["t_inter"], n_local_heads=-1,
                     head_dim=spec["t_head_dim"], rope_base=10000, norm_eps=1e-5,
                     dropout_rate=0.1, attn_dropout_rate=0.1, channels_first=True)
    post = WindowLimitedTransformer(causal=True, window_size=spec["window"],
                                    input_dim=spec["latent"], config=tcfg)
    quant = DownsampleResidualVectorQuantize(
        input_dim=spec["latent"], n_codebooks=spec["n_codebooks"],
        codebook_size=spec["codebook_size"], codebook_dim=spec["codebook_dim"],
        quantizer_dropout=0.5, downsample_factor=[2, 2], post_module=post,
        pre_module=(WindowLimitedTransformer(causal=True, window_size=spec["window"], input_dim=spec["latent"],
                                             config=tcfg) if enc_layers else None),
        semantic_codebook_size=spec["semantic_codebook_size"])
    gen = functools.partial(ModelArgs, block_size=8192, n_local_heads=-1, head_dim=64,
                            rope_base=10000, norm_eps=1e-5, dropout_rate=0.1,
                            attn_dropout_rate=0.1, channels_first=True)
    dac = DAC(encoder_dim=spec["encoder_dim"], encoder_rates=[2, 4, 8, 8],
              decoder_dim=spec["decoder_dim"], decoder_rates=[8, 8, 4, 2], quantizer=quant,
              sample_rate=44100, causal=True, encoder_transformer_layers=enc_layers or [0, 0, 0, 0],
              decoder_transformer_layers=[0, 0, 0, 0], transformer_general_config=gen)
    sd = dac.state_dict()
    keys = [(k, tuple(v.shape)) for k, v in sd.items()
            if enc_layers or k.startswith("decoder.") or k.startswith("quantizer.")]
    state = synth_state(keys, seed, synth.codec_rule)
    state = OrderedDict((k, v.float()) for k, v in state.items())
    err = dac.load_state_dict(state, strict=False)
    assert not err.unexpected_keys, err.unexpected_keys
    missing = [k for k in err.missing_keys if enc_layers or not k.startswith("encoder.")]
    assert not missing, missing
    return dac.eval()


def codec_codes(spec, T, seed):
    return signals.codec_codes(spec["n_codebooks"], spec["semantic_codebook_size"], spec["codebook_size"],
                               T, seed)


def run_codec(name, spec, seed, T, clamp_test: bool):
    dac = build_codec(spec, seed)
    codes = codec_codes(spec, T, seed + 1)
    if clamp_test:  # out-of-range codes are clamped in place by rvq.py:354-359
        codes[0, 0, 3] = spec["semantic_codebook_size"] + 9
        codes[0, 2, 5] = spec["codebook_size"] + 3
    res = {"codes": codes.astype(np.int32), "synth_seed": seed, "spec": json.dumps(spec),
           "torch_version": torch.__version__}
    with torch.inference_mode():
        t0 = time.time()
        y32 = dac.from_indices(torch.from_numpy(codes.copy()))
        res["wave_fp32"] = y32.float().numpy()
        dt = time.time() - t0
        half = T // 2
        yp = dac.from_indices(torch.from_numpy(codes[..., :half].copy()))
        res["prefix_T"] = half
        res["prefix_maxdiff"] = float((yp - y32[..., :yp.shape[-1]]).abs().max())
        # intermediate: latent after RVQ decode + post transformer + upsample (B,1024,4T)
        z = dac.quantizer.decode(torch.from_numpy(codes.copy()))
        res["latent_fp32"] = z.float().numpy()
        dac_bf = dac.to(torch.bfloat16)
        ybf = dac_bf.from_indices(torch.from_numpy(codes.copy()))
        res["wave_bf16"] = ybf.float().numpy()
    np.savez_compressed(os.path.join(GOLD, f"{name}.npz"), **res)
    print(f"{name}: T={T} -> {res['wave_fp32'].shape} fp32 {dt:.1f}s; prefix maxdiff "
          f"{res['prefix_maxdiff']:.3g}; bf16-vs-fp32 rms "
          f"{np.sqrt(np.mean((res['wave_bf16'] - res['wave_fp32'])**2)):.3g} "
          f"(signal rms {np.sqrt(np.mean(res['wave_fp32']**2)):.3g})")


# --------------------------------------------------------------------------------------
# Codec ENCODE: DAC.encode (modded_dac.py:874-923) = Encoder
# (modded_dac.py:623-709) + DownsampleResidualVectorQuantize.forward (rvq.py:293-343) with the
# descript 1.0.0 VQ encode restated in ref_stubs (parity at that boundary unpinned, as for decode)
# --------------------------------------------------------------------------------------
def encode_audio(n, seed):
    return signals.reference_audio(n, seed)


def run_codec_enc(name, spec, seed, n_samples, enc_layers, tail_steps=None):
    """tail_steps: keep only the last `tail_steps` encoder-transformer steps of the z_enc taps and
    regenerate the audio in the test (signals.reference_audio(n_samples, audio_seed)), so a long
    clip's fixture stays small."""
    dac = build_codec(spec, seed, enc_layers)
    audio = encode_audio(n_samples, seed + 2)
    margins = []

    def track(vq):
        orig = vq.decode_latents

        def dl(latents):
            enc = F.normalize(latents.transpose(1, 2).reshape(-1, latents.shape[1]))
            cbk = F.normalize(vq.codebook.weight)
            dist = enc.pow(2).sum(1, keepdim=True) - 2 * enc @ cbk.t() + cbk.pow(2).sum(1, keepdim=True).t()
            top2 = torch.topk(-dist, 2, dim=1).values
            margins.append((top2[:, 0] - top2[:, 1]).float().numpy().copy())
            return orig(latents)

        vq.decode_latents = dl

    for vq in list(dac.quantizer.semantic_quantizer.quantizers) + list(dac.quantizer.quantizer.quantizers):
        track(vq)
    res = {"audio": audio, "synth_seed": seed, "spec": json.dumps(spec), "audio_seed": seed + 2,
           "n_samples": n_samples, "enc_layers": np.array(enc_layers, np.int32),
           "torch_version": torch.__version__}
    with torch.inference_mode():
        x = torch.from_numpy(audio)[None, None]
        t0 = time.time()
        codes, lens = dac.encode(x)
        dt = time.time() - t0
        res["codes"] = codes.numpy().astype(np.int32)
        res["lens"] = lens.numpy().astype(np.int32)
        res["margin"] = np.stack(margins[:codes.shape[1]], 0).astype(np.float32)  # [nq+1][T]
        # intermediate taps: encoder output (before the quantizer) and the quantizer's input to
        # the first VQ stage (after downsample + pre_module)
        pad = (-audio.shape[0]) % dac.frame_length
        xp = F.pad(x, (0, pad))
        z = dac.encoder(xp)
        res["z_enc"] = z.float().numpy()
        zq = dac.quantizer.pre_module(dac.quantizer.downsample(z))
        res["z_pre"] = zq.float().numpy()
        # the reference's own bf16 run (the bound a bf16 build is held to)
        dac_bf = dac.to(torch.bfloat16)
        res["z_enc_bf16"] = dac_bf.encoder(xp.bfloat16()).float().numpy()
        res["codes_bf16"] = dac_bf.encode(x.bfloat16())[0].numpy().astype(np.int32)
    if tail_steps:
        del res["audio"]
        for k in ("z_enc", "z_enc_bf16"):
            res[k] = np.ascontiguousarray(res[k][..., -tail_steps:])
        res["tail_steps"] = tail_steps
    np.savez_compressed(os.path.join(GOLD, f"{name}.npz"), **res)
    print(f"{name}: {n_samples} samples -> codes {res['codes'].shape} in {dt:.1f}s; "
          f"min margin {res['margin'].min():.3g}; z_enc {res['z_enc'].shape} z_pre {res['z_pre'].shape}")


def cmd_codec_enc():
    run_codec_enc("codec_enc_tiny", CODEC_TINY, seed=41, n_samples=6 * 2048 - 700, enc_layers=[0, 0, 0, 2])


def cmd_codec_enc_full():
    run_codec_enc("codec_enc_full", CODEC_FULL, seed=43, n_samples=8 * 2048 - 300, enc_layers=[0, 0, 0, 4])


def cmd_codec_enc_long():
    """160 code frames = 640 encoder-transformer steps (7.4 s): the encoder transformer's 512-step
    causal window (modded_dac.py:380-398) is crossed, as in config 5's 30 s clip."""
    run_codec_enc("codec_enc_long", CODEC_FULL, seed=47, n_samples=160 * 2048 - 300, enc_layers=[0, 0, 0, 4],
                  tail_steps=96)


def cmd_codec_keys():
    """The state_dict key layout of the reference's own DAC at the real modded_dac_vq.yaml dims with
    the encoder (enc_layers [0,0,0,4]): names and shapes only. Loader tests push a checkpoint with
    exactly this layout through FishMICodec.from_checkpoint (dac/inference.py:23-47)."""
    dac = build_codec(CODEC_FULL, 1, [0, 0, 0, 4])
    keys = [[k, list(v.shape), str(v.dtype)] for k, v in dac.state_dict().items()]
    with open(os.path.join(GOLD, "codec_keys.json"), "w") as f:
        json.dump({"spec": CODEC_FULL, "enc_layers": [0, 0, 0, 4], "torch_version": torch.__version__,
                   "keys": keys}, f, indent=0)
    print(f"codec_keys: {len(keys)} tensors")


def cmd_codec():
    run_codec("codec_tiny", CODEC_TINY, seed=31, T=12, clamp_test=True)


def cmd_codec_full():
    run_codec("codec_full", CODEC_FULL, seed=37, T=4, clamp_test=False)


def cmd_codec_long():
    """Config-2 length (216 frames = 10 s) at the real modded_dac_vq.yaml shapes, so the post
    transformer's 128-frame causal window (modded_dac.py:380-398) is crossed.  The waveform is kept
    at two segments (frames [0, 8) and the last 40), in three reference modes: fp32; the CLI's
    dac.to(bf16) (inference.py:416); and the engine's autocast(bf16) over fp32 weights
    (vq_manager.py:16-21, fish_speech/inference_engine/__init__.py:179-192; CPU autocast here)."""
    spec, seed, T, head, tail = CODEC_FULL, 37, 216, 8, 40
    dac = build_codec(spec, seed)
    codes = codec_codes(spec, T, seed + 101)
    segs = lambda y: np.concatenate([y.reshape(-1)[: head * 2048], y.reshape(-1)[(T - tail) * 2048:]])
    res = {"codes": codes.astype(np.int32), "synth_seed": seed, "spec": json.dumps(spec),
           "torch_version": torch.__version__, "head_frames": head, "tail_frames": tail}
    with torch.inference_mode():
        t0 = time.time()
        y32 = dac.from_indices(torch.from_numpy(codes.copy())).float().numpy()
        res["wave_fp32"] = segs(y32)
        print(f"codec_long fp32 {time.time() - t0:.1f}s")
        with torch.autocast(device_type="cpu", dtype=torch.bfloat16):
            ya = dac.from_indices(torch.from_numpy(codes.copy())).float().numpy()
        res["wave_autocast"] = segs(ya)
        ybf = dac.to(torch.bfloat16).from_indices(torch.from_numpy(codes.copy())).float().numpy()
        res["wave_bf16"] = segs(ybf)
    for k in ("wave_bf16", "wave_autocast"):
        e = res[k] - res["wave_fp32"]
        res[k + "_rms_err"] = float(np.sqrt(np.mean(e.astype(np.float64) ** 2)))
        res[k + "_stft_db"] = signals.stft_logmag_error_db(res[k][head * 2048:], res["wave_fp32"][head * 2048:])
    np.savez_compressed(os.path.join(GOLD, "codec_long.npz"), **res)
    print(f"codec_long: T={T} in {time.time() - t0:.1f}s; signal rms {np.sqrt(np.mean(res['wave_fp32'] ** 2)):.4g}; "
          f"bf16 rms err {res['wave_bf16_rms_err']:.4g} ({res['wave_bf16_stft_db']:.4g} dB); autocast rms err "
          f"{res['wave_autocast_rms_err']:.4g} ({res['wave_autocast_stft_db']:.4g} dB)")


# --------------------------------------------------------------------------------------
# LLM at the real S2-Pro widths, reduced depth (synthetic weights, nothing committed but
# the outputs).  Shapes per SURVEY.md §2.3.
# --------------------------------------------------------------------------------------
LLM_WIDE_CONFIG = {
    "model_type": "fish_qwen3_omni",
    "text_config": {
        "vocab_size": 155776, "n_layer": 2, "n_head": 32, "n_local_heads": 8,
        "head_dim": 128, "dim": 2560, "intermediate_size": 9728, "rope_base": 1000000,
        "norm_eps": 1e-6, "max_seq_len": 128, "tie_word_embeddings": True,
        "attention_qkv_bias": False, "attention_o_bias": False, "attention_qk_norm": True,
    },
    "audio_decoder_config": {
        "vocab_size": 4096, "num_codebooks": 10, "n_layer": 1, "dim": 2560, "n_head": 32,
        "n_local_heads": 8, "head_dim": 128, "intermediate_size": 9728,
    },
    "semantic_start_token_id": 151678,
    "semantic_end_token_id": 155773,
}


def cmd_llm_wide():
    os.makedirs(os.path.join(GOLD, "llm_wide"), exist_ok=True)
    with open(os.path.join(GOLD, "llm_wide", "config.json"), "w") as f:
        json.dump(LLM_WIDE_CONFIG, f, indent=1)
    from fish_speech.models.text2semantic import inference

    T = 64  # >= 64 prompt tokens, then 16 single-column decode steps (SURVEY.md §8d config 2 shape)
    model = build_llm(LLM_WIDE_CONFIG, None, seed=41, log2_half=5).to(torch.bfloat16)
    cfg = model.config
    prompt = make_prompt(cfg, T, 3)
    t0 = time.time()
    seq = inference.generate(model=model, prompt=prompt.clone(), max_new_tokens=17,
                             audio_masks=None, audio_parts=None, temperature=0.7, top_p=0.9,
                             top_k=1)
    n = seq.shape[1] - T
    slow, fast, hid = teacher_forced(model, seq, T, n, torch.bfloat16)
    del model
    m32 = build_llm(LLM_WIDE_CONFIG, None, seed=41, log2_half=5).to(torch.float32)
    s32, f32, _ = teacher_forced(m32, seq, T, n, torch.float32)
    del m32
    # keep the constrained rows only (semantic range + im_end); the rest are -inf
    keep = np.r_[IM_END_ID, cfg.semantic_begin_id:cfg.semantic_end_id + 1]
    np.savez_compressed(os.path.join(GOLD, "llm_wide_bf16.npz"),
                        prompt=prompt.numpy().astype(np.int32), seq=seq.numpy().astype(np.int32),
                        slow_rows=keep.astype(np.int32), slow_logits=slow[:, keep],
                        fast_logits=fast, hidden=hid, slow_logits_f32=s32[:, keep], fast_logits_f32=f32,
                        synth_seed=41, log2_half=5, torch_version=torch.__version__,
                        threads=torch.get_num_threads())
    e_s = np.abs(slow[:, keep] - s32[:, keep])
    print(f"llm_wide: T={T}, {n} frames in {time.time() - t0:.1f}s; reference bf16-vs-fp32 slow logits "
          f"max {e_s.max():.4g} rms {np.sqrt((e_s ** 2).mean()):.4g}; first cols", seq[:, T:T + 2].T.tolist())


# --------------------------------------------------------------------------------------
# The configurations the bench times (round 3): BASELINE config 2 at FULL S2-Pro depth (36 slow
# + 4 fast layers), a >= 3000-token context at S2-Pro widths (config 5's flash-decode regime),
# and config 3's ragged batch (32 prompts of uniform 16..256 tokens, seed 2).  Weights are the
# synthetic rule of fishmi.synth (regenerated on the device from the seed), so only prompts,
# the reference's columns and its teacher-forced logits are stored: slow logits for the 4097
# rows the semantic bias leaves finite, the bf16 ones as exact bf16 bit patterns.
# --------------------------------------------------------------------------------------
def _wide_config(n_layer, n_fast_layer, max_seq_len):
    import copy as _copy

    c = _copy.deepcopy(LLM_WIDE_CONFIG)
    c["text_config"]["n_layer"] = n_layer
    c["text_config"]["max_seq_len"] = max_seq_len
    c["audio_decoder_config"]["n_layer"] = n_fast_layer
    return c


def _llm_state(config, seed, log2_half):
    """The synthetic bf16 state dict of a config (built once, shared by the bf16 and fp32 models)."""
    from fish_speech.models.text2semantic import llama

    cfg_path = os.path.join("/tmp/fishmi_cfg", "config.json")
    os.makedirs(os.path.dirname(cfg_path), exist_ok=True)
    with open(cfg_path, "w") as f:
        json.dump(config, f, indent=1)
    cfg = llama.BaseModelArgs.from_pretrained(cfg_path)
    with torch.device("meta"):
        keys = [(k, tuple(v.shape)) for k, v in llama.DualARTransformer(cfg).state_dict().items()]
    return cfg, synth_state(keys, seed, functools.partial(synth.llm_rule, log2_half_linear=log2_half))


def _llm_from_state(cfg, state, dtype):
    """bf16: the state's tensors assigned (no copy); fp32: copied into fp32 parameters (the same as
    build_llm(...).to(torch.float32), without a second full-size bf16 copy)."""
    from fish_speech.models.text2semantic import llama

    torch.manual_seed(0)
    model = llama.DualARTransformer(cfg)
    err = model.load_state_dict(state, strict=False, assign=(dtype == torch.bfloat16))
    assert not err.missing_keys and not err.unexpected_keys, err
    model.tokenizer = StubTokenizer()
    return model.to(dtype).eval()


def _bf16_bits(x: np.ndarray) -> np.ndarray:
    b = synth.f32_to_bf16_bits(x)
    assert np.array_equal(synth.bf16_bits_to_f32(b), x)  # the reference's bf16 logits are bf16-exact
    return b


def _timed_case(out_name, config, T, n_new, prompt_seed, fast_last_only=False):
    """fast_last_only: keep the fast logits of the last codebook only (long runs: its pass reads
    every fast cache position), as fast_last_bits / fast_last_f32."""
    from fish_speech.models.text2semantic import inference

    t0 = time.time()
    cfg, state = _llm_state(config, 41, 5)
    print(f"{out_name}: synthetic state in {time.time() - t0:.0f}s")
    model = _llm_from_state(cfg, state, torch.bfloat16)
    prompt = make_prompt(cfg, T, prompt_seed)
    seq = inference.generate(model=model, prompt=prompt.clone(), max_new_tokens=n_new, audio_masks=None,
                             audio_parts=None, temperature=0.7, top_p=0.9, top_k=1)
    n = seq.shape[1] - T
    slow, fast, _ = teacher_forced(model, seq, T, n, torch.bfloat16)
    del model
    print(f"{out_name}: bf16 generate + teacher forcing done at {time.time() - t0:.0f}s")
    m32 = _llm_from_state(cfg, state, torch.float32)
    del state
    s32, f32, _ = teacher_forced(m32, seq, T, n, torch.float32)
    del m32
    keep = np.r_[IM_END_ID, cfg.semantic_begin_id:cfg.semantic_end_id + 1]
    fast_fields = dict(fast_last_bits=_bf16_bits(fast[:, -1]), fast_last_f32=f32[:, -1]) if fast_last_only else \
        dict(fast_logits_bits=_bf16_bits(fast), fast_logits_f32=f32)
    np.savez_compressed(os.path.join(GOLD, f"{out_name}.npz"), config=np.array(json.dumps(config)),
                        prompt=prompt.numpy().astype(np.int32), seq=seq.numpy().astype(np.int32),
                        slow_rows=keep.astype(np.int32), slow_logits_bits=_bf16_bits(slow[:, keep]),
                        slow_logits_f32=s32[:, keep], synth_seed=41, log2_half=5,
                        torch_version=torch.__version__, threads=torch.get_num_threads(), **fast_fields)
    e_s = np.abs(slow[:, keep] - s32[:, keep])
    print(f"{out_name}: T={T}, {n} frames in {time.time() - t0:.0f}s; reference bf16-vs-fp32 slow logits max "
          f"{e_s.max():.4g} rms {np.sqrt((e_s ** 2).mean()):.4g}; first cols", seq[:, T:T + 2].T.tolist())


def cmd_llm_full():
    """Config 2 at full depth: 36 slow + 4 fast layers, 64-token prompt, prefill + 8 frames."""
    _timed_case("llm_full_bf16", _wide_config(36, 4, 128), T=64, n_new=9, prompt_seed=3)


def cmd_llm_full64():
    """Config 2 at full depth over 64 decode frames (positions 64..128): prefill + 64 frames,
    every frame's slow logits and the last codebook's fast logits."""
    _timed_case("llm_full64_bf16", _wide_config(36, 4, 160), T=64, n_new=65, prompt_seed=7, fast_last_only=True)


def cmd_llm_full216():
    """Config 2's bench run at full depth: prefill + 216 decode frames (positions 64..280, the
    positions bench.py decodes to), every frame's slow logits and the last codebook's fast logits."""
    _timed_case("llm_full216_bf16", _wide_config(36, 4, 296), T=64, n_new=217, prompt_seed=11, fast_last_only=True)


def cmd_llm_long4():
    """A 3000-token context through 4 slow layers (+ 1 fast) at S2-Pro widths."""
    _timed_case("llm_long4_bf16", _wide_config(4, 1, 3072), T=3000, n_new=7, prompt_seed=9)


def cmd_llm_long():
    """A 3000-token context at S2-Pro widths (2 slow + 1 fast layers): every decode frame's slow
    attention spans many flash-decode splits."""
    _timed_case("llm_long_bf16", _wide_config(2, 1, 3072), T=3000, n_new=7, prompt_seed=5)


def cmd_llm_ragged64():
    """Config 3's ragged batch over 64 decode frames (positions up to 256 + 64): the same 32
    prompt lengths as llm_ragged, each run by the reference at batch 1; greedy columns for all 65
    frames, teacher-forced logits (slow rows + the last codebook's fast logits) kept at frames 0,
    32 and 64 (the file stays small; the GPU run teacher-forces every frame in between)."""
    _ragged_case("llm_ragged64_bf16", n_new=65, keep_frames=(0, 32, 64), max_seq_len=336, prompt_seed0=200)


def cmd_llm_ragged_full():
    """Config 3's ragged batch at FULL depth (36 slow + 4 fast layers): the 32 prompt lengths of
    llm_ragged, prefill + 8 decode frames, logits kept at frames 0, 4 and 8."""
    _ragged_case("llm_ragged_full_bf16", n_new=9, keep_frames=(0, 4, 8), max_seq_len=272, prompt_seed0=300,
                 n_layer=36, n_fast_layer=4)


def cmd_llm_ragged():
    """Config 3's ragged batch at S2-Pro widths (2 slow + 1 fast layers): 32 prompts with lengths
    uniform over 16..256 (seed 2), each run by the reference at batch 1 (its only
    mode): greedy columns + teacher-forced logits for the prefill frame and 2 decode frames.  Fast
    logits are kept for the last codebook only (its pass reads every fast cache position)."""
    _ragged_case("llm_ragged_bf16", n_new=3, keep_frames=(0, 1, 2), max_seq_len=272, prompt_seed0=100)


def _ragged_case(out_name, n_new, keep_frames, max_seq_len, prompt_seed0, n_layer=2, n_fast_layer=1):
    from fish_speech.models.text2semantic import inference

    B = 32
    config = _wide_config(n_layer, n_fast_layer, max_seq_len)
    lens = np.random.default_rng(2).integers(16, 257, B)
    t0 = time.time()
    cfg, state = _llm_state(config, 41, 5)
    model = _llm_from_state(cfg, state, torch.bfloat16)
    m32 = _llm_from_state(cfg, state, torch.float32)
    del state
    keep = np.r_[IM_END_ID, cfg.semantic_begin_id:cfg.semantic_end_id + 1]
    kf = list(keep_frames)
    res = {k: [] for k in ("seq", "slow_bits", "fast_bits", "slow_f32", "fast_f32")}
    prompts = {}
    for i, T in enumerate(lens):
        T = int(T)
        prompt = make_prompt(cfg, T, prompt_seed0 + i)
        prompts[f"prompt_{i}"] = prompt.numpy().astype(np.int32)
        seq = inference.generate(model=model, prompt=prompt.clone(), max_new_tokens=n_new, audio_masks=None,
                                 audio_parts=None, temperature=0.7, top_p=0.9, top_k=1)
        assert seq.shape[1] - T == n_new
        slow, fast, _ = teacher_forced(model, seq, T, n_new, torch.bfloat16)
        s32, f32, _ = teacher_forced(m32, seq, T, n_new, torch.float32)
        res["seq"].append(seq[:, T:].numpy().astype(np.int32))
        res["slow_bits"].append(_bf16_bits(slow[kf][:, keep]))
        res["fast_bits"].append(_bf16_bits(fast[kf][:, -1]))
        res["slow_f32"].append(s32[kf][:, keep])
        res["fast_f32"].append(f32[kf][:, -1])
        print(f"{out_name}: prompt {i} (T={T}) done at {time.time() - t0:.0f}s", flush=True)
    np.savez_compressed(os.path.join(GOLD, f"{out_name}.npz"), config=np.array(json.dumps(config)),
                        lens=lens.astype(np.int32), cols=np.stack(res["seq"]), slow_rows=keep.astype(np.int32),
                        keep_frames=np.array(kf, np.int32),
                        slow_logits_bits=np.stack(res["slow_bits"]), fast_last_bits=np.stack(res["fast_bits"]),
                        slow_logits_f32=np.stack(res["slow_f32"]), fast_last_f32=np.stack(res["fast_f32"]),
                        synth_seed=41, log2_half=5, torch_version=torch.__version__,
                        threads=torch.get_num_threads(), **prompts)
    print(f"{out_name}: {B} prompts (lens {lens.min()}..{lens.max()}) x {n_new} frames in {time.time() - t0:.0f}s")


# --------------------------------------------------------------------------------------
# Weight-only int8: tools/llama/quantize.py's WeightOnlyInt8QuantHandler
# (create_quantized_state_dict on the bf16 model, as quantize.py:441-458 runs it, then
# convert_for_runtime + load, llama.py:528-535) and the reference's generate / teacher forcing
# on that int8 model.  llm_q: biases on qkv/o, an untied output head and fast_project_in (all
# three nn.Linear -> WeightOnlyInt8Linear, biases dropped); every in_features a multiple of 64.
# --------------------------------------------------------------------------------------
LLM_Q_CONFIG = {
    "model_type": "dual_ar",
    "vocab_size": 400, "n_layer": 3, "n_head": 4, "n_local_heads": 2, "head_dim": 32,
    "dim": 128, "intermediate_size": 256, "rope_base": 10000, "norm_eps": 1e-5,
    "max_seq_len": 192, "tie_word_embeddings": False, "attention_qkv_bias": True,
    "attention_o_bias": True, "attention_qk_norm": False, "codebook_size": 64,
    "num_codebooks": 6, "semantic_begin_id": 300, "semantic_end_id": 363,
    "n_fast_layer": 2, "fast_dim": 64, "fast_n_head": 2, "fast_n_local_heads": 1,
    "fast_head_dim": 32, "fast_intermediate_size": 128, "scale_codebook_embeddings": False,
    "norm_fastlayer_input": False,
}


def _quantize_module():
    """tools/llama/quantize.py as shipped imports inference.load_model, which the reference's
    inference.py no longer defines (it has init_model): the module fails to import.  Its quantization
    classes do not use that name, so it is aliased before the import (test infrastructure only)."""
    from fish_speech.models.text2semantic import inference

    if not hasattr(inference, "load_model"):
        inference.load_model = inference.init_model
    from tools.llama import quantize

    return quantize


def cmd_int4_quant():
    """Weight-only int4 groupwise quantization (the int4 half): the reference's
    own group_quantize_tensor / group_dequantize_tensor (tools/llama/quantize.py:57-160) on seeded
    bf16 matrices, every group size the handler accepts (quantize.py:366), with rows that hit the
    clamp (a constant row: max == min), wide and tiny magnitudes.  Its packed matmul
    (_weight_int4pack_mm, quantize.py:249-257) does not run on this CPU: the build is pinned here at
    the quantizer, not at the packed-matmul level."""
    q = _quantize_module()
    out = {}
    rng = np.random.default_rng(17)
    for gs, (N, K) in ((32, (24, 256)), (64, (24, 512)), (128, (48, 1024)), (256, (32, 1024))):
        w = rng.standard_normal((N, K)).astype(np.float32) * 0.05
        w[1] = 0.0371  # constant row: scales clamp to 1e-6
        w[2] *= 400.0  # wide range
        w[3] *= 1e-4  # tiny range
        w[4, ::7] = 3.5  # outliers
        wb = torch.from_numpy(w).to(torch.bfloat16)
        w_int32, sz = q.group_quantize_tensor(wb, n_bit=4, groupsize=gs)
        wdq = q.group_dequantize_tensor(w_int32, sz.float(), n_bit=4, groupsize=gs)
        out[f"w_bits_g{gs}"] = synth.f32_to_bf16_bits(wb.float().numpy())
        out[f"q_g{gs}"] = w_int32.numpy().astype(np.uint8)
        out[f"sz_bits_g{gs}"] = synth.f32_to_bf16_bits(sz.float().numpy())  # [K/gs][N][2] (scale, zero)
        out[f"dq_g{gs}"] = wdq.float().numpy()
    np.savez_compressed(os.path.join(GOLD, "int4_quant.npz"), torch_version=torch.__version__, **out)
    print("int4_quant:", {k: v.shape for k, v in out.items() if k.startswith("q_")})


def int8_model(config, qsd, seed, log2_half, dtype):
    """The reference's int8 model: modules converted, the quantized state_dict loaded."""
    WeightOnlyInt8QuantHandler = _quantize_module().WeightOnlyInt8QuantHandler

    model = build_llm(config, None, seed, log2_half)
    model = WeightOnlyInt8QuantHandler(model).convert_for_runtime()
    err = model.load_state_dict(qsd, strict=False, assign=True)
    assert not err.missing_keys, err.missing_keys
    assert all(k.endswith(".bias") for k in err.unexpected_keys), err.unexpected_keys
    return model.to(dtype).eval()


def quantized_state(config, seed, log2_half):
    WeightOnlyInt8QuantHandler = _quantize_module().WeightOnlyInt8QuantHandler

    model = build_llm(config, None, seed, log2_half).to(torch.bfloat16)
    return WeightOnlyInt8QuantHandler(model).create_quantized_state_dict()


def cmd_llm_int8():
    from fish_speech.models.text2semantic import inference

    qdir = os.path.join(GOLD, "llm_q_int8")
    os.makedirs(qdir, exist_ok=True)
    with open(os.path.join(qdir, "config.json"), "w") as f:
        json.dump(LLM_Q_CONFIG, f, indent=1)
    qsd = quantized_state(LLM_Q_CONFIG, 29, 3)
    torch.save(OrderedDict((k, v.contiguous()) for k, v in qsd.items()), os.path.join(qdir, "model.pth"))
    T, n_new = 19, 24
    for dtype in (torch.float32, torch.bfloat16):
        model = int8_model(LLM_Q_CONFIG, qsd, 29, 3, dtype)
        prompt = make_prompt(model.config, T, 4)
        seq = inference.generate(model=model, prompt=prompt.clone(), max_new_tokens=n_new,
                                 audio_masks=None, audio_parts=None, temperature=0.7, top_p=0.9, top_k=1)
        n = seq.shape[1] - T
        slow, fast, hid = teacher_forced(model, seq, T, n, dtype)
        tag = {torch.float32: "fp32", torch.bfloat16: "bf16"}[dtype]
        extra = {}
        if dtype == torch.bfloat16:
            s32, f32, _ = teacher_forced(int8_model(LLM_Q_CONFIG, qsd, 29, 3, torch.float32), seq, T, n,
                                         torch.float32)
            extra = dict(slow_logits_f32=s32, fast_logits_f32=f32)
        np.savez_compressed(os.path.join(GOLD, f"llm_q_int8_{tag}.npz"), prompt=prompt.numpy().astype(np.int32),
                            seq=seq.numpy().astype(np.int32), slow_logits=slow, fast_logits=fast, hidden=hid,
                            torch_version=torch.__version__, **extra)
        print(f"llm_q_int8 {tag}: T={T} generated {n} frames; first columns", seq[:, T:T + 3].T.tolist())


def cmd_llm_wide_int8():
    """S2-Pro widths, int8: the same synthetic bf16 weights as llm_wide, quantized by the reference's
    handler.  The build quantizes them on the device (quant_rows_kernel); only logits are stored."""
    from fish_speech.models.text2semantic import inference

    T = 64
    qsd = quantized_state(LLM_WIDE_CONFIG, 41, 5)
    model = int8_model(LLM_WIDE_CONFIG, qsd, 41, 5, torch.bfloat16)
    cfg = model.config
    prompt = make_prompt(cfg, T, 3)
    t0 = time.time()
    seq = inference.generate(model=model, prompt=prompt.clone(), max_new_tokens=9,
                             audio_masks=None, audio_parts=None, temperature=0.7, top_p=0.9, top_k=1)
    n = seq.shape[1] - T
    slow, fast, hid = teacher_forced(model, seq, T, n, torch.bfloat16)
    del model
    s32, f32, _ = teacher_forced(int8_model(LLM_WIDE_CONFIG, qsd, 41, 5, torch.float32), seq, T, n, torch.float32)
    keep = np.r_[IM_END_ID, cfg.semantic_begin_id:cfg.semantic_end_id + 1]
    # per-tensor checksums of the reference's quantization (int8 sum, scale sum) for the device rule
    sums = {k: (int(v.to(torch.int64).sum()), float(qsd[k[:-len("weight")] + "scales"].float().sum()))
            for k, v in qsd.items() if v.dtype == torch.int8}
    np.savez_compressed(os.path.join(GOLD, "llm_wide_int8_bf16.npz"),
                        prompt=prompt.numpy().astype(np.int32), seq=seq.numpy().astype(np.int32),
                        slow_rows=keep.astype(np.int32), slow_logits=slow[:, keep], fast_logits=fast,
                        slow_logits_f32=s32[:, keep], fast_logits_f32=f32, synth_seed=41, log2_half=5,
                        qsums=json.dumps(sums), torch_version=torch.__version__)
    print(f"llm_wide_int8: {n} frames in {time.time() - t0:.1f}s; first cols", seq[:, T:T + 2].T.tolist())


# --------------------------------------------------------------------------------------
# Prompt side: the reference's own Conversation / ContentSequence
# encode_for_inference and the speaker batching of generate_long (inference.py:454-651),
# driven with a tiny local tokenizer (tests/golden/tok_tiny, written here) whose ids match the
# llm_a fixture (semantic 200..327, <|im_end|> = 4).
# --------------------------------------------------------------------------------------
def write_tiny_tokenizer(path):
    from tokenizers import AddedToken, Regex, Tokenizer, models, pre_tokenizers

    specials = ["<|endoftext|>", "<|pad|>", "<|im_start|>", "<|phoneme_start|>", "<|im_end|>",
                "<|phoneme_end|>", "<|text|>", "<|voice|>", "<|interleave|>", "<|audio_start|>",
                "<|audio_end|>", "<|audio_pad|>"] + [f"<|speaker:{i}|>" for i in range(5)]
    vocab = {t: i for i, t in enumerate(specials)}
    for ch in [chr(c) for c in range(32, 127)] + ["\n"]:
        vocab[ch] = len(vocab)
    vocab["[UNK]"] = len(vocab)
    while len(vocab) < 200:
        vocab[f"<|reserved_{len(vocab)}|>"] = len(vocab)
    sem = [f"<|semantic:{i}|>" for i in range(128)]
    for t in sem:
        vocab[t] = len(vocab)
    while len(vocab) < 512:
        vocab[f"<|reserved_{len(vocab)}|>"] = len(vocab)
    tk = Tokenizer(models.WordLevel(vocab=vocab, unk_token="[UNK]"))
    tk.pre_tokenizer = pre_tokenizers.Split(Regex("."), behavior="isolated")
    tk.add_special_tokens([AddedToken(t, special=True, normalized=False) for t in specials + sem])
    os.makedirs(path, exist_ok=True)
    tk.save(os.path.join(path, "tokenizer.json"))
    with open(os.path.join(path, "tokenizer_config.json"), "w") as f:
        json.dump({"tokenizer_class": "PreTrainedTokenizerFast", "eos_token": "<|endoftext|>",
                   "pad_token": "<|pad|>"}, f)


def cmd_prompt():
    import torch
    from fish_speech.content_sequence import TextPart, VQPart
    from fish_speech.conversation import Conversation, Message
    from fish_speech.models.text2semantic.inference import group_turns_into_batches, split_text_by_speaker
    from fish_speech.tokenizer import FishTokenizer
    from copy import deepcopy

    tdir = os.path.join(GOLD, "tok_tiny")
    write_tiny_tokenizer(tdir)
    tok = FishTokenizer(tdir)
    C = 10
    rng = np.random.default_rng(5)
    texts = ["Hello there, how are you today?",
             "<|speaker:0|>Hi! <|speaker:1|>Hey, long time. <|speaker:0|>Indeed, it has been a while "
             "since we last met at the station. <|speaker:2|>Third voice here.",
             "no speaker tags at all, just a sentence that is longer than the chunk length limit of "
             "this test so that grouping has to split it into several batches? no, without tags it "
             "stays one batch."]
    out = {}
    cases = []
    for ti, text in enumerate(texts):
        turns = split_text_by_speaker(text)
        batches = group_turns_into_batches(turns, max_speakers=5, max_bytes=40) if turns else [text]
        out[f"turns_{ti}"] = np.array(json.dumps(turns))
        out[f"batches_{ti}"] = np.array(json.dumps(batches))
        for use_prompt in (False, True):
            # base conversation exactly as generate_long builds it (inference.py:558-600)
            base = Conversation()
            ptoks = None
            if use_prompt:
                ptext = ["reference one", "<|speaker:1|>second reference"]
                ptoks = [torch.from_numpy(rng.integers(0, 128, (C, 6))), torch.from_numpy(rng.integers(0, 128, (C, 4)))]
                tagged = [t if "<|speaker:" in t else f"<|speaker:{i}|>{t}" for i, t in enumerate(ptext)]
                parts = [TextPart(text="convert the provided text to speech reference to the following:\n\nText:\n",
                                  cal_loss=False),
                         TextPart(text="\n".join(tagged), cal_loss=False),
                         TextPart(text="\n\nSpeech:\n", cal_loss=False),
                         VQPart(codes=torch.cat(ptoks, dim=1), cal_loss=False)]
                out[f"ptoks_{ti}"] = np.concatenate([p.numpy() for p in ptoks], axis=1)
            else:
                parts = [TextPart(text="convert the provided text to speech", cal_loss=False)]
            base.append(Message(role="system", parts=parts, cal_loss=False, add_im_start=True, add_im_end=True))
            conv = deepcopy(base)
            for bi, bt in enumerate(batches):
                conv.append(Message(role="user", parts=[TextPart(text=bt, cal_loss=False)], cal_loss=False,
                                    add_im_start=True, add_im_end=True))
                gen = deepcopy(conv)
                gen.append(Message(role="assistant", parts=[], cal_loss=False, modality="voice",
                                   add_im_start=True, add_im_end=False))
                enc, am, ap = gen.encode_for_inference(tok, num_codebooks=C)
                key = f"enc_{ti}_{int(use_prompt)}_{bi}"
                out[key] = enc.numpy().astype(np.int64)
                # the "generated" codes appended back (inference.py:696-707), synthetic here
                codes = torch.from_numpy(rng.integers(0, 128, (C, 3 + bi)))
                out[f"gen_{ti}_{int(use_prompt)}_{bi}"] = codes.numpy()
                conv.append(Message(role="assistant", parts=[VQPart(codes=codes.cpu(), cal_loss=False)],
                                    cal_loss=False, modality="voice", add_im_start=True, add_im_end=True))
                cases.append(key)
    out["texts"] = np.array(json.dumps(texts))
    out["cases"] = np.array(json.dumps(cases))
    np.savez_compressed(os.path.join(GOLD, "prompt.npz"), **out)
    print(f"prompt: {len(cases)} encoded conversations; e.g. {cases[:3]} shape {out[cases[0]].shape}")


def cmd_engine():
    """generate_long (inference.py:523-733) end to end, greedy fp32, on the llm_a weights with the
    tiny tokenizer: reference prompt (speaker-tagged text + VQ codes), a multi-speaker text split
    into batches, the conversation growing with each batch's codes."""
    import copy as _copy

    from fish_speech.models.text2semantic import inference
    from fish_speech.tokenizer import FishTokenizer

    cfg = _copy.deepcopy(LLM_A_CONFIG)
    cfg["text_config"]["max_seq_len"] = 2560  # generate_long refuses prompts > max_len - 2048
    model = build_llm(cfg, None, seed=11, log2_half=3).to(torch.float32)
    model.tokenizer = FishTokenizer(os.path.join(GOLD, "tok_tiny"))
    rng = np.random.default_rng(9)
    ptoks = [torch.from_numpy(rng.integers(0, 128, (10, 5))), torch.from_numpy(rng.integers(0, 128, (10, 3)))]
    text = "<|speaker:0|>Good morning. <|speaker:1|>Morning! Coffee? <|speaker:0|>Yes please, black."
    outs = list(inference.generate_long(model=model, device="cpu", decode_one_token=inference.decode_one_token_ar,
                                        text=text, max_new_tokens=7, top_p=0.9, top_k=1, temperature=0.7,
                                        chunk_length=30, prompt_text=["ref a", "<|speaker:1|>ref b"],
                                        prompt_tokens=ptoks))
    res = {"text": np.array(text), "ptok0": ptoks[0].numpy(), "ptok1": ptoks[1].numpy(),
           "actions": np.array(json.dumps([o.action for o in outs])),
           "batch_texts": np.array(json.dumps([o.text for o in outs if o.action == "sample"]))}
    for i, o in enumerate([o for o in outs if o.action == "sample"]):
        res[f"codes_{i}"] = o.codes.numpy().astype(np.int32)
    np.savez_compressed(os.path.join(GOLD, "engine.npz"), **res)
    print("engine:", [o.action for o in outs], [res[k].shape for k in res if k.startswith("codes_")])


def cmd_engine_bf16():
    """generate_long (inference.py:523-733) in bf16 -- the reference's production precision -- on
    the engine golden's request, recording what each batch's generate() saw: the encoded whole
    conversation (its prompt) and every emitted column.  Each batch is then replayed teacher-forced
    (teacher_forced above: the reference's own prefill + decode_one_token_ar forwards with its emitted
    columns) by the bf16 model and by the fp32 model on the same columns, so the test can hold the
    native reused-prefix flow (fm_llm_generate_at) to the reference's own bf16-vs-fp32 error batch by
    batch, instead of to bit-identity with another native flow."""
    import copy as _copy

    from fish_speech.models.text2semantic import inference
    from fish_speech.tokenizer import FishTokenizer

    cfg = _copy.deepcopy(LLM_A_CONFIG)
    cfg["text_config"]["max_seq_len"] = 2560
    g = np.load(os.path.join(GOLD, "engine.npz"))
    tok = FishTokenizer(os.path.join(GOLD, "tok_tiny"))
    model = build_llm(cfg, None, seed=11, log2_half=3).to(torch.bfloat16)
    model.tokenizer = tok
    seen = []
    real_generate = inference.generate

    def recording_generate(*, model, prompt, **kw):  # instrumentation only: the reference's generate runs
        y = real_generate(model=model, prompt=prompt, **kw)
        seen.append((prompt.clone(), y.clone()))
        return y

    inference.generate = recording_generate
    try:
        outs = list(inference.generate_long(
            model=model, device="cpu", decode_one_token=inference.decode_one_token_ar, text=str(g["text"]),
            max_new_tokens=7, top_p=0.9, top_k=1, temperature=0.7, chunk_length=30,
            prompt_text=["ref a", "<|speaker:1|>ref b"],
            prompt_tokens=[torch.from_numpy(g["ptok0"]), torch.from_numpy(g["ptok1"])]))
    finally:
        inference.generate = real_generate
    m32 = build_llm(cfg, None, seed=11, log2_half=3).to(torch.float32)
    res = {"actions": np.array(json.dumps([o.action for o in outs])), "n_batches": len(seen)}
    for i, (prompt, y) in enumerate(seen):
        T = prompt.shape[1]
        n = y.shape[1] - T
        slow, fast, _ = teacher_forced(model, y, T, n, torch.bfloat16)
        s32, f32, _ = teacher_forced(m32, y, T, n, torch.float32)
        res[f"prompt_{i}"] = prompt.numpy().astype(np.int32)
        res[f"cols_{i}"] = y[:, T:].numpy().astype(np.int32)
        res[f"slow_{i}"], res[f"fast_{i}"] = slow, fast
        res[f"slow32_{i}"], res[f"fast32_{i}"] = s32, f32
    for i, o in enumerate([o for o in outs if o.action == "sample"]):
        res[f"codes_{i}"] = o.codes.numpy().astype(np.int32)
    np.savez_compressed(os.path.join(GOLD, "engine_bf16.npz"), **res)
    print("engine_bf16:", [o.action for o in outs],
          [(res[f"prompt_{i}"].shape[1], res[f"cols_{i}"].shape[1]) for i in range(len(seen))])


def cmd_engine_clone():
    """BASELINE config 5's chain at tiny shapes: reference audio -> the reference's own DAC.encode
    (codec_enc_tiny weights, fp32; vq_manager.py:24-52) -> those codes as the voice-clone prompt of
    the reference's generate_long (llm_a weights, tiny tokenizer, greedy fp32, several speaker
    batches) -> codes.  The GPU test runs the same chain through fm_codec_encode + the native
    generate_long."""
    import copy as _copy

    from fish_speech.models.text2semantic import inference
    from fish_speech.tokenizer import FishTokenizer

    dac = build_codec(CODEC_TINY, 41, [0, 0, 0, 2])
    n = 9 * 2048 - 500
    audio = encode_audio(n, 77)
    with torch.inference_mode():
        ref_codes = dac.encode(torch.from_numpy(audio)[None, None])[0][0]
    cfg = _copy.deepcopy(LLM_A_CONFIG)
    cfg["text_config"]["max_seq_len"] = 2560
    model = build_llm(cfg, None, seed=11, log2_half=3).to(torch.float32)
    model.tokenizer = FishTokenizer(os.path.join(GOLD, "tok_tiny"))
    text = "<|speaker:0|>Read this aloud. <|speaker:0|>Then a second sentence follows here."
    outs = list(inference.generate_long(model=model, device="cpu", decode_one_token=inference.decode_one_token_ar,
                                        text=text, max_new_tokens=9, top_p=0.9, top_k=1, temperature=0.7,
                                        chunk_length=30, prompt_text=["the reference transcript"],
                                        prompt_tokens=[ref_codes.clone()]))
    res = {"text": np.array(text), "audio_seed": 77, "n_samples": n, "ref_codes": ref_codes.numpy().astype(np.int32),
           "prompt_text": np.array("the reference transcript"),
           "actions": np.array(json.dumps([o.action for o in outs]))}
    for i, o in enumerate([o for o in outs if o.action == "sample"]):
        res[f"codes_{i}"] = o.codes.numpy().astype(np.int32)
    np.savez_compressed(os.path.join(GOLD, "engine_clone.npz"), **res)
    print("engine_clone:", res["ref_codes"].shape, [o.action for o in outs],
          [res[k].shape for k in res if k.startswith("codes_")])

if __name__ == "__main__":
    cmds = sys.argv[1:] or ["all"]
    if cmds == ["all"]:
        cmds = ["ops", "llm", "codec", "codec_full", "codec_long", "codec_enc", "codec_enc_full",
                "codec_enc_long", "codec_keys", "llm_wide", "llm_int8", "llm_wide_int8", "prompt", "engine", "engine_bf16",
                "engine_clone"]
    for c in cmds:
        globals()[f"cmd_{c}"]()
