#!/usr/bin/env python3
"""bench.py -- BASELINE.json's headline metric on the MI355X-native path.

Metric: synthesised audio-seconds per wall-second (aggregate over all GPUs) + p50 first-sample
latency, S2-Pro 4B.  One "step" = one utterance per GPU of BASELINE config 2:
a 64-token prompt, 216 decode frames (10.03 s of 44.1 kHz audio at 21.533 frames/s) with
<|im_end|> masked so the length is fixed, and the codec decode of the [1, 10, 216] codes.
The first 8 frames are vocoded as soon as they exist (the codec is causal end to end, so that
chunk is exactly the prefix of the final waveform); the time from request to that PCM is the
first-sample latency.  N>1: one process per GPU (torch.distributed.run), rank 0 scatters the
request descriptors and gathers the int16 PCM over RCCL (fishmi/dp.py), weak scaling.

Weights are seeded synthetic bf16 at the S2-Pro shapes (there is no checkpoint on the box).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--no-cpu-baseline]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "fish-speech_amd"))

METRIC = "audio-sec/wall-sec (RTF) + p50 first-sample latency, S2-Pro 4B @1/2/4/8 GPU"
FRAME_RATE = 44100.0 / 2048.0          # codec frames per audio second (modded_dac.py:833,861)
HBM_PEAK_GBPS = 8000.0                 # MI355X HBM3E (MI355X_MICROARCH.md §HBM)
BF16_DENSE_TFLOPS = 2500.0             # MI355X dense bf16 MFMA peak (no sparsity)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--frames", type=int, default=216)
    ap.add_argument("--prompt-len", type=int, default=64)
    ap.add_argument("--first-chunk", type=int, default=1,
                    help="frames in the first vocoded chunk (later chunks grow 4x)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-frames", type=int, default=0,
                    help="oracle decode frames timed (0: the whole utterance, --frames)")
    ap.add_argument("--cpu-codec-frames", type=int, default=0,
                    help="oracle codec frames timed (0: the whole utterance)")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--batch", type=int, default=32,
                    help="throughput leg (BASELINE config 3): concurrent streams per GPU (0: skip)")
    ap.add_argument("--batch-frames", type=int, default=512, help="throughput leg: frames per request")
    ap.add_argument("--overlap-vocode", action="store_true",
                    help="configs 2 and 5: vocode the chunks after the first on a host thread, overlapped with "
                         "the next chunk's decode (default: each chunk before decoding the next; measured "
                         "neutral, profiles/r06_vocoder_overlap_ab.txt)")
    ap.add_argument("--vocode-chunk", type=int, default=128,
                    help="throughput leg: frames per streamed codec chunk, vocoded on a host thread of its "
                         "own while the decode goes on (0: each stream vocoded at its end, serially)")
    ap.add_argument("--waves", type=int, default=1,
                    help="throughput leg: requests = batch x GPUs x waves, pulled from rank 0's tick queue")
    ap.add_argument("--longform-turns", type=int, default=4,
                    help="config-5 leg: speaker turns (0: skip), each --longform-frames frames")
    ap.add_argument("--longform-frames", type=int, default=323, help="config-5 leg: frames per turn (15 s)")
    ap.add_argument("--no-int8", action="store_true", help="skip the opt-in weight-only int8 leg")
    ap.add_argument("--tune", action="append", default=[], metavar="KEY=VALUE",
                    help="fm_tune developer knob before the run (repeatable)")
    ap.add_argument("--no-pmc", action="store_true",
                    help="skip the in-run rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes on the GEMV")
    ap.add_argument("--encode-seconds", type=float, default=30.0,
                    help="encode leg: seconds of reference audio through the codec encoder (0: skip)")
    return ap.parse_args()


def make_prompt(cfg, T, seed):
    """Template + text token ids: ids from [16, semantic_begin)."""
    rng = np.random.default_rng(seed + 10**6)  # warmup steps use negative step ids
    p = np.zeros((cfg.num_codebooks + 1, T), np.int32)
    p[0] = rng.integers(16, cfg.semantic_begin_id, T)
    return p


def utterance(llm, codec, prompt, sp, frames, first_chunk, voc=None):
    """Request -> PCM for one stream.  Returns (pcm, timings in seconds).  The vocoder streams:
    each chunk of frames is vocoded as soon as its frames exist -- first_chunk frames, then chunks
    growing 4x, so a chunk's generation (4^k frames at ~10x real time) takes less time than the
    audio already delivered (>= 4^k frames) takes to play -- continuing one codec stream (carried
    causal state, fm_codec_decode_chunk), so no frame is vocoded twice and the waveform is
    bit-identical to a one-shot decode (tests/test_gpu_codec_stream.py).  With voc (a
    scheduler.StreamVocoder), the chunks after the first are vocoded on its host thread, on the
    codec's own HIP stream, while the next chunk decodes; the first chunk's PCM is waited for (the
    first-sample latency), the rest at the end.  timings: decode = host time in decode_frames,
    codec = time inside the codec calls after the first chunk."""
    t0 = time.perf_counter()
    col0 = llm.prefill(0, prompt, sp)
    t1 = time.perf_counter()
    durs = []

    def vocode(codes):
        ta = time.perf_counter()
        out = codec.decode_chunk(codes)
        durs.append(time.perf_counter() - ta)
        return out

    if voc is None:
        codec.stream_reset()
    else:
        voc.submit(codec.stream_reset)
    pcm, jobs, done, n = [], [], 0, min(first_chunk, frames)
    cols = col0[None]
    first = decode = 0.0
    while done < frames:
        ta = time.perf_counter()
        if n > cols.shape[0]:
            cols = np.concatenate([cols, llm.decode_frames([0], n - cols.shape[0])[:, 0, :]], axis=0)
        tb = time.perf_counter()
        codes = np.ascontiguousarray(cols[:, 1:].T)
        if voc is None:
            pcm.append(vocode(codes))
        else:
            ev, box = voc.submit(lambda c=codes: vocode(c))
            jobs.append((ev, box))
            if done == 0:
                ev.wait()
        tc = time.perf_counter()
        if done == 0:
            first = tc - t0
        else:
            decode += tb - ta
        done += n
        cols = cols[:0]
        n = min(4 * n, frames - done)
    for ev, box in jobs:
        ev.wait()
        if isinstance(box[0], BaseException):
            raise box[0]
        pcm.append(box[0])
    t4 = time.perf_counter()
    return np.concatenate(pcm), dict(first=first, prefill=t1 - t0, head=first - (t1 - t0), decode=decode,
                                     codec=float(sum(durs[1:])), total=t4 - t0)


def throughput_leg(llm, codec, cfg, batch, frames, waves, sync, dist, world, vocode_chunk=128):
    """BASELINE config 3 at N=1 (32 concurrent prompts per GPU) and config 4 at N=8 (256 requests
    over 8 GPUs), end to end: rank 0 owns batch x world x waves requests (prompt lengths uniform in
    [16, 256], seed 2; `frames` frames each) and hands them out through the tick queue
    (fishmi/scheduler.py). Each rank prefills its requests into KV slots and decodes them together,
    one batched Dual-AR frame per graph replay (slow pass + 10 fast passes + samplers of every
    stream). It vocodes each stream through the streamed codec -- with vocode_chunk > 0 on a
    host thread of its own (scheduler.StreamVocoder), each live stream's finished columns in chunks
    of vocode_chunk frames while the next tick decodes; 0: each stream at its end, serially -- and
    the int16 PCM is gathered to rank 0 over RCCL. Value = audio seconds of PCM gathered at rank 0 / wall time
    (max over ranks)."""
    from fishmi import dp
    from fishmi import scheduler as S
    from fishmi.llm import DualARModel

    rank = dist.get_rank() if dist is not None else 0
    C1 = cfg.num_codebooks + 1
    reqs = None
    if rank == 0:
        rng = np.random.default_rng(2)
        n = batch * world * waves
        lens = rng.integers(16, 257, n)
        reqs = [S.Request(i, make_prompt(cfg, int(lens[i]), 5000 + i), frames, 31 * i + 7) for i in range(n)]
    if dist is None:  # the tick queue runs on a one-rank gloo group at N=1
        import torch.distributed as tdist

        tdist.init_process_group("gloo", store=tdist.HashStore(), rank=0, world_size=1)
    # graph capture of the batch-wide frame before the clock starts
    warm = [s for s in range(batch)]
    for s in warm:
        llm.prefill(s, make_prompt(cfg, 16, 77 + s), DualARModel.sampling(mask_im_end=True))
    llm.decode_frames(warm, 2)

    phase = {"prefill": 0.0, "decode": 0.0, "codec": 0.0}  # host wall per phase (each call syncs)

    def timed(name, f):
        t = time.perf_counter()
        r = f()
        phase[name] += time.perf_counter() - t
        return r

    def start(slot, req):
        return timed("prefill", lambda: llm.prefill(
            slot, req.prompt, DualARModel.sampling(temperature=0.8, top_p=0.8, top_k=30, seed=req.seed,
                                                   mask_im_end=True)))

    def start_batch(pairs):  # a tick's new requests prefilled together (one GEMM pass over all prompts)
        return timed("prefill", lambda: llm.prefill_batch(
            [sl for sl, _ in pairs], [r.prompt for _, r in pairs],
            [DualARModel.sampling(temperature=0.8, top_p=0.8, top_k=30, seed=r.seed, mask_im_end=True)
             for _, r in pairs]))

    def step(slots, n):
        return timed("decode", lambda: llm.decode_frames(slots, n))

    voc = S.StreamVocoder(codec, vocode_chunk) if vocode_chunk > 0 else None

    def finish(slot, req, cols):
        if voc is not None:  # the rest of the stream; earlier chunks were vocoded during the decode
            return timed("codec", lambda: dp.pcm_to_int16(voc.finish(slot, req, cols)))

        def vocode():
            codec.stream_reset()
            mx = codec.max_frames
            return dp.pcm_to_int16(np.concatenate([codec.decode_chunk(np.ascontiguousarray(cols[1:, t:t + mx]))
                                                   for t in range(0, cols.shape[1], mx)]))
        return timed("codec", vocode)

    sync()
    t0 = time.perf_counter()
    q = S.TickQueue(reqs, C1)
    stats = S.serve(q, batch, start, step, finish, tick_frames=32, start_batch=start_batch,
                    progress=voc.progress if voc is not None else None)
    sync()
    dt = time.perf_counter() - t0
    codec_busy = voc.busy_s if voc is not None else phase["codec"]
    if voc is not None:
        voc.close()
    if dist is not None:
        import torch

        e = torch.tensor([dt], dtype=torch.float64, device="cuda")
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        dt = float(e.item())
    else:
        import torch.distributed as tdist

        tdist.destroy_process_group()
    if rank != 0:
        return None
    samples = sum(r.data.size for r in q.results)
    audio_s = samples / 44100.0
    return {"workload": f"BASELINE config {3 if world == 1 else 4}: {len(q.results)} requests (prompt lengths "
                        f"uniform 16-256, seed 2; {frames} frames each, top_k 30, top_p 0.8, temp 0.8) over "
                        f"{world} GPU(s), {batch} concurrent per GPU via rank 0's tick queue; end to end: "
                        f"prefill + batched hipGraph decode + streamed codec decode + int16 PCM gathered "
                        f"to rank 0",
            "requests": len(q.results), "batch_per_gpu": batch, "frames": frames,
            "value": round(audio_s / dt, 2), "unit": "audio-sec/wall-sec", "wall_s": round(dt, 3),
            "decode_frames_rank0": stats["frames"], "ticks": stats["ticks"],
            "phase_s_rank0": {k: round(v, 3) for k, v in phase.items()},
            "vocode_chunk": vocode_chunk, "codec_busy_s_rank0": round(codec_busy, 3),
            "per_stream_rtf": round(audio_s / len(q.results) / dt, 3)}


def encode_leg(ccfg, device, seconds, seed):
    """BASELINE config 5's voice-clone input: `seconds` of reference audio -> codes through the codec
    ENCODER (DAC.encode, modded_dac_vq.yaml shapes, bf16, random-init weights, synthetic audio).
    Device time from HIP events around the encode; FLOPs are the implicit-GEMM convs/linears."""
    from fishmi.codec import FishMICodec

    T = int(np.ceil(seconds * FRAME_RATE))
    m = FishMICodec(ccfg, device, "bf16", max_frames=T)
    m.enable_encoder(64, (0, 0, 0, 4))
    m.synth(seed + 2)
    m.synth_encoder(seed + 2)
    m.finalize()
    n = T * ccfg.hop
    t = np.arange(n) / ccfg.sample_rate
    audio = (0.4 * np.sin(2 * np.pi * 220 * t) + 0.05 * np.random.default_rng(seed).standard_normal(n)).astype(np.float32)
    m.encode_audio(audio)  # warm-up
    ms0, _, fl0 = m.profile()
    reps = 3
    t0 = time.perf_counter()
    for _ in range(reps):
        m.encode_audio(audio)
    wall = (time.perf_counter() - t0) / reps
    ms1, _, fl1 = m.profile()
    dev_ms = (ms1 - ms0) / reps
    tflops = (fl1 - fl0) / reps / (dev_ms * 1e-3) / 1e12
    m.close()
    return {"workload": f"codec encode of {n / ccfg.sample_rate:.1f} s of reference audio ({T} code frames), bf16",
            "value": round(n / ccfg.sample_rate / wall, 2), "unit": "audio-sec/wall-sec",
            "wall_ms": round(wall * 1e3, 2), "device_ms": round(dev_ms, 2),
            "roofline": {"bound": "mfma", "achieved": round(tflops, 2), "peak": BF16_DENSE_TFLOPS,
                         "unit": "TFLOP/s", "frac": round(tflops / BF16_DENSE_TFLOPS, 4)}}


def longform_leg(ccfg, device, turns, frames_per_turn, seed, serial=False):
    """BASELINE config 5 on one GPU: voice clone from 30 s of reference audio (codec encode), then
    `turns` speaker turns of `frames_per_turn` frames through the native generate_long (conversation
    growing with each turn's codes, prefix KV reused), codes streamed into the causal streamed
    vocoder in chunks of 1, 4, 16, then 64 frames per turn (each chunk generated faster than the
    audio before it plays).  Synthetic S2-Pro weights and a synthetic tokenizer at the S2-Pro vocab
    layout; <|im_end|> masked so every turn has its full length.  Timed from the request (reference
    audio in host memory) to the last PCM sample."""
    import tempfile

    from fishmi import engine as E
    from fishmi.codec import FishMICodec
    from fishmi.config import S2_PRO_CONFIG, S2_PRO_IM_END_ID, DualARConfig
    from fishmi.llm import DualARModel
    from fishmi.prompt import FishTokenizer
    from fishmi.synth import write_synthetic_tokenizer

    cfg = DualARConfig._from_fish_qwen3_omni(S2_PRO_CONFIG)
    cfg.im_end_id = S2_PRO_IM_END_ID
    cfg.max_seq_len = 5120  # generate_long refuses prompts longer than max_seq_len - 2048
    llm = DualARModel.synthetic(cfg, seed=seed, log2_half=5, device=device, precision="bf16", max_slots=1)
    tdir = tempfile.mkdtemp(prefix="fishmi_tok_", dir="/tmp")
    llm.tokenizer = FishTokenizer(write_synthetic_tokenizer(tdir, cfg.vocab_size, S2_PRO_IM_END_ID,
                                                            cfg.semantic_begin_id))
    ref_frames = int(np.ceil(30.0 * FRAME_RATE))
    codec = FishMICodec(ccfg, device, "bf16", max_frames=ref_frames)
    codec.enable_encoder(64, (0, 0, 0, 4))
    codec.synth(seed + 1)
    codec.synth_encoder(seed + 1)
    codec.finalize()
    n = ref_frames * ccfg.hop
    t = np.arange(n) / ccfg.sample_rate
    audio = (0.4 * np.sin(2 * np.pi * 220 * t) * (0.6 + 0.4 * np.sin(2 * np.pi * 3 * t)) +
             0.05 * np.random.default_rng(seed).standard_normal(n)).astype(np.float32)
    words = "the quick brown fox jumps over a lazy dog while the river runs past the old mill "
    text = " ".join(f"<|speaker:{i % 2}|>" + (words * 2)[: 150 + 7 * i] for i in range(turns))

    from fishmi import scheduler as S

    # chunks after a turn's first go to the vocoder thread (codec HIP stream) while the generator
    # decodes on; a turn's first chunk is waited for (its latency is the turn's first-chunk time)
    voc = None if serial else S.StreamVocoder(codec)

    def run():
        t0 = time.perf_counter()
        ptok = codec.encode_audio(audio)
        firsts, samples, turn_t0, jobs = [], 0, t0, []
        for o in E.generate_long(model=llm, text=text, max_new_tokens=frames_per_turn, top_p=0.8, top_k=30,
                                 temperature=0.8, chunk_length=200, prompt_text=["a thirty second reference"],
                                 prompt_tokens=[ptok], seed=seed, stream_frames=1, stream_growth=4,
                                 stream_max=64, mask_im_end=True, reuse_prefix=True):
            if o.action != "sample":
                continue
            if voc is None:
                if o.stream == 0:
                    codec.stream_reset()
                samples += codec.decode_chunk(o.codes).size
            else:
                if o.stream == 0:
                    voc.submit(codec.stream_reset)
                ev, box = voc.submit(lambda c=o.codes: codec.decode_chunk(c))
                jobs.append((ev, box))
                if o.stream == 0:
                    ev.wait()
            now = time.perf_counter()
            if o.stream == 0:
                # turn start (the previous turn's last chunk vocoded, or handed to the vocoder) -> first PCM
                firsts.append(now - turn_t0)
            turn_t0 = now
        for ev, box in jobs:
            ev.wait()
            if isinstance(box[0], BaseException):
                raise box[0]
            samples += box[0].size
        return time.perf_counter() - t0, firsts, samples, ptok.shape[1]

    run()  # warm-up: graph capture, tokenizer, allocation
    wall, firsts, samples, ref_codes = run()
    if voc is not None:
        voc.close()
    llm.close()
    codec.close()
    audio_s = samples / ccfg.sample_rate
    f = np.array(firsts) * 1e3
    return {"workload": f"BASELINE config 5: voice clone from {n / ccfg.sample_rate:.1f} s of reference audio "
                        f"({ref_codes} code frames, HIP encode) + {turns} speaker turns x {frames_per_turn} frames "
                        f"through generate_long (prefix KV reused across turns), codes streamed in chunks of 1, 4, 16, "
                        f"then 64 frames into the causal streamed vocoder; bf16, synthetic weights + tokenizer",
            "value": round(audio_s / wall, 3), "unit": "audio-sec/wall-sec", "audio_s": round(audio_s, 2),
            "wall_s": round(wall, 3), "vocoder": "serial" if serial else "host thread, overlapped with generation",
            "first_sample_ms": round(float(f[0]), 2),
            "turn_first_chunk_ms_p50": round(float(np.median(f)), 2),
            "turn_first_chunk_ms_p90": round(float(np.percentile(f, 90)), 2)}


def quant_leg(cfg, codec, args, local, quant):
    """Config 2 with weight-only int8 / int4 linears (opt-in; tools/llama/
    quantize.py's per-channel int8 rule or groupwise int4 rule (group 128) applied on the device to the
    same synthetic weights): the same utterance loop, and the quantized decode GEMV's roofline at its
    own algorithmic bytes (int8: 1 byte per weight + row scales; int4: half a byte + a (scale, zero)
    word per row and 128-k unit)."""
    from fishmi.llm import DualARModel

    llm = DualARModel.synthetic(cfg, seed=args.seed, log2_half=5, device=local, precision="bf16",
                                max_slots=1, quant=quant)
    def go(step):
        sp = DualARModel.sampling(temperature=0.8, top_p=0.8, top_k=30, seed=7919 * step, mask_im_end=True)
        return utterance(llm, codec, make_prompt(cfg, args.prompt_len, 1000 * step), sp, args.frames,
                         args.first_chunk)[1]

    go(-1)
    import torch

    torch.cuda.synchronize()
    t0 = time.perf_counter()
    tms = [go(k) for k in range(args.steps)]
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    pos = args.prompt_len + args.frames // 2
    llm.prefill(0, make_prompt(cfg, args.prompt_len, 99), DualARModel.sampling(mask_im_end=True))
    llm.decode_frames([0], args.frames // 2)
    avg_us, n, b = llm.kernel_bench("linear", reps=20)
    dec_s = np.mean([t["decode"] for t in tms]) / (args.frames - args.first_chunk)
    fb = llm.frame_bytes(1, pos)
    llm.close()
    ach = b / n / (avg_us * 1e-6) / 1e9
    what = ("weight-only int8 linears (round(round(x.q) * scale), biases dropped, as WeightOnlyInt8Linear)"
            if quant == "int8" else
            "weight-only int4 linears, group 128 (quantize.py's group_quantize_tensor on the device, bit-exact; "
            "weights bf16(fma(q - 8, scale, zero)), 4-bit codes streamed by the batch-1 GEMVs)")
    return {"workload": f"config 2 as above with {what}; opt-in, off the bf16 parity contract",
            "value": round(args.steps * args.frames / FRAME_RATE / el, 4), "unit": "audio-sec/wall-sec",
            "ms_per_frame": round(dec_s * 1e3, 4), "bytes_per_frame": int(fb),
            "frame_frac": round(fb / dec_s / 1e9 / HBM_PEAK_GBPS, 4),
            "gemv": {"achieved": round(ach, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                     "frac": round(ach / HBM_PEAK_GBPS, 4), "bytes_per_launch": int(b / n),
                     "avg_launch_us": round(avg_us, 3), "launches_per_frame": int(n)}}


def cpu_baseline(cfg, ccfg, prompt, frames, n_frames, n_codec, seed):
    """The C oracle (oracle/, a restatement of the reference's CPU path) at full S2-Pro shapes on
    the host cores: the prompt pass + n_frames decode frames and a codec decode of n_codec frames.
    n_frames = n_codec = frames (the default): the whole config-2 utterance, timed as it runs; a
    smaller sample is extrapolated.  Also BASELINE config 1 (the reference's CPU plumbing case): a
    16-token prompt + chat template, 32 greedy frames, on the tiny fixture model (tests/golden/llm_a)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O

    n_frames = n_frames or frames
    n_codec = n_codec or frames
    llm = O.OracleLLM(cfg, True)
    llm.synth(seed, 5)
    out = llm.generate(prompt, n_frames, temperature=0.8, top_p=0.8, top_k=30, seed=seed, mask_im_end=True)
    t_pre, t_fr = O.OracleLLM.last_generate_timing()
    n_fr = max(out.shape[1] - 1, 1)
    del llm
    codec = O.OracleCodec(ccfg)
    codec.synth(seed)
    codes = np.ascontiguousarray(out[1:, :n_codec]) if out.shape[1] >= n_codec else \
        np.ascontiguousarray(out[1:, :1].repeat(n_codec, axis=1))
    t0 = time.perf_counter()
    codec.decode(codes)
    t_codec = time.perf_counter() - t0
    del codec
    per_frame, per_codec = t_fr / n_fr, t_codec / n_codec
    whole = n_fr == frames - 1 and n_codec == frames
    est = t_pre + (frames - 1) * per_frame + frames * per_codec
    # config 1: tiny fixture model, 16 text tokens inside the chat template, 32 greedy frames
    from fishmi.checkpoint import load_llm_weights
    from fishmi.config import DualARConfig

    gold = os.path.join(ROOT, "tests", "golden")
    c1 = DualARConfig.from_pretrained(os.path.join(gold, "llm_a"))
    c1.im_end_id = 4
    p1 = np.zeros((c1.num_codebooks + 1, 16 + 8), np.int32)
    rng = np.random.default_rng(1)
    p1[0] = rng.integers(16, c1.semantic_begin_id, p1.shape[1])
    p1[0, :3], p1[0, -5:] = (1, 2, 3), (4, 1, 2, 3, 5)  # template specials around the 16 text ids
    o1 = O.OracleLLM(c1, False)
    o1.load(load_llm_weights(os.path.join(gold, "llm_a")))
    t1 = time.perf_counter()
    y1 = o1.generate(p1, 32, top_k=1)
    t1 = time.perf_counter() - t1
    del o1
    what = (f"the whole config-2 utterance: {prompt.shape[1]}-token prompt pass {t_pre:.2f}s + {n_fr} decode frames "
            f"{t_fr:.2f}s ({per_frame:.3f}s/frame) + codec decode of {n_codec} frames {t_codec:.2f}s = {est:.1f}s"
            if whole else
            f"{prompt.shape[1]}-token prompt pass {t_pre:.2f}s, {n_fr} decode frames {per_frame:.3f}s/frame, codec "
            f"{n_codec} frames {per_codec:.3f}s/frame; extrapolated to prefill + {frames} frames + codec of "
            f"{frames} frames = {est:.1f}s")
    return {"value": round(frames / FRAME_RATE / est, 5), "unit": "audio-sec/wall-sec",
            "cores": O.threads(), "kind": "port",
            "sample": f"C oracle at full S2-Pro shapes, bf16-rounded arithmetic, {what}",
            "config1": {"workload": "BASELINE config 1: tiny fixture model (tests/golden/llm_a), 16 text ids in the "
                                    "chat template, greedy, 32 frames, C oracle on CPU",
                        "frames": int(y1.shape[1]), "ms": round(t1 * 1e3, 2),
                        "frames_per_s": round(y1.shape[1] / t1, 1)}}


def spawn_ranks(n):
    """`bench.py --gpus N` outside torch.distributed.run: start N rank processes through it (one per
    GPU, RCCL rendezvous on 127.0.0.1) before this process touches the GPU, and exit with their
    status. The driver's own launch (WORLD_SIZE set) skips this."""
    import socket
    import subprocess

    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def pmc_gemv_traffic(timeout_s=150):
    """HBM bytes per decode-GEMV launch at HEAD, measured in this run: two rocprofv3 --pmc passes
    (FETCH_SIZE, then WRITE_SIZE; one counter group per pass) over scripts/pmc_probe.py in child
    processes. FETCH_SIZE is doubled per the gfx950 wide-read correction (MI355X_MICROARCH.md §HBM).
    Returns (bytes per launch or None, note)."""
    import glob
    import shutil
    import subprocess
    import tempfile

    sys.path.insert(0, os.path.join(ROOT, "scripts"))
    from rocprof_summary import is_decode_linear, load_pmc

    exe = shutil.which("rocprofv3")
    if exe is None:
        return None, "rocprofv3 not on PATH"
    vals = {}
    for counter in ("FETCH_SIZE", "WRITE_SIZE"):
        d = tempfile.mkdtemp(prefix="fishmi_pmc_", dir="/tmp")
        env = dict(os.environ, FISHMI_GRAPH="0")
        cmd = ["timeout", "-s", "KILL", str(timeout_s), exe, "--pmc", counter, "-d", d, "-o", "pmc", "--",
               sys.executable, os.path.join(ROOT, "scripts", "pmc_probe.py")]
        r = subprocess.run(cmd, env=env, cwd="/tmp", stdout=subprocess.DEVNULL, stderr=subprocess.PIPE)
        dbs = glob.glob(os.path.join(d, "**", "*results.db"), recursive=True) + \
            glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
        if r.returncode != 0 or not dbs:
            return None, f"rocprofv3 --pmc {counter} failed (rc {r.returncode}): {r.stderr[-300:].decode(errors='replace')}"
        v = [x for name, xs in load_pmc(dbs[0], counter).items() if is_decode_linear(name) for x in xs]
        shutil.rmtree(d, ignore_errors=True)
        if not v:
            return None, f"no decode-linear dispatches in the {counter} pass"
        vals[counter] = 1024.0 * sum(v) / len(v)
    fetch = 2.0 * vals["FETCH_SIZE"]
    return int(round(fetch + vals["WRITE_SIZE"])), (
        f"rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE passes over scripts/pmc_probe.py in this run: "
        f"{fetch / 1e6:.2f} MB fetched (FETCH_SIZE KB x1024 x2, gfx950 wide-read correction) + "
        f"{vals['WRITE_SIZE'] / 1e6:.3f} MB written per decode-linear launch (gemv_kernel, rowgemv_kernel)")


def trace_decode_kernels(timeout_s=150):
    """Per-launch durations of the decode kernels from a rocprofv3 --kernel-trace pass over
    scripts/pmc_probe.py (a child process; prefill + 4 batch-1 frames at S2-Pro shapes): the decode
    linear class and the fused fast attention + wo (fattn_wo_kernel), which streams the fast model's
    wo weights but sits outside the "linear" class.  Returns {name: (launches, avg_us)} or a note."""
    import glob
    import shutil
    import subprocess
    import tempfile

    sys.path.insert(0, os.path.join(ROOT, "scripts"))
    from rocprof_summary import is_decode_linear, load_dispatches

    exe = shutil.which("rocprofv3")
    if exe is None:
        return {"note": "rocprofv3 not on PATH"}
    d = tempfile.mkdtemp(prefix="fishmi_tr_", dir="/tmp")
    cmd = ["timeout", "-s", "KILL", str(timeout_s), exe, "--kernel-trace", "--output-format", "csv", "-d", d, "-o",
           "tr", "--", sys.executable, os.path.join(ROOT, "scripts", "pmc_probe.py")]
    r = subprocess.run(cmd, cwd="/tmp", stdout=subprocess.DEVNULL, stderr=subprocess.PIPE)
    csvs = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    if r.returncode != 0 or not csvs:
        return {"note": f"rocprofv3 --kernel-trace failed (rc {r.returncode}): {r.stderr[-300:].decode(errors='replace')}"}
    disp = load_dispatches(csvs[0])
    shutil.rmtree(d, ignore_errors=True)
    lin = [ns for n, ns, _ in disp if is_decode_linear(n)]
    fw = [ns for n, ns, _ in disp if n.startswith("void fattn_wo_kernel")]
    out = {}
    if lin:
        out["linear"] = (len(lin), sum(lin) / len(lin) / 1e3)
    if fw:
        out["fattn_wo"] = (len(fw), sum(fw) / len(fw) / 1e3)
    return out


def pmc_codec_mfma(codec_ms, timeout_s=120):
    """MFMA utilisation of the codec decode from the hardware counters, measured in this run: one
    rocprofv3 --pmc pass (SQ_VALU_MFMA_BUSY_CYCLES, SQ_INSTS_VALU_MFMA_MOPS_BF16, SQ_ACTIVE_INST_VALU,
    SQ_WAVE_CYCLES, GRBM_GUI_ACTIVE) over scripts/codec_pmc_probe.py (config 2's 216-frame decode) in
    a child process.  mfma_busy is rocprofiler-compute's MfmaUtil: busy MFMA cycles over (elapsed
    cycles x 1024 SIMDs), per kernel family; it is set beside the FLOP-derived frac (see note)."""
    import glob
    import shutil
    import subprocess
    import tempfile

    sys.path.insert(0, os.path.join(ROOT, "scripts"))
    import codec_pmc_probe as P

    exe = shutil.which("rocprofv3")
    if exe is None:
        return {"note": "rocprofv3 not on PATH"}
    d = tempfile.mkdtemp(prefix="fishmi_cpmc_", dir="/tmp")
    cmd = ["timeout", "-s", "KILL", str(timeout_s), exe, "--pmc", *P.COUNTERS, "--output-format", "csv", "-d", d,
           "-o", "pmc", "--", sys.executable, os.path.join(ROOT, "scripts", "codec_pmc_probe.py")]
    r = subprocess.run(cmd, cwd="/tmp", stdout=subprocess.DEVNULL, stderr=subprocess.PIPE)
    csvs = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if r.returncode != 0 or not csvs:
        return {"note": f"rocprofv3 --pmc failed (rc {r.returncode}): {r.stderr[-300:].decode(errors='replace')}"}
    fams = P.summarise(csvs[0])
    shutil.rmtree(d, ignore_errors=True)
    a = fams.get("all", {})
    el_ms = a.get("elapsed_Mcycles", 0) * 1e6 / 2.4e9 * 1e3
    return {"mfma_busy": a.get("mfma_busy"), "per_kernel": {k: v for k, v in fams.items() if k != "all"},
            "bf16_mfma_gflop_counted": a.get("bf16_mfma_gflop"),
            "elapsed_ms_at_2.4GHz": round(el_ms, 3),
            "note": "mfma_busy = sum SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs) over one "
                    "config-2 codec decode (rocprofiler-compute MfmaUtil).  Busy cycles = MOPS x 512 / 1024 "
                    "(1024 bf16 flop per busy cycle per SIMD, the dense peak rate).  It reads below the "
                    "FLOP-derived frac because GRBM_GUI_ACTIVE spans each counter-serialised dispatch's ramp "
                    f"and tail ({el_ms:.2f} ms at 2.4 GHz vs {codec_ms:.2f} ms unprofiled) and above it by the "
                    "padded MFMA work (counted vs analytic flops)"}


def stream_peak_gbps(nbytes=2 << 30, reps=10):
    """Measured HBM stream peak (SURVEY.md §8d's STREAM-like figure beside the vendor 8 TB/s):
    libfishmi's fm_stream_peak: the best of several non-temporal read streams (register float4 and
    LDS-DMA forms) and of two float4 copies over 2 GiB buffers (far past the 256 MiB MALL), HIP
    events.  The read stream is the ceiling a weight stream can reach; the copy counts read +
    written bytes."""
    from fishmi import native

    r, c = native.stream_peak(0, nbytes, reps)
    return round(r, 1), round(c, 1)


def box_identity():
    """Which machine and GPU a line was measured on (so per-box speed differences can be checked)."""
    import socket

    import torch

    out = {"host": socket.gethostname()}
    try:
        p = torch.cuda.get_device_properties(0)
        out["gpu"] = p.name
        uuid = getattr(p, "uuid", None)
        if uuid is not None:
            out["gpu_uuid"] = str(uuid)
        out["pci_bus_id"] = getattr(p, "pci_bus_id", None)
        out["cus"] = p.multi_processor_count
    except Exception as e:  # identity is informative only
        out["error"] = str(e)
    return out


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}: launch one rank per GPU")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch

    dist = None
    if world > 1:
        import torch.distributed as dist

        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    from fishmi import dp
    from fishmi.codec import FishMICodec
    from fishmi.config import S2_PRO_CONFIG, S2_PRO_IM_END_ID, CodecConfig, DualARConfig
    from fishmi.llm import DualARModel

    from fishmi import native

    for kv in args.tune:
        k, v = kv.split("=")
        native.tune(k, int(v))
    cfg = DualARConfig._from_fish_qwen3_omni(S2_PRO_CONFIG)
    cfg.im_end_id = S2_PRO_IM_END_ID
    cfg.max_seq_len = max(1024, args.prompt_len + args.frames + 8, 256 + args.batch_frames + 8)
    ccfg = CodecConfig()
    llm = DualARModel.synthetic(cfg, seed=args.seed, log2_half=5, device=local, precision="bf16",
                                max_slots=max(1, args.batch))
    # one codec handle for the utterance leg and the config-3 streams: sized so a 512-frame request
    # vocodes in one pass (the reference decodes a request's codes in one decode_vq_tokens call)
    codec = FishMICodec.synthetic(ccfg, args.seed + 1, local, "bf16", max_frames=max(args.frames, args.batch_frames))

    def sync():
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
            torch.cuda.synchronize()

    def one_step(step):
        # rank 0 owns the request list; each rank gets one utterance (weak scaling)
        if dist is not None:
            prompts = [make_prompt(cfg, args.prompt_len, 1000 * step + r) for r in range(world)] \
                if rank == 0 else None
            prompt = dp.scatter_prompts(prompts, cfg.num_codebooks + 1)
        else:
            prompt = make_prompt(cfg, args.prompt_len, 1000 * step)
        sp = DualARModel.sampling(temperature=0.8, top_p=0.8, top_k=30, seed=7919 * step + rank,
                                  mask_im_end=True)
        pcm, tm = utterance(llm, codec, prompt, sp, args.frames, args.first_chunk, voc2)
        if dist is not None:
            dp.gather_pcm(dp.pcm_to_int16(pcm))
        return tm

    from fishmi import scheduler as S

    voc2 = S.StreamVocoder(codec) if args.overlap_vocode else None
    for w in range(args.warmup):
        one_step(-1 - w)
    sync()
    t0 = time.perf_counter()
    tms = [one_step(k) for k in range(args.steps)]
    sync()
    elapsed = time.perf_counter() - t0
    if voc2 is not None:
        voc2.close()
    firsts = np.array([t["first"] for t in tms], np.float64)
    if dist is not None:
        e = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed = float(e.item())
        f = torch.tensor(firsts, device="cuda")
        fl = [torch.zeros_like(f) for _ in range(world)]
        dist.all_gather(fl, f)
        firsts = torch.cat(fl).cpu().numpy()

    # ---- roofline of the dominant kernel: the decode GEMV ("linear" class).  One decode frame's
    # GEMV launches (exact args, weights and shapes of the timed frames) are recorded and
    # replayed back to back as a graph between two HIP events on the compute stream. ----
    pos = args.prompt_len + args.frames // 2
    llm.prefill(0, make_prompt(cfg, args.prompt_len, 99), DualARModel.sampling(mask_im_end=True))
    llm.decode_frames([0], args.frames // 2)
    avg_us, lin_n, lin_bytes = llm.kernel_bench("linear", reps=20)
    per_launch = lin_bytes / lin_n
    achieved = per_launch / (avg_us * 1e-6) / 1e9
    # per-class split of an eager frame (event-bracketed launches: diagnostic only)
    llm.profile(True)
    llm.decode_frames([0], 8)
    cls_ms = {c: llm.profile_read(c)[0] / 8 for c in ("linear", "attn", "rope", "norm", "sample", "other")}
    llm.profile(False)

    # frame-level: algorithmic frame bytes / graph-replayed frame time inside the timed region
    dec_s = np.mean([t["decode"] for t in tms]) / (args.frames - args.first_chunk)
    frame_bytes = llm.frame_bytes(1, pos)
    ms0, n0, fl0 = codec.profile()
    codec.decode_codes(np.zeros((ccfg.n_codebooks + 1, args.frames), np.int32))
    ms1, n1, fl1 = codec.profile()
    codec_tflops = (fl1 - fl0) / ((ms1 - ms0) * 1e-3) / 1e12
    codec_pmc = {"mfma_busy": None, "note": "not measured (--no-pmc or N>1)"}
    if rank == 0 and world == 1 and not args.no_pmc:
        codec_pmc = pmc_codec_mfma(ms1 - ms0)

    thr = throughput_leg(llm, codec, cfg, args.batch, args.batch_frames, args.waves, sync, dist, world,
                         args.vocode_chunk) \
        if args.batch > 0 else None
    enc = encode_leg(ccfg, local, args.encode_seconds, args.seed) if args.encode_seconds > 0 else None
    longf = longform_leg(ccfg, local, args.longform_turns, args.longform_frames, args.seed,
                         not args.overlap_vocode) \
        if args.longform_turns > 0 and rank == 0 else None

    q8 = q4 = None
    if rank == 0 and not args.no_int8:
        llm.close()
        q8 = quant_leg(cfg, codec, args, local, "int8")
        q4 = quant_leg(cfg, codec, args, local, "int4")
    stream_gbps = stream_peak_gbps() if rank == 0 else (None, None)
    box = box_identity() if rank == 0 else None
    traffic, traffic_note = None, "not measured (--no-pmc or N>1)"
    fused_wo = {"note": "not measured (--no-pmc or N>1)"}
    if rank == 0 and world == 1 and not args.no_pmc:
        traffic, traffic_note = pmc_gemv_traffic()
        tr = trace_decode_kernels()
        if "fattn_wo" in tr and "linear" in tr:
            # the fused fast attention + wo (fm_rowgemv.hip fattn_wo_kernel): its wo weights count as
            # decode-linear bytes; one launch per fast layer and codebook, less codebook 0's last layer
            # (fast_tail: only its K / V rows are needed)
            fw_n = cfg.num_codebooks * cfg.n_fast_layer - 1
            fw_bytes = 2 * cfg.fast_dim * cfg.fast_n_head * cfg.fast_head_dim
            fw_us, lin_tr_us = tr["fattn_wo"][1], tr["linear"][1]
            both = (lin_bytes + fw_n * fw_bytes) / (lin_n * lin_tr_us + fw_n * fw_us) / 1e3  # GB/s
            fused_wo = {"launches_per_frame": fw_n, "bytes_per_launch": fw_bytes,
                        "avg_launch_us_rocprof": round(fw_us, 3),
                        "achieved": round(fw_bytes / fw_us / 1e3, 1), "unit": "GB/s",
                        "frac": round(fw_bytes / fw_us / 1e3 / HBM_PEAK_GBPS, 4),
                        "linear_avg_launch_us_rocprof": round(lin_tr_us, 3),
                        "linear_incl_fused_wo_frac": round(both / HBM_PEAK_GBPS, 4),
                        "method": "rocprofv3 --kernel-trace pass over scripts/pmc_probe.py in this run (prefill + 4 "
                                  "batch-1 frames): per-launch durations; bytes = the fast model's wo weights "
                                  "(the attention's <= 10 cached K / V rows are not counted)"}
        else:
            fused_wo = tr

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        del llm, codec
        cpu = cpu_baseline(cfg, ccfg, make_prompt(cfg, args.prompt_len, 0), args.frames,
                           args.cpu_frames, args.cpu_codec_frames, args.seed)

    if rank == 0:
        audio_s = world * args.steps * args.frames / FRAME_RATE
        out = {
            "metric": METRIC,
            "value": round(audio_s / elapsed, 4),
            "unit": "audio-sec/wall-sec",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16",
            "data": "synthetic: seeded random bf16 weights at S2-Pro 4B shapes, random prompt ids, "
                    "<|im_end|> masked (fixed length)",
            "config": {"workload": f"BASELINE config 2 per GPU: one utterance = {args.prompt_len}-token "
                                   f"prompt + {args.frames} Dual-AR frames (top_k 30, top_p 0.8, temp 0.8) "
                                   f"+ codec decode [1,10,{args.frames}] -> {args.frames * 2048} samples",
                       "global_batch": world, "frames": args.frames, "prompt_len": args.prompt_len,
                       "first_chunk_frames": args.first_chunk, "vocoder_chunks": "first_chunk_frames, then growing 4x",
                       "vocoder": "serial" if not args.overlap_vocode else
                                  "host thread, codec HIP stream overlapped with the next chunk's decode",
                       "parallelism": f"dp{world}"},
            "p50_first_sample_ms": round(float(np.median(firsts)) * 1e3, 2),
            "p90_first_sample_ms": round(float(np.percentile(firsts, 90)) * 1e3, 2),
            "per_stream_rtf": round(args.frames / FRAME_RATE / np.mean([t["total"] for t in tms]), 4),
            "breakdown_ms": {k: round(float(np.mean([t[k] for t in tms])) * 1e3, 2)
                             for k in ("prefill", "head", "decode", "codec", "total")},
            "roofline": {"kernel": "decode linear layers: gemv_kernel (16-row MFMA tiles: w1||w3, heads, first-layer "
                                   "wqkv) + rowgemv_kernel (row blocks: wo / w2 with the residual epilogue, wqkv "
                                   "with the RMSNorm prologue)",
                         "bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 4),
                         "traffic": traffic, "traffic_source": traffic_note,
                         "stream_peak_measured": {"read": stream_gbps[0], "copy": stream_gbps[1], "unit": "GB/s",
                                                  "frac_of_read_peak": round(achieved / stream_gbps[0], 4)
                                                  if stream_gbps[0] else None,
                                                  "method": "fm_stream_peak: best of non-temporal float4 "
                                                            "read streams (4 / 8 in flight per thread, 8 / 16 "
                                                            "blocks per CU) and non-temporal LDS-DMA streams "
                                                            "(16 / 32 KiB in flight per wave); best of two "
                                                            "float4 copies (read + write bytes); 2 GiB "
                                                            "buffers, 10 launches each, HIP events"},
                         "fused_fast_wo": fused_wo,
                         "bytes_per_launch": int(per_launch),
                         "avg_launch_us": round(avg_us, 3), "launches_per_frame": int(lin_n),
                         "method": "one frame's GEMV launches replayed x20 as a graph, HIP events on "
                                   "the compute stream"},
            "frame_roofline": {"bytes_per_frame": int(frame_bytes), "ms_per_frame": round(dec_s * 1e3, 4),
                               "achieved": round(frame_bytes / dec_s / 1e9, 1), "unit": "GB/s",
                               "frac": round(frame_bytes / dec_s / 1e9 / HBM_PEAK_GBPS, 4),
                               "eager_event_class_ms_per_frame": {k: round(v, 4) for k, v in cls_ms.items()}},
            "codec_roofline": {"bound": "mfma", "achieved": round(codec_tflops, 2),
                               "peak": BF16_DENSE_TFLOPS, "unit": "TFLOP/s",
                               "frac": round(codec_tflops / BF16_DENSE_TFLOPS, 4), **codec_pmc},
            "throughput": thr,
            "encode": enc,
            "longform": longf,
            "int8": q8,
            "int4": q4,
            "cpu_baseline": cpu,
            "box": box,
        }
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
