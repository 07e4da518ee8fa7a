"""GPU: BASELINE config 5's voice-clone chain and the TTS engine / HTTP seam on libfishmi.

* Chain parity (tests/golden/engine_clone.npz, oracle/gen_goldens.py engine_clone): reference
  audio -> fm_codec_encode (codec_enc_tiny weights, fp32) must give the reference DAC.encode's
  codes, and the native generate_long (llm_a, tiny tokenizer, greedy fp32) voice-cloned on them
  must give the reference generate_long's codes, batch by batch.
* Engine / wire: TTSInferenceEngine over the real B1 worker and HIP codec streams a WAV header then
  int16 chunks equal to the codec decode of each batch's codes (tools/server/inference.py:12-45),
  and POST /v1/tts returns the same audio."""
import io
import json
import os
import shutil
import wave

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu


def _ckpt(tmp_path):
    d = tmp_path / "ckpt"
    shutil.copytree(os.path.join(GOLDEN, "llm_a"), d)
    for f in ("tokenizer.json", "tokenizer_config.json"):
        shutil.copy(os.path.join(GOLDEN, "tok_tiny", f), d / f)
    return str(d)


def _codec(golden):
    from fishmi.codec import FishMICodec
    from fishmi.config import CodecConfig

    g = golden("codec_enc_tiny.npz")
    spec = json.loads(str(g["spec"]))
    m = FishMICodec(CodecConfig.from_spec(spec), 0, "fp32", max_frames=64)
    m.enable_encoder(spec["encoder_dim"], [int(v) for v in g["enc_layers"]])
    m.synth(int(g["synth_seed"]))
    m.synth_encoder(int(g["synth_seed"]))
    m.finalize()
    return m


def test_voice_clone_chain_matches_reference(golden, tmp_path):
    import signals

    from fishmi import engine
    from fishmi.llm import DualARModel

    g = golden("engine_clone.npz")
    codec = _codec(golden)
    codes = codec.encode_audio(signals.reference_audio(int(g["n_samples"]), int(g["audio_seed"])))
    np.testing.assert_array_equal(codes, g["ref_codes"])
    m = DualARModel.from_pretrained(_ckpt(tmp_path), device=0, precision="fp32", max_length=2560)
    outs = list(engine.generate_long(model=m, text=str(g["text"]), max_new_tokens=9, top_p=0.9, top_k=1,
                                     temperature=0.7, chunk_length=30, prompt_text=[str(g["prompt_text"])],
                                     prompt_tokens=[codes]))
    assert [o.action for o in outs] == json.loads(str(g["actions"]))
    for i, o in enumerate([o for o in outs if o.action == "sample"]):
        np.testing.assert_array_equal(o.codes, g[f"codes_{i}"])


def _wav(x, sr):
    buf = io.BytesIO()
    with wave.open(buf, "wb") as w:
        w.setnchannels(1)
        w.setsampwidth(2)
        w.setframerate(sr)
        w.writeframes((np.clip(x, -1, 1) * 32767).astype("<i2").tobytes())
    return buf.getvalue()


def test_tts_engine_and_http_stream(golden, tmp_path):
    import signals

    from fishmi import engine as E
    from fishmi.llm import DualARModel
    from fishmi.tts import ServeReferenceAudio, ServeTTSRequest, TTSInferenceEngine, wav_chunk_header

    m = DualARModel.from_pretrained(_ckpt(tmp_path), device=0, precision="bf16", max_length=2560)
    codec = _codec(golden)
    q = E.launch_thread_safe_queue(None, 0, "bf16", model=m)
    eng = TTSInferenceEngine(q, codec)
    wav = _wav(signals.reference_audio(6 * 2048, 5), 44100)
    req = dict(text="<|speaker:0|>One sentence. <|speaker:0|>And another one here.", chunk_length=100,
               references=[ServeReferenceAudio(audio=wav, text="ref words")], seed=123, max_new_tokens=12,
               streaming=True)
    res = list(eng.inference(ServeTTSRequest(**req)))
    assert res[0].code == "header" and res[-1].code == "final"
    segs = [r.audio[1] for r in res if r.code == "segment"]
    assert segs and all(s.size % 2048 == 0 for s in segs)
    np.testing.assert_array_equal(res[-1].audio[1], np.concatenate(segs))
    # the same request straight through generate_long: the engine's segments are the codec decode
    # of those codes (same seed -> same sampled streams)
    ptok = codec.encode_audio(__import__("fishmi.tts", fromlist=["read_wav"]).read_wav(wav, 44100))
    outs = [o for o in E.generate_long(model=m, text=req["text"], max_new_tokens=12, top_p=0.8, temperature=0.8,
                                       chunk_length=100, prompt_text=["ref words"], prompt_tokens=[ptok], seed=123)
            if o.action == "sample"]
    assert len(outs) == len(segs)
    for o, s in zip(outs, segs):
        np.testing.assert_array_equal(codec.decode_codes(o.codes), s)
    # HTTP: the streamed body is the header + int16 chunks of the same segments
    from fastapi.testclient import TestClient

    from fishmi.server import create_app

    c = TestClient(create_app(eng))
    body = dict(req, references=[{"audio": __import__("base64").b64encode(wav).decode(), "text": "ref words"}])
    r = c.post("/v1/tts", json=body)
    assert r.status_code == 200
    hdr = wav_chunk_header(44100)
    assert r.content[: len(hdr)] == hdr
    pcm = np.frombuffer(r.content[len(hdr):], "<i2")
    np.testing.assert_array_equal(pcm, np.concatenate([(s * 32768).astype(np.int16) for s in segs]))
    q.put(None)


def test_streamed_generation_and_vocoding(golden, tmp_path):
    """generate_long(stream_frames=K) yields each batch's codes K columns at a time; their
    concatenation equals the batch's codes from the one-shot flow (same seed), and the engine's
    latency="balanced" stream vocodes them as one causal stream: the PCM equals the one-shot decode
    of the batch's codes (the codec is causal end to end)."""
    from fishmi import engine as E
    from fishmi.llm import DualARModel
    from fishmi.tts import ServeTTSRequest, TTSInferenceEngine

    m = DualARModel.from_pretrained(_ckpt(tmp_path), device=0, precision="bf16", max_length=2560)
    kw = dict(model=m, text="<|speaker:0|>Streaming turn one, long enough to fill most of a batch by itself. "
                             "<|speaker:1|>Streaming turn two, which has to land in a second text batch.",
              max_new_tokens=23, top_p=0.8, temperature=0.8, chunk_length=100, seed=7)
    whole = [o for o in E.generate_long(**kw) if o.action == "sample"]
    chunks = [o for o in E.generate_long(stream_frames=5, **kw) if o.action == "sample"]
    assert all(c.stream is not None for c in chunks) and max(c.codes.shape[1] for c in chunks) <= 5
    per_batch, cur = [], None
    for c in chunks:
        if c.stream == 0:
            cur = []
            per_batch.append(cur)
        cur.append(c.codes)
    assert len(per_batch) == len(whole) == 2
    for w, parts in zip(whole, per_batch):
        np.testing.assert_array_equal(np.concatenate(parts, axis=1), w.codes)
    # geometric chunks (the config-5 bench schedule: 1, 4, 8, 8, ... frames) give the same codes
    grown = [o for o in E.generate_long(stream_frames=1, stream_growth=4, stream_max=8, **kw) if o.action == "sample"]
    per_batch, cur = [], None
    for c in grown:
        if c.stream == 0:
            assert c.codes.shape[1] == 1
            cur = []
            per_batch.append(cur)
        cur.append(c.codes)
    assert len(per_batch) == 2 and max(c.codes.shape[1] for c in grown) <= 8
    for w, parts in zip(whole, per_batch):
        np.testing.assert_array_equal(np.concatenate(parts, axis=1), w.codes)
    codec = _codec(golden)
    q = E.launch_thread_safe_queue(None, 0, "bf16", model=m)
    eng = TTSInferenceEngine(q, codec, stream_frames=5)
    res = list(eng.inference(ServeTTSRequest(text=kw["text"], max_new_tokens=23, chunk_length=100, seed=7,
                                             streaming=True, latency="balanced")))
    segs = [r.audio[1] for r in res if r.code == "segment"]
    assert len(segs) == len(chunks)
    np.testing.assert_array_equal(np.concatenate(segs),
                                  np.concatenate([codec.decode_codes(w.codes) for w in whole]))
    q.put(None)
