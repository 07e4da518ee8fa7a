"""Engine and HTTP wire layer (fishmi.tts / fishmi.server) against the reference's contract
(fish_speech/inference_engine/__init__.py:41-131, tools/server/inference.py:12-45,
tools/server/views.py:146-205, tools/api_server.py:33-45), on CPU with a scripted LLM worker and a
numpy codec stand-in.  The GPU path (real worker + HIP codec) is tests/test_gpu_tts.py."""
import io
import queue
import threading
import wave

import numpy as np
import pytest

fastapi = pytest.importorskip("fastapi")
msgpack = pytest.importorskip("msgpack")


class FakeCodec:
    sample_rate = 44100
    frame_length = 2048
    device = "cpu"

    def __init__(self):
        self.encoded = []

    def decode_codes(self, codes):
        c = np.asarray(codes)
        t = np.arange(c.shape[1] * self.frame_length, dtype=np.float32)
        return (0.5 * np.sin(t * 0.01 + float(c[0, 0]))).astype(np.float32)

    def encode_audio(self, audio):
        self.encoded.append(audio.size)
        return np.full((10, (audio.size + 2047) // 2048), 7, np.int32)


def fake_worker(batches, fail=False):
    """Scripted B1 worker: one (10, n) code matrix per text batch, then "next" (or an error)."""
    from fishmi.engine import GenerateResponse, WrappedGenerateResponse

    q = queue.Queue()
    seen = []

    def run():
        while True:
            item = q.get()
            if item is None:
                return
            seen.append(item.request)
            if fail:
                item.response_queue.put(WrappedGenerateResponse("error", RuntimeError("boom")))
                continue
            for i, n in enumerate(batches):
                codes = np.full((10, n), i + 1, np.int32)
                item.response_queue.put(WrappedGenerateResponse("success", GenerateResponse("sample", codes, f"b{i}")))
            item.response_queue.put(WrappedGenerateResponse("success", GenerateResponse("next")))

    threading.Thread(target=run, daemon=True).start()
    return q, seen


def _engine(batches=(3, 2), fail=False, tmp_path=None):
    from fishmi.tts import TTSInferenceEngine

    q, seen = fake_worker(batches, fail)
    eng = TTSInferenceEngine(q, FakeCodec(), references_dir=str(tmp_path) if tmp_path else "references")
    return eng, seen


def _wav(x, sr=22050, width=2):
    buf = io.BytesIO()
    with wave.open(buf, "wb") as w:
        w.setnchannels(1)
        w.setsampwidth(width)
        w.setframerate(sr)
        w.writeframes((x * 32767).astype("<i2").tobytes())
    return buf.getvalue()


def test_engine_streaming_results():
    from fishmi.tts import ServeTTSRequest, wav_chunk_header

    eng, seen = _engine()
    res = list(eng.inference(ServeTTSRequest(text="hello", streaming=True, seed=3)))
    assert [r.code for r in res] == ["header", "segment", "segment", "final"]
    assert res[0].audio[1].tobytes() == wav_chunk_header(44100)
    segs = [r.audio[1] for r in res[1:3]]
    assert [s.size for s in segs] == [3 * 2048, 2 * 2048]
    np.testing.assert_array_equal(res[-1].audio[1], np.concatenate(segs))
    assert seen[0]["text"] == "hello" and seen[0]["seed"] == 3 and seen[0]["chunk_length"] == 200


def test_engine_error_and_empty():
    from fishmi.tts import ServeTTSRequest

    eng, _ = _engine(fail=True)
    res = list(eng.inference(ServeTTSRequest(text="x")))
    # the reference yields the worker's error, then (no segments) its "No audio generated" error
    assert [r.code for r in res] == ["error", "error"] and "boom" in str(res[0].error)
    eng, _ = _engine(batches=())
    res = list(eng.inference(ServeTTSRequest(text="x")))
    assert res[-1].code == "error" and "No audio" in str(res[-1].error)


def test_references_encoded_once_per_hash(tmp_path):
    from fishmi.tts import ServeReferenceAudio, ServeTTSRequest

    eng, seen = _engine(tmp_path=tmp_path)
    ref = ServeReferenceAudio(audio=_wav(np.sin(np.arange(22050) * 0.05)), text="ref text")
    list(eng.inference(ServeTTSRequest(text="a", references=[ref], use_memory_cache="on")))
    list(eng.inference(ServeTTSRequest(text="b", references=[ref], use_memory_cache="on")))
    assert eng.decoder_model.encoded == [44100]  # resampled 22.05 -> 44.1 kHz, encoded once
    assert seen[1]["prompt_text"] == ["ref text"] and seen[1]["prompt_tokens"][0].shape == (10, 22)
    # reference_id folder with .wav + .lab
    d = tmp_path / "alice"
    d.mkdir()
    (d / "a.wav").write_bytes(_wav(np.zeros(4410), 44100))
    (d / "a.lab").write_text("alice says hi")
    list(eng.inference(ServeTTSRequest(text="c", reference_id="alice")))
    assert seen[2]["prompt_text"] == ["alice says hi"] and eng.list_reference_ids() == ["alice"]


def test_read_wav_formats():
    from fishmi.tts import read_wav

    x = (0.25 * np.sin(np.arange(1000) * 0.1)).astype(np.float32)
    np.testing.assert_allclose(read_wav(_wav(x, 44100), 44100), x, atol=1e-4)
    with pytest.raises(ValueError):
        read_wav(b"ID3\x03mp3data...", 44100)


def _client(**kw):
    from fastapi.testclient import TestClient

    from fishmi.server import create_app

    eng, seen = _engine(**{k: v for k, v in kw.items() if k in ("batches", "fail")})
    app = create_app(eng, max_text_length=kw.get("max_text_length", 0), api_key=kw.get("api_key"))
    return TestClient(app), eng, seen


def test_http_health_and_auth():
    c, _, _ = _client(api_key="sekrit")
    assert c.get("/v1/health").status_code == 401
    r = c.get("/v1/health", headers={"Authorization": "Bearer sekrit"})
    assert r.status_code == 200 and r.json() == {"status": "ok"}
    c, _, _ = _client()
    assert c.post("/v1/health").json() == {"status": "ok"}


def test_http_reference_management(tmp_path):
    """/v1/references/add | list | update | delete (tools/server/views.py:208-470): the reference's
    status codes (400 bad input, 404 unknown id, 409 existing id) and folder layout (sample.wav +
    sample.lab), over msgpack, JSON (base64 audio) and multipart/form-data; the added voice is then
    usable as a reference_id."""
    import base64

    from fastapi.testclient import TestClient

    from fishmi.server import create_app
    from fishmi.tts import ServeTTSRequest

    eng, seen = _engine(tmp_path=tmp_path)
    c = TestClient(create_app(eng))
    wav = _wav(np.sin(np.arange(4410) * 0.05), 44100)
    mp = lambda d: dict(content=msgpack.packb(d, use_bin_type=True),  # noqa: E731
                        headers={"Content-Type": "application/msgpack"})
    r = c.post("/v1/references/add", **mp({"id": "alice", "audio": wav, "text": "alice says hi"}))
    assert r.status_code == 200
    assert msgpack.unpackb(r.content, raw=False) == {"success": True, "reference_id": "alice",
                                                      "message": "Reference voice 'alice' added successfully"}
    assert (tmp_path / "alice" / "sample.wav").read_bytes() == wav
    assert (tmp_path / "alice" / "sample.lab").read_text() == "alice says hi"
    assert c.post("/v1/references/add", **mp({"id": "alice", "audio": wav, "text": "x"})).status_code == 409
    assert c.post("/v1/references/add", **mp({"id": "bad/id", "audio": wav, "text": "x"})).status_code == 400
    assert c.post("/v1/references/add", **mp({"id": "e", "audio": wav, "text": " "})).status_code == 400
    assert c.post("/v1/references/add", **mp({"id": "e", "audio": b"", "text": "t"})).status_code == 400
    r = c.post("/v1/references/add?format=json", json={"id": "bob", "audio": base64.b64encode(wav).decode(),
                                                       "text": "bob text"})
    assert r.status_code == 200 and r.json()["success"] is True
    r = c.post("/v1/references/add", data={"id": "carol", "text": "carol text"},
               files={"audio": ("c.wav", wav, "audio/wav")})
    assert r.status_code == 200 and (tmp_path / "carol" / "sample.wav").read_bytes() == wav
    r = c.get("/v1/references/list?format=json")
    assert r.json()["reference_ids"] == ["alice", "bob", "carol"]
    # the added voice conditions a request by id
    list(eng.inference(ServeTTSRequest(text="x", reference_id="alice", use_memory_cache="on")))
    assert seen[-1]["prompt_text"] == ["alice says hi"]
    # rename: cache entry follows; 409 onto an existing id, 404 from an unknown one, 400 same id
    r = c.post("/v1/references/update?format=json", json={"old_reference_id": "alice", "new_reference_id": "alicia"})
    assert r.status_code == 200 and r.json()["new_reference_id"] == "alicia"
    assert "alicia" in eng.ref_by_id and "alice" not in eng.ref_by_id
    assert c.post("/v1/references/update", json={"old_reference_id": "bob",
                                                 "new_reference_id": "carol"}).status_code == 409
    assert c.post("/v1/references/update", json={"old_reference_id": "nobody",
                                                 "new_reference_id": "x"}).status_code == 404
    assert c.post("/v1/references/update", json={"old_reference_id": "bob",
                                                 "new_reference_id": "bob"}).status_code == 400
    r = c.request("DELETE", "/v1/references/delete?format=json", json={"reference_id": "bob"})
    assert r.status_code == 200 and not (tmp_path / "bob").exists()
    assert c.request("DELETE", "/v1/references/delete", json={"reference_id": "bob"}).status_code == 404
    assert c.get("/v1/references/list?format=json").json()["reference_ids"] == ["alicia", "carol"]
    # an unexpected failure: the reference's 500 body, not FastAPI's plain-text error
    orig = eng.rename_reference

    def broken(old, new):
        raise RuntimeError("disk on fire")

    eng.rename_reference = broken
    try:
        r = c.post("/v1/references/update?format=json", json={"old_reference_id": "carol", "new_reference_id": "z"})
        assert r.status_code == 500
        assert r.json() == {"success": False, "message": "Internal server error occurred",
                            "old_reference_id": "carol", "new_reference_id": "z"}
    finally:
        eng.rename_reference = orig


def test_http_tts_wav_and_stream_json_and_msgpack():
    from fishmi.tts import wav_chunk_header

    c, eng, _ = _client()
    r = c.post("/v1/tts", json={"text": "hello"})
    assert r.status_code == 200 and r.headers["content-type"] == "audio/wav"
    with wave.open(io.BytesIO(r.content)) as w:
        assert w.getframerate() == 44100 and w.getnframes() == 5 * 2048
    body = msgpack.packb({"text": "hello", "streaming": True}, use_bin_type=True)
    r = c.post("/v1/tts", content=body, headers={"Content-Type": "application/msgpack"})
    assert r.status_code == 200
    hdr = wav_chunk_header(44100)
    assert r.content[: len(hdr)] == hdr
    pcm = np.frombuffer(r.content[len(hdr):], "<i2")
    exp = np.concatenate([(eng.decoder_model.decode_codes(np.full((10, n), i + 1)) * 32768).astype(np.int16)
                          for i, n in enumerate((3, 2))])
    np.testing.assert_array_equal(pcm, exp)  # the reference's x * 32768 -> int16 chunks


def test_http_tts_errors():
    c, _, _ = _client(max_text_length=5)
    assert c.post("/v1/tts", json={"text": "too long text"}).status_code == 400
    c, _, _ = _client()
    assert c.post("/v1/tts", json={"text": "x", "streaming": True, "format": "mp3"}).status_code == 400
    assert c.post("/v1/tts", json={"text": "x", "chunk_length": 5}).status_code == 422
    c, _, _ = _client(fail=True)
    assert c.post("/v1/tts", json={"text": "x"}).status_code == 500
    # streaming: the header has gone out before the worker fails, so the body just ends there
    from fishmi.tts import wav_chunk_header

    r = c.post("/v1/tts", json={"text": "x", "streaming": True})
    assert r.status_code == 200 and r.content == wav_chunk_header(44100)


def test_http_vqgan_routes():
    c, eng, _ = _client()
    wav = _wav(np.zeros(44100 + 100), 44100)
    r = c.post("/v1/vqgan/encode", content=msgpack.packb({"audios": [wav]}, use_bin_type=True),
               headers={"Content-Type": "application/msgpack"})
    tok = msgpack.unpackb(r.content, raw=False)["tokens"]
    assert np.asarray(tok).shape == (1, 10, 22)
    r = c.post("/v1/vqgan/decode?format=json", json={"tokens": [[[1] * 4] * 10]})
    assert r.status_code == 200
    r = c.post("/v1/vqgan/decode", content=msgpack.packb({"tokens": [[[1] * 4] * 10]}, use_bin_type=True),
               headers={"Content-Type": "application/msgpack"})
    a = np.frombuffer(msgpack.unpackb(r.content, raw=False)["audios"][0], np.float16)
    assert a.size == 4 * 2048


class FakeStreamCodec(FakeCodec):
    """A codec whose streamed chunks continue a carried position, like the HIP codec's causal state:
    a chunk decoded on the wrong context comes out shifted."""

    def decode_codes(self, codes):
        c = np.asarray(codes)
        t = np.arange(c.shape[1] * self.frame_length, dtype=np.float32)
        return (0.5 * np.sin(t * 0.01 + np.repeat(c[0].astype(np.float32), self.frame_length))).astype(np.float32)

    def open_stream(self):
        codec = self

        class S:
            pos = 0
            closed = False

            def decode_chunk(self, codes):
                assert not self.closed
                c = np.asarray(codes)
                t = np.arange(self.pos, self.pos + c.shape[1] * codec.frame_length, dtype=np.float32)
                self.pos += c.shape[1] * codec.frame_length
                return (0.5 * np.sin(t * 0.01 + np.repeat(c[0].astype(np.float32), codec.frame_length))).astype(np.float32)

            def close(self):
                self.closed = True

        return S()

    def stream_reset(self):  # the handle's single stream must not be used by concurrent requests
        raise AssertionError("shared codec stream used")

    decode_chunk = stream_reset


def test_interleaved_streaming_requests_keep_their_own_codec_state():
    """Two latency=balanced streaming requests consumed alternately: each one's audio equals the
    one-shot decode of its own codes (one shared carried state corrupted the other)."""
    from fishmi.engine import GenerateResponse, WrappedGenerateResponse
    from fishmi.tts import ServeTTSRequest, TTSInferenceEngine

    q = queue.Queue()
    codes_of = {}

    def run():
        while True:
            item = q.get()
            if item is None:
                return
            base = 3 if item.request["text"] == "a" else 40
            chunks = [np.full((10, n), base + i, np.int32) for i, n in enumerate((2, 3, 1))]
            codes_of[item.request["text"]] = np.concatenate(chunks, axis=1)
            for i, c in enumerate(chunks):
                item.response_queue.put(WrappedGenerateResponse("success", GenerateResponse("sample", c, "t", stream=i)))
            item.response_queue.put(WrappedGenerateResponse("success", GenerateResponse("next")))

    threading.Thread(target=run, daemon=True).start()
    codec = FakeStreamCodec()
    eng = TTSInferenceEngine(q, codec)
    ga = eng.inference(ServeTTSRequest(text="a", streaming=True, latency="balanced"))
    gb = eng.inference(ServeTTSRequest(text="b", streaming=True, latency="balanced"))
    outs = {"a": [], "b": []}
    live = {"a": ga, "b": gb}
    while live:
        for k in list(live):
            try:
                r = next(live[k])
            except StopIteration:
                del live[k]
                continue
            if r.code == "segment":
                outs[k].append(r.audio[1])
    q.put(None)
    for k in ("a", "b"):
        np.testing.assert_allclose(np.concatenate(outs[k]), codec.decode_codes(codes_of[k]), atol=1e-6)
