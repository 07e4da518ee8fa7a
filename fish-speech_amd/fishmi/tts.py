"""TTS inference engine on libfishmi: the drop-in for fish_speech.inference_engine (SURVEY.md §8b B5,
§8f row 3).

Mirrors the reference's engine-side seam:
  * ServeTTSRequest / ServeReferenceAudio      fish_speech/utils/schema.py:61-107 (request fields and
                                               ranges: the wire contract of POST /v1/tts)
  * InferenceResult, wav_chunk_header          fish_speech/inference_engine/utils.py:9-29
  * TTSInferenceEngine.inference               fish_speech/inference_engine/__init__.py:22-131
      references by hash / by id               inference_engine/reference_loader.py:20-107
      encode_reference, decode_vq_tokens       inference_engine/vq_manager.py:16-52
      send_Llama_request                       inference_engine/__init__.py:144-177
  * inference_wrapper (header, int16 chunks)   tools/server/inference.py:12-45

The LLM side is the B1 worker (fishmi.engine.launch_thread_safe_queue); the codec is
fishmi.codec.FishMICodec (HIP encode for voice-clone references, HIP decode per segment).

Audio I/O: reference audio arrives as WAV bytes (PCM 16/24/32-bit or float32, any rate, mono or
multi-channel: channels are averaged, and the rate is converted to 44.1 kHz by a polyphase
resampler). The reference decodes with torchaudio/ffmpeg, which are absent here. Compressed
formats (mp3, opus, flac) are rejected with a clear error.
"""
from __future__ import annotations

import io
import logging
import queue
import re
import threading
import wave
from dataclasses import dataclass
from fractions import Fraction
from hashlib import sha256
from pathlib import Path
from typing import Generator, List, Literal, Optional, Tuple

import numpy as np

from .engine import GenerateRequest, GenerateResponse, WrappedGenerateResponse

log = logging.getLogger("fishmi.tts")

AMPLITUDE = 32768  # tools/server/inference.py:9


# ---------------------------------------------------------------------------------------------
# wire schema (fish_speech/utils/schema.py)
# ---------------------------------------------------------------------------------------------
try:
    import base64

    from pydantic import BaseModel, Field, model_validator

    class ServeReferenceAudio(BaseModel):
        audio: bytes
        text: str

        @model_validator(mode="before")
        @classmethod
        def _b64(cls, values):
            a = values.get("audio") if isinstance(values, dict) else None
            if isinstance(a, str) and len(a) > 255:  # base64 in JSON bodies
                try:
                    values["audio"] = base64.b64decode(a)
                except Exception:
                    pass
            return values

    class ServeTTSRequest(BaseModel):
        text: str
        chunk_length: int = Field(200, ge=100, le=1000)
        format: Literal["wav", "pcm", "mp3", "opus"] = "wav"
        latency: Literal["normal", "balanced"] = "normal"
        references: List[ServeReferenceAudio] = []
        reference_id: Optional[str] = None
        seed: Optional[int] = None
        use_memory_cache: Literal["on", "off"] = "off"
        normalize: bool = True
        streaming: bool = False
        max_new_tokens: int = 1024
        top_p: float = Field(0.8, ge=0.1, le=1.0)
        repetition_penalty: float = Field(1.1, ge=0.9, le=2.0)
        temperature: float = Field(0.8, ge=0.1, le=1.0)
except ImportError:  # pragma: no cover - pydantic is part of the image
    ServeReferenceAudio = ServeTTSRequest = None


@dataclass
class InferenceResult:
    code: Literal["header", "segment", "error", "final"]
    audio: Optional[Tuple[int, np.ndarray]]
    error: Optional[Exception]


def wav_chunk_header(sample_rate: int = 44100, bit_depth: int = 16, channels: int = 1) -> bytes:
    """A WAV header with zero data length: streaming clients read int16 PCM until EOF."""
    buf = io.BytesIO()
    with wave.open(buf, "wb") as w:
        w.setnchannels(channels)
        w.setsampwidth(bit_depth // 8)
        w.setframerate(sample_rate)
    return buf.getvalue()


def wav_bytes(pcm: np.ndarray, sample_rate: int) -> bytes:
    """float PCM in [-1, 1] -> a complete 16-bit mono WAV file."""
    buf = io.BytesIO()
    with wave.open(buf, "wb") as w:
        w.setnchannels(1)
        w.setsampwidth(2)
        w.setframerate(sample_rate)
        w.writeframes((np.clip(pcm, -1.0, 1.0) * 32767.0).astype("<i2").tobytes())
    return buf.getvalue()


def read_wav(data: bytes, target_sr: int) -> np.ndarray:
    """WAV bytes -> mono float32 at target_sr (ReferenceLoader.load_audio, reference_loader.py:109-128)."""
    if len(data) >= 4 and data[:4] != b"RIFF":
        raise ValueError("reference audio must be WAV (RIFF); compressed formats need ffmpeg, absent here")
    with wave.open(io.BytesIO(data), "rb") as w:
        sr, ch, width, n = w.getframerate(), w.getnchannels(), w.getsampwidth(), w.getnframes()
        raw = w.readframes(n)
    if width == 2:
        x = np.frombuffer(raw, "<i2").astype(np.float32) / 32768.0
    elif width == 4:
        x = np.frombuffer(raw, "<i4").astype(np.float32) / 2147483648.0
    elif width == 3:
        b = np.frombuffer(raw, np.uint8).reshape(-1, 3).astype(np.int32)
        v = b[:, 0] | (b[:, 1] << 8) | (b[:, 2] << 16)
        x = (np.where(v >= 1 << 23, v - (1 << 24), v)).astype(np.float32) / 8388608.0
    elif width == 1:
        x = (np.frombuffer(raw, np.uint8).astype(np.float32) - 128.0) / 128.0
    else:
        raise ValueError(f"unsupported WAV sample width {width}")
    x = x.reshape(-1, ch).mean(axis=1) if ch > 1 else x
    if sr != target_sr:
        from scipy.signal import resample_poly

        f = Fraction(target_sr, sr).limit_denominator(1000)
        x = resample_poly(x, f.numerator, f.denominator).astype(np.float32)
    return np.ascontiguousarray(x, np.float32)


AUDIO_EXTENSIONS = {".wav"}


# ---------------------------------------------------------------------------------------------
# engine
# ---------------------------------------------------------------------------------------------
class TTSInferenceEngine:
    """fish_speech.inference_engine.TTSInferenceEngine on libfishmi.

    llama_queue: the B1 worker's input queue (fishmi.engine.launch_thread_safe_queue).
    decoder_model: a FishMICodec (its encoder enabled for voice-clone references)."""

    def __init__(self, llama_queue: "queue.Queue", decoder_model, precision="bf16", compile: bool = False,
                 references_dir: str = "references", stream_frames: int = 22, reuse_prefix: bool = False):
        self.llama_queue = llama_queue
        self.decoder_model = decoder_model
        self.precision = precision
        self.compile = compile
        self.references_dir = Path(references_dir)
        self.ref_by_id: dict = {}
        self.ref_by_hash: dict = {}
        self._codec_lock = threading.Lock()  # one codec handle, called from request threads
        # streaming requests with latency="balanced": codes arrive `stream_frames` columns at a time
        # (generate_long(stream_frames=...)) and are vocoded as one causal stream per text batch
        self.stream_frames = stream_frames
        # prefix-KV reuse across a request's text batches (generate_long reuse_prefix): opt-in, the
        # default is the reference's whole-conversation re-prefill
        self.reuse_prefix = reuse_prefix

    # ---- references (reference_loader.py) -------------------------------------------------
    def encode_reference(self, reference_audio: bytes, enable_reference_audio: bool = True):
        """VQManager.encode_reference (vq_manager.py:24-52): audio -> codes (C, T) via DAC.encode."""
        if not enable_reference_audio or reference_audio is None:
            return None
        audio = read_wav(reference_audio, self.decoder_model.sample_rate)
        log.info("Loaded audio with %.2f seconds", audio.size / self.decoder_model.sample_rate)
        with self._codec_lock:
            codes = self.decoder_model.encode_audio(audio)
        log.info("Encoded prompt: %s", codes.shape)
        return codes

    def load_by_hash(self, references, use_cache: str):
        tokens, texts = [], []
        for ref in references:
            h = sha256(ref.audio).hexdigest()
            if use_cache == "off" or h not in self.ref_by_hash:
                t = self.encode_reference(ref.audio, True)
                self.ref_by_hash[h] = (t, ref.text)
            t, txt = self.ref_by_hash[h]
            tokens.append(t)
            texts.append(txt)
        return tokens, texts

    def load_by_id(self, ref_id: str, use_cache: str):
        if not valid_reference_id(ref_id):
            raise ValueError(f"invalid reference_id {ref_id!r}")
        folder = self.references_dir / ref_id
        root = self.references_dir.resolve()
        if root not in folder.resolve().parents:
            raise ValueError(f"reference_id {ref_id!r} leaves the references directory")
        if use_cache == "off" or ref_id not in self.ref_by_id:
            audios = sorted(p for p in folder.rglob("*") if p.suffix.lower() in AUDIO_EXTENSIONS) \
                if folder.exists() else []
            tokens = [self.encode_reference(p.read_bytes(), True) for p in audios]
            texts = [p.with_suffix(".lab").read_text(encoding="utf-8").strip() if p.with_suffix(".lab").exists()
                     else "" for p in audios]
            self.ref_by_id[ref_id] = (tokens, texts)
        return self.ref_by_id[ref_id]

    def list_reference_ids(self) -> List[str]:
        if not self.references_dir.exists():
            return []
        out = []
        for d in self.references_dir.iterdir():
            if d.is_dir() and any(p.suffix.lower() in AUDIO_EXTENSIONS and p.with_suffix(".lab").exists()
                                  for p in d.iterdir()):
                out.append(d.name)
        return sorted(out)

    # ---- reference management (inference_engine/reference_loader.py:167-271, views.py:380-470)
    def add_reference(self, ref_id: str, audio: bytes, text: str) -> None:
        """references/<id>/sample.wav + sample.lab.  ValueError: bad id / text / audio;
        FileExistsError: the id exists."""
        if not ref_id or not ref_id.strip():
            raise ValueError("Reference ID cannot be empty")
        if not text or not text.strip():
            raise ValueError("Reference text cannot be empty")
        if not valid_reference_id(ref_id):
            raise ValueError("Reference ID contains invalid characters. Only alphanumeric, hyphens, "
                             "underscores, and spaces are allowed." if len(ref_id) <= 255 else
                             "Reference ID is too long. Maximum length is 255 characters.")
        if not audio:
            raise ValueError("Audio file is empty or could not be read")
        folder = self.references_dir / ref_id
        if folder.exists():
            raise FileExistsError(f"Reference ID '{ref_id}' already exists")
        try:
            folder.mkdir(parents=True, exist_ok=False)
            (folder / "sample.wav").write_bytes(audio)
            (folder / "sample.lab").write_text(text, encoding="utf-8")
        except Exception:
            import shutil

            shutil.rmtree(folder, ignore_errors=True)
            raise
        self.ref_by_id.pop(ref_id, None)

    def delete_reference(self, ref_id: str) -> None:
        """FileNotFoundError: no such id."""
        if not ref_id or not ref_id.strip():
            raise ValueError("Reference ID cannot be empty")
        if not valid_reference_id(ref_id):
            raise ValueError(f"invalid reference_id {ref_id!r}")
        folder = self.references_dir / ref_id
        if not folder.exists():
            raise FileNotFoundError(f"Reference ID '{ref_id}' does not exist")
        import shutil

        try:
            shutil.rmtree(folder)
        except Exception as e:
            raise OSError(f"Failed to delete reference '{ref_id}': {e}")
        self.ref_by_id.pop(ref_id, None)

    def rename_reference(self, old_id: str, new_id: str) -> None:
        """FileNotFoundError: no old id; FileExistsError: the new id exists; ValueError: bad ids."""
        if not old_id or not old_id.strip():
            raise ValueError("Old reference ID cannot be empty")
        if not new_id or not new_id.strip():
            raise ValueError("New reference ID cannot be empty")
        if old_id == new_id:
            raise ValueError("New reference ID must be different from old reference ID")
        if not valid_reference_id(new_id):
            raise ValueError("New reference ID contains invalid characters or is too long")
        if not valid_reference_id(old_id):
            raise FileNotFoundError(f"Reference ID '{old_id}' not found")
        old, new = self.references_dir / old_id, self.references_dir / new_id
        if not old.is_dir():
            raise FileNotFoundError(f"Reference ID '{old_id}' not found")
        if new.exists():
            raise FileExistsError(f"Reference ID '{new_id}' already exists")
        old.rename(new)
        if old_id in self.ref_by_id:
            self.ref_by_id[new_id] = self.ref_by_id.pop(old_id)

    # ---- LLM request (inference_engine/__init__.py:144-177) ---------------------------------
    def send_Llama_request(self, req, prompt_tokens: list, prompt_texts: list) -> "queue.Queue":
        request = dict(device=getattr(self.decoder_model, "device", 0), max_new_tokens=req.max_new_tokens,
                       text=req.text, top_p=req.top_p, repetition_penalty=req.repetition_penalty,
                       temperature=req.temperature, compile=self.compile, iterative_prompt=req.chunk_length > 0,
                       chunk_length=req.chunk_length, prompt_tokens=prompt_tokens, prompt_text=prompt_texts)
        if req.seed is not None:
            request["seed"] = int(req.seed)
        if self.reuse_prefix:
            request["reuse_prefix"] = True
        if req.streaming and req.latency == "balanced" and self.stream_frames > 0:
            request["stream_frames"] = self.stream_frames
        rq: "queue.Queue" = queue.Queue()
        self.llama_queue.put(GenerateRequest(request=request, response_queue=rq))
        return rq

    def decode_vq_tokens(self, codes) -> np.ndarray:
        """VQManager.decode_vq_tokens: DAC.from_indices(codes[None])[0].squeeze()."""
        c = np.asarray(codes)
        log.info("VQ features: %s", c.shape)
        with self._codec_lock:
            return self.decoder_model.decode_codes(c)

    def get_audio_segment(self, result: GenerateResponse, streams: Optional[dict] = None) -> np.ndarray:
        """One "sample" response -> PCM.  A streamed chunk (result.stream set) continues its text
        batch's causal stream, whose carried codec state belongs to the calling request alone:
        `streams` is that request's holder ({"ctx": CodecStream}); chunk 0 replaces its context
        with a fresh one.  Without a holder the handle's own stream is used (one caller only)."""
        if getattr(result, "audio", None) is not None:  # vocoded where it was decoded (dist_serving)
            return np.asarray(result.audio, np.float32)
        if result.stream is not None:  # a chunk of one batch's causal stream: carried codec state
            codes = np.asarray(result.codes)
            with self._codec_lock:
                if streams is None or not hasattr(self.decoder_model, "open_stream"):
                    if result.stream == 0:
                        self.decoder_model.stream_reset()
                    return np.asarray(self.decoder_model.decode_chunk(codes), np.float32)
                if result.stream == 0 or streams.get("ctx") is None:
                    if streams.get("ctx") is not None:
                        streams["ctx"].close()
                    streams["ctx"] = self.decoder_model.open_stream()
                return np.asarray(streams["ctx"].decode_chunk(codes), np.float32)
        return np.asarray(self.decode_vq_tokens(result.codes), np.float32)

    def _close_streams(self, streams: dict):
        if streams.get("ctx") is not None:
            with self._codec_lock:
                streams["ctx"].close()
            streams["ctx"] = None

    # ---- main entry (inference_engine/__init__.py:41-131) -----------------------------------
    def inference(self, req) -> Generator[InferenceResult, None, None]:
        prompt_tokens, prompt_texts = [], []
        if req.reference_id is not None:
            prompt_tokens, prompt_texts = self.load_by_id(req.reference_id, req.use_memory_cache)
        elif req.references:
            prompt_tokens, prompt_texts = self.load_by_hash(req.references, req.use_memory_cache)
        rq = self.send_Llama_request(req, prompt_tokens, prompt_texts)
        sr = self.decoder_model.sample_rate
        if req.streaming:
            yield InferenceResult(code="header", audio=(sr, np.frombuffer(wav_chunk_header(sr), np.uint8)), error=None)
        segments = []
        streams: dict = {}  # this request's codec stream context (latency="balanced" chunks)
        try:
            while True:
                wrapped: WrappedGenerateResponse = rq.get()
                if wrapped.status == "error":
                    err = wrapped.response if isinstance(wrapped.response, Exception) else Exception("Unknown error")
                    yield InferenceResult(code="error", audio=None, error=err)
                    break
                result = wrapped.response
                if not isinstance(result, GenerateResponse):
                    raise TypeError(f"Expected GenerateResponse, got {type(result).__name__}")
                if result.action == "next":
                    break
                seg = self.get_audio_segment(result, streams)
                if req.streaming:
                    yield InferenceResult(code="segment", audio=(sr, seg), error=None)
                segments.append(seg)
        finally:
            self._close_streams(streams)
        if not segments:
            yield InferenceResult(code="error", audio=None,
                                  error=RuntimeError("No audio generated, please check the input text."))
        else:
            yield InferenceResult(code="final", audio=(sr, np.concatenate(segments, axis=0)), error=None)


class EngineError(RuntimeError):
    """An error result of the engine (the HTTP layer maps it to 500)."""


def inference_wrapper(req, engine: TTSInferenceEngine):
    """tools/server/inference.py:12-45: header bytes, int16 PCM bytes per segment, then the final
    float audio (the non-streaming caller takes it)."""
    count = 0
    for result in engine.inference(req):
        if result.code == "header":
            yield result.audio[1].tobytes()
        elif result.code == "error":
            raise EngineError(str(result.error))
        elif result.code == "segment":
            count += 1
            yield (result.audio[1] * AMPLITUDE).astype(np.int16).tobytes()
        elif result.code == "final":
            count += 1
            yield result.audio[1]
            return
    if count == 0:
        raise EngineError("No audio generated, please check the input text.")


_SAFE_ID = re.compile(r"^[a-zA-Z0-9\-_ ]+$")


def valid_reference_id(ref_id: str) -> bool:
    return bool(_SAFE_ID.match(ref_id)) and len(ref_id) <= 255
