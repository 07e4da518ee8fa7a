"""Modded-DAC codec decode on libfishmi: the drop-in for ``DAC.from_indices``.

Mirrors ``fish_speech.models.dac.modded_dac.DAC`` (modded_dac.py:804-996) for the decode half:
``from_indices(indices[B, C, T]) -> [B, 1, 2048*T]`` at 44.1 kHz, ``sample_rate``,
``frame_length``.  Unlike the reference (rvq.py:354-359 clamps ``indices`` in place) the caller's
array is not mutated; the clamp itself is applied identically on the device.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

from . import native
from .checkpoint import Tensor, codec_encoder_tensor_shapes, codec_tensor_shapes, load_codec_weights
from .config import CodecConfig
from .synth import codec_rule


class FishMICodec:
    def __init__(self, cfg: CodecConfig = None, device: int = 0, precision: str = "bf16",
                 max_frames: int = 1024):
        self.cfg = cfg or CodecConfig()
        self.device = device
        self.precision = precision
        self.max_frames = max_frames
        self.sample_rate = self.cfg.sample_rate
        self.frame_length = self.cfg.hop
        L = native.lib()
        if native.device_count() < 1:
            raise native.FishMIError("no HIP device visible; libfishmi has no CPU fallback")
        self._c = self.cfg.to_c()
        h = ctypes.c_void_p()
        prec = native.FM_PREC_BF16 if precision == "bf16" else native.FM_PREC_FP32
        native.check(L.fm_codec_open(ctypes.byref(self._c), device, prec, max_frames, ctypes.byref(h)))
        self.h = h

    @classmethod
    def from_checkpoint(cls, codec_pth, device=0, precision="bf16", max_frames=1024,
                        cfg: CodecConfig = None, encoder: bool = False, encoder_dim: int = 64,
                        enc_layers=(0, 0, 0, 4)):
        """load_codec_model / dac.inference.load_model (inference.py:395-417,
        fish_speech/models/dac/inference.py:23-47). `encoder=True` also loads the encode half
        (Encoder, quantizer downsample / pre_module, VQ in_proj), which VQManager.encode_reference
        needs (vq_manager.py:24-52); the decode-only inventory is the default."""
        m = cls(cfg or CodecConfig(), device, precision, max_frames)
        w = load_codec_weights(codec_pth)
        if encoder:
            m.enable_encoder(encoder_dim, enc_layers)
            m.load_encoder_weights(w)
        m.load_weights(w)
        m.finalize()
        return m

    @classmethod
    def synthetic(cls, cfg: CodecConfig, seed: int, device=0, precision="bf16", max_frames=1024):
        m = cls(cfg, device, precision, max_frames)
        m.synth(seed)
        m.finalize()
        return m

    def load_weights(self, weights: "dict[str, Tensor]"):
        L = native.lib()
        for name, shape in codec_tensor_shapes(self.cfg).items():
            if name not in weights:
                raise KeyError(f"codec checkpoint lacks {name}")
            t = weights[name]
            a = np.ascontiguousarray(t.data if t.bf16 else np.asarray(t.data, np.float32))
            native.check(L.fm_codec_set_tensor(self.h, name.encode(), a.ctypes.data_as(ctypes.c_void_p),
                                               native.FM_DT_BF16 if t.bf16 else native.FM_DT_F32, a.size))

    def synth(self, seed: int):
        L = native.lib()
        for name, shape in codec_tensor_shapes(self.cfg).items():
            c, e = codec_rule(name)
            native.check(L.fm_codec_synth_tensor(self.h, name.encode(), int(np.prod(shape)), seed, c, e))

    def finalize(self):
        native.check(native.lib().fm_codec_finalize(self.h))

    # ---- encode side: DAC.encode (modded_dac.py:874-923), voice-clone reference audio ----------
    def enable_encoder(self, encoder_dim: int = 64, enc_layers=(0, 0, 0, 4)):
        """Before load/synth + finalize: adds the encoder, quantizer.downsample / pre_module and
        VQ in_proj tensors (the decode-only inventory is the default)."""
        if tuple(enc_layers[:3]) != (0, 0, 0):
            raise ValueError("only the last encoder block carries a transformer (modded_dac_vq.yaml)")
        self.encoder_dim, self.enc_layers = encoder_dim, tuple(enc_layers)
        native.check(native.lib().fm_codec_enable_encoder(self.h, encoder_dim, int(enc_layers[3])))

    def _encoder_shapes(self):
        return codec_encoder_tensor_shapes(self.cfg, self.encoder_dim, self.enc_layers)

    def load_encoder_weights(self, weights: "dict[str, Tensor]"):
        L = native.lib()
        for name, shape in self._encoder_shapes().items():
            if name not in weights:
                raise KeyError(f"codec checkpoint lacks {name}")
            t = weights[name]
            a = np.ascontiguousarray(t.data if t.bf16 else np.asarray(t.data, np.float32))
            native.check(L.fm_codec_set_tensor(self.h, name.encode(), a.ctypes.data_as(ctypes.c_void_p),
                                               native.FM_DT_BF16 if t.bf16 else native.FM_DT_F32, a.size))

    def synth_encoder(self, seed: int):
        L = native.lib()
        for name, shape in self._encoder_shapes().items():
            c, e = codec_rule(name)
            native.check(L.fm_codec_synth_tensor(self.h, name.encode(), int(np.prod(shape)), seed, c, e))

    def encode_audio(self, audio: np.ndarray) -> np.ndarray:
        """mono 44.1 kHz samples -> codes (n_codebooks+1, ceil(n/2048)) int32 (DAC.encode with the
        right pad to a multiple of frame_length; lens = T)."""
        a = np.ascontiguousarray(np.asarray(audio, np.float32).reshape(-1))
        T = (a.size + self.frame_length - 1) // self.frame_length
        codes = np.zeros((self.cfg.n_codebooks + 1, T), np.int32)
        t_out = ctypes.c_int(0)
        native.check(native.lib().fm_codec_encode(self.h, native.f32p(a), a.size, native.i32p(codes),
                                                  ctypes.byref(t_out)))
        assert t_out.value == T
        return codes

    def encode(self, audio_data, audio_lengths=None):
        """DAC.encode(audio[B, 1, N], audio_lengths) -> (codes[B, C, T], lens[B])."""
        x = np.asarray(audio_data, np.float32)
        if x.ndim == 2:
            x = x[:, None]
        outs, lens = [], []
        for b in range(x.shape[0]):
            n = int(audio_lengths[b]) if audio_lengths is not None else x.shape[-1]
            outs.append(self.encode_audio(x[b, 0, :x.shape[-1]]))
            lens.append((n + self.frame_length - 1) // self.frame_length)
        return np.stack(outs), np.array(lens, np.int64)

    def decode_codes(self, codes: np.ndarray) -> np.ndarray:
        """codes (C, T) int -> float32 PCM (2048*T,)."""
        cd = np.ascontiguousarray(codes, dtype=np.int32)
        assert cd.ndim == 2 and cd.shape[0] == self.cfg.n_codebooks + 1
        out = np.zeros(cd.shape[1] * self.frame_length, np.float32)
        native.check(native.lib().fm_codec_decode(self.h, native.i32p(cd), cd.shape[1], native.f32p(out)))
        return out

    # ---- streamed decode (BASELINE config 5) -----------------------------------------------
    def stream_reset(self):
        """Start a new stream: the carried causal context is zeroed (== the causal padding)."""
        native.check(native.lib().fm_codec_stream_reset(self.h))

    def decode_chunk(self, codes: np.ndarray) -> np.ndarray:
        """Next chunk of the stream: codes (C, T) int -> float32 PCM (2048*T,).  The chunks'
        concatenated PCM equals decode_codes of the concatenated codes (causal decode with the
        previous chunk's rows carried, fm_codec_decode_chunk)."""
        cd = np.ascontiguousarray(codes, dtype=np.int32)
        assert cd.ndim == 2 and cd.shape[0] == self.cfg.n_codebooks + 1
        out = np.zeros(cd.shape[1] * self.frame_length, np.float32)
        native.check(native.lib().fm_codec_decode_chunk(self.h, native.i32p(cd), cd.shape[1], native.f32p(out)))
        return out

    def open_stream(self) -> "CodecStream":
        """A stream context of its own (fm_codec_stream_open): its carried causal rows and RoPE
        position are independent of the handle's stream and of every other context, so several
        streamed requests can share one handle (calls still serialised by the caller)."""
        sid = ctypes.c_int(0)
        native.check(native.lib().fm_codec_stream_open(self.h, ctypes.byref(sid)))
        return CodecStream(self, sid.value)

    def from_indices(self, indices) -> np.ndarray:
        idx = np.asarray(indices)
        if idx.ndim == 2:
            idx = idx[None]
        return np.stack([self.decode_codes(b)[None] for b in idx])

    def debug_read(self, stage: int, T: int) -> np.ndarray:
        """Test hook: 1 = transformer output [T][D], 2 = first upsample [2T][D],
        3 = decoder input latent [4T][D] of the last decode; 10 = encoder output [4T][D],
        11 = quantizer input after downsample + pre_module [T][D] of the last encode (fp32,
        time-major)."""
        D = self.cfg.latent
        shape = {1: (T, D), 2: (2 * T, D), 3: (4 * T, D), 10: (4 * T, D), 11: (T, D)}[stage]
        out = np.zeros(shape, np.float32)
        native.check(native.lib().fm_codec_debug_read(self.h, stage, T, native.f32p(out)))
        return out

    def profile(self):
        ms, n, fl = ctypes.c_double(), ctypes.c_int64(), ctypes.c_double()
        native.check(native.lib().fm_codec_profile_read(self.h, ctypes.byref(ms), ctypes.byref(n), ctypes.byref(fl)))
        return ms.value, n.value, fl.value

    def close(self):
        if getattr(self, "h", None):
            native.lib().fm_codec_close(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class CodecStream:
    """One streamed vocoding context on a FishMICodec (open_stream); starts at zero state."""

    def __init__(self, codec: FishMICodec, sid: int):
        self.codec, self.sid = codec, sid

    def decode_chunk(self, codes: np.ndarray) -> np.ndarray:
        """As FishMICodec.decode_chunk, on this context's carried state."""
        cd = np.ascontiguousarray(codes, dtype=np.int32)
        assert cd.ndim == 2 and cd.shape[0] == self.codec.cfg.n_codebooks + 1
        out = np.zeros(cd.shape[1] * self.codec.frame_length, np.float32)
        native.check(native.lib().fm_codec_stream_decode(self.codec.h, self.sid, native.i32p(cd), cd.shape[1],
                                                          native.f32p(out)))
        return out

    def rewind(self):
        """Back to zero state for the next request (fm_codec_stream_rewind: no reallocation)."""
        native.check(native.lib().fm_codec_stream_rewind(self.codec.h, self.sid))

    def close(self):
        if self.sid and getattr(self.codec, "h", None):
            native.check(native.lib().fm_codec_stream_close(self.codec.h, self.sid))
        self.sid = 0


def smoke_codec(golden_dir: str):
    """Tiny codec (reference-generated golden) in fp32 on cuda:0 vs the reference waveform."""
    import json

    g = np.load(os.path.join(golden_dir, "codec_tiny.npz"))
    cfg = CodecConfig.from_spec(json.loads(str(g["spec"])))
    m = FishMICodec.synthetic(cfg, int(g["synth_seed"]), 0, "fp32", 64)
    wave = m.decode_codes(g["codes"][0])
    ref = g["wave_fp32"].reshape(-1)
    err = float(np.abs(wave - ref).max())
    m.close()
    if err > 2e-3:
        raise AssertionError(f"codec fp32 waveform off by {err}")
