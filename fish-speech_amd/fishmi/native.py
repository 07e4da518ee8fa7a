"""ctypes binding of libfishmi.so (include/fishmi.h).

The product path is this library and nothing else: if it is missing or no GPU is visible,
construction fails loudly (there is no CPU fallback).
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libfishmi.so")

FM_PREC_BF16, FM_PREC_FP32 = 0, 1
FM_DT_F32, FM_DT_BF16, FM_DT_I8 = 0, 1, 2
FM_QUANT_NONE, FM_QUANT_INT8, FM_QUANT_INT4 = 0, 1, 2

_lib = None

# every symbol include/fishmi.h declares (checked by tests/test_abi.py)
ABI_SYMBOLS = [
    "fm_device_count", "fm_last_error", "fm_stream_peak", "fm_llm_open", "fm_llm_set_quant", "fm_llm_set_quant_int4", "fm_llm_set_tensor", "fm_llm_synth_tensor",
    "fm_llm_finalize", "fm_llm_prefill", "fm_llm_prefill_batch", "fm_llm_decode", "fm_llm_decode_frames", "fm_llm_generate", "fm_llm_generate_at", "fm_llm_prefill_at", "fm_llm_slot_pos", "fm_llm_teacher_step",
    "fm_llm_frame_bytes", "fm_llm_profile", "fm_llm_profile_read", "fm_llm_kernel_bench", "fm_llm_use_graph", "fm_llm_debug_vec", "fm_tune", "fm_debug_ts_read",
    "fm_llm_close", "fm_source_hash", "fm_codec_open", "fm_codec_set_tensor", "fm_codec_synth_tensor",
    "fm_codec_finalize", "fm_codec_decode", "fm_codec_stream_reset", "fm_codec_decode_chunk",
    "fm_codec_stream_open", "fm_codec_stream_decode", "fm_codec_stream_rewind", "fm_codec_stream_close",
    "fm_codec_profile_read", "fm_codec_debug_read", "fm_codec_enable_encoder", "fm_codec_encode",
    "fm_codec_close", "fm_llm_force", "fm_llm_read_logits", "fm_op_rmsnorm", "fm_op_qk_rope", "fm_op_decode_attn", "fm_op_prompt_attn",
    "fm_op_embed", "fm_op_quant4", "fm_rope_table",
]


class FishMIError(RuntimeError):
    pass


def tree_source_hash() -> str:
    """sha256 (first 16 hex digits) over the files fish-speech_amd/Makefile's HASHED names, in its
    order: the compiled sources (SRCS), the csrc headers sorted by name, include/fishmi.h."""
    import hashlib
    import re

    pkg = os.path.dirname(HERE)
    mk = open(os.path.join(pkg, "Makefile")).read()
    srcs = re.search(r"^SRCS\s*=\s*(.+)$", mk, re.M).group(1).split()
    heads = sorted(f for f in os.listdir(os.path.join(pkg, "csrc")) if f.endswith(".h"))
    files = srcs + [os.path.join("csrc", h) for h in heads] + [os.path.join("..", "include", "fishmi.h")]
    h = hashlib.sha256()
    for f in files:
        with open(os.path.join(pkg, f), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


class SamplingC(ctypes.Structure):
    _fields_ = [("temperature", ctypes.c_float), ("top_p", ctypes.c_float),
                ("top_k", ctypes.c_int), ("seed", ctypes.c_uint64), ("mask_im_end", ctypes.c_int)]


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise FishMIError(f"{LIB_PATH} is missing: build it with `make -C fish-speech_amd` "
                          "(or __graft_entry__.build()); there is no CPU fallback")
    # torch bundles its own libamdhip64 (same soname).  Whichever HIP runtime is mapped first is
    # the one both use; if this library pulled /opt/rocm's in first, torch's later device init
    # fails ("No HIP GPUs are available", measured on the MI355X box), which would break every
    # torch.distributed / RCCL caller that loads fishmi first.  Map torch's runtime first.
    if not os.environ.get("FISHMI_NO_TORCH_FIRST"):  # (developer: the rocprofv3 fault investigation)
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
    L = ctypes.CDLL(LIB_PATH)
    # build provenance: the library must have been compiled from the sources in this tree
    L.fm_source_hash.restype = ctypes.c_char_p
    if not os.environ.get("FISHMI_ALLOW_STALE"):  # (the escape hatch skips the sources entirely)
        built = L.fm_source_hash().decode()
        try:
            tree = tree_source_hash()
        except OSError as e:
            raise FishMIError(f"cannot check {LIB_PATH} against its sources ({e}): deploy the package with "
                              "its Makefile, csrc/ and include/, or set FISHMI_ALLOW_STALE=1") from e
        if built != tree:
            raise FishMIError(f"{LIB_PATH} was built from other sources (hash {built}, tree {tree}): "
                              "rebuild it with `make -C fish-speech_amd`")
    # developer: FISHMI_TUNE="key=value,..." applies fm_tune knobs at load (run a test suite under a variant)
    for kv in filter(None, os.environ.get("FISHMI_TUNE", "").split(",")):
        k, v = kv.split("=")
        L.fm_tune.argtypes = [ctypes.c_char_p, ctypes.c_int]
        if L.fm_tune(k.strip().encode(), int(v)) != 0:
            raise FishMIError(f"FISHMI_TUNE: fm_tune({k}, {v}) failed")
    vp, i32, i64, u64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_uint64
    f32 = ctypes.c_float
    pi32 = ctypes.POINTER(ctypes.c_int32)
    pf32 = ctypes.POINTER(ctypes.c_float)
    L.fm_last_error.restype = ctypes.c_char_p
    L.fm_device_count.restype = i32
    L.fm_stream_peak.argtypes = [i32, i64, i32, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double)]
    L.fm_llm_open.argtypes = [vp, i32, i32, i32, ctypes.POINTER(vp)]
    L.fm_llm_set_quant.argtypes = [vp, i32]
    L.fm_llm_set_quant_int4.argtypes = [vp, i32]
    L.fm_llm_set_tensor.argtypes = [vp, ctypes.c_char_p, vp, i32, i64]
    L.fm_llm_synth_tensor.argtypes = [vp, ctypes.c_char_p, i64, u64, f32, i32]
    L.fm_llm_finalize.argtypes = [vp]
    L.fm_llm_prefill.argtypes = [vp, i32, pi32, i32, ctypes.POINTER(SamplingC), pi32]
    L.fm_llm_prefill_batch.argtypes = [vp, i32, pi32, pi32, pi32, ctypes.POINTER(SamplingC), pi32]
    L.fm_llm_decode.argtypes = [vp, pi32, i32, pi32]
    L.fm_llm_decode_frames.argtypes = [vp, pi32, i32, i32, pi32]
    L.fm_llm_generate.argtypes = [vp, i32, pi32, i32, i32, ctypes.POINTER(SamplingC), pi32,
                                  ctypes.POINTER(ctypes.c_int)]
    L.fm_llm_generate_at.argtypes = [vp, i32, pi32, i32, i32, i32, ctypes.POINTER(SamplingC), pi32,
                                     ctypes.POINTER(ctypes.c_int)]
    L.fm_llm_prefill_at.argtypes = [vp, i32, pi32, i32, i32, ctypes.POINTER(SamplingC), pi32]
    L.fm_llm_slot_pos.argtypes = [vp, i32, ctypes.POINTER(ctypes.c_int)]
    L.fm_llm_teacher_step.argtypes = [vp, i32, pi32, i32, i32, pi32, pf32, pf32, pf32]
    L.fm_llm_frame_bytes.argtypes = [vp, i32, i32]
    L.fm_llm_frame_bytes.restype = i64
    L.fm_llm_profile.argtypes = [vp, i32]
    L.fm_llm_profile_read.argtypes = [vp, ctypes.c_char_p, ctypes.POINTER(ctypes.c_double),
                                      ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64)]
    L.fm_llm_kernel_bench.argtypes = [vp, ctypes.c_char_p, i32, ctypes.POINTER(ctypes.c_double),
                                      ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64)]
    L.fm_llm_use_graph.argtypes = [vp, i32]
    L.fm_llm_debug_vec.argtypes = [vp, ctypes.c_char_p, i32, pf32, i64]
    L.fm_tune.argtypes = [ctypes.c_char_p, i32]
    L.fm_debug_ts_read.argtypes = [ctypes.POINTER(ctypes.c_uint64), i64, ctypes.POINTER(ctypes.c_int64)]
    L.fm_llm_close.argtypes = [vp]
    L.fm_llm_force.argtypes = [vp, i32, pi32]
    L.fm_llm_read_logits.argtypes = [vp, i32, pf32, pf32]
    L.fm_op_rmsnorm.argtypes = [i32, i32, i32, pf32, pf32, i32, i32, f32, pf32]
    L.fm_op_qk_rope.argtypes = [i32, i32, i32, pf32, i32, i32, i32, pf32, pf32, i32, f32, f32, i32, pf32, pf32]
    L.fm_op_prompt_attn.argtypes = [i32, i32, i32, pf32, i32, i32, i32, i32, i32, pf32, pf32, i32, pf32]
    L.fm_op_decode_attn.argtypes = [i32, i32, i32, pf32, i32, i32, i32, i32, pf32, pf32, i32, f32, f32, pi32, pf32,
                                    pf32, i32, i32, pf32, pf32, pf32]
    L.fm_op_embed.argtypes = [i32, i32, pi32, i32, pf32, i32, pf32, i32, i32, i32, i32, i32, i32, pf32]
    L.fm_op_quant4.argtypes = [i32, pf32, i32, i32, i32, ctypes.POINTER(ctypes.c_uint8), pf32, pf32, pf32, pf32, i32,
                               pf32, pf32]
    L.fm_rope_table.argtypes = [i32, i32, f32, pf32]
    if hasattr(L, "fm_codec_open"):
        L.fm_codec_open.argtypes = [vp, i32, i32, i32, ctypes.POINTER(vp)]
        L.fm_codec_set_tensor.argtypes = [vp, ctypes.c_char_p, vp, i32, i64]
        L.fm_codec_synth_tensor.argtypes = [vp, ctypes.c_char_p, i64, u64, f32, i32]
        L.fm_codec_finalize.argtypes = [vp]
        L.fm_codec_decode.argtypes = [vp, pi32, i32, pf32]
        L.fm_codec_stream_reset.argtypes = [vp]
        L.fm_codec_decode_chunk.argtypes = [vp, pi32, i32, pf32]
        L.fm_codec_stream_open.argtypes = [vp, ctypes.POINTER(ctypes.c_int)]
        L.fm_codec_stream_decode.argtypes = [vp, i32, pi32, i32, pf32]
        L.fm_codec_stream_rewind.argtypes = [vp, i32]
        L.fm_codec_stream_close.argtypes = [vp, i32]
        L.fm_codec_profile_read.argtypes = [vp, ctypes.POINTER(ctypes.c_double),
                                            ctypes.POINTER(ctypes.c_int64),
                                            ctypes.POINTER(ctypes.c_double)]
        L.fm_codec_close.argtypes = [vp]
        L.fm_codec_debug_read.argtypes = [vp, i32, i32, pf32]
        L.fm_codec_enable_encoder.argtypes = [vp, i32, i32]
        L.fm_codec_encode.argtypes = [vp, pf32, i64, pi32, ctypes.POINTER(ctypes.c_int)]
    _lib = L
    return L


def check(rc: int):
    if rc != 0:
        raise FishMIError(f"libfishmi error {rc}: {lib().fm_last_error().decode()}")
    return rc


def device_count() -> int:
    return lib().fm_device_count()


def stream_peak(device: int = 0, nbytes: int = 2 << 30, reps: int = 10):
    """(read GB/s, copy GB/s) of the measured HBM stream peak (fm_stream_peak)."""
    r, c = ctypes.c_double(), ctypes.c_double()
    check(lib().fm_stream_peak(int(device), int(nbytes), int(reps), ctypes.byref(r), ctypes.byref(c)))
    return r.value, c.value


def i32p(a: np.ndarray):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))


def f32p(a: np.ndarray):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))


def tune(key: str, value: int):
    """Process-wide developer knob of the decode GEMV (see fm_tune in include/fishmi.h)."""
    check(lib().fm_tune(key.encode(), int(value)))


def debug_ts_read(max_records: int = 1 << 20) -> np.ndarray:
    """Per-block GEMV phase timestamps (developer hook, see fm_debug_ts_read): (n, 8) uint64."""
    out = np.zeros((max_records, 8), np.uint64)
    n = ctypes.c_int64(0)
    check(lib().fm_debug_ts_read(out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), max_records,
                                 ctypes.byref(n)))
    return out[: n.value]
