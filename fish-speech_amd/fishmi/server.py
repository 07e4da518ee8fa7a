"""Wire-compatible HTTP API on libfishmi: the drop-in for tools/api_server.py.

Routes and contract, as the reference serves them (tools/server/views.py, api_utils.py):
  GET|POST /v1/health          {"status": "ok"}
  POST /v1/tts                 ServeTTSRequest as application/json or application/msgpack;
                               streaming: WAV header then int16 little-endian PCM chunks, one per
                               text batch (format must be wav, else 400); otherwise a whole file in
                               `format` (wav; pcm = raw int16; mp3/opus need encoders absent here: 400).
                               400 when the text exceeds --max-text-length, 500 on engine errors.
  POST /v1/vqgan/encode        msgpack {"audios": [wav bytes]} -> {"tokens": [[[int]]]}
  POST /v1/vqgan/decode        msgpack {"tokens": [[[int]]]} -> {"audios": [float16 PCM bytes]}.
                               The reference's batch_vqgan_decode calls DAC.decode(x, feature_lengths),
                               which its DAC does not have, so this route is broken
                               there; here it decodes each token matrix through the codec.
  GET  /v1/references/list     {"success": true, "reference_ids": [...]}
  POST /v1/references/add      {id, audio (bytes), text} as msgpack, JSON (audio base64) or
                               multipart/form-data -> {success, message, reference_id};
                               400 bad input, 409 id exists, 500 file-system error
  DELETE /v1/references/delete {reference_id} -> 404 unknown id
  POST /v1/references/update   {old_reference_id, new_reference_id} (rename) -> 404 / 409 / 400
                               (tools/server/views.py:208-470)
Optional bearer auth (--api-key): 401 "Invalid token" otherwise (tools/api_server.py:33-45).

    python -m fishmi.server --llama-checkpoint-path DIR --decoder-checkpoint-path codec.pth [--slots 32]

--slots N serves up to N requests at once on one GPU (fishmi.batching.BatchedWorker: batched decode
frames, each request on its own KV slot); handlers run the blocking engine work in the thread pool, so
concurrent HTTP requests reach the worker together.

Several GPUs (BASELINE config 4): launch one process per GPU,

    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 -m fishmi.server --slots 32 ...

Rank 0 serves HTTP and vocodes; every rank decodes requests on its own KV slots
(fishmi.dist_serving.DistributedWorker: requests scattered and codes gathered at ticks).
"""
import argparse
import io
import logging
import os
from typing import Optional

import numpy as np

from . import tts as TTS

log = logging.getLogger("fishmi.server")


def _content_type(fmt: str) -> str:
    return {"wav": "audio/wav", "flac": "audio/flac", "mp3": "audio/mpeg", "opus": "audio/ogg"}.get(
        fmt, "application/octet-stream")


def create_app(engine: "TTS.TTSInferenceEngine", max_text_length: int = 0, api_key: Optional[str] = None):
    import msgpack
    from fastapi import FastAPI, HTTPException, Request
    from fastapi.responses import JSONResponse, Response, StreamingResponse

    app = FastAPI(title="Fish Speech API (libfishmi)", version="1.5.0")

    @app.middleware("http")
    async def auth(request: Request, call_next):
        if api_key is not None:
            h = request.headers.get("authorization", "")
            if not h.lower().startswith("bearer ") or h[7:].strip() != api_key:
                return JSONResponse({"detail": "Invalid token"}, status_code=401)
        return await call_next(request)

    async def body(request: Request) -> dict:
        ct = request.headers.get("content-type", "").split(";")[0].strip().lower()
        raw = await request.body()
        if ct == "application/msgpack":
            return msgpack.unpackb(raw, raw=False)
        if ct in ("application/json", ""):
            import json

            return json.loads(raw or b"{}")
        raise HTTPException(415, detail="Accept: application/msgpack, application/json")

    def wants_json(request: Request) -> bool:
        q = request.query_params.get("format", "").strip().lower()
        if q in {"json", "application/json", "msgpack", "application/msgpack"}:
            return q in ("json", "application/json")
        accept = request.headers.get("accept", "").lower()
        return "application/json" in accept and "application/msgpack" not in accept

    def respond(request: Request, obj: dict, status: int = 200):
        if wants_json(request):  # bytes fields travel base64-encoded in JSON
            import base64

            def enc(v):
                if isinstance(v, bytes):
                    return base64.b64encode(v).decode()
                if isinstance(v, list):
                    return [enc(x) for x in v]
                return v

            return JSONResponse({k: enc(v) for k, v in obj.items()}, status_code=status)
        return Response(msgpack.packb(obj, use_bin_type=True), media_type="application/msgpack", status_code=status)

    @app.get("/v1/health")
    @app.post("/v1/health")
    async def health():
        return {"status": "ok"}

    @app.post("/v1/tts")
    async def tts(request: Request):
        try:
            req = TTS.ServeTTSRequest(**(await body(request)))
        except HTTPException:
            raise
        except Exception as e:
            raise HTTPException(422, detail=str(e))
        sr = engine.decoder_model.sample_rate
        if max_text_length > 0 and len(req.text) > max_text_length:
            raise HTTPException(400, detail=f"Text is too long, max length is {max_text_length}")
        if req.streaming and req.format != "wav":
            raise HTTPException(400, detail="Streaming only supports WAV format")
        headers = {"Content-Disposition": f"attachment; filename=audio.{req.format}"}
        if req.reference_id is not None and not TTS.valid_reference_id(req.reference_id):
            raise HTTPException(400, detail="Invalid reference_id")
        if req.streaming:
            from starlette.concurrency import run_in_threadpool

            gen = TTS.inference_wrapper(req, engine)
            try:  # the header (and any immediate engine error) before the response starts
                first = await run_in_threadpool(next, gen)
            except TTS.EngineError as e:
                raise HTTPException(500, detail=str(e))

            def stream():
                # the status line is already out once the header is: an engine error ends the
                # body early, as the reference's HTTPException inside its stream generator does
                yield first
                try:
                    for chunk in gen:
                        if isinstance(chunk, bytes):
                            yield chunk
                except TTS.EngineError as e:
                    log.error("TTS stream aborted: %s", e)

            return StreamingResponse(stream(), media_type=_content_type("wav"), headers=headers)
        if req.format not in ("wav", "pcm"):
            raise HTTPException(400, detail=f"format {req.format!r} needs an encoder absent from this build")
        def run():  # blocking engine work off the event loop: concurrent requests reach the worker
            out = None
            for chunk in TTS.inference_wrapper(req, engine):
                if isinstance(chunk, np.ndarray):
                    out = chunk
            return out

        from starlette.concurrency import run_in_threadpool

        try:
            audio = await run_in_threadpool(run)
        except TTS.EngineError as e:
            raise HTTPException(500, detail=str(e))
        data = TTS.wav_bytes(audio, sr) if req.format == "wav" else \
            (np.clip(audio, -1, 1) * 32767).astype("<i2").tobytes()
        return Response(data, media_type=_content_type(req.format), headers=headers)

    @app.post("/v1/vqgan/encode")
    async def vqgan_encode(request: Request):
        d = await body(request)
        try:
            tokens = [engine.encode_reference(a, True).tolist() for a in d["audios"]]
        except Exception as e:
            log.error("VQGAN encode failed: %s", e)
            raise HTTPException(500, detail="Failed to encode audio")
        return respond(request, {"tokens": tokens})

    @app.post("/v1/vqgan/decode")
    async def vqgan_decode(request: Request):
        d = await body(request)
        try:
            audios = [engine.decode_vq_tokens(np.asarray(t, np.int32)).astype(np.float16).tobytes()
                      for t in d["tokens"]]
        except Exception as e:
            log.error("VQGAN decode failed: %s", e)
            raise HTTPException(500, detail="Failed to decode tokens to audio")
        return respond(request, {"audios": audios})

    @app.get("/v1/references/list")
    async def list_refs(request: Request):
        try:
            ids = engine.list_reference_ids()
        except Exception as e:
            log.error("listing references failed: %s", e)
            return respond(request, {"success": False, "reference_ids": [], "message": "Internal server error occurred"},
                           500)
        return respond(request, {"success": True, "reference_ids": ids,
                                 "message": f"Found {len(ids)} reference voices"})

    async def fields(request: Request) -> dict:
        """msgpack / JSON body, or multipart/form-data (parsed with the stdlib email parser: the
        multipart package FastAPI's Form() needs is absent here)."""
        ct = request.headers.get("content-type", "")
        if ct.split(";")[0].strip().lower() != "multipart/form-data":
            return await body(request)
        from email.parser import BytesParser
        from email.policy import HTTP

        raw = await request.body()
        msg = BytesParser(policy=HTTP).parsebytes(b"Content-Type: " + ct.encode() + b"\r\n\r\n" + raw)
        out = {}
        for part in msg.iter_parts():
            name = part.get_param("name", header="content-disposition")
            if name:
                data = part.get_payload(decode=True) or b""
                out[name] = data if part.get_filename() is not None else data.decode("utf-8", "replace")
        return out

    def ref_reply(request: Request, ok: bool, message: str, status: int = 200, **ids):
        return respond(request, {"success": ok, "message": message, **ids}, status)

    @app.post("/v1/references/add")
    async def add_ref(request: Request):
        rid = ""
        try:
            d = await fields(request)
            rid, audio, text = d.get("id") or "", d.get("audio"), d.get("text") or ""
            if isinstance(audio, str):  # JSON: base64
                import base64

                audio = base64.b64decode(audio)
            engine.add_reference(rid, audio or b"", text)
            return ref_reply(request, True, f"Reference voice '{rid}' added successfully", reference_id=rid)
        except FileExistsError:
            return ref_reply(request, False, f"Reference ID '{rid}' already exists", 409, reference_id=rid)
        except ValueError as e:
            return ref_reply(request, False, str(e), 400, reference_id=rid)
        except OSError as e:
            log.error("adding reference %r: %s", rid, e)
            return ref_reply(request, False, "File system error occurred", 500, reference_id=rid)
        except Exception as e:
            log.error("adding reference %r: %s", rid, e)
            return ref_reply(request, False, "Internal server error occurred", 500, reference_id=rid)

    @app.delete("/v1/references/delete")
    async def delete_ref(request: Request):
        rid = ""
        try:
            d = await fields(request)
            rid = d.get("reference_id") or ""
            engine.delete_reference(rid)
            return ref_reply(request, True, f"Reference voice '{rid}' deleted successfully", reference_id=rid)
        except FileNotFoundError:
            return ref_reply(request, False, f"Reference ID '{rid}' not found", 404, reference_id=rid)
        except ValueError as e:
            return ref_reply(request, False, str(e), 400, reference_id=rid)
        except OSError as e:
            log.error("deleting reference %r: %s", rid, e)
            return ref_reply(request, False, "File system error occurred", 500, reference_id=rid)
        except Exception as e:
            log.error("deleting reference %r: %s", rid, e)
            return ref_reply(request, False, "Internal server error occurred", 500, reference_id=rid)

    @app.post("/v1/references/update")
    async def update_ref(request: Request):
        old = new = ""
        try:
            d = await fields(request)
            old, new = d.get("old_reference_id") or "", d.get("new_reference_id") or ""
            engine.rename_reference(old, new)
            return ref_reply(request, True, f"Reference voice renamed from '{old}' to '{new}' successfully",
                             old_reference_id=old, new_reference_id=new)
        except FileNotFoundError as e:
            return ref_reply(request, False, str(e), 404, old_reference_id=old, new_reference_id=new)
        except FileExistsError:
            return ref_reply(request, False, f"Reference ID '{new}' already exists", 409,
                             old_reference_id=old, new_reference_id=new)
        except ValueError as e:
            return ref_reply(request, False, str(e), 400, old_reference_id=old, new_reference_id=new)
        except OSError as e:
            log.error("renaming reference %r: %s", old, e)
            return ref_reply(request, False, "File system error occurred", 500,
                             old_reference_id=old, new_reference_id=new)
        except Exception as e:  # the reference's update route answers these too (views.py:472-480)
            log.error("renaming reference %r: %s", old, e)
            return ref_reply(request, False, "Internal server error occurred", 500,
                             old_reference_id=old, new_reference_id=new)

    return app


def build_engine(llama_checkpoint_path: str, decoder_checkpoint_path: str, device=0, precision="bf16",
                 compile: bool = False, max_frames: int = 2048, slots: int = 1, reuse_prefix: bool = False,
                 llama_queue=None):
    """ModelManager (tools/server/model_manager.py): the LLM worker + the codec with its encoder.
    slots > 1: concurrent requests decode together on their own KV slots (fishmi.batching).
    llama_queue: an already-launched worker queue (the multi-GPU worker's, rank 0)."""
    from .codec import FishMICodec
    from .engine import launch_thread_safe_queue

    q = llama_queue if llama_queue is not None else \
        launch_thread_safe_queue(llama_checkpoint_path, device, precision, compile, max_slots=slots)
    codec = FishMICodec.from_checkpoint(decoder_checkpoint_path, device, precision, max_frames, encoder=True)
    return TTS.TTSInferenceEngine(q, codec, precision, compile, reuse_prefix=reuse_prefix)


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", choices=["tts"], default="tts")
    ap.add_argument("--llama-checkpoint-path", default="checkpoints/s2-pro")
    ap.add_argument("--decoder-checkpoint-path", default="checkpoints/s2-pro/codec.pth")
    ap.add_argument("--decoder-config-name", default="modded_dac_vq")
    ap.add_argument("--device", default="cuda")
    ap.add_argument("--half", action="store_true")
    ap.add_argument("--compile", action="store_true")
    ap.add_argument("--max-text-length", type=int, default=0)
    ap.add_argument("--listen", default="127.0.0.1:8080")
    ap.add_argument("--workers", type=int, default=1)
    ap.add_argument("--api-key", default=None)
    ap.add_argument("--slots", type=int, default=1,
                    help="concurrent requests decoded together on one GPU (KV slots); 1 = the reference's serial worker")
    ap.add_argument("--reuse-prefix", action="store_true",
                    help="keep a request's conversation KV across its text batches (opt-in; default re-prefills)")
    a = ap.parse_args(argv)
    import uvicorn

    from .engine import _device_index

    # flags of tools/server/api_utils.py:21-43 that this build cannot honour as given are refused or
    # mapped explicitly (an operator must not get a different precision or worker count silently)
    if a.decoder_config_name != "modded_dac_vq":
        ap.error(f"--decoder-config-name {a.decoder_config_name!r}: only modded_dac_vq (the S2-Pro codec) is built")
    if a.workers != 1:
        ap.error("--workers > 1: one process drives one GPU here; run one server per GPU (or use --slots for "
                 "concurrent requests on one GPU)")
    if a.half:
        log.warning("--half: fp16 is not built; the HIP path runs bf16 (the reference's default precision)")
    if a.compile:
        log.info("--compile: decode frames are always hipGraph-captured; the flag changes nothing")
    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        return _main_distributed(a)
    engine = build_engine(a.llama_checkpoint_path, a.decoder_checkpoint_path, _device_index(a.device), "bf16",
                          slots=a.slots, reuse_prefix=a.reuse_prefix)
    host, port = a.listen.rsplit(":", 1)
    uvicorn.run(create_app(engine, a.max_text_length, a.api_key), host=host, port=int(port), workers=1)


def _main_distributed(a):
    """One rank per GPU under torchrun: every rank decodes and vocodes what it decoded (its own codec
    handle); rank 0 also serves HTTP (its engine's codec encodes the voice-clone references)."""
    import torch
    import torch.distributed as dist
    import uvicorn

    from .dist_serving import launch_distributed_queue

    local = int(os.environ.get("LOCAL_RANK", "0"))
    backend = "nccl" if torch.cuda.is_available() else "gloo"
    if backend == "nccl":
        torch.cuda.set_device(local)
    dist.init_process_group(backend)
    try:
        from .codec import FishMICodec

        def vocoder():
            return FishMICodec.from_checkpoint(a.decoder_checkpoint_path, local, "bf16", 2048, encoder=False)

        q, th = launch_distributed_queue(a.llama_checkpoint_path, local, "bf16", max_slots=max(a.slots, 1),
                                         vocoder=vocoder)
        if dist.get_rank() == 0:
            engine = build_engine(a.llama_checkpoint_path, a.decoder_checkpoint_path, local, "bf16",
                                  reuse_prefix=a.reuse_prefix, llama_queue=q)
            host, port = a.listen.rsplit(":", 1)
            try:
                uvicorn.run(create_app(engine, a.max_text_length, a.api_key), host=host, port=int(port), workers=1)
            finally:
                q.put(None)  # stops every rank's worker
        th.join()
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
