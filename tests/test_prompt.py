"""Prompt side vs the reference (tests/golden/prompt.npz from the reference's own
Conversation.encode_for_inference / split_text_by_speaker / group_turns_into_batches, driven
through generate_long's conversation flow, inference.py:558-707).  Bit-exact (integer ids)."""
import copy
import json
import os

import numpy as np

from conftest import GOLDEN


def _flow(P, tok, text, ptoks, gen_codes, C=10):
    """generate_long's conversation bookkeeping for one sample; returns the encoded prompts."""
    turns = P.split_text_by_speaker(text)
    batches = P.group_turns_into_batches(turns, max_speakers=5, max_bytes=40) if turns else [text]
    if ptoks is not None:
        base = P.base_conversation(["reference one", "<|speaker:1|>second reference"],
                                   [ptoks[:, :6], ptoks[:, 6:]])
    else:
        base = P.base_conversation()
    conv = copy.deepcopy(base)
    encs = []
    for bi, bt in enumerate(batches):
        conv.append(P.Message(role="user", parts=[P.TextPart(text=bt)]))
        gen = copy.deepcopy(conv)
        gen.append(P.Message(role="assistant", parts=[], modality="voice", add_im_end=False))
        encs.append(gen.encode_for_inference(tok, num_codebooks=C)[0])
        conv.append(P.Message(role="assistant", parts=[P.VQPart(codes=gen_codes[bi])], modality="voice"))
    return turns, batches, encs


def test_prompt_encoding_matches_reference(golden):
    from fishmi import prompt as P

    g = golden("prompt.npz")
    tok = P.FishTokenizer(os.path.join(GOLDEN, "tok_tiny"))
    assert (tok.semantic_begin_id, tok.semantic_end_id, tok.get_token_id("<|im_end|>")) == (200, 327, 4)
    texts = json.loads(str(g["texts"]))
    n = 0
    for ti, text in enumerate(texts):
        for use_prompt in (0, 1):
            ptoks = g[f"ptoks_{ti}"] if use_prompt else None
            nb = len(json.loads(str(g[f"batches_{ti}"])))
            gens = [g[f"gen_{ti}_{use_prompt}_{bi}"] for bi in range(nb)]
            turns, batches, encs = _flow(P, tok, text, ptoks, gens)
            assert turns == json.loads(str(g[f"turns_{ti}"]))
            assert batches == json.loads(str(g[f"batches_{ti}"]))
            for bi, e in enumerate(encs):
                np.testing.assert_array_equal(e, g[f"enc_{ti}_{use_prompt}_{bi}"])
                n += 1
    assert n == len(json.loads(str(g["cases"])))


def test_split_and_group_edge_cases():
    from fishmi import prompt as P

    assert P.split_text_by_speaker("no tags") == []
    assert P.split_text_by_speaker("<|speaker:3|>") == ["<|speaker:3|>"]
    assert P.split_text_by_speaker("lead <|speaker:0|> a <|speaker:1|>b ") == ["<|speaker:0|> a", "<|speaker:1|>b"]
    assert P.group_turns_into_batches([], 2, 10) == []
    assert P.group_turns_into_batches(["aaaa", "bbbb", "cc"], 5, 8) == ["aaaa\nbbbb", "cc"]
    assert P.group_turns_into_batches(["x" * 50], 5, 8) == ["x" * 50]  # an oversize turn stays whole
    assert P.group_turns_into_batches(["a", "b", "c", "d"], 3, 100) == ["a\nb\nc", "d"]


def test_engine_device_and_precision_parsing():
    import torch

    from fishmi import engine

    assert engine._device_index("cuda:3") == 3 and engine._device_index("cuda") == 0
    assert engine._device_index(torch.device("cuda", 2)) == 2 and engine._device_index(5) == 5
    assert engine._precision(torch.bfloat16) == "bf16" and engine._precision(torch.float32) == "fp32"
    assert engine._precision("bf16") == "bf16" and engine._precision("fp32") == "fp32"


def test_single_prompt_text_and_tokens():
    """generate_long(prompt_text="...", prompt_tokens=<one (C, T) array>) wraps both together
    (inference.py:544-547): the system message is the same as for one-element lists, with a 2-D
    VQ part."""
    from fishmi import prompt as P

    tok = P.FishTokenizer(os.path.join(GOLDEN, "tok_tiny"))
    codes = np.random.default_rng(0).integers(0, 128, (10, 7))
    one = P.base_conversation("reference one", codes)
    lst = P.base_conversation(["reference one"], [codes])
    assert one.messages[0].parts[-1].codes.shape == (10, 7)
    np.testing.assert_array_equal(one.encode_for_inference(tok, num_codebooks=10)[0],
                                  lst.encode_for_inference(tok, num_codebooks=10)[0])
