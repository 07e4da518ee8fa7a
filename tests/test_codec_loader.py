"""Codec checkpoint loading (B3 loader: fish_speech/models/dac/inference.py:23-47).

tests/golden/codec_keys.json holds the names and shapes of the reference's own DAC state_dict at the
real modded_dac_vq.yaml dims (oracle/gen_goldens.py codec_keys). The real layout mixes two
weight-norm spellings: the modded DAC's own convs use `conv.parametrizations.weight.original0/1`,
and the descript VQ projections use `weight_g/weight_v`. These CPU tests pin the build's tensor
inventory and loader to that layout; test_gpu_codec_loader.py pushes a checkpoint through
FishMICodec.from_checkpoint on the GPU.
"""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN


def _ref_keys():
    with open(os.path.join(GOLDEN, "codec_keys.json")) as f:
        return json.load(f)


def test_inventory_equals_reference_state_dict():
    from fishmi.checkpoint import codec_encoder_tensor_shapes, codec_tensor_shapes
    from fishmi.config import CodecConfig

    d = _ref_keys()
    ref = {k: tuple(s) for k, s, _ in d["keys"]}
    cfg = CodecConfig.from_spec(d["spec"])
    ours = dict(codec_tensor_shapes(cfg))
    enc = codec_encoder_tensor_shapes(cfg, d["spec"]["encoder_dim"], tuple(d["enc_layers"]))
    assert not set(ours) & set(enc)
    ours.update(enc)
    assert set(ours) == set(ref)
    assert all(tuple(ours[k]) == ref[k] for k in ref)
    # both weight-norm spellings occur in the real layout
    assert any(k.endswith("weight_g") for k in ref) and any(k.endswith("original0") for k in ref)


@pytest.mark.parametrize("wrapped", [False, True])
def test_load_codec_weights_layouts(tmp_path, wrapped):
    """A plain state_dict and a Lightning-style {"state_dict": {"generator.*": ...}} checkpoint
    load to the same tensors; bf16 tensors keep their bits, fp32 stay fp32."""
    torch = pytest.importorskip("torch")
    from fishmi.checkpoint import load_codec_weights

    d = _ref_keys()
    g = torch.Generator().manual_seed(0)
    sd = {}
    for i, (k, s, _) in enumerate(d["keys"][:40]):
        t = torch.randn(*s, generator=g) if np.prod(s) < 1 << 16 else torch.zeros(*s)
        sd[k] = t.bfloat16() if i % 3 == 0 else t
    obj = {"state_dict": {"generator." + k: v for k, v in sd.items()} | {"discriminator.x": torch.ones(1)}} \
        if wrapped else sd
    path = tmp_path / "codec.pth"
    torch.save(obj, path)
    w = load_codec_weights(str(path))
    assert list(w) == list(sd)
    for k, v in sd.items():
        if v.dtype == torch.bfloat16:
            assert w[k].bf16 and np.array_equal(w[k].data, v.view(torch.int16).numpy().view(np.uint16))
        else:
            assert not w[k].bf16 and np.array_equal(w[k].data, v.numpy())
