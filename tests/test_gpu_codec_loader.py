"""GPU: FishMICodec.from_checkpoint on a checkpoint in the reference's key layout (the
parametrizations.weight.original0/1 convs plus the descript weight_g/weight_v VQ projections),
wrapped as a Lightning {"state_dict": {"generator.*"}} file like the released codec.pth.

The tensors are the deterministic synthetic weights (fishmi/synth.py) at the codec_enc_tiny
shapes, so the loaded codec must decode and encode bit-for-bit like FishMICodec.synthetic with
the same seed, which the other codec tests pin to the reference."""
import json

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("prec", ["fp32", "bf16"])
def test_from_checkpoint_equals_synthetic(tmp_path, golden, prec):
    import torch

    from fishmi.checkpoint import codec_encoder_tensor_shapes, codec_tensor_shapes
    from fishmi.codec import FishMICodec
    from fishmi.config import CodecConfig
    from fishmi.synth import codec_rule, synth_f32

    g = golden("codec_enc_tiny.npz")
    spec = json.loads(str(g["spec"]))
    cfg = CodecConfig.from_spec(spec)
    layers = tuple(int(v) for v in g["enc_layers"])
    seed = int(g["synth_seed"])
    shapes = dict(codec_tensor_shapes(cfg))
    shapes.update(codec_encoder_tensor_shapes(cfg, spec["encoder_dim"], layers))
    sd = {}
    for i, (name, shape) in enumerate(shapes.items()):
        c, e = codec_rule(name)
        # synthetic weights are bf16-valued (fishmi/synth.py); store every other tensor as a bf16
        # tensor and the rest as bf16-rounded fp32, so both checkpoint dtypes are loaded
        t = torch.from_numpy(synth_f32(seed, name, int(np.prod(shape)), c, e).reshape(shape)).bfloat16()
        sd["generator." + name] = t if i % 2 else t.float()
    path = tmp_path / "codec.pth"
    torch.save({"state_dict": sd}, path)

    a = FishMICodec.from_checkpoint(str(path), 0, prec, 16, cfg=cfg, encoder=True,
                                    encoder_dim=spec["encoder_dim"], enc_layers=layers)
    b = FishMICodec(cfg, 0, prec, 16)
    b.enable_encoder(spec["encoder_dim"], layers)
    b.synth(seed)
    b.synth_encoder(seed)
    b.finalize()
    codes_a, codes_b = a.encode_audio(g["audio"]), b.encode_audio(g["audio"])
    np.testing.assert_array_equal(codes_a, codes_b)
    np.testing.assert_array_equal(a.decode_codes(codes_a), b.decode_codes(codes_a))
    a.close()
    b.close()
