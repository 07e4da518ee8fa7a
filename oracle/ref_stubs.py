"""Stand-ins that let the read-only reference (/root/reference) import on this CPU box.

TEST INFRASTRUCTURE ONLY (used by oracle/gen_goldens.py in the survey container; never
shipped, never imported by the product path).

Absent packages and what replaces them:
  * loguru                 -> stdlib logging (logging only, no arithmetic)
  * loralib                -> empty module (LoRA is never constructed at inference)
  * audiotools             -> BaseModel = nn.Module, AudioSignal placeholder
  * dac.model.base         -> CodecMixin.get_delay() = 0 (only used in DAC.__init__)
  * dac.nn.layers          -> Snake1d, WNConv1d, WNConvTranspose1d restated from
                              descript-audio-codec==1.0.0 (uv.lock:861-863):
                              snake(x) = x + (alpha + 1e-9)^-1 * sin(alpha * x)^2,
                              WN convs = torch.nn.utils.weight_norm (keys weight_g/weight_v)
  * dac.nn.quantize        -> ResidualVectorQuantize with the decode half used by
                              rvq.py:352-366: quantizers[i].{in_proj,out_proj,codebook};
                              from_codes sums out_proj(embedding(code).T)
The descript arithmetic is third-party and absent here, so the codec oracle is pinned
against this restatement of descript 1.0.0's published formulas (parity on the
descript boundary is "unpinned" in the strict sense).
"""
from __future__ import annotations

import logging
import sys
import types

import torch
import torch.nn as nn
import torch.nn.functional as F

REFERENCE = "/root/reference"


def install() -> None:
    if "loguru" not in sys.modules:
        m = types.ModuleType("loguru")
        m.logger = logging.getLogger("reference")
        sys.modules["loguru"] = m
    if "loralib" not in sys.modules:
        sys.modules["loralib"] = types.ModuleType("loralib")

    # ---- audiotools ------------------------------------------------------------------
    at = types.ModuleType("audiotools")
    at_ml = types.ModuleType("audiotools.ml")

    class AudioSignal:  # placeholder, never used on the decode path
        pass

    at.AudioSignal = AudioSignal
    at_ml.BaseModel = nn.Module
    at.ml = at_ml
    sys.modules["audiotools"] = at
    sys.modules["audiotools.ml"] = at_ml

    # ---- dac ---------------------------------------------------------------------------
    dac = types.ModuleType("dac")
    dac_model = types.ModuleType("dac.model")
    dac_base = types.ModuleType("dac.model.base")
    dac_nn = types.ModuleType("dac.nn")
    dac_layers = types.ModuleType("dac.nn.layers")
    dac_quant = types.ModuleType("dac.nn.quantize")

    class CodecMixin:
        def get_delay(self):
            return 0

    dac_base.CodecMixin = CodecMixin

    def snake(x, alpha):
        shape = x.shape
        x = x.reshape(shape[0], shape[1], -1)
        x = x + (alpha + 1e-9).reciprocal() * torch.sin(alpha * x).pow(2)
        return x.reshape(shape)

    class Snake1d(nn.Module):
        def __init__(self, channels):
            super().__init__()
            self.alpha = nn.Parameter(torch.ones(1, channels, 1))

        def forward(self, x):
            return snake(x, self.alpha)

    def WNConv1d(*args, **kwargs):
        return torch.nn.utils.weight_norm(nn.Conv1d(*args, **kwargs))

    def WNConvTranspose1d(*args, **kwargs):
        return torch.nn.utils.weight_norm(nn.ConvTranspose1d(*args, **kwargs))

    dac_layers.Snake1d = Snake1d
    dac_layers.WNConv1d = WNConv1d
    dac_layers.WNConvTranspose1d = WNConvTranspose1d

    class VectorQuantize(nn.Module):
        def __init__(self, input_dim, codebook_size, codebook_dim):
            super().__init__()
            self.codebook_size = codebook_size
            self.codebook_dim = codebook_dim
            self.in_proj = WNConv1d(input_dim, codebook_dim, kernel_size=1)
            self.out_proj = WNConv1d(codebook_dim, input_dim, kernel_size=1)
            self.codebook = nn.Embedding(codebook_size, codebook_dim)

        def decode_code(self, embed_id):
            return F.embedding(embed_id, self.codebook.weight).transpose(1, 2)

        # encode side (descript-audio-codec 1.0.0 dac/nn/quantize.py VectorQuantize.forward /
        # decode_latents, restated): in_proj, nearest codebook entry by l2-normalised
        # distance, straight-through z_q, out_proj.  Losses are training-only and omitted.
        def decode_latents(self, latents):
            b = latents.shape[0]
            enc = latents.transpose(1, 2).reshape(-1, latents.shape[1])
            enc = F.normalize(enc)
            cbk = F.normalize(self.codebook.weight)
            dist = enc.pow(2).sum(1, keepdim=True) - 2 * enc @ cbk.t() + cbk.pow(2).sum(1, keepdim=True).t()
            indices = (-dist).max(1)[1].reshape(b, -1)
            return self.decode_code(indices), indices

        def forward(self, z):
            z_e = self.in_proj(z)
            z_q, indices = self.decode_latents(z_e)
            z_q = z_e + (z_q - z_e).detach()
            z_q = self.out_proj(z_q)
            zero = torch.zeros(z.shape[0])
            return z_q, zero, zero, indices, z_e

    class ResidualVectorQuantize(nn.Module):
        def __init__(self, input_dim=512, n_codebooks=9, codebook_size=1024,
                     codebook_dim=8, quantizer_dropout=0.0):
            super().__init__()
            if isinstance(codebook_dim, int):
                codebook_dim = [codebook_dim for _ in range(n_codebooks)]
            self.n_codebooks = n_codebooks
            self.codebook_dim = codebook_dim
            self.codebook_size = codebook_size
            self.quantizers = nn.ModuleList(
                VectorQuantize(input_dim, codebook_size, codebook_dim[i])
                for i in range(n_codebooks)
            )
            self.quantizer_dropout = quantizer_dropout

        # descript 1.0.0 ResidualVectorQuantize.forward, eval mode (no quantizer dropout)
        def forward(self, z, n_quantizers=None):
            z_q = 0
            residual = z
            codes, latents = [], []
            if n_quantizers is None:
                n_quantizers = self.n_codebooks
            zero = torch.zeros(z.shape[0])
            for i, quantizer in enumerate(self.quantizers):
                if i >= n_quantizers:
                    break
                z_q_i, _, _, indices_i, z_e_i = quantizer(residual)
                z_q = z_q + z_q_i
                residual = residual - z_q_i
                codes.append(indices_i)
                latents.append(z_e_i)
            return z_q, torch.stack(codes, dim=1), torch.cat(latents, dim=1), zero, zero

        def from_codes(self, codes):
            z_q = 0.0
            z_p = []
            for i in range(codes.shape[1]):
                z_p_i = self.quantizers[i].decode_code(codes[:, i, :])
                z_p.append(z_p_i)
                z_q = z_q + self.quantizers[i].out_proj(z_p_i)
            return z_q, torch.cat(z_p, dim=1), codes

    dac_quant.ResidualVectorQuantize = ResidualVectorQuantize
    dac.model = dac_model
    dac_model.base = dac_base
    dac.nn = dac_nn
    dac_nn.layers = dac_layers
    dac_nn.quantize = dac_quant
    for name, mod in [("dac", dac), ("dac.model", dac_model), ("dac.model.base", dac_base),
                      ("dac.nn", dac_nn), ("dac.nn.layers", dac_layers),
                      ("dac.nn.quantize", dac_quant)]:
        sys.modules[name] = mod

    if REFERENCE not in sys.path:
        sys.path.insert(0, REFERENCE)
