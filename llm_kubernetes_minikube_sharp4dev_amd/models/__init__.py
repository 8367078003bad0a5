"""Model construction: presets (``configs``), random-init or checkpoint weights."""
from __future__ import annotations

from pathlib import Path
from typing import Optional

import torch

from ..parallel.tp import SINGLE, TPGroup
from .bert import EncoderModel
from .configs import DECODERS, ENCODERS, DecoderConfig, EncoderConfig, decoder_config, encoder_config
from . import llama
from .llama import LlamaModel
from .opt import OPTModel


def _load_safetensors_dir(path: str) -> dict:
    from safetensors.torch import load_file

    sd = {}
    for f in sorted(Path(path).glob("*.safetensors")):
        sd.update(load_file(str(f)))
    if not sd:
        raise FileNotFoundError(f"no *.safetensors in {path}")
    return sd


def build_decoder(name: str | DecoderConfig, device="cpu", dtype=torch.bfloat16, tp: TPGroup = SINGLE,
                  seed: int = 0, checkpoint: Optional[str] = None, **overrides):
    cfg = name if isinstance(name, DecoderConfig) else decoder_config(name, **overrides)
    cls = LlamaModel if cfg.arch == "llama" else OPTModel
    m = cls(cfg, tp, dtype, device)
    if checkpoint:
        m.load_hf_state_dict(_load_safetensors_dir(checkpoint))  # folds on the GPU itself
    else:
        m.random_init(seed)
        if isinstance(m, LlamaModel) and m.device.type == "cuda" and llama.FOLD_NORMS:
            m.fold_norms()
    return m.eval()


def build_encoder(name: str | EncoderConfig, device="cpu", dtype=torch.bfloat16, seed: int = 0,
                  checkpoint: Optional[str] = None, **overrides):
    cfg = name if isinstance(name, EncoderConfig) else encoder_config(name, **overrides)
    m = EncoderModel(cfg, dtype, device)
    if checkpoint:
        m.load_hf_state_dict(_load_safetensors_dir(checkpoint))
    else:
        m.random_init(seed)
    return m.eval()


__all__ = ["build_decoder", "build_encoder", "DECODERS", "ENCODERS", "DecoderConfig", "EncoderConfig",
           "LlamaModel", "OPTModel", "EncoderModel"]
