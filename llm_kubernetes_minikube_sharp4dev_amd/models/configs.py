"""Architecture presets for every model the reference names or BASELINE.json configs use
(SURVEY Appendix B).  Dimensions are public model-card facts; weights are random-init
(fixed seed) unless a safetensors checkpoint directory is supplied."""
from __future__ import annotations

import dataclasses
from dataclasses import dataclass, field
from typing import Optional


@dataclass
class DecoderConfig:
    name: str
    arch: str                    # "llama" | "opt"
    num_layers: int
    hidden: int
    num_heads: int
    num_kv_heads: int
    head_dim: int
    intermediate: int
    vocab_size: int
    max_position: int = 8192
    norm_eps: float = 1e-5
    rope_theta: float = 500000.0
    rope_scaling: Optional[dict] = None
    tie_word_embeddings: bool = False
    bos_token_id: int = 1
    eos_token_ids: tuple = (2,)
    # OPT specifics
    pos_offset: int = 2
    activation: str = "silu"     # silu (SwiGLU) | relu | gelu
    bias: bool = False


@dataclass
class EncoderConfig:
    name: str
    arch: str                    # "bert" | "nomic_bert"
    num_layers: int
    hidden: int
    num_heads: int
    intermediate: int
    vocab_size: int
    max_position: int = 512
    type_vocab_size: int = 2
    norm_eps: float = 1e-12
    pooling: str = "mean"        # mean | cls
    normalize: bool = True
    activation: str = "gelu"     # gelu | swiglu
    rotary: bool = False
    rope_theta: float = 1000.0
    bias: bool = True
    dim: int = field(init=False, default=0)

    def __post_init__(self):
        self.dim = self.hidden

    @property
    def head_dim(self) -> int:
        return self.hidden // self.num_heads


LLAMA3_SCALING = {"rope_type": "llama3", "factor": 8.0, "low_freq_factor": 1.0,
                  "high_freq_factor": 4.0, "original_max_position_embeddings": 8192}

DECODERS = {
    "llama-3-8b": DecoderConfig("llama-3-8b", "llama", 32, 4096, 32, 8, 128, 14336, 128256,
                                max_position=131072, rope_scaling=LLAMA3_SCALING,
                                bos_token_id=128000, eos_token_ids=(128001, 128008, 128009)),
    "llama-3-70b": DecoderConfig("llama-3-70b", "llama", 80, 8192, 64, 8, 128, 28672, 128256,
                                 max_position=131072, rope_scaling=LLAMA3_SCALING,
                                 bos_token_id=128000, eos_token_ids=(128001, 128008, 128009)),
    "opt-125m": DecoderConfig("opt-125m", "opt", 12, 768, 12, 12, 64, 3072, 50272,
                              max_position=2048, norm_eps=1e-5, tie_word_embeddings=True,
                              bos_token_id=2, eos_token_ids=(2,), activation="relu", bias=True),
    # small shapes for tests / smoke runs (same code paths, tiny weights)
    # (vocab = the built-in tokenizer's 32768 so text round-trips through the servers)
    "llama-tiny": DecoderConfig("llama-tiny", "llama", 2, 256, 4, 2, 64, 512, 32768,
                                max_position=4096, rope_theta=10000.0),
    "opt-tiny": DecoderConfig("opt-tiny", "opt", 2, 128, 2, 2, 64, 256, 32768, max_position=512,
                              tie_word_embeddings=True, activation="relu", bias=True,
                              bos_token_id=2, eos_token_ids=(2,)),
}

ENCODERS = {
    "bge-base": EncoderConfig("bge-base", "bert", 12, 768, 12, 3072, 30522, pooling="cls"),
    "minilm-l6": EncoderConfig("minilm-l6", "bert", 6, 384, 12, 1536, 30522, pooling="mean"),
    "nomic-embed-text": EncoderConfig("nomic-embed-text", "nomic_bert", 12, 768, 12, 3072, 30528,
                                      max_position=8192, pooling="mean", activation="swiglu",
                                      rotary=True, rope_theta=1000.0, bias=False),
    "bert-tiny": EncoderConfig("bert-tiny", "bert", 2, 128, 2, 256, 32768, max_position=512),
    "nomic-tiny": EncoderConfig("nomic-tiny", "nomic_bert", 2, 128, 2, 256, 32768,
                                max_position=2048, activation="swiglu", rotary=True, bias=False),
}


def decoder_config(name: str, **overrides) -> DecoderConfig:
    cfg = dataclasses.replace(DECODERS[name])
    for k, v in overrides.items():
        setattr(cfg, k, v)
    return cfg


def encoder_config(name: str, **overrides) -> EncoderConfig:
    cfg = dataclasses.replace(ENCODERS[name])
    for k, v in overrides.items():
        setattr(cfg, k, v)
    return cfg


def param_count(cfg: DecoderConfig) -> int:
    H, I, L, V = cfg.hidden, cfg.intermediate, cfg.num_layers, cfg.vocab_size
    qkv = H * (cfg.num_heads + 2 * cfg.num_kv_heads) * cfg.head_dim
    o = cfg.num_heads * cfg.head_dim * H
    mlp = (3 if cfg.activation == "silu" else 2) * H * I
    emb = V * H * (1 if cfg.tie_word_embeddings else 2)
    return L * (qkv + o + mlp + 2 * H) + emb + H


def pad_vocab(n: int, tile: int = 256) -> int:
    """Rows of an LM head padded to the MFMA GEMM kernels' 256-column tile."""
    return -(-n // tile) * tile
