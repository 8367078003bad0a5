"""Sentence-embedding encoders: BERT (bge-base, all-MiniLM-L6) and nomic-bert
(``nomic-embed-text``, the embedder the reference hard-codes at
``Minimal_RAG/Program.cs:18``).  Replaces Ollama's ``/api/embeddings`` compute.

Varlen packed batches ([T, H] rows + cu_seqlens) — no padding FLOPs:
  K1 embedding gather + LayerNorm (one kernel) -> per layer: QKV GEMM ->
  (rotary for nomic) -> bidirectional flash attention (K3, dense K/V rows) ->
  O GEMM (+bias) -> residual+LayerNorm (K4, one kernel) -> FFN up GEMM with the bias+GELU or
  SwiGLU epilogue fused -> down GEMM (+bias) ->
  residual+LayerNorm -> K5 mean/CLS pooling + L2 normalisation.
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn

from .. import ops
from .configs import EncoderConfig


class EncoderLayerWeights(nn.Module):
    def __init__(self, cfg: EncoderConfig, dtype, device):
        super().__init__()
        H, I = cfg.hidden, cfg.intermediate
        e = dict(dtype=dtype, device=device)

        def P(*shape, fill=None):
            t = torch.empty(*shape, **e) if fill is None else torch.full(shape, fill, **e)
            return nn.Parameter(t, requires_grad=False)

        self.qkv = P(3 * H, H)
        self.qkv_b = P(3 * H, fill=0.0) if cfg.bias else None
        self.o = P(H, H)
        self.o_b = P(H, fill=0.0) if cfg.bias else None
        self.ln1_w, self.ln1_b = P(H, fill=1.0), P(H, fill=0.0)
        n_up = 2 * I if cfg.activation == "swiglu" else I
        self.fc1 = P(n_up, H)
        self.fc1_b = P(n_up, fill=0.0) if cfg.bias else None
        self.fc2 = P(H, I)
        self.fc2_b = P(H, fill=0.0) if cfg.bias else None
        self.ln2_w, self.ln2_b = P(H, fill=1.0), P(H, fill=0.0)


class EncoderModel(nn.Module):
    def __init__(self, cfg: EncoderConfig, dtype=torch.bfloat16, device="cpu"):
        super().__init__()
        self.cfg, self.dtype, self.device = cfg, dtype, torch.device(device)
        H = cfg.hidden
        e = dict(dtype=dtype, device=device)
        self.tok = nn.Parameter(torch.empty(cfg.vocab_size, H, **e), requires_grad=False)
        self.pos = None if cfg.rotary else nn.Parameter(torch.empty(cfg.max_position, H, **e),
                                                         requires_grad=False)
        self.typ = nn.Parameter(torch.empty(cfg.type_vocab_size, H, **e), requires_grad=False)
        self.emb_ln_w = nn.Parameter(torch.ones(H, **e), requires_grad=False)
        self.emb_ln_b = nn.Parameter(torch.zeros(H, **e), requires_grad=False)
        self.layers = nn.ModuleList([EncoderLayerWeights(cfg, dtype, device) for _ in range(cfg.num_layers)])
        self.nh, self.D = cfg.num_heads, cfg.head_dim
        self.scale = 1.0 / math.sqrt(self.D)
        if cfg.rotary:
            self.register_buffer("cos_sin", ops.rope_cos_sin(cfg.max_position, self.D, cfg.rope_theta,
                                                             device=device), persistent=False)

    @property
    def dim(self) -> int:
        return self.cfg.hidden

    @torch.no_grad()
    def random_init(self, seed: int = 0, std: float = 0.02):
        gen_dev = self.device if self.device.type == "cuda" else torch.device("cpu")
        for i, (name, p) in enumerate(self.named_parameters()):
            if name.endswith("ln_w") or name.endswith("ln1_w") or name.endswith("ln2_w"):
                p.fill_(1.0)
            elif name.endswith("_b"):
                p.zero_()
            else:
                g = torch.Generator(device=gen_dev).manual_seed(seed * 7919 + i * 104729)
                p.copy_(torch.randn(p.shape, generator=g, device=gen_dev).mul_(std).to(p.dtype))
        return self

    def forward(self, ids: torch.Tensor, cu: torch.Tensor, positions: torch.Tensor,
                lens_cpu: list, type_ids=None, pool: bool = True, out=None, tiles=None):
        """ids/positions [T] int32 packed; cu [B+1] int32 -> [B, H] f32 embeddings (``out``: the
        pooling kernel writes these rows instead, f32 or bf16; ``tiles``: the attention's device
        tile list, precomputed -- a hipGraph capture cannot upload it)."""
        cfg, nh, D, H = self.cfg, self.nh, self.D, self.cfg.hidden
        h = ops.embed_layernorm(ids, None if cfg.rotary else positions, type_ids, self.tok, self.pos,
                                self.typ, self.emb_ln_w, self.emb_ln_b, cfg.norm_eps)
        for L in self.layers:
            qkv = ops.linear(h, L.qkv, L.qkv_b)
            if cfg.rotary:
                ops.rope_kv_(qkv, positions, self.cos_sin, nh, nh, D, None, None, None, True, True)
            a = ops.flash_prefill(qkv[:, :H], qkv[:, H:2 * H], qkv[:, 2 * H:], cu, nh, nh, D, self.scale,
                                  False, q_lens_cpu=lens_cpu, tiles=tiles)
            o = ops.linear(a, L.o, L.o_b)
            h = ops.layernorm(o, L.ln1_w, L.ln1_b, cfg.norm_eps, residual=h)
            if cfg.activation == "swiglu":
                f = ops.linear_swiglu(h, L.fc1) if L.fc1_b is None else ops.silu_mul(ops.linear(h, L.fc1, L.fc1_b))
            else:
                f = ops.linear(h, L.fc1, L.fc1_b, act="gelu")  # bias + GELU fused into the GEMM
            d = ops.linear(f, L.fc2, L.fc2_b)
            h = ops.layernorm(d, L.ln2_w, L.ln2_b, cfg.norm_eps, residual=h)
        if not pool:
            return h
        return ops.pool_normalize(h, cu, 1 if cfg.pooling == "cls" else 0, cfg.normalize, out=out)

    @torch.no_grad()
    def load_hf_state_dict(self, sd: dict):
        """HuggingFace ``BertModel`` names (bge / MiniLM)."""
        def t(n):
            for k in (n, "bert." + n, n.replace("embeddings.", "bert.embeddings.")):
                if k in sd:
                    return sd[k].to(self.dtype)
            raise KeyError(n)

        self.tok.copy_(t("embeddings.word_embeddings.weight"))
        if self.pos is not None:
            self.pos.copy_(t("embeddings.position_embeddings.weight"))
        self.typ.copy_(t("embeddings.token_type_embeddings.weight"))
        self.emb_ln_w.copy_(t("embeddings.LayerNorm.weight"))
        self.emb_ln_b.copy_(t("embeddings.LayerNorm.bias"))
        for i, L in enumerate(self.layers):
            p = f"encoder.layer.{i}."
            L.qkv.copy_(torch.cat([t(p + f"attention.self.{n}.weight") for n in ("query", "key", "value")]))
            if L.qkv_b is not None:
                L.qkv_b.copy_(torch.cat([t(p + f"attention.self.{n}.bias") for n in ("query", "key", "value")]))
            L.o.copy_(t(p + "attention.output.dense.weight"))
            if L.o_b is not None:
                L.o_b.copy_(t(p + "attention.output.dense.bias"))
            L.ln1_w.copy_(t(p + "attention.output.LayerNorm.weight"))
            L.ln1_b.copy_(t(p + "attention.output.LayerNorm.bias"))
            L.fc1.copy_(t(p + "intermediate.dense.weight"))
            if L.fc1_b is not None:
                L.fc1_b.copy_(t(p + "intermediate.dense.bias"))
            L.fc2.copy_(t(p + "output.dense.weight"))
            if L.fc2_b is not None:
                L.fc2_b.copy_(t(p + "output.dense.bias"))
            L.ln2_w.copy_(t(p + "output.LayerNorm.weight"))
            L.ln2_b.copy_(t(p + "output.LayerNorm.bias"))
        return self
