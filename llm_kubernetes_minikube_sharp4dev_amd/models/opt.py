"""OPT decoder (OPT-125m: the CPU-config generator of BASELINE.json:7).

Pre-LN LayerNorm blocks, learned positions (offset 2), ReLU FFN with biases, tied
LM head.  Residual adds are folded into the LayerNorm kernel exactly like the
Llama RMSNorm path; attention shares the paged flash / decode kernels.
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn

from .. import ops
from ..parallel.tp import SINGLE, TPGroup
from .attention import AttnMeta, paged_attention
from .configs import DecoderConfig, pad_vocab


class OPTLayerWeights(nn.Module):
    def __init__(self, cfg: DecoderConfig, tp: TPGroup, dtype, device):
        super().__init__()
        H, D = cfg.hidden, cfg.head_dim
        hq = cfg.num_heads // tp.size
        I = cfg.intermediate // tp.size
        e = dict(dtype=dtype, device=device)

        def P(*shape, fill=None):
            t = torch.empty(*shape, **e) if fill is None else torch.full(shape, fill, **e)
            return nn.Parameter(t, requires_grad=False)

        self.attn_ln_w, self.attn_ln_b = P(H, fill=1.0), P(H, fill=0.0)
        self.ffn_ln_w, self.ffn_ln_b = P(H, fill=1.0), P(H, fill=0.0)
        self.qkv, self.qkv_b = P(3 * hq * D, H), P(3 * hq * D, fill=0.0)
        self.o, self.o_b = P(H, hq * D), P(H, fill=0.0)
        self.fc1, self.fc1_b = P(I, H), P(I, fill=0.0)
        self.fc2, self.fc2_b = P(H, I), P(H, fill=0.0)


class OPTModel(nn.Module):
    def __init__(self, cfg: DecoderConfig, tp: TPGroup = SINGLE, dtype=torch.bfloat16, device="cpu"):
        super().__init__()
        self.cfg, self.tp, self.dtype, self.device = cfg, tp, dtype, torch.device(device)
        self.hq = self.hkv = cfg.num_heads // tp.size
        self.D = cfg.head_dim
        self.scale = 1.0 / math.sqrt(self.D)
        # context-parallel group for attention (models/attention.py cp_paged_attention); None = off
        self.cp_group = None
        e = dict(dtype=dtype, device=device)
        self.vocab_lo, self.vocab_hi = 0, cfg.vocab_size
        self.vocab_local = cfg.vocab_size
        # tied embedding / LM head padded to the GEMM's 256-column tile (50272 -> 50432 zero
        # rows; logits sliced back): the head runs on the MFMA kernels, not the vendor library
        self.embed = nn.Parameter(torch.empty(pad_vocab(cfg.vocab_size), cfg.hidden, **e), requires_grad=False)
        self.pos_embed = nn.Parameter(torch.empty(cfg.max_position + cfg.pos_offset, cfg.hidden, **e),
                                      requires_grad=False)
        self.layers = nn.ModuleList([OPTLayerWeights(cfg, tp, dtype, device) for _ in range(cfg.num_layers)])
        self.final_ln_w = nn.Parameter(torch.ones(cfg.hidden, **e), requires_grad=False)
        self.final_ln_b = nn.Parameter(torch.zeros(cfg.hidden, **e), requires_grad=False)
        self.lm_head = self.embed

    @torch.no_grad()
    def random_init(self, seed: int = 0, std: float = 0.02):
        gen_dev = self.device if self.device.type == "cuda" else torch.device("cpu")
        for i, (name, p) in enumerate(self.named_parameters()):
            if name.endswith("_ln_w"):
                p.fill_(1.0)
            elif name.endswith("_b"):
                p.zero_()
            else:
                g = torch.Generator(device=gen_dev).manual_seed(seed * 7919 + i * 104729 + self.tp.rank)
                p.copy_(torch.randn(p.shape, generator=g, device=gen_dev).mul_(std).to(p.dtype))
        self.embed[self.vocab_local:].zero_()
        return self

    def forward(self, ids: torch.Tensor, meta: AttnMeta, kv_caches) -> torch.Tensor:
        cfg, hq, D = self.cfg, self.hq, self.D
        res = self.embed[ids.long()] + self.pos_embed[meta.positions.long() + cfg.pos_offset]
        if self.tp.enabled:
            res = res.contiguous()
        L0 = self.layers[0]
        x = ops.layernorm(res, L0.attn_ln_w, L0.attn_ln_b, cfg.norm_eps)
        attn_out = None
        n = len(self.layers)
        for li, L in enumerate(self.layers):
            qkv = ops.linear(x, L.qkv, L.qkv_b)
            T = qkv.shape[0]
            kc, vc = kv_caches[li]
            k = qkv[:, hq * D:2 * hq * D].view(T, hq, D)
            v = qkv[:, 2 * hq * D:3 * hq * D].view(T, hq, D)
            ops.kv_write(k, v, kc, vc, meta.slots)
            attn_out = paged_attention(qkv, kc, vc, meta, hq, hq, D, self.scale, attn_out, cp_group=self.cp_group)
            o = ops.linear(attn_out, L.o, L.o_b if self.tp.rank == 0 else None)
            self.tp.all_reduce_(o)
            x = ops.layernorm(o, L.ffn_ln_w, L.ffn_ln_b, cfg.norm_eps, residual=res, write_residual=True)
            f = ops.linear(x, L.fc1, L.fc1_b, act="relu")
            d = ops.linear(f, L.fc2, L.fc2_b if self.tp.rank == 0 else None)
            self.tp.all_reduce_(d)
            if li + 1 < n:
                nx = self.layers[li + 1]
                x = ops.layernorm(d, nx.attn_ln_w, nx.attn_ln_b, cfg.norm_eps, residual=res, write_residual=True)
            else:
                x = ops.layernorm(d, self.final_ln_w, self.final_ln_b, cfg.norm_eps, residual=res,
                                  write_residual=True)
        if meta.logits_idx is not None:
            x = x.index_select(0, meta.logits_idx)
        return x

    def head(self, hidden):
        lg = ops.linear(hidden, self.lm_head)
        return lg[:, : self.vocab_local] if lg.shape[1] != self.vocab_local else lg

    def logits(self, hidden, gather: bool = True, dtype=torch.float32):
        lg = self.head(hidden)
        return lg.to(dtype) if dtype is not None else lg

    def greedy(self, hidden):
        return self.tp.greedy_ids(self.head(hidden), self.vocab_lo)

    @torch.no_grad()
    def load_hf_state_dict(self, sd: dict):
        """HuggingFace ``OPTForCausalLM`` names (``model.decoder.*``)."""
        tp, D, cfg = self.tp, self.D, self.cfg

        def t(n):
            key = n if n in sd else n.replace("model.decoder.", "decoder.")
            return sd[key].to(self.dtype)

        s, e = tp.shard(cfg.num_heads)
        fs, fe = tp.shard(cfg.intermediate)
        self.embed[: self.vocab_local].copy_(t("model.decoder.embed_tokens.weight"))
        self.embed[self.vocab_local:].zero_()
        self.pos_embed.copy_(t("model.decoder.embed_positions.weight")[: self.pos_embed.shape[0]])
        for i, L in enumerate(self.layers):
            p = f"model.decoder.layers.{i}."
            w = [t(p + f"self_attn.{n}_proj.weight")[s * D:e * D] for n in "qkv"]
            b = [t(p + f"self_attn.{n}_proj.bias")[s * D:e * D] for n in "qkv"]
            L.qkv.copy_(torch.cat(w, 0))
            L.qkv_b.copy_(torch.cat(b, 0))
            L.o.copy_(t(p + "self_attn.out_proj.weight")[:, s * D:e * D])
            L.o_b.copy_(t(p + "self_attn.out_proj.bias"))
            L.attn_ln_w.copy_(t(p + "self_attn_layer_norm.weight"))
            L.attn_ln_b.copy_(t(p + "self_attn_layer_norm.bias"))
            L.ffn_ln_w.copy_(t(p + "final_layer_norm.weight"))
            L.ffn_ln_b.copy_(t(p + "final_layer_norm.bias"))
            L.fc1.copy_(t(p + "fc1.weight")[fs:fe])
            L.fc1_b.copy_(t(p + "fc1.bias")[fs:fe])
            L.fc2.copy_(t(p + "fc2.weight")[:, fs:fe])
            L.fc2_b.copy_(t(p + "fc2.bias"))
        self.final_ln_w.copy_(t("model.decoder.final_layer_norm.weight"))
        self.final_ln_b.copy_(t("model.decoder.final_layer_norm.bias"))
        return self

    def kv_cache_shape(self, num_blocks: int, block_size: int):
        return (num_blocks, self.hkv, block_size, self.D)

    def kv_bytes_per_token(self) -> int:
        return 2 * self.cfg.num_layers * self.hkv * self.D * 2
