"""Weight creation: seeded random init (synthetic benchmarks) and HF safetensors loading, with TP/EP sharding.

Sharding (Megatron, ``tp`` ranks):
  qkv      [(Hq + 2 Hkv) D, d]  column-parallel: rank r keeps its Hq/tp query heads, Hkv/tp key heads, Hkv/tp value heads
  o        [d, Hq D]            row-parallel:    the input columns of its query heads
  gate_up  [2F, d]              column-parallel: its F/tp gate rows and its F/tp up rows
  down     [d, F]               row-parallel
  embed / lm_head [V, d]        vocab-parallel rows (padded to a multiple of tp)
  Mixtral experts               expert-parallel over the same ranks (models/moe.py)

Random init: small models (and every test) draw each FULL tensor from a per-name seed on the CPU and slice it, so a
TP=k model computes the same function as TP=1 (tests/test_tp_equivalence.py). Large models draw each rank's shard
directly on the GPU (per-(name, rank) seed) — 8B/70B bf16 in seconds, no host round trip.
"""
from __future__ import annotations

import hashlib
import json
from pathlib import Path

import torch

from kafka_llm_service_amd.models.config import ModelConfig
from kafka_llm_service_amd.models.llama import TransformerLM

INIT_STD = 0.02


def _seed(name: str, base: int) -> int:
    return int(hashlib.sha1(f"{base}:{name}".encode()).hexdigest()[:12], 16)


def _randn(shape, seed: int, device, dtype, std=INIT_STD) -> torch.Tensor:
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    t = torch.empty(shape, dtype=torch.float32 if device.type == "cpu" else dtype, device=device)
    t.normal_(0.0, std, generator=g)
    return t.to(dtype)


class _Shard:
    def __init__(self, cfg: ModelConfig, tp: int, r: int):
        self.cfg, self.tp, self.r = cfg, tp, r
        D = cfg.head_dim
        self.hq, self.hkv = cfg.num_heads // tp, cfg.num_kv_heads // tp
        self.q_rows = slice(r * self.hq * D, (r + 1) * self.hq * D)
        qn, kn = cfg.num_heads * D, cfg.num_kv_heads * D
        self.k_rows = slice(qn + r * self.hkv * D, qn + (r + 1) * self.hkv * D)
        self.v_rows = slice(qn + kn + r * self.hkv * D, qn + kn + (r + 1) * self.hkv * D)
        F = cfg.intermediate_size
        self.f = F // tp
        self.g_rows = slice(r * self.f, (r + 1) * self.f)
        self.u_rows = slice(F + r * self.f, F + (r + 1) * self.f)
        self.v_local = (cfg.vocab_size + tp - 1) // tp
        self.vocab = slice(r * self.v_local, (r + 1) * self.v_local)

    def qkv(self, w):
        return torch.cat([w[self.q_rows], w[self.k_rows], w[self.v_rows]], 0)

    def o(self, w):
        return w[:, self.q_rows]

    def gate_up(self, w):
        return torch.cat([w[self.g_rows], w[self.u_rows]], 0)

    def down(self, w):
        return w[:, self.g_rows]

    def vocab_rows(self, w):
        out = w[self.vocab]
        if out.shape[0] < self.v_local:
            out = torch.cat([out, out.new_zeros(self.v_local - out.shape[0], out.shape[1])], 0)
        return out


def full_shapes(cfg: ModelConfig) -> dict[str, tuple]:
    d, D = cfg.hidden_size, cfg.head_dim
    qkv = (cfg.num_heads + 2 * cfg.num_kv_heads) * D
    s = {"embed": (cfg.vocab_size, d), "lm_head": (cfg.vocab_size, d), "final_norm": (d,)}
    for i in range(cfg.num_layers):
        p = f"layers.{i}."
        s[p + "input_norm"] = (d,)
        s[p + "post_norm"] = (d,)
        s[p + "qkv"] = (qkv, d)
        s[p + "o"] = (d, cfg.num_heads * D)
        if cfg.num_experts:
            s[p + "router"] = (cfg.num_experts, d)
            s[p + "w13"] = (cfg.num_experts, 2 * cfg.intermediate_size, d)
            s[p + "w2"] = (cfg.num_experts, d, cfg.intermediate_size)
        else:
            s[p + "gate_up"] = (2 * cfg.intermediate_size, d)
            s[p + "down"] = (d, cfg.intermediate_size)
    return s


def _shard_tensor(sh: _Shard, key: str, w: torch.Tensor, ep_slice: slice | None) -> torch.Tensor:
    if key in ("embed", "lm_head"):
        return sh.vocab_rows(w)
    kind = key.split(".")[-1]
    if kind == "qkv":
        return sh.qkv(w)
    if kind == "o":
        return sh.o(w)
    if kind == "gate_up":
        return sh.gate_up(w)
    if kind == "down":
        return sh.down(w)
    if kind in ("w13", "w2") and ep_slice is not None:
        return w[ep_slice]
    return w


def _assign(model: TransformerLM, key: str, t: torch.Tensor) -> None:
    if key in ("embed", "lm_head", "final_norm"):
        setattr(model, key, t)
        return
    _, i, kind = key.split(".")
    setattr(model.layers[int(i)], kind, t)


def ep_slice(cfg: ModelConfig, tp: int, r: int) -> slice | None:
    if not cfg.num_experts:
        return None
    if tp == 1:
        return slice(0, cfg.num_experts)
    if cfg.num_experts % tp:
        raise ValueError("num_experts must be divisible by the EP size")
    n = cfg.num_experts // tp
    return slice(r * n, (r + 1) * n)


def random_init(model: TransformerLM, seed: int = 0, exact_tp: bool | None = None) -> TransformerLM:
    cfg, tp, r = model.cfg, model.tp, model.tp_rank
    dev, dt = model.device, model.dtype
    if exact_tp is None:
        exact_tp = cfg.num_params() < 2e9 or tp == 1
    sh = _Shard(cfg, tp, r)
    eps = ep_slice(cfg, model.ep, model.ep_rank)
    er = model.ep_rank if model.dp_attention else r  # the rank whose shard a per-rank seed draws
    for key, shape in full_shapes(cfg).items():
        kind = key.split(".")[-1]
        if kind in ("input_norm", "post_norm", "final_norm"):
            t = torch.ones(shape, dtype=dt, device=dev)
        elif exact_tp:
            # drawn on this rank's device with the device's generator, like the TP=1 model: the shards of a TP group
            # are then exact slices of the TP=1 weights on the same kind of device
            full = _randn(shape, _seed(key, seed), dev, dt)
            t = _shard_tensor(sh, key, full, eps).to(dev).contiguous()
        else:
            # same shapes as the shard, drawn directly on the device
            probe = torch.empty(shape, device="meta")
            lshape = _shard_tensor(sh, key, probe, eps).shape
            t = _randn(lshape, _seed(f"{key}@{er}" if key.endswith(("w13", "w2")) else f"{key}@{r}", seed), dev, dt)
        _assign(model, key, t)
    _finish(model)
    return model


def _finish(model: TransformerLM) -> None:
    if model.cfg.num_experts:
        from kafka_llm_service_amd.models.moe import MoEBlock

        model.moe = MoEBlock(model)


# ---------------------------------------------------------------------------------------------------------------
# HF safetensors checkpoints (Llama / Mixtral naming). Loaded with safetensors only (never pickle).
def _hf_names(cfg: ModelConfig, i: int) -> dict:
    p = f"model.layers.{i}."
    return {
        "input_norm": p + "input_layernorm.weight", "post_norm": p + "post_attention_layernorm.weight",
        "q": p + "self_attn.q_proj.weight", "k": p + "self_attn.k_proj.weight", "v": p + "self_attn.v_proj.weight",
        "o": p + "self_attn.o_proj.weight", "gate": p + "mlp.gate_proj.weight", "up": p + "mlp.up_proj.weight",
        "down": p + "mlp.down_proj.weight", "router": p + "block_sparse_moe.gate.weight",
        "expert": p + "block_sparse_moe.experts.{e}.{w}.weight",
    }


def load_safetensors(model: TransformerLM, path: str | Path) -> TransformerLM:
    from safetensors import safe_open

    path = Path(path)
    files = sorted(path.glob("*.safetensors")) if path.is_dir() else [path]
    handles = [safe_open(str(f), framework="pt", device="cpu") for f in files]
    index = {}
    for h in handles:
        for k in h.keys():
            index[k] = h

    def get(name):
        return index[name].get_tensor(name)

    cfg, tp, r = model.cfg, model.tp, model.tp_rank
    sh = _Shard(cfg, tp, r)
    eps = ep_slice(cfg, model.ep, model.ep_rank)
    dev, dt = model.device, model.dtype

    def put(key, t):
        _assign(model, key, _shard_tensor(sh, key, t, eps).to(device=dev, dtype=dt).contiguous())

    put("embed", get("model.embed_tokens.weight"))
    put("lm_head", get("lm_head.weight") if "lm_head.weight" in index else get("model.embed_tokens.weight"))
    put("final_norm", get("model.norm.weight"))
    for i in range(cfg.num_layers):
        n = _hf_names(cfg, i)
        put(f"layers.{i}.input_norm", get(n["input_norm"]))
        put(f"layers.{i}.post_norm", get(n["post_norm"]))
        put(f"layers.{i}.qkv", torch.cat([get(n["q"]), get(n["k"]), get(n["v"])], 0))
        put(f"layers.{i}.o", get(n["o"]))
        if cfg.num_experts:
            put(f"layers.{i}.router", get(n["router"]))
            w13 = torch.stack([torch.cat([get(n["expert"].format(e=e, w="w1")), get(n["expert"].format(e=e, w="w3"))], 0)
                               for e in range(cfg.num_experts)])
            w2 = torch.stack([get(n["expert"].format(e=e, w="w2")) for e in range(cfg.num_experts)])
            put(f"layers.{i}.w13", w13)
            put(f"layers.{i}.w2", w2)
        else:
            put(f"layers.{i}.gate_up", torch.cat([get(n["gate"]), get(n["up"])], 0))
            put(f"layers.{i}.down", get(n["down"]))
    _finish(model)
    return model


def save_safetensors(model: TransformerLM, path: str | Path) -> None:
    """Write a TP=1 model in HF naming (used by tests to round-trip the loader)."""
    from safetensors.torch import save_file

    cfg = model.cfg
    assert model.tp == 1
    D, F = cfg.head_dim, cfg.intermediate_size
    qn, kn = cfg.num_heads * D, cfg.num_kv_heads * D
    from kafka_llm_service_amd import ops

    def dense(lw, name):  # tiled-only models keep just the wave-tiled copy: untile it for export
        w = getattr(lw, name)
        return w if w is not None else ops.untile_weight(getattr(lw, name + "_t"), glu=bool(lw.glu) and
                                                         name == "gate_up")

    lm_head = model.lm_head if model.lm_head is not None else ops.untile_weight(model.lm_head_t)
    out = {"model.embed_tokens.weight": model.embed, "lm_head.weight": lm_head,
           "model.norm.weight": model.final_norm}
    for i, lw in enumerate(model.layers):
        qkv, o = dense(lw, "qkv"), dense(lw, "o")
        n = _hf_names(cfg, i)
        out[n["input_norm"]] = lw.input_norm
        out[n["post_norm"]] = lw.post_norm
        out[n["q"]], out[n["k"]], out[n["v"]] = qkv[:qn], qkv[qn:qn + kn], qkv[qn + kn:]
        out[n["o"]] = o
        if cfg.num_experts:
            out[n["router"]] = lw.router
            for e in range(cfg.num_experts):
                out[n["expert"].format(e=e, w="w1")] = lw.w13[e, :F]
                out[n["expert"].format(e=e, w="w3")] = lw.w13[e, F:]
                out[n["expert"].format(e=e, w="w2")] = lw.w2[e]
        else:
            gu = dense(lw, "gate_up")
            out[n["gate"]], out[n["up"]] = gu[:F], gu[F:]
            out[n["down"]] = dense(lw, "down")
    out = {k: v.detach().cpu().contiguous() for k, v in out.items()}
    Path(path).parent.mkdir(parents=True, exist_ok=True)
    save_file(out, str(path))
    (Path(path).parent / "config.json").write_text(json.dumps({
        "hidden_size": cfg.hidden_size, "intermediate_size": cfg.intermediate_size,
        "num_hidden_layers": cfg.num_layers, "num_attention_heads": cfg.num_heads,
        "num_key_value_heads": cfg.num_kv_heads, "head_dim": cfg.head_dim, "vocab_size": cfg.vocab_size,
        "rms_norm_eps": cfg.rms_norm_eps, "rope_theta": cfg.rope_theta, "rope_scaling": cfg.rope_scaling,
        "max_position_embeddings": cfg.max_position_embeddings, "num_local_experts": cfg.num_experts or None,
        "num_experts_per_tok": cfg.num_experts_per_tok or None, "bos_token_id": cfg.bos_token_id,
        "eos_token_id": cfg.eos_token_ids}))


def build_model(cfg: ModelConfig, device, tp: int = 1, tp_rank: int = 0, seed: int = 0, weights: str | None = None,
                max_positions: int | None = None, dp_attention: tuple[int, int] | None = None) -> TransformerLM:
    """``dp_attention = (ep, ep_rank)``: whole attention on this rank, experts sharded over the EP group."""
    model = TransformerLM(cfg, device, tp=tp, tp_rank=tp_rank, max_positions=max_positions)
    if dp_attention is not None:
        model.enable_dp_attention(*dp_attention)
    if weights:
        return load_safetensors(model, weights)
    return random_init(model, seed)
