"""Model architecture configs (public HF configs of the benchmark models; random-init weights)."""
from __future__ import annotations

import json
from dataclasses import asdict, dataclass, field
from pathlib import Path


@dataclass
class ModelConfig:
    name: str
    arch: str = "llama"  # "llama" | "mixtral"
    hidden_size: int = 4096
    intermediate_size: int = 14336
    num_layers: int = 32
    num_heads: int = 32
    num_kv_heads: int = 8
    head_dim: int = 128
    vocab_size: int = 128256
    rms_norm_eps: float = 1e-5
    rope_theta: float = 500000.0
    rope_scaling: dict | None = None
    max_position_embeddings: int = 8192
    tie_word_embeddings: bool = False
    # MoE
    num_experts: int = 0
    num_experts_per_tok: int = 0
    # special tokens (Llama-3 family ids; Mixtral uses its own)
    bos_token_id: int = 128000
    eos_token_ids: list[int] = field(default_factory=lambda: [128001, 128008, 128009])

    @property
    def q_size(self) -> int:
        return self.num_heads * self.head_dim

    @property
    def kv_size(self) -> int:
        return self.num_kv_heads * self.head_dim

    def num_params(self) -> int:
        d, f, L, V = self.hidden_size, self.intermediate_size, self.num_layers, self.vocab_size
        attn = d * (self.q_size + 2 * self.kv_size) + self.q_size * d
        if self.num_experts:
            mlp = self.num_experts * 3 * d * f + d * self.num_experts
        else:
            mlp = 3 * d * f
        emb = V * d * (1 if self.tie_word_embeddings else 2)
        return L * (attn + mlp + 2 * d) + emb + d

    def kv_bytes_per_token(self, dtype_bytes: int = 2) -> int:
        return 2 * self.num_layers * self.kv_size * dtype_bytes

    def to_json(self) -> str:
        return json.dumps(asdict(self))

    @staticmethod
    def from_hf(path: str | Path) -> "ModelConfig":
        """Build from a HF ``config.json`` (for loading real safetensors checkpoints when available)."""
        c = json.loads(Path(path).read_text())
        arch = "mixtral" if c.get("num_local_experts") else "llama"
        eos = c.get("eos_token_id", 2)
        return ModelConfig(
            name=c.get("_name_or_path", Path(path).parent.name), arch=arch, hidden_size=c["hidden_size"],
            intermediate_size=c["intermediate_size"], num_layers=c["num_hidden_layers"],
            num_heads=c["num_attention_heads"], num_kv_heads=c.get("num_key_value_heads", c["num_attention_heads"]),
            head_dim=c.get("head_dim", c["hidden_size"] // c["num_attention_heads"]), vocab_size=c["vocab_size"],
            rms_norm_eps=c.get("rms_norm_eps", 1e-5), rope_theta=c.get("rope_theta", 10000.0),
            rope_scaling=c.get("rope_scaling"), max_position_embeddings=c.get("max_position_embeddings", 8192),
            tie_word_embeddings=c.get("tie_word_embeddings", False), num_experts=c.get("num_local_experts", 0),
            num_experts_per_tok=c.get("num_experts_per_tok", 0), bos_token_id=c.get("bos_token_id", 1),
            eos_token_ids=eos if isinstance(eos, list) else [eos])


LLAMA31_SCALING = {"rope_type": "llama3", "factor": 8.0, "low_freq_factor": 1.0, "high_freq_factor": 4.0,
                   "original_max_position_embeddings": 8192}

PRESETS: dict[str, ModelConfig] = {
    # Llama-3-8B shapes with Llama-3.1 RoPE scaling: the ~18k-token Kafka prompt exceeds 8k.
    "llama3-8b": ModelConfig(name="llama3-8b", rope_scaling=LLAMA31_SCALING, max_position_embeddings=131072),
    "llama3-8b-8k": ModelConfig(name="llama3-8b-8k"),
    "llama3-70b": ModelConfig(name="llama3-70b", hidden_size=8192, intermediate_size=28672, num_layers=80,
                              num_heads=64, num_kv_heads=8, rope_scaling=LLAMA31_SCALING,
                              max_position_embeddings=131072),
    "mixtral-8x7b": ModelConfig(name="mixtral-8x7b", arch="mixtral", vocab_size=32000, rope_theta=1e6,
                                max_position_embeddings=32768, num_experts=8, num_experts_per_tok=2,
                                bos_token_id=1, eos_token_ids=[2]),
    # small configs with the same head geometry (head_dim 128, GQA) for tests and smoke runs
    "tiny-llama": ModelConfig(name="tiny-llama", hidden_size=512, intermediate_size=1024, num_layers=2,
                              num_heads=8, num_kv_heads=2, vocab_size=128256, max_position_embeddings=131072,
                              rope_scaling=LLAMA31_SCALING),
    "tiny-mixtral": ModelConfig(name="tiny-mixtral", arch="mixtral", hidden_size=512, intermediate_size=512,
                                num_layers=2, num_heads=8, num_kv_heads=2, vocab_size=32000, rope_theta=1e6,
                                max_position_embeddings=32768, num_experts=4, num_experts_per_tok=2,
                                bos_token_id=1, eos_token_ids=[2]),
    "small-llama": ModelConfig(name="small-llama", hidden_size=1024, intermediate_size=3584, num_layers=4,
                               num_heads=16, num_kv_heads=4, max_position_embeddings=131072,
                               rope_scaling=LLAMA31_SCALING),
}


def get_config(name: str) -> ModelConfig:
    if name in PRESETS:
        return PRESETS[name]
    p = Path(name)
    if p.is_dir() and (p / "config.json").exists():
        return ModelConfig.from_hf(p / "config.json")
    if p.suffix == ".json" and p.exists():
        return ModelConfig.from_hf(p)
    raise KeyError(f"unknown model {name!r}; presets: {sorted(PRESETS)}")
