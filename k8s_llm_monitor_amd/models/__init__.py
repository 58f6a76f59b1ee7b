"""Model definitions (Llama-3 / Mixtral / GPT-2) and architecture presets."""
from .config import PRESETS, ModelConfig, get_config  # noqa: F401
from .llama import AttnMeta, CausalLM  # noqa: F401
