"""Model definitions (Llama-3 / Mixtral / GPT-2) and architecture presets."""
from .config import PRESETS, ModelConfig, get_config  # noqa: F401
from .llama import AttnMeta, CausalLM  # noqa: F401
from .checkpoint import config_from_hf, load_checkpoint, save_checkpoint  # noqa: F401
