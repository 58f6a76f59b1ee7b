"""``config.yaml`` loader with the reference's schema, defaults and env semantics
(``internal/config/config.go:12-182``).

Order of precedence, as viper applies it: defaults < YAML file < environment.  Every key can be
overridden by its upper-cased, ``_``-joined path (``SERVER_PORT=8081``, ``METRICS_NAMESPACES=a,b``)
and ``OPENAI_API_KEY`` / ``OPENAI_BASE_URL`` map to ``llm.api_key`` / ``llm.base_url``.  Unknown
keys are ignored.  A missing file is an error, like ``viper.ReadInConfig``.

New engine knobs live under ``llm`` next to the reference's keys: ``provider: local-rocm`` selects
the in-process MI355X engine (``openai`` keeps the reference's remote semantics: no local model),
plus ``tp_size``, ``dp_replicas``, ``max_batch``, ``kv_cache_gb``, ``max_model_len``, ``dtype``,
``seed``, ``use_graphs``.
"""
from __future__ import annotations

import dataclasses
import os
from dataclasses import dataclass, field
from typing import Any, Optional

import yaml


@dataclass
class ServerConfig:
    host: str = "0.0.0.0"
    port: int = 8080
    debug: bool = False


@dataclass
class K8sConfig:
    kubeconfig: str = ""
    namespace: str = "default"
    watch_namespaces: str = "default"  # CSV
    backend: str = "auto"  # new: auto | kube | fake | none


@dataclass
class LLMConfig:
    provider: str = "openai"
    api_key: str = ""
    base_url: str = ""
    model: str = "gpt-4"
    max_tokens: int = 2000
    temperature: float = 0.1
    timeout: int = 30
    # in-process engine (provider local-rocm)
    tp_size: int = 1
    dp_replicas: int = 1
    max_batch: int = 64
    kv_cache_gb: float = 32.0
    max_model_len: int = 8192
    dtype: str = "bf16"
    seed: int = 0
    use_graphs: bool = True
    top_p: float = 1.0
    top_k: int = 0
    max_prefill_tokens: int = 16384  # token budget of one prefill step
    chunked_prefill: bool = True  # longer prompts prefill in chunks of that budget
    prefix_caching: bool = True  # reuse the KV blocks of shared prompt prefixes
    weights: str = ""  # Hugging Face model dir (config.json + *.safetensors); "" = random init
    # analysis type -> OpenAI-compatible base URL of the deployment that serves it (e.g.
    # root_cause -> a Llama-3-70B TP=8 server's ".../v1"); unrouted types use this server's backend.
    # YAML mapping, or "type=url,type=url" from the environment (LLM_ROUTES)
    routes: dict = field(default_factory=dict)


@dataclass
class RedisConfig:
    addr: str = ""
    password: str = ""
    db: int = 0


@dataclass
class PostgresConfig:
    host: str = ""
    port: int = 0
    user: str = ""
    password: str = ""
    database: str = ""


@dataclass
class StorageConfig:
    type: str = "memory"
    redis: RedisConfig = field(default_factory=RedisConfig)
    postgres: PostgresConfig = field(default_factory=PostgresConfig)
    path: str = ""  # new: directory for type "file" (analysis records as JSON lines)


@dataclass
class MonitoringConfig:
    metrics_interval: int = 30
    event_retention: int = 168
    log_retention: int = 24


@dataclass
class MetricsConfig:
    enabled: bool = True
    collect_interval: int = 30
    namespaces: list = field(default_factory=lambda: ["default"])
    enable_node: bool = True
    enable_pod: bool = True
    enable_network: bool = False
    enable_custom: bool = False
    cache_retention: int = 300


@dataclass
class AnalysisConfig:
    enable_prediction: bool = True
    enable_auto_fix: bool = False
    max_context_events: int = 100
    prompt_token_budget: int = 6144  # new: cap on the cluster-context part of a prompt


@dataclass
class LoggingConfig:
    level: str = "info"
    format: str = "json"
    output: str = "stdout"


@dataclass
class Config:
    server: ServerConfig = field(default_factory=ServerConfig)
    k8s: K8sConfig = field(default_factory=K8sConfig)
    llm: LLMConfig = field(default_factory=LLMConfig)
    storage: StorageConfig = field(default_factory=StorageConfig)
    monitoring: MonitoringConfig = field(default_factory=MonitoringConfig)
    metrics: MetricsConfig = field(default_factory=MetricsConfig)
    analysis: AnalysisConfig = field(default_factory=AnalysisConfig)
    logging: LoggingConfig = field(default_factory=LoggingConfig)


class ConfigError(Exception):
    pass


def _coerce(value: Any, default: Any, key: str) -> Any:
    """mapstructure's weakly-typed decode: strings from env/YAML into the field's type."""
    try:
        if isinstance(default, bool):
            if isinstance(value, bool):
                return value
            if isinstance(value, (int, float)):
                return value != 0
            s = str(value).strip().lower()
            if s in ("1", "t", "true", "yes", "on"):
                return True
            if s in ("", "0", "f", "false", "no", "off"):
                return False
            raise ValueError(value)
        if isinstance(default, int):
            if isinstance(value, str):
                return int(float(value)) if value.strip() else 0
            return int(value)
        if isinstance(default, float):
            return float(value) if value != "" else 0.0
        if isinstance(default, list):
            if value is None:
                return []
            if isinstance(value, str):
                return [x.strip() for x in value.split(",") if x.strip()] if value else []
            return [str(x) for x in value]
        if isinstance(default, str):
            return "" if value is None else str(value)
        if isinstance(default, dict):
            if value is None or value == "":
                return {}
            if isinstance(value, str):
                pairs = [p.split("=", 1) for p in value.split(",") if p.strip()]
                if any(len(p) != 2 for p in pairs):
                    raise ValueError(value)
                return {k.strip(): v.strip() for k, v in pairs}
            if not isinstance(value, dict):
                raise ValueError(value)
            return {str(k): str(v) for k, v in value.items()}
    except (TypeError, ValueError) as e:
        raise ConfigError(f"failed to unmarshal config: key {key!r}: cannot decode {value!r}") from e
    return value


def _apply(obj: Any, data: dict, prefix: str) -> None:
    for f in dataclasses.fields(obj):
        key = f"{prefix}{f.name}"
        cur = getattr(obj, f.name)
        if dataclasses.is_dataclass(cur):
            sub = data.get(f.name) if isinstance(data, dict) else None
            _apply(cur, sub if isinstance(sub, dict) else {}, key + ".")
            continue
        if isinstance(data, dict) and f.name in data:
            setattr(obj, f.name, _coerce(data[f.name], cur, key))
        env = os.environ.get(key.upper().replace(".", "_"))
        if env is not None:
            setattr(obj, f.name, _coerce(env, cur, key))


def load(path: str) -> Config:
    """``config.Load`` (config.go:105-129)."""
    if not path or not os.path.isfile(path):
        raise ConfigError(f"failed to read config file: open {path}: no such file or directory")
    with open(path, "rb") as fh:
        try:
            data = yaml.safe_load(fh) or {}
        except yaml.YAMLError as e:
            raise ConfigError(f"failed to read config file: {e}") from e
    if not isinstance(data, dict):
        raise ConfigError("failed to read config file: top level must be a mapping")
    cfg = Config()
    _apply(cfg, data, "")
    # processEnvVars (config.go:172-182)
    if os.environ.get("OPENAI_API_KEY"):
        cfg.llm.api_key = os.environ["OPENAI_API_KEY"]
    if os.environ.get("OPENAI_BASE_URL"):
        cfg.llm.base_url = os.environ["OPENAI_BASE_URL"]
    return cfg


def from_dict(data: Optional[dict] = None) -> Config:
    cfg = Config()
    _apply(cfg, data or {}, "")
    return cfg


def parse_namespaces(csv: str) -> list[str]:
    """``parseNamespaces`` (client.go:80-100): CSV, trimmed, empty -> ["default"]."""
    out = [p.strip() for p in (csv or "").split(",") if p.strip()]
    return out or ["default"]


DEFAULT_YAML = """\
server:
  host: "0.0.0.0"
  port: 8080
  debug: false
k8s:
  kubeconfig: ""
  namespace: "default"
  watch_namespaces: "default,kube-system"
llm:
  provider: "local-rocm"
  model: "llama-3-8b"
  max_tokens: 2000
  temperature: 0.1
  timeout: 30
  tp_size: 1
  max_batch: 64
  kv_cache_gb: 32
storage:
  type: "memory"
monitoring:
  metrics_interval: 30
  event_retention: 168
  log_retention: 24
metrics:
  enabled: true
  collect_interval: 30
  namespaces: ["default", "kube-system"]
  enable_node: true
  enable_pod: true
  enable_network: true
  enable_custom: false
  cache_retention: 300
analysis:
  enable_prediction: true
  enable_auto_fix: false
  max_context_events: 100
logging:
  level: "info"
  format: "json"
  output: "stdout"
"""
