"""Native (C++) serving runtime: KV block allocator, BPE encoder, decode-batch packing.

Built in-tree by ``python -m k8s_llm_monitor_amd.ops.build --only runtime``; optional on CPU
(pure-Python equivalents exist), but ``__graft_entry__.build()`` requires it to load.
"""
from __future__ import annotations

import importlib

_RT = None
_TRIED = False


def native_runtime():
    """The ``_k8sllm_runtime`` module, or None if it is not built."""
    global _RT, _TRIED
    if not _TRIED:
        _TRIED = True
        try:
            _RT = importlib.import_module("k8s_llm_monitor_amd.runtime._k8sllm_runtime")
        except ImportError:
            _RT = None
    return _RT
