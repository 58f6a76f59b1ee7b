"""Diagnostic LLM layer: prompt construction, analysis service, synthetic workloads."""
