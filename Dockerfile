# k8s-llm-monitor-amd image: ROCm PyTorch base + in-tree gfx950 kernels and C++ runtime.
# The same image runs the server (GPU), the scheduler controller and the UAV agent (CPU only).
ARG BASE=rocm/pytorch:latest
FROM ${BASE}
WORKDIR /app
ENV PYTORCH_ROCM_ARCH=gfx950 HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
COPY k8s_llm_monitor_amd ./k8s_llm_monitor_amd
COPY web ./web
COPY configs ./configs
COPY __graft_entry__.py bench.py ./
RUN python -c "import __graft_entry__ as g; g.build()"
EXPOSE 8081 9090
HEALTHCHECK --interval=30s --timeout=5s CMD python -c "import urllib.request;urllib.request.urlopen('http://127.0.0.1:8081/health',timeout=4)"
CMD ["python", "-m", "k8s_llm_monitor_amd.cmd.server", "-config", "/app/configs/config.yaml"]
