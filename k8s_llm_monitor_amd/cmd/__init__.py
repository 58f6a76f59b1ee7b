"""Process entry points mirroring the reference's binaries (``cmd/*``):
``server``, ``scheduler``, ``uav_agent``, ``test_k8s`` and ``demos``."""
