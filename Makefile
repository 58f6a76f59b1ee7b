# Build / test / run targets (the reference's Makefile equivalents).
PY ?= python
CONFIG ?= ./configs/config.yaml

.PHONY: build native test test-gpu run dev scheduler agent bench smoke docker lint clean

build native:
	$(PY) -c "import __graft_entry__ as g; g.build()"

test:
	$(PY) -m pytest tests/ -x -q -m "not gpu"

test-gpu:
	$(PY) -m pytest tests/ -x -q -m gpu

run: build
	$(PY) -m k8s_llm_monitor_amd.cmd.server -config $(CONFIG)

dev:
	$(PY) -m k8s_llm_monitor_amd.cmd.server -config ./configs/config.dev.yaml

scheduler:
	$(PY) -m k8s_llm_monitor_amd.cmd.scheduler -config $(CONFIG) -interval 15s

agent:
	$(PY) -m k8s_llm_monitor_amd.cmd.uav_agent -port 9090

bench: build
	$(PY) bench.py --gpus 1 --steps 3 --warmup 1

smoke: build
	$(PY) -c "import __graft_entry__ as g; g.smoke()"

docker:
	docker build -t k8s-llm-monitor-amd:dev .

lint:
	$(PY) -m pyflakes k8s_llm_monitor_amd tests || true

clean:
	rm -rf build k8s_llm_monitor_amd/ops/*.so k8s_llm_monitor_amd/runtime/*.so
