# llmtrain (MI355X) developer targets
PY ?= python
NPROC ?= 8
GPURUN ?= /usr/local/graft/bin/gpurun

.PHONY: build test test-gpu bench bench-module profile train-smoke train-ddp train-gpt2 train-gpt2-ddp8 \
        k8s-build k8s-train k8s-logs k8s-clean k8s-e2e lint

build:                 ## compile every HIP kernel for gfx950 into llmtrain/ops/_llmtrain_hip.so
	$(PY) -m llmtrain.ops.build

test:                  ## CPU test suite (contracts, fused engine on CPU, multi-process gloo DDP)
	$(PY) -m pytest tests -m "not gpu" -q

test-gpu: build        ## kernel numerics + fused engine on a MI355X
	$(PY) -m pytest tests -m gpu -q

bench: build           ## GPT-2 124M tokens/s on one GPU (see bench.py for N GPUs)
	$(PY) bench.py --gpus 1 --steps 20 --warmup 5

bench-module:          ## same benchmark through plain PyTorch (autocast + SDPA) for A/B
	$(PY) bench.py --gpus 1 --steps 20 --warmup 5 --path module

profile: build         ## rocprofv3 kernel trace + per-kernel stats of the bench
	bash scripts/profile.sh

train-smoke:
	$(PY) -m llmtrain train --config configs/presets/gpt_smoke.yaml

train-ddp:             ## reference DDP smoke: 2 CPU ranks over gloo
	$(PY) -m torch.distributed.run --nproc_per_node=2 --master-addr 127.0.0.1 -m llmtrain train --config configs/presets/ddp_smoke.yaml

train-gpt2: build
	$(PY) -m llmtrain train --config configs/presets/gpt2_124m_mi355x.yaml

train-gpt2-ddp8: build ## 8x MI355X, one rank per GPU over RCCL/xGMI
	$(PY) -m torch.distributed.run --standalone --local-addr 127.0.0.1 --nproc_per_node=$(NPROC) -m llmtrain train --config configs/presets/gpt2_124m_mi355x_ddp8.yaml

k8s-build:
	docker build -t llmtrain-mi355x:dev -f k8s/Dockerfile .

k8s-train:
	kubectl apply -f k8s/rbac.yaml -f k8s/storage.yaml -f k8s/configmap.yaml -f k8s/service.yaml -f k8s/job.yaml
	kubectl wait --for=condition=complete --timeout=1800s job/llmtrain

k8s-logs:
	kubectl logs -l app=llmtrain --all-containers --prefix

k8s-clean:
	kubectl delete -f k8s/job.yaml -f k8s/service.yaml -f k8s/configmap.yaml -f k8s/storage.yaml -f k8s/rbac.yaml --ignore-not-found

k8s-e2e:
	bash k8s/test_e2e.sh
