# llmtrain (MI355X) developer targets
PY ?= python
NPROC ?= 8
GPURUN ?= /usr/local/graft/bin/gpurun

.PHONY: build test test-gpu bench bench-module profile parity train-smoke train-ddp train-gpt2 train-gpt2-ddp8 \
        generate mlflow format k8s-build k8s-train k8s-logs k8s-clean k8s-e2e k8s-e2e-cpu k8s-train-resilient lint \
        k8s-kind-cluster k8s-kind-delete k8s-kind-smoke k8s-mlflow \
        k8s-cluster k8s-cluster-delete k8s-full k8s-kind-load train-gpt-ddp \
        k8s-dashboard k8s-dashboard-token k8s-dashboard-proxy k8s-dashboard-delete

build:                 ## compile every HIP kernel for gfx950 into llmtrain/ops/_llmtrain_hip.so
	$(PY) -m llmtrain.ops.build

lint:                  ## ruff + mypy when installed, plus the built-in checker (scripts/lint.py)
	$(PY) scripts/lint.py

format:                ## ruff format (when installed)
	$(PY) -m ruff format llmtrain tests bench scripts examples bench.py __graft_entry__.py

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

parity: build          ## val-loss parity: fused engine vs torch bf16 vs fp32 oracle (one GPU)
	$(PY) bench/parity.py --steps 300

generate:              ## sample from the newest checkpoint of a run: make generate RUN=<run_id> PROMPT="..."
	$(PY) -m llmtrain generate --config $(or $(CONFIG),configs/presets/gpt2_124m_mi355x.yaml) \
	  --checkpoint $(RUN) --prompt "$(or $(PROMPT),Hello)" --top-next 5

mlflow:                ## MLflow UI over the local SQLite store
	mlflow ui --backend-store-uri sqlite:///./mlflow.db

train-smoke:
	$(PY) -m llmtrain train --config configs/presets/gpt_smoke.yaml

train-ddp:             ## reference DDP smoke: 2 CPU ranks over gloo
	$(PY) -m torch.distributed.run --nproc_per_node=2 --master-addr 127.0.0.1 -m llmtrain train --config configs/presets/ddp_smoke.yaml

train-gpt-ddp:         ## reference target name: 2 CPU ranks over gloo on the wikitext DDP preset
	$(PY) -m torch.distributed.run --nproc_per_node=2 --master-addr 127.0.0.1 -m llmtrain train --config configs/presets/gpt_wikitext_ddp.yaml

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

k8s-train-resilient:   ## the Job under the gang-restart controller (fail fast, restart all ranks, resume)
	kubectl apply -f k8s/rbac.yaml -f k8s/storage.yaml -f k8s/configmap.yaml -f k8s/service.yaml
	bash k8s/gang_restart.sh --job k8s/job.yaml --max-restarts 3

k8s-e2e-cpu:           ## kind: create/reuse cluster, build+load image, 2-pod gloo Job with one injected crash
	bash k8s/test_e2e.sh --cpu --inject-failure

# ---- local kind cluster: CPU smoke of the same IndexedJob plumbing (gloo, 2 pods) -------------
DASHBOARD_URL ?= https://raw.githubusercontent.com/kubernetes/dashboard/v2.7.0/aio/deploy/recommended.yaml

k8s-kind-cluster:
	mkdir -p runs mlflow-k8s
	kind create cluster --name llmtrain --config k8s/kind/kind-config.yaml

k8s-kind-delete:
	kind delete cluster --name llmtrain

# reference target names (Makefile:30-51 of the reference): kind cluster, then the GPU Job
k8s-cluster: k8s-kind-cluster

k8s-cluster-delete: k8s-kind-delete

k8s-kind-load: k8s-build
	kind load docker-image llmtrain-mi355x:dev --name llmtrain

# kind has no AMD GPU device plugin: the reference-named end-to-end target runs the CPU Job on kind
# (k8s/kind/*), exactly like the reference's CPU-only k8s-full; the GPU Job (k8s-train) needs a
# cluster with the AMD device plugin and MI355X nodes
k8s-full: k8s-cluster k8s-kind-smoke k8s-logs

k8s-kind-smoke: k8s-build
	kind load docker-image llmtrain-mi355x:dev --name llmtrain
	kubectl apply -f k8s/rbac.yaml -f k8s/kind/storage-kind.yaml -f k8s/kind/configmap-cpu.yaml -f k8s/service.yaml -f k8s/kind/job-cpu.yaml
	kubectl wait --for=condition=complete --timeout=600s job/llmtrain

k8s-mlflow:
	mlflow ui --backend-store-uri sqlite:///mlflow-k8s/mlflow.db

k8s-dashboard:
	kubectl apply -f $(DASHBOARD_URL)
	kubectl apply -f k8s/dashboard-admin.yaml
	@$(MAKE) --no-print-directory k8s-dashboard-token
	@echo "then: make k8s-dashboard-proxy and open http://localhost:8001/api/v1/namespaces/kubernetes-dashboard/services/https:kubernetes-dashboard:/proxy/"

k8s-dashboard-token:
	@kubectl -n kubernetes-dashboard create token llmtrain-dashboard-admin

k8s-dashboard-proxy:
	kubectl proxy

k8s-dashboard-delete:
	kubectl delete -f k8s/dashboard-admin.yaml --ignore-not-found
	kubectl delete -f $(DASHBOARD_URL) --ignore-not-found
