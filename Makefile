# polykey (MI355X-native) — developer targets, mirroring the reference's Makefile
# (build / run-server / run-test-client / test / test-integration / compose-*) plus the
# GPU-side targets (kernels, gpu tests, bench, profiling).
.DEFAULT_GOAL := help
PY        ?= python3
SERVER_ADDR ?= localhost:50051
PORT      ?= 50051

.PHONY: help build clean run-server run-llm-server run-test-client test test-gpu test-dist test-integration test-integration-local health \
        bench bench-gpu8 prof compose-up compose-down compose-logs lint ci-check kill-local-server

help: ## show targets
	@grep -E '^[a-zA-Z0-9_-]+:.*## ' $(MAKEFILE_LIST) | awk -F':.*## ' '{printf "  \033[36m%-18s\033[0m %s\n", $$1, $$2}'

build: ## compile HIP kernels (gfx950), comm lib and C++ runtime/crypto extensions in-tree
	PYTORCH_ROCM_ARCH=gfx950 $(PY) -m polykey_service_amd._native.build -j 8

clean: ## remove native build artefacts
	$(PY) -m polykey_service_amd._native.build --clean

run-server: build ## run the gRPC server with the mock backend (reference behaviour)
	LISTEN_ADDR=:$(PORT) $(PY) -m polykey_service_amd.server

run-llm-server: build ## run the gRPC + OpenAI server with the on-node Llama-3-8B backend (random init)
	LISTEN_ADDR=:$(PORT) POLYKEY_BACKEND=local POLYKEY_HTTP_ADDR=:8000 POLYKEY_METRICS_ADDR=:9100 \
	  $(PY) -m polykey_service_amd.server

run-llm-server-tp8: build ## 70B TP=8 server (one process per GPU over RCCL; rank 0 serves)
	$(PY) -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 -m polykey_service_amd.server \
	  -backend local -model llama3-70b -tp 8 -http-addr :8000

run-test-client: ## dev client against $(SERVER_ADDR) with the Jest-style report
	POLYKEY_SERVER_ADDR=$(SERVER_ADDR) $(PY) -m polykey_service_amd.client

test: build ## CPU test suite (unit + integration + gloo multi-process) with a Jest-style summary
	$(PY) -m pytest tests -q -m "not gpu" -p polykey_service_amd.report.pytest_plugin --jest-json=.jest.jsonl; \
	  rc=$$?; $(PY) -m polykey_service_amd.report jest < .jest.jsonl; exit $$rc

test-gpu: build ## kernel numerics + GPU engine tests (needs an MI355X)
	$(PY) -m pytest tests -q -m gpu

test-dist: ## multi-process TP/EP/SP/DP-EP tests on gloo (CPU, 2/4/8 ranks)
	$(PY) -m pytest tests/parallel -q

test-integration-local: build ## in-process server + dev client, health, reflection, LLM tools
	$(PY) -m pytest tests/integration -q

test-integration: compose-up ## container flow: compose up -> wait healthy -> remote tests + dev client -> down
	@echo "waiting for polykey-server to become healthy"
	@until [ "$$(docker inspect -f {{.State.Health.Status}} $$(docker compose -f compose.yml ps -q polykey-server))" = "healthy" ]; do \
		sleep 1; \
	done
	POLYKEY_SERVER_ADDR=$(SERVER_ADDR) $(PY) -m pytest tests/integration/test_remote_server.py -q; \
	  rc=$$?; $(MAKE) run-test-client || rc=1; $(MAKE) compose-down; exit $$rc

health: ## gRPC health probe of $(SERVER_ADDR) (grpc_health_probe contract)
	$(PY) -m polykey_service_amd.client.health_probe -addr=$(SERVER_ADDR)

bench: build ## headline benchmark on 1 GPU (output tokens/s via gRPC, Llama-3-8B)
	$(PY) bench.py --gpus 1

bench-gpu8: build ## 1/2/4/8-GPU weak-scaling curve
	for n in 1 2 4 8; do $(PY) bench.py --gpus $$n --steps 3 --warmup 1; done

prof: build ## rocprofv3 kernel trace + stats of a short bench run into gpurun_out/prof
	cd /tmp && TMPDIR=/tmp rocprofv3 --kernel-trace --stats --output-format csv -d $(CURDIR)/gpurun_out/prof -o run \
	  -- $(PY) $(CURDIR)/bench.py --steps 1 --warmup 1

compose-up: ## docker compose up (server image)
	docker compose -f compose.yml up -d --build

compose-down: ## docker compose down
	docker compose -f compose.yml down

compose-logs: ## follow server logs through the Jest-style beautifier
	docker compose -f compose.yml logs -f | $(PY) -m polykey_service_amd.report

kill-local-server: ## kill whatever listens on $(PORT)
	@pid=$$(lsof -t -i :$(PORT) 2>/dev/null); if [ -n "$$pid" ]; then kill $$pid; fi

test-race: ## native cores under ASan/UBSan + concurrency stress (the reference's go test -race)
	$(PY) -m pytest tests/unit/test_native_sanitizers.py tests/integration -q -k "sanitizer or concurrent or cancel"

security-scan: ## Trivy filesystem + image scan (CRITICAL/HIGH fail), if trivy is installed
	@if command -v trivy >/dev/null 2>&1; then \
	  trivy fs --severity CRITICAL,HIGH --exit-code 1 . && \
	  trivy image --severity CRITICAL,HIGH --exit-code 1 polykey-amd:latest; \
	else echo "trivy not installed (no network in this image); CI runs the scan"; fi

sbom: ## SPDX SBOM of the server image (trivy), if available
	@if command -v trivy >/dev/null 2>&1; then trivy image --format spdx-json -o sbom.spdx.json polykey-amd:latest; \
	else echo "trivy not installed"; fi

docker-build: ## build the server image (ROCm base)
	docker build --target server -t polykey-amd:latest .

install-deps: ## verify the offline Python dependencies this repo needs are importable
	$(PY) -c "import grpc, google.protobuf, fastapi, uvicorn, prometheus_client, safetensors, tokenizers, pybind11; print('ok')"

ci-check: build test ## what CI runs on a CPU runner

lint: ## ruff (as in CI) when installed, else a byte-compile pass over every Python file
	@if command -v ruff >/dev/null 2>&1; then \
	  ruff check --select E9,F,I --line-length 120 polykey_service_amd tests bench.py __graft_entry__.py tools; \
	else $(PY) -m compileall -q polykey_service_amd tests tools bench.py __graft_entry__.py && echo "compile ok"; fi
