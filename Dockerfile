# polykey (MI355X-native) images.  ROCm 7.x + PyTorch-ROCm, no CUDA anywhere.
#   docker build --target server -t polykey-amd .      (slim runtime image, the one compose runs)
#   docker build --target test   -t polykey-amd-test . (full tree + toolchain: CPU test suite)
#   docker run --device=/dev/kfd --device=/dev/dri --group-add video --shm-size 16g -p 50051:50051 polykey-amd
#
# Stages mirror the reference's builder / tester / production / server split
# (/root/reference/Dockerfile:1-66): `build` compiles every HIP / C++ extension for gfx950 with the
# ROCm toolchain; `runtime` starts from a plain OS image, installs only the ROCm *runtime*
# libraries the extensions and PyTorch link against plus a PyTorch-ROCm wheel, and copies in the
# Python package with its built .so files -- no compilers, no sources under csrc/, no tests, no
# build objects; `server` is the runtime with the non-root user, health check and entry point.

ARG BUILD_BASE=rocm/pytorch:latest
ARG RUNTIME_BASE=ubuntu:22.04
ARG ROCM_APT=https://repo.radeon.com/rocm/apt/7.0
ARG TORCH_INDEX=https://download.pytorch.org/whl/rocm7.0

# ---------------------------------------------------------------- build: compile the extensions
FROM ${BUILD_BASE} AS build
WORKDIR /app
COPY . /app
ENV PYTORCH_ROCM_ARCH=gfx950
RUN python3 -m polykey_service_amd._native.build -j 8

# ---------------------------------------------------------------- test: full tree, CPU suite
FROM build AS test
CMD ["python3", "-m", "pytest", "tests", "-q", "-m", "not gpu"]

# ---------------------------------------------------------------- runtime: slim
FROM ${RUNTIME_BASE} AS runtime
ARG ROCM_APT
ARG TORCH_INDEX
ENV DEBIAN_FRONTEND=noninteractive
# ROCm runtime only: HIP runtime, hipBLASLt / rocBLAS (PyTorch GEMMs), RCCL; python; OpenSSL (AES-GCM)
RUN apt-get update && apt-get install -y --no-install-recommends ca-certificates curl gnupg python3 python3-pip \
        libssl3 libnuma1 \
    && curl -fsSL https://repo.radeon.com/rocm/rocm.gpg.key | gpg --dearmor -o /usr/share/keyrings/rocm.gpg \
    && echo "deb [signed-by=/usr/share/keyrings/rocm.gpg] ${ROCM_APT} jammy main" > /etc/apt/sources.list.d/rocm.list \
    && apt-get update && apt-get install -y --no-install-recommends rocm-hip-runtime hipblaslt rocblas rccl \
    && apt-get purge -y curl gnupg && apt-get autoremove -y && rm -rf /var/lib/apt/lists/*
RUN python3 -m pip install --no-cache-dir --index-url ${TORCH_INDEX} torch \
    && python3 -m pip install --no-cache-dir grpcio protobuf fastapi uvicorn prometheus_client msgpack numpy \
        safetensors tokenizers
WORKDIR /app
# the package with its compiled extensions (polykey_service_amd/_lib/*.so); nothing else
COPY --from=build /app/polykey_service_amd /app/polykey_service_amd
RUN find /app -name '__pycache__' -prune -exec rm -rf {} + && find /app -name '*.stamp' -delete
ENV PYTHONPATH=/app HSA_ENABLE_IPC_MODE_LEGACY=0

# ---------------------------------------------------------------- server: non-root entry point
FROM runtime AS server
RUN useradd -m -u 10001 appuser
USER appuser
ENV LISTEN_ADDR=:50051 POLYKEY_BACKEND=mock
EXPOSE 50051 8000 9100
HEALTHCHECK --interval=10s --timeout=5s --start-period=20s --retries=3 \
  CMD ["python3", "-m", "polykey_service_amd.client.health_probe", "-addr=:50051"]
ENTRYPOINT ["python3", "-m", "polykey_service_amd.server"]
