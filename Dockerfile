# polykey (MI355X-native) server image.  Base: ROCm 7.x + PyTorch-ROCm (no CUDA anywhere).
#   docker build -t polykey-amd .
#   docker run --device=/dev/kfd --device=/dev/dri --group-add video --shm-size 16g -p 50051:50051 polykey-amd
ARG BASE=rocm/pytorch:latest
FROM ${BASE} AS build
WORKDIR /app
COPY . /app
ENV PYTORCH_ROCM_ARCH=gfx950
RUN python3 -m polykey_service_amd._native.build -j 8

FROM build AS test
CMD ["python3", "-m", "pytest", "tests", "-q", "-m", "not gpu"]

FROM build AS server
RUN useradd -m appuser && chown -R appuser /app
USER appuser
ENV LISTEN_ADDR=:50051 POLYKEY_BACKEND=mock HSA_ENABLE_IPC_MODE_LEGACY=0
EXPOSE 50051 8000 9100
HEALTHCHECK --interval=10s --timeout=5s --start-period=20s --retries=3 \
  CMD ["python3", "-m", "polykey_service_amd.client.health_probe", "-addr=:50051"]
ENTRYPOINT ["python3", "-m", "polykey_service_amd.server"]
