#!/bin/bash
# Environment for building and running on MI355X (gfx950) nodes, ROCm 7.x.
# Parity: ref config/g5k-module-load.sh, config/lumi-module-load.sh (module loads
# for CUDA 12 / HIP 5.2 / ROCm 6.0.3 + cray-mpich). Source it: `. scripts/env-mi355x.sh`.
export ROCM_PATH=${ROCM_PATH:-/opt/rocm}
export PATH=$ROCM_PATH/bin:$ROCM_PATH/llvm/bin:$PATH
export LD_LIBRARY_PATH=$ROCM_PATH/lib:${LD_LIBRARY_PATH:-}
export HIPCC=${HIPCC:-$ROCM_PATH/bin/hipcc}
export TTS_OFFLOAD_ARCH=${TTS_OFFLOAD_ARCH:-gfx950}
export PYTORCH_ROCM_ARCH=$TTS_OFFLOAD_ARCH
# dmabuf IPC only on this driver: required by RCCL / cross-process tensor sharing
export HSA_ENABLE_IPC_MODE_LEGACY=0
# one host thread drives each device; keep HIP's default of 4 hardware queues
export GPU_MAX_HW_QUEUES=${GPU_MAX_HW_QUEUES:-4}
# RCCL over xGMI within a node: small status records dominate (latency-bound);
# no IB/RoCE on a single node
export NCCL_IB_DISABLE=${NCCL_IB_DISABLE:-1}
export RCCL_MSCCL_ENABLE=${RCCL_MSCCL_ENABLE:-0}
export TORCH_NCCL_ASYNC_ERROR_HANDLING=${TORCH_NCCL_ASYNC_ERROR_HANDLING:-1}
# rendezvous on loopback for single-node runs
export MASTER_ADDR=${MASTER_ADDR:-127.0.0.1}
export OMP_NUM_THREADS=${OMP_NUM_THREADS:-16}
# optional failure detection (see csrc/core/runner.hpp, parallel/faults.py)
# export TTS_WATCHDOG_S=60 TTS_WATCHDOG_ABORT=1
echo "[env-mi355x] ROCm at $ROCM_PATH, arch $TTS_OFFLOAD_ARCH"
