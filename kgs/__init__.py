"""kgs -- an MI355X-native kind GPU provisioner.

Capabilities of ``maryamtahhan/kind-gpu-sim`` (create/delete/load a kind
cluster whose workers carry ``amd.com/gpu``), rebuilt MI355X-first: real
``/dev/kfd`` + ``/dev/dri`` passthrough, a from-scratch kubelet device plugin,
and an in-pod PyTorch-ROCm workload whose hot path is a hand-written gfx950 bf16
MFMA GEMM plus an RCCL all-reduce over xGMI.

Subpackages:
  kgs.cli / kgs.cluster...  orchestration (the reference's kind-gpu-sim.sh)
  kgs.deviceplugin          kubelet v1beta1 gRPC device plugin
  kgs.gpuinfo               native GPU/xGMI enumeration core (C++)
  kgs.ops                   HIP kernels (GEMM, vector add, ...)
  kgs.parallel              RCCL collectives via torch.distributed
  kgs.models                the in-pod workload models (GEMM step, MLP)
  kgs.workload              the rocm-gpu-test pod entrypoint
"""

__version__ = "0.1.0"
