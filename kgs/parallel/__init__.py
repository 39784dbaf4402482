"""Distributed runtime for the in-pod workload: one process per GPU, RCCL over xGMI.

* :mod:`kgs.parallel.dist` -- process-group bootstrap from torchrun env (RCCL on
  GPUs, gloo on CPU for tests), barrier / max-over-ranks helpers.
* :mod:`kgs.parallel.allreduce` -- all-reduce bandwidth sweep (algbw/busbw) and
  the bucketed, backward-overlapped gradient all-reduce used for data parallel.
"""
