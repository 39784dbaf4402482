"""Distributed runtime for the in-pod workload: one process per GPU, RCCL over xGMI.

* :mod:`kgs.parallel.dist` -- process-group bootstrap from torchrun env (RCCL on
  GPUs, gloo on CPU for tests), barrier / max-over-ranks helpers.
* :mod:`kgs.parallel.allreduce` -- all-reduce bandwidth sweep (algbw/busbw) and
  the bucketed, backward-overlapped gradient all-reduce used for data parallel.
* :mod:`kgs.parallel.p2p_allreduce` -- one-kernel P2P all-reduce over IPC-mapped
  xGMI peers (small/medium messages; hipGraph-capturable).
* :mod:`kgs.parallel.tensor_parallel` -- column/row-parallel Linear and the TP
  MLP, whose row-parallel reduction runs on the P2P all-reduce.
"""
