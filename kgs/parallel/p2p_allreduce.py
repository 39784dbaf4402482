"""Peer-to-peer all-reduce over xGMI, the small/medium
message path next to RCCL.

A :class:`P2PAllReduce` is created collectively by every rank of a group (one
process per GPU). Each rank allocates an IPC-shareable staging buffer and an
uncached signal block outside torch's caching allocator, the ranks swap IPC
handles over the (gloo or RCCL) process group, and every rank maps every
peer's buffers. :meth:`all_reduce` is then ONE kernel launch on the current
stream -- no host round trip, no RCCL proxy thread -- which makes it the
latency path for tensor-parallel activations (the vLLM custom all-reduce that
the reference disables on its CPU pod, /root/reference/pods/vllm-cpu-pod.yaml:19).

Algorithms (native/kernels/allreduce_p2p.hip):

* ``oneshot`` -- every rank reads all N staging buffers and sums: N-1 remote
  reads of the whole message, each over its own xGMI link. Lowest latency.
* ``twoshot`` -- reduce-scatter into the staging buffers, then all-gather:
  2(N-1)/N of the message per rank. Wins once the message is bandwidth-bound.

Every call is one kernel whose barrier epoch lives on the device (a per-block
counter in the rank's signal block), so calls can be captured in a hipGraph
(``torch.cuda.CUDAGraph``) and replayed: a TP layer's GEMM + all-reduce chain
becomes one graph launch.

``algo="auto"`` picks one-shot up to :attr:`oneshot_max_bytes` (256 KiB at
8 ranks, 1 MiB at <= 4), two-shot above, and RCCL (``dist.all_reduce``) beyond
``max_bytes`` or for unsupported dtypes/shapes -- results are then identical in
meaning, only the transport differs.

:meth:`local_ranks` builds N "ranks" inside ONE process on one GPU: N staging
buffers and ONE launch of N x blocks workgroups in which workgroup r*blocks+b
plays block b of rank r. The flag protocol and the kernels are the ones that run
across GPUs, all workgroups are co-resident, and no IPC is involved -- the
single-GPU test path.
"""
from __future__ import annotations

import ctypes
import math

import torch

from ..ops import _lib

THREADS = 512
_DTYPES = {torch.float32: 0, torch.bfloat16: 1}


def _lib_checked():
    so = _lib.lib()
    if not hasattr(so, "kgs_ar_run"):
        raise _lib.NativeUnavailable("libkgs_kernels.so predates the P2P all-reduce: rebuild (python -m kgs.utils.build)")
    return so


def _alloc(nbytes: int, uncached: bool) -> int:
    ptr = ctypes.c_void_p()
    _lib.check(_lib_checked().kgs_ar_alloc(nbytes, int(uncached), ctypes.byref(ptr)), "kgs_ar_alloc")
    return int(ptr.value)


class P2PAllReduce:
    """One-kernel all-reduce across the GPUs of a process group (<= 8 ranks)."""

    def __init__(self, group=None, max_bytes: int = 8 << 20, device=None, timeout_s: float = 10.0,
                 oneshot_max_bytes: int | None = None, _local_world: int | None = None,
                 staging_uncached: bool = True):
        """``staging_uncached``: the staging (data) buffers from uncached device
        memory, like the signal blocks (round 6 default). The flag protocol also
        writes L2 back before a flag and invalidates after a poll
        (allreduce_p2p.hip block_barrier, pinned by tests/test_kernel_resources.py),
        but with uncached staging no peer's data ever waits in an L2. The
        single-GPU A/B (bench/p2p_staging_ab.py, profiles/r6/p2p/README.md): equal
        or faster in 16 of 18 cells, 0.79-0.90x the time at 4 MiB, at most
        1.04x; and the one wrong result ever seen in local-rank runs came from a
        cached-staging instance."""
        so = _lib_checked()
        self.max_bytes = int(max_bytes)
        if self.max_bytes <= 0 or self.max_bytes % 16:
            raise ValueError("max_bytes must be a positive multiple of 16")
        self.timeout_s = float(timeout_s)
        self.group = group
        dev = torch.device(device) if device is not None else torch.device("cuda")
        self.device = dev if dev.index is not None else torch.device("cuda", torch.cuda.current_device())
        self.max_blocks = so.kgs_ar_max_blocks()
        self._closed = False
        self._owned: list[int] = []   # allocations to hipFree
        self._opened: list[int] = []  # peer mappings to hipIpcCloseMemHandle
        sig_bytes = so.kgs_ar_signal_bytes()
        with torch.cuda.device(self.device):
            if _local_world is not None:
                # N ranks in one process: all buffers local, one stream per rank
                self.world, self.rank = int(_local_world), 0
                self.data = [_alloc(self.max_bytes, staging_uncached) for _ in range(self.world)]
                self.sigs = [_alloc(sig_bytes, True) for _ in range(self.world)]
                self._owned += self.data + self.sigs
                self.local = True
            else:
                import torch.distributed as dist

                self.world = dist.get_world_size(group)
                self.rank = dist.get_rank(group)
                my_data = _alloc(self.max_bytes, staging_uncached)
                my_sig = _alloc(sig_bytes, True)
                self._owned += [my_data, my_sig]
                hbytes = so.kgs_ar_ipc_handle_bytes()
                hd = ctypes.create_string_buffer(hbytes)
                hs = ctypes.create_string_buffer(hbytes)
                _lib.check(so.kgs_ar_ipc_handle(my_data, hd), "hipIpcGetMemHandle(data)")
                _lib.check(so.kgs_ar_ipc_handle(my_sig, hs), "hipIpcGetMemHandle(signal)")
                gathered: list = [None] * self.world
                dist.all_gather_object(gathered, (hd.raw, hs.raw), group=group)
                self.data, self.sigs = [], []
                for r, (hdr, hsr) in enumerate(gathered):
                    if r == self.rank:
                        self.data.append(my_data)
                        self.sigs.append(my_sig)
                        continue
                    self.data.append(self._open(hdr))
                    self.sigs.append(self._open(hsr))
                self.local = False
        if not 1 <= self.world <= so.kgs_ar_max_ranks():
            raise ValueError(f"P2P all-reduce supports 1..{so.kgs_ar_max_ranks()} ranks, got {self.world}")
        self.err = torch.zeros(1, dtype=torch.int32, device=self.device)
        self.oneshot_max_bytes = oneshot_max_bytes if oneshot_max_bytes is not None else (
            (1 << 20) if self.world <= 4 else (256 << 10))
        self._epoch = 0
        n = self.world
        self._data_arr = (ctypes.c_void_p * n)(*self.data)
        self._sig_arr = (ctypes.c_void_p * n)(*self.sigs)

    @classmethod
    def local_ranks(cls, world: int, max_bytes: int = 8 << 20, device=None, timeout_s: float = 10.0, **kw):
        """``world`` ranks inside this process (one GPU, one launch plays them all)."""
        return cls(group=None, max_bytes=max_bytes, device=device, timeout_s=timeout_s, _local_world=world, **kw)

    def _open(self, handle: bytes) -> int:
        ptr = ctypes.c_void_p()
        _lib.check(_lib_checked().kgs_ar_ipc_open(handle, ctypes.byref(ptr)), "hipIpcOpenMemHandle")
        self._opened.append(int(ptr.value))
        return int(ptr.value)

    # ------------------------------------------------------------------ API --
    def supports(self, t: torch.Tensor) -> bool:
        nbytes = t.numel() * t.element_size()
        return (t.dtype in _DTYPES and t.is_contiguous() and t.device == self.device and 0 < nbytes <= self.max_bytes
                and nbytes % 16 == 0 and t.data_ptr() % 16 == 0)

    def pick_algo(self, nbytes: int) -> str:
        return "oneshot" if nbytes <= self.oneshot_max_bytes or self.world <= 2 else "twoshot"

    def blocks_for(self, nbytes: int, algo: str) -> int:
        nvec = nbytes // 16
        per_block = THREADS * (1 if algo == "oneshot" else 2)
        cap = self.max_blocks
        if getattr(self, "local", False):
            cap = min(cap, max(1, 256 // self.world))  # one launch of world x blocks must be co-resident
        return max(1, min(cap, math.ceil(nvec / per_block)))

    def _next_epoch(self) -> int:
        """Host-side call numbers (diagnostics only; the API uses the device
        counters -- never mix the two on one instance). Flags start at 0, so
        epoch 0 is never used; the uint32 wrap skips it too."""
        self._epoch = self._epoch % 0xFFFFFFFF + 1
        return self._epoch

    def _run(self, rank: int, inp, out, nbytes: int, dtype, algo: str, epoch: int, stream) -> None:
        if algo not in ("oneshot", "twoshot"):
            raise ValueError(f"unknown algo {algo!r}")
        rc = _lib_checked().kgs_ar_run(
            self._data_arr, self._sig_arr, self.world, rank, inp, out, nbytes, self.max_bytes, _DTYPES[dtype],
            0 if algo == "oneshot" else 1, epoch, self.blocks_for(nbytes, algo), self.timeout_s, self.err.data_ptr(),
            stream)
        _lib.check(rc, f"p2p all_reduce[{algo}, {nbytes} B, rank {rank}/{self.world}]")

    def _launch(self, rank: int, inp: torch.Tensor, out: torch.Tensor, algo: str, epoch: int, stream) -> None:
        self._run(rank, inp.data_ptr(), out.data_ptr(), inp.numel() * inp.element_size(), inp.dtype, algo, epoch,
                  stream)

    def all_reduce(self, t: torch.Tensor, out: torch.Tensor | None = None, algo: str = "auto") -> torch.Tensor:
        """Sum ``t`` over the group. Returns ``out`` (a new tensor unless given;
        ``out=t`` is allowed). Falls back to RCCL when the tensor does not fit."""
        if self._closed:
            raise RuntimeError("P2PAllReduce is closed")
        if self.local:
            raise RuntimeError("local_ranks instance: use all_reduce_local")
        if not self.supports(t):
            import torch.distributed as dist

            res = t.clone() if out is None else out.copy_(t)
            dist.all_reduce(res, group=self.group)
            return res
        nbytes = t.numel() * t.element_size()
        algo = self.pick_algo(nbytes) if algo == "auto" else algo
        out = torch.empty_like(t) if out is None else out
        # epoch 0: the kernel keeps the call count on the device, so the call
        # can be captured in a hipGraph (torch.cuda.CUDAGraph) and replayed
        self._launch(self.rank, t, out, algo, 0, _lib.stream_handle(self.device))
        return out

    def all_reduce_local(self, inputs: list, algo: str = "auto", outs: list | None = None) -> list:
        """local_ranks instances: reduce ``inputs[r]`` (rank r's tensor) with one
        launch on the current stream; returns the N outputs (``outs`` if given)."""
        if not self.local:
            raise RuntimeError("not a local_ranks instance")
        if len(inputs) != self.world:
            raise ValueError(f"need {self.world} inputs")
        t0 = inputs[0]
        if not all(self.supports(x) and x.shape == t0.shape and x.dtype == t0.dtype for x in inputs):
            raise ValueError("inputs must be equal-shape contiguous f32/bf16 tensors on this device, 16-B sized")
        nbytes = t0.numel() * t0.element_size()
        algo = self.pick_algo(nbytes) if algo == "auto" else algo
        outs = [torch.empty_like(x) for x in inputs] if outs is None else outs
        ins = (ctypes.c_void_p * self.world)(*[x.data_ptr() for x in inputs])
        outp = (ctypes.c_void_p * self.world)(*[o.data_ptr() for o in outs])
        self._run(-1, ins, outp, nbytes, t0.dtype, algo, 0, _lib.stream_handle(self.device))
        return outs

    def check(self) -> None:
        """Synchronise and raise if any barrier timed out (a peer never arrived)."""
        v = int(self.err.item())
        if v:
            phases = [p for p in range(4) if v & (1 << p)]
            raise RuntimeError(f"P2P all-reduce barrier timed out on rank {self.rank} (phases {phases})")

    def close(self) -> None:
        if self._closed:
            return
        self._closed = True
        torch.cuda.synchronize(self.device)
        so = _lib_checked()
        for p in self._opened:
            so.kgs_ar_ipc_close(p)
        for p in self._owned:
            so.kgs_ar_free(p)
        self._opened, self._owned = [], []

    def __del__(self):  # pragma: no cover - best effort
        try:
            self.close()
        except Exception:
            pass


def latency_sweep(ar: P2PAllReduce, sizes=None, dtype=torch.bfloat16, iters: int = 50, warmup: int = 10,
                  compare_rccl: bool = True) -> list[dict]:
    """Per-size latency of the P2P path (and RCCL for comparison); run on every rank."""
    import time

    import torch.distributed as dist

    sizes = sizes or [1 << s for s in range(10, 24)]  # 1 KiB .. 8 MiB
    esz = torch.tensor([], dtype=dtype).element_size()
    rows = []
    for nbytes in sizes:
        if nbytes > ar.max_bytes:
            break
        x = torch.ones(nbytes // esz, dtype=dtype, device=ar.device)
        row = {"bytes": nbytes, "algo": ar.pick_algo(nbytes)}
        for name, fn in (("p2p", lambda: ar.all_reduce(x)), ("rccl", lambda: dist.all_reduce(x.clone()))):
            if name == "rccl" and not compare_rccl:
                continue
            for _ in range(warmup):
                fn()
            torch.cuda.synchronize(ar.device)
            dist.barrier(group=ar.group)
            t0 = time.perf_counter()
            for _ in range(iters):
                y = fn()
            torch.cuda.synchronize(ar.device)
            dt = (time.perf_counter() - t0) / iters
            row[f"{name}_us"] = round(dt * 1e6, 2)
            if name == "p2p":
                row["p2p_correct"] = bool(torch.all(y == float(ar.world)).item())
        ar.check()
        rows.append(row)
    return rows


def main(argv=None) -> int:  # pragma: no cover - needs >= 2 GPUs
    """torchrun --nproc-per-node N -m kgs.parallel.p2p_allreduce [--max-mib 8]"""
    import argparse
    import json

    from . import dist as kdist

    ap = argparse.ArgumentParser(description="P2P (xGMI) all-reduce latency vs RCCL")
    ap.add_argument("--max-mib", type=int, default=8)
    ap.add_argument("--iters", type=int, default=50)
    a = ap.parse_args(argv)
    ctx = kdist.init_from_env()
    ar = P2PAllReduce(group=ctx.group, max_bytes=a.max_mib << 20, device=ctx.device)
    rows = latency_sweep(ar, iters=a.iters)
    if ctx.rank == 0:
        for r in rows:
            print(json.dumps({"world": ctx.world_size, **r}), flush=True)
    ar.close()
    kdist.shutdown(ctx)
    return 0


if __name__ == "__main__":  # pragma: no cover
    raise SystemExit(main())
