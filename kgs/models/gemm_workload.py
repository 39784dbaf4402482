"""The rocm-gpu-test pod's compute workload: bf16 MFMA GEMMs + RCCL gradient sync.

One :class:`GemmWorkload` per rank (one process per GPU). A step is
``gemms_per_step`` GEMMs ``C = A . B^T`` on the hand-written gfx950 kernel
(:func:`kgs.ops.gemm_nt`) plus, when the pod holds more than one GPU, an RCCL
all-reduce of a gradient-sized bucket on its own HIP stream so the collective
overlaps the MFMA work (the data-parallel pattern; xGMI traffic while the
matrix cores run).

Replaces the reference's ``echo Hello from fake ROCm GPU node``
(pods/rocm-gpu-test-pod.yaml:9).
"""
from __future__ import annotations

import torch


class GemmWorkload:
    def __init__(self, m=8192, n=8192, k=8192, gemms_per_step=4, allreduce_bytes=0, overlap=True,
                 device=None, group=None, seed=0, backend="kgs", dtype="bf16"):
        self.m, self.n, self.k = m, n, k
        self.g = gemms_per_step
        self.device = torch.device(device) if device is not None else torch.device("cuda")
        self.group = group
        self.overlap = overlap
        self.backend = backend
        gen = torch.Generator(device=self.device)
        gen.manual_seed(seed)
        # U[-1, 1) operands: random data (zeros inflate TFLOPS via DVFS)
        self.a = (torch.rand((m, k), generator=gen, device=self.device) * 2 - 1).to(torch.bfloat16)
        self.b = (torch.rand((n, k), generator=gen, device=self.device) * 2 - 1).to(torch.bfloat16)
        self.c = [torch.empty((m, n), dtype=torch.bfloat16, device=self.device) for _ in range(2)]
        self.bucket = None
        self.cuda = self.device.type == "cuda"
        if not self.cuda:
            self.overlap = False  # CPU (gloo) path for tests: no streams
            if backend == "kgs":
                raise ValueError("the kgs HIP GEMM needs a GPU; use backend='torch' on CPU")
        if allreduce_bytes > 0:
            self.bucket = torch.rand(allreduce_bytes // 4, generator=gen, device=self.device)
            if self.cuda:
                self.comm_stream = torch.cuda.Stream(device=self.device)
        self.dtype = dtype
        self.reset_stats()
        if dtype == "fp8":
            # e4m3 operands (per-tensor scales), bf16 out: the scaled fp8 MFMA path
            from kgs.ops import quantize_fp8

            self.qa, self.sa = quantize_fp8(self.a)
            self.qb, self.sb = quantize_fp8(self.b)
            if backend == "kgs":
                from kgs.ops import gemm_fp8_nt

                self._gemm = lambda i: gemm_fp8_nt(self.qa, self.qb, self.sa, self.sb, out=self.c[i & 1])
            else:
                ta = torch.tensor(self.sa, device=self.device)
                tb = torch.tensor(self.sb, device=self.device)
                self._gemm = lambda i: torch._scaled_mm(self.qa, self.qb.T, scale_a=ta, scale_b=tb,
                                                        out_dtype=torch.bfloat16, out=self.c[i & 1])
        elif backend == "kgs":
            from kgs.ops import gemm_nt

            self._gemm = lambda i: gemm_nt(self.a, self.b, out=self.c[i & 1])
        else:
            self._gemm = lambda i: torch.matmul(self.a, self.b.T, out=self.c[i & 1])
        # the yardstick: the vendor library (hipBLASLt behind torch) on the same
        # operands, into its own outputs (the timed outputs stay checkable)
        if dtype == "fp8":
            ta = torch.tensor(self.sa, device=self.device)
            tb = torch.tensor(self.sb, device=self.device)
            self._ref_gemm = lambda i: torch._scaled_mm(self.qa, self.qb.T, scale_a=ta, scale_b=tb,
                                                        out_dtype=torch.bfloat16, out=self._c_ref(i))
        else:
            self._ref_gemm = lambda i: torch.matmul(self.a, self.b.T, out=self._c_ref(i))
        self._cref = None

    def flops_per_step(self) -> float:
        return 2.0 * self.m * self.n * self.k * self.g

    def path_name(self) -> str:
        if self.dtype == "fp8":
            return "kgs gemm_fp8_nt (scaled e4m3 MFMA)" if self.backend == "kgs" else "torch._scaled_mm"
        if self.backend != "kgs":
            return "torch.matmul"
        from kgs.ops import fast_path_ok

        return "kgs gemm_nt_w4p (persistent 4-wave 256x256 LDS-DMA pipeline)" if fast_path_ok(self.a, self.b, self.c[0]) else \
            "kgs gemm_nt_generic"

    def reference_path_name(self) -> str:
        lib = "hipBLASLt" if self.cuda else "CPU BLAS"
        return f"torch._scaled_mm ({lib})" if self.dtype == "fp8" else f"torch.matmul ({lib})"

    def _allreduce(self):
        import time

        import torch.distributed as dist

        if self.cuda:
            ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            ev[0].record()
            dist.all_reduce(self.bucket, group=self.group)
            ev[1].record()
            self._ar_events.append(ev)
        else:
            t0 = time.perf_counter()
            dist.all_reduce(self.bucket, group=self.group)
            self._ar_wall.append((time.perf_counter() - t0) * 1e3)

    def reset_stats(self) -> None:
        self._ar_events, self._ar_wall = [], []

    def allreduce_ms(self):
        """Mean duration of the in-step all-reduce (stream time between its
        start and end events: includes waiting for CUs the GEMM holds)."""
        if self.bucket is None:
            return None
        if self.cuda:
            torch.cuda.synchronize(self.device)
            ts = [a.elapsed_time(b) for a, b in self._ar_events]
        else:
            ts = list(self._ar_wall)
        return sum(ts) / len(ts) if ts else None

    def _c_ref(self, i):
        if self._cref is None:
            self._cref = [torch.empty_like(self.c[0]) for _ in range(2)]
        return self._cref[i & 1]

    def step(self, reference: bool = False) -> None:
        """One workload step. ``reference``: the same step with the vendor GEMM
        (torch.matmul -> hipBLASLt; torch._scaled_mm for fp8) in place of the
        kgs kernel -- the same-box yardstick bench.py interleaves with it."""
        gemm = self._ref_gemm if reference else self._gemm
        if not self.cuda:
            for i in range(self.g):
                gemm(i)
            if self.bucket is not None:
                self._allreduce()
            return
        cur = torch.cuda.current_stream(self.device)
        if self.bucket is not None and self.overlap:
            self.comm_stream.wait_stream(cur)
            with torch.cuda.stream(self.comm_stream):
                self._allreduce()
        for i in range(self.g):
            gemm(i)
        if self.bucket is not None:
            if self.overlap:
                cur.wait_stream(self.comm_stream)
            else:
                self._allreduce()

    @torch.no_grad()
    def verify(self, rows: int = 256) -> float:
        """Relative max error of one GEMM's first ``rows`` rows vs fp32 torch."""
        self._gemm(0)
        if self.dtype == "fp8":
            ref = (self.qa[:rows].float() * self.sa) @ (self.qb.float() * self.sb).T
        else:
            ref = self.a[:rows].float() @ self.b.float().T
        got = self.c[0][:rows].float()
        return ((got - ref).abs().max() / ref.abs().max()).item()

    @torch.no_grad()
    def check_output(self, chunk_rows: int = 2048) -> float:
        """Relative max error of the LAST timed GEMM's whole output (``C`` of
        the step's final GEMM, as the timed loop left it) against an fp32
        reference of the same operands: ``max|C - A.B^T| / max|A.B^T|``.
        Row chunks keep the fp32 temporaries small; TF32 is off."""
        got = self.c[(self.g - 1) & 1]
        prev = torch.backends.cuda.matmul.allow_tf32 if self.cuda else None
        if self.cuda:
            torch.backends.cuda.matmul.allow_tf32 = False
        try:
            if self.dtype == "fp8":
                bf = self.qb.float() * self.sb
            else:
                bf = self.b.float()
            err = ref_max = 0.0
            for r0 in range(0, self.m, chunk_rows):
                a = self.qa[r0:r0 + chunk_rows].float() * self.sa if self.dtype == "fp8" else \
                    self.a[r0:r0 + chunk_rows].float()
                ref = a @ bf.T
                err = max(err, (got[r0:r0 + chunk_rows].float() - ref).abs().max().item())
                ref_max = max(ref_max, ref.abs().max().item())
            return err / ref_max if ref_max > 0 else float(err)
        finally:
            if self.cuda:
                torch.backends.cuda.matmul.allow_tf32 = prev

    def torch_reference_tflops(self, iters: int = 10) -> float:
        """hipBLASLt (torch.matmul) TFLOP/s on the same operands, for comparison."""
        out = torch.empty_like(self.c[0])
        for _ in range(3):
            torch.matmul(self.a, self.b.T, out=out)
        torch.cuda.synchronize(self.device)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(iters):
            torch.matmul(self.a, self.b.T, out=out)
        e.record()
        torch.cuda.synchronize(self.device)
        ms = s.elapsed_time(e) / iters
        return 2.0 * self.m * self.n * self.k / (ms * 1e-3) / 1e12
