#!/usr/bin/env python3
"""Flagship benchmark: the rocm-gpu-test pod's in-pod workload step.

BASELINE.json metric: "cluster-create->GPU-pod-Running sec; in-pod bf16 GEMM
TFLOPS at 1/2/4/8 MI355X". The cluster-create half needs docker + kind + a GPU
host (see ``bench/e2e.py``); this script measures the in-pod half exactly as the
pod runs it, one process per GPU:

  step (per rank) = G x bf16 GEMM C = A . B^T  (M=N=K=8192, hand-written gfx950
                    MFMA kernel, kgs.ops.gemm_nt)
                  + an RCCL all-reduce of a gradient bucket (default 64 MiB
                    fp32) on a separate HIP stream, overlapped with the GEMMs
                    (the data-parallel gradient-sync pattern; skipped at N=1)

Timing: W untimed warmup steps, then K steps bracketed by barrier +
torch.cuda.synchronize() on both sides; the MAX over ranks is reported.
value = aggregate GEMM TFLOP/s over all N GPUs (weak scaling: per-GPU work is
fixed). Synthetic U[-1,1) operands (random data, not zeros: DVFS reads zeros
fast, cdna_hip_programming.md rule 25).

Self-normalising and self-checking (after the timed region, which alone gives
``value`` and ``ms_per_step``): the last timed GEMM's whole output is compared
with an fp32 reference (``rel_err``; the run fails above ``--max-rel-err``),
and ``--yardstick-rounds`` interleaved rounds of S kgs steps and S steps of the
same workload on the vendor GEMM (torch.matmul -> hipBLASLt) give
``hipblaslt_tflops`` and ``ratio_vs_hipblaslt`` on the same box, so a change in
``value`` between runs reads as box speed or kernel change.

Usage:  python bench.py [--gpus N] [--steps K] [--warmup W]
        torchrun --nproc-per-node N bench.py --gpus N ...

With ``--gpus N > 1`` and no WORLD_SIZE in the environment the script launches
itself: the parent (which never touches the GPU) spawns N ranks with the
torchrun env contract (kgs.parallel.launch) and exits with their status.

Failure is loud and bounded, under torchrun or the self-launch alike: the
rendezvous has its own timeout (``--rendezvous-timeout``, 120 s), every rank
checks it owns a distinct GPU before the RCCL communicator exists, and a
per-rank watchdog ends the run after ``--launch-timeout`` (300 s). Whatever
fails, ONE JSON line with ``"status": "error"``, the failing rank, the phase
each rank reached and (self-launch) the failing rank's stderr tail is printed
and the exit status is non-zero -- never a silent hang.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

BASELINE_VALUE = None  # the reference publishes no numbers


def parse(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    # --gemm-m/n/k (not --m/--n/--k: torchrun's parser would take those as
    # abbreviations of its own options)
    ap.add_argument("--gemm-m", "--m", dest="m", type=int, default=8192)
    ap.add_argument("--gemm-n", "--n", dest="n", type=int, default=8192)
    ap.add_argument("--gemm-k", "--k", dest="k", type=int, default=8192)
    ap.add_argument("--gemms-per-step", type=int, default=4)
    ap.add_argument("--allreduce-mb", type=float, default=64.0, help="gradient bucket all-reduced per step (MiB)")
    ap.add_argument("--no-overlap", action="store_true", help="run the all-reduce after the GEMMs, same stream")
    ap.add_argument("--compare-torch", action="store_true", help="also time torch.matmul (hipBLASLt), untimed part")
    ap.add_argument("--yardstick-rounds", type=int, default=3,
                    help="after the timed region: this many interleaved rounds of (S kgs steps, S vendor-GEMM "
                         "steps) on the same operands, medians -> ratio_vs_hipblaslt (0 = off)")
    ap.add_argument("--yardstick-steps", type=int, default=20, help="S, steps per yardstick block")
    ap.add_argument("--max-rel-err", type=float, default=1e-2,
                    help="the last timed GEMM's whole output is checked against fp32; above this the run fails")
    ap.add_argument("--verify", action="store_true", help="check one GEMM against fp32 torch before timing")
    ap.add_argument("--backend", choices=("kgs", "torch"), default="kgs",
                    help="kgs = hand-written gfx950 kernel (the benchmark); torch = reference / CPU test path")
    ap.add_argument("--cpu", action="store_true", help="CPU + gloo (tests of the distributed plumbing only)")
    ap.add_argument("--dist-backend", choices=("auto", "nccl", "gloo"), default="auto",
                    help="collective backend: auto = RCCL on GPUs (the benchmark), gloo on CPU")
    ap.add_argument("--oversubscribe", action="store_true",
                    help="allow more ranks than GPUs (rank r on GPU r %% n): tests the multi-rank GPU path on a "
                         "1-GPU box, with --dist-backend gloo; not a benchmark configuration")
    ap.add_argument("--dtype", choices=("bf16", "fp8"), default="bf16",
                    help="bf16 = the headline (BASELINE.json); fp8 = e4m3 operands on the scaled MFMA (extra)")
    ap.add_argument("--launch-timeout", type=float, default=300.0,
                    help="per-rank bound from `import torch` to the end (watchdog); the self-launch parent, whose "
                         "clock includes the ranks' imports, kills at +180 s")
    ap.add_argument("--rendezvous-timeout", type=float, default=120.0,
                    help="how long a rank waits for the others to join")
    return ap.parse_args(argv)


def metric_name(dtype: str) -> str:
    return ("in-pod bf16 GEMM TFLOPS (gpu-rocm-test workload, 8192^3 MFMA GEMM + RCCL grad all-reduce)"
            if dtype == "bf16" else
            "in-pod fp8 e4m3 GEMM TFLOPS (gpu-rocm-test workload, 8192^3 scaled-MFMA GEMM + RCCL all-reduce)")


def error_report(args, world: int) -> dict:
    """The fields of the success line that are known before the run, for the
    error line (so a parser keyed on ``metric`` finds the failure)."""
    return {"metric": metric_name(args.dtype), "value": None, "unit": "TFLOP/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "higher_is_better": True, "scaling": "weak",
            "dtype": args.dtype if args.dtype == "bf16" else "fp8_e4m3"}


def main(argv=None) -> int:
    args = parse(argv)
    from kgs.parallel import launch

    if launch.needs_self_launch(args.gpus):
        raw = list(sys.argv[1:] if argv is None else argv)
        os.environ["KGS_LAUNCH_PARENT"] = "1"
        return launch.spawn_local(args.gpus, [os.path.abspath(__file__), *raw],
                                  require_gpus=not (args.cpu or args.oversubscribe),
                                  timeout_s=args.launch_timeout + 180, error_report=error_report(args, args.gpus))

    env_rank = int(os.environ.get("RANK", "0") or 0)
    env_world = int(os.environ.get("WORLD_SIZE", "1") or 1)
    # the watchdog's clock starts after `import torch`, which alone can take 1-2
    # minutes on a freshly booted box (image paging), so that cost never reads as a hang
    import torch  # noqa: F401

    wd = launch.Watchdog(args.launch_timeout, env_rank, env_world, error_report(args, env_world))
    if env_rank == 0 and env_world > 1 and not os.environ.get("KGS_LAUNCH_PARENT"):
        # under torchrun: a peer's failure reaches rank 0 as SIGTERM from the agent
        import signal

        def _term(signum, frame):
            launch.report_once({**error_report(args, env_world), "status": "error", "exit_code": 128 + signum,
                                "reason": f"rank 0 stopped by signal {signum} in phase {wd.phase!r} "
                                          "(a peer rank failed or the launcher stopped the job)"})
            os._exit(128 + signum)

        signal.signal(signal.SIGTERM, _term)
    try:
        rc = run(args, wd)
    except BaseException as e:
        if env_rank == 0 and not (isinstance(e, SystemExit) and e.code in (0, None)):
            launch.report_once({**error_report(args, env_world), "status": "error", "exit_code": 1,
                                "failing_rank": env_rank, "phase": wd.phase, "reason": f"{type(e).__name__}: {e}"})
        raise
    finally:
        wd.cancel()
    return rc


def yardstick(wl, ctx, sync, rounds: int, steps: int) -> dict:
    """Interleaved medians of ``rounds`` x (``steps`` kgs steps, ``steps``
    vendor-GEMM steps), each block bracketed like the timed region (barrier +
    synchronize, max over ranks). Same operands, same all-reduce, same box."""
    import statistics

    from kgs.parallel import dist as kdist

    for _ in range(min(3, steps)):  # the vendor path's first calls pick its kernel
        wl.step(reference=True)

    def block(reference: bool) -> float:
        sync()
        kdist.barrier(ctx)
        sync()
        t0 = time.perf_counter()
        for _ in range(steps):
            wl.step(reference=reference)
        sync()
        kdist.barrier(ctx)
        sync()
        return kdist.max_over_ranks(ctx, time.perf_counter() - t0) / steps * 1e3

    kgs, ref = [], []
    for _ in range(rounds):
        kgs.append(block(False))
        ref.append(block(True))
    return {"rounds": rounds, "steps": steps, "kgs_ms_per_step": round(statistics.median(kgs), 4),
            "ref_ms_per_step": round(statistics.median(ref), 4), "kgs_ms": [round(t, 4) for t in kgs],
            "ref_ms": [round(t, 4) for t in ref]}


def run(args, wd) -> int:
    import torch
    from kgs.models.gemm_workload import GemmWorkload
    from kgs.parallel import dist as kdist
    from kgs.parallel import launch

    wd.set_phase("rendezvous")
    ctx = kdist.init_from_env(expected_world=args.gpus, device_type="cpu" if args.cpu else None,
                              backend=None if args.dist_backend == "auto" else args.dist_backend,
                              rendezvous_timeout_s=args.rendezvous_timeout,
                              timeout_s=max(args.launch_timeout, args.rendezvous_timeout),
                              allow_shared_device=args.oversubscribe)
    rank, world = ctx.rank, ctx.world_size
    dev = ctx.device
    if world > 1:
        wd.store = ctx.store
    wd.set_phase("setup")
    launch.inject_fault(rank, "setup")

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)

    wl = GemmWorkload(
        m=args.m,
        n=args.n,
        k=args.k,
        gemms_per_step=args.gemms_per_step,
        allreduce_bytes=int(args.allreduce_mb * (1 << 20)) if world > 1 else 0,
        overlap=not args.no_overlap,
        device=dev,
        group=ctx.group,
        seed=1234 + rank,
        backend=args.backend,
        dtype=args.dtype,
    )
    if args.verify:
        err = wl.verify()
        if rank == 0:
            print(f"[bench] verify rel err {err:.3e}", file=sys.stderr)
        if err > 2e-2:
            raise SystemExit(f"GEMM verification failed: rel err {err}")

    launch.inject_fault(rank, "warmup")  # before the marker: a stalled rank stays behind in "setup"
    wd.set_phase("warmup")
    for _ in range(args.warmup):
        wl.step()
    sync()
    wd.set_phase("warmup-barrier")
    kdist.barrier(ctx)
    sync()
    wl.reset_stats()
    wd.set_phase("timed")
    t0 = time.perf_counter()
    for _ in range(args.steps):
        wl.step()
    sync()
    wd.set_phase("timed-barrier")
    kdist.barrier(ctx)
    sync()
    elapsed = time.perf_counter() - t0
    elapsed_max = kdist.max_over_ranks(ctx, elapsed)
    # --- untimed from here: the check and the same-box yardstick ---
    wd.set_phase("check")
    rel_err = kdist.max_over_ranks(ctx, wl.check_output())
    ys = None
    if args.yardstick_rounds > 0 and rel_err <= args.max_rel_err:
        wd.set_phase("yardstick")
        ys = yardstick(wl, ctx, sync, args.yardstick_rounds, args.yardstick_steps)
    wd.set_phase("report")

    per_rank_ms = [round(t / max(1, args.steps) * 1e3, 4) for t in kdist.all_gather_object(ctx, elapsed)]
    ar_ms = wl.allreduce_ms()  # mean in-step all-reduce time over the timed steps (None at N=1)
    ms_per_step = elapsed_max / max(1, args.steps) * 1e3
    flops_per_step = wl.flops_per_step()
    per_gpu_tflops = flops_per_step / (ms_per_step * 1e-3) / 1e12
    total_tflops = per_gpu_tflops * world

    extra = {}
    if ar_ms:
        ar_bytes = wl.bucket.numel() * wl.bucket.element_size()
        extra["allreduce_ms_in_step"] = round(ar_ms, 4)
        # nccl-tests convention: busBW = algBW * 2 (N-1) / N
        extra["allreduce_busbw_gbs"] = round(ar_bytes / (ar_ms * 1e-3) * 2 * (world - 1) / world / 1e9, 2)
    if args.compare_torch:
        extra["torch_matmul_tflops_per_gpu"] = round(wl.torch_reference_tflops(), 1)
    extra["rel_err"] = float(f"{rel_err:.3e}")
    if ys is not None:
        kgs_ms, ref_ms = ys["kgs_ms_per_step"], ys["ref_ms_per_step"]
        extra["hipblaslt_tflops"] = round(flops_per_step / (ref_ms * 1e-3) / 1e12 * world, 2)
        extra["ratio_vs_hipblaslt"] = round(ref_ms / kgs_ms, 4)  # > 1: the kgs step is faster
        extra["yardstick"] = {**ys, "path": wl.reference_path_name(),
                              "kgs_tflops": round(flops_per_step / (kgs_ms * 1e-3) / 1e12 * world, 2)}
    if rel_err > args.max_rel_err:
        if rank == 0:
            launch.report_once({**error_report(args, world), "status": "error", "exit_code": 1, "phase": "check",
                                "rel_err": rel_err, "reason": f"timed GEMM output rel err {rel_err:.3e} > "
                                                              f"{args.max_rel_err:g} against fp32"})
        wd.shutdown_bound(90.0)
        kdist.shutdown(ctx)
        return 1

    if rank == 0:
        out = {
            "metric": metric_name(args.dtype),
            "value": round(total_tflops, 2),
            "unit": "TFLOP/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": (round(total_tflops / BASELINE_VALUE, 4) if BASELINE_VALUE else None),
            "dtype": args.dtype if args.dtype == "bf16" else "fp8_e4m3",
            "data": "synthetic U[-1,1) operands, random-init",
            "config": {
                "model": f"rocm-gpu-test in-pod workload: {args.dtype} GEMM C=A.B^T (kgs gfx950 MFMA kernel)",
                "global_batch": args.gemms_per_step * world,
                "seq_len": args.m,
                "parallelism": f"dp{world}",
                "m": args.m,
                "n": args.n,
                "k": args.k,
                "gemms_per_step_per_gpu": args.gemms_per_step,
                "allreduce_mb": args.allreduce_mb if world > 1 else 0,
                "allreduce_overlap": not args.no_overlap,
            },
            "per_gpu_tflops": round(per_gpu_tflops, 2),
            "per_rank_ms_per_step": per_rank_ms,
            "gemm_path": wl.path_name(),
            "backend": args.backend,
            **extra,
        }
        launch.report_once(out)  # the one JSON line (a later signal cannot add an error line)
    # the measurement is done on every rank: from here only the teardown is bounded
    # (its store exit barrier waits up to 60 s for a lagging peer)
    wd.shutdown_bound(90.0)
    kdist.shutdown(ctx)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
