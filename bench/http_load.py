#!/usr/bin/env python3
"""End-to-end HTTP load test of ``python -m kgs.serve serve`` -- the process the
kgs-serve pod runs (BASELINE config 5 stand-in), measured through its
OpenAI-style API the way a vLLM deployment is: N concurrent streaming clients,
each sending its requests back to back, token-id prompts (no tokenizer on the
critical path), EOS ignored.

Starts the server as a child process (it owns the GPU; this process never
touches it), waits for ``/health``, runs the load, prints one JSON line with
throughput and TTFT / ITL percentiles over HTTP, and stops the server.

  python bench/http_load.py [--clients 64] [--requests 256] [--input-len 512] [--output-len 128]
                            [--server-args "--chunked-prefill 2048 --prefix-caching"]
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import shlex
import signal
import subprocess
import sys
import time

import numpy as np


def _pct(v, q):
    v = sorted(v)
    return v[min(len(v) - 1, int(q * len(v)))] if v else float("nan")


async def _client(http, url, prompts, out_len, stats):
    for prompt in prompts:
        t0 = time.perf_counter()
        times = []
        body = {"prompt": prompt, "max_tokens": out_len, "ignore_eos": True, "stream": True}
        async with http.stream("POST", url + "/v1/completions", json=body, timeout=600) as r:
            r.raise_for_status()
            async for line in r.aiter_lines():
                if not line.startswith("data: ") or line == "data: [DONE]":
                    continue
                times.append(time.perf_counter())
        stats["ttft"].append(times[0] - t0)
        stats["itl"].extend(b - a for a, b in zip(times, times[1:]))
        stats["tokens"] += len(times)


async def _load(url, prompts, clients, out_len):
    import httpx

    stats = {"ttft": [], "itl": [], "tokens": 0}
    shards = [prompts[i::clients] for i in range(clients)]
    limits = httpx.Limits(max_connections=clients + 4, max_keepalive_connections=clients + 4)
    async with httpx.AsyncClient(limits=limits) as http:
        t0 = time.perf_counter()
        await asyncio.gather(*(_client(http, url, s, out_len, stats) for s in shards if s))
        dt = time.perf_counter() - t0
    return stats, dt


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--clients", type=int, default=64)
    ap.add_argument("--requests", type=int, default=256)
    ap.add_argument("--input-len", type=int, default=512)
    ap.add_argument("--output-len", type=int, default=128)
    ap.add_argument("--port", type=int, default=8011)
    ap.add_argument("--server-args", default="--max-batch 256 --max-model-len 2048")
    ap.add_argument("--startup-timeout", type=float, default=600)
    ap.add_argument("--server-log", default="http_load_server.log")
    a = ap.parse_args(argv)
    import httpx

    cmd = [sys.executable, "-m", "kgs.serve", "serve", "--host", "127.0.0.1", "--port", str(a.port),
           *shlex.split(a.server_args)]
    log = open(a.server_log, "w")  # a file, not a pipe: uvicorn's access log would fill a pipe and block
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, PYTHONPATH=root + os.pathsep + os.environ.get("PYTHONPATH", ""))
    srv = subprocess.Popen(cmd, stdout=log, stderr=subprocess.STDOUT, start_new_session=True, cwd=root, env=env)
    url = f"http://127.0.0.1:{a.port}"
    try:
        t0 = time.time()
        while True:
            if srv.poll() is not None:
                raise SystemExit(f"server exited ({srv.returncode}): {open(a.server_log).read()[-2000:]}")
            try:
                if httpx.get(url + "/health", timeout=2).status_code == 200:
                    break
            except httpx.HTTPError:
                pass
            if time.time() - t0 > a.startup_timeout:
                raise SystemExit("server did not come up")
            time.sleep(1)
        startup = time.time() - t0
        rng = np.random.default_rng(0)
        prompts = [rng.integers(3, 128256, size=a.input_len).tolist() for _ in range(a.requests)]
        stats, dt = asyncio.run(_load(url, prompts, a.clients, a.output_len))
        metrics = httpx.get(url + "/metrics", timeout=10).text
        ms = lambda v: round(1e3 * v, 2)  # noqa: E731
        print(json.dumps({
            "metric": "kgs.serve over HTTP (OpenAI /v1/completions, streaming), Llama-3-8B arch, random init",
            "clients": a.clients, "requests": a.requests, "input_len": a.input_len, "output_len": a.output_len,
            "server_args": a.server_args, "server_startup_s": round(startup, 1), "seconds": round(dt, 3),
            "output_tok_per_s": round(stats["tokens"] / dt, 1),
            "total_tok_per_s": round((stats["tokens"] + a.requests * a.input_len) / dt, 1),
            "ttft_ms": {"p50": ms(_pct(stats["ttft"], .5)), "p99": ms(_pct(stats["ttft"], .99))},
            "itl_ms": {"p50": ms(_pct(stats["itl"], .5)), "p99": ms(_pct(stats["itl"], .99))},
            "server_requests_total": next((ln.split()[1] for ln in metrics.splitlines()
                                           if ln.startswith("kgs_requests_total")), None),
        }), flush=True)
    finally:
        if srv.poll() is None:
            os.killpg(srv.pid, signal.SIGINT)  # the server's own process group: uvicorn shuts down cleanly
            try:
                srv.wait(timeout=60)
            except subprocess.TimeoutExpired:
                os.killpg(srv.pid, signal.SIGKILL)
                srv.wait(timeout=30)
        log.close()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
