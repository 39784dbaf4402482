#!/usr/bin/env python3
"""Summarise a bench/gemm_sweep.py JSON: per shape, production ("fast") vs
the non-temporal-store variant of the tile map production uses for that
shape (gemm_persistent.hip: tall -> mirrored order, K > 8192 -> groups of 8)
vs hipBLASLt, interleaved medians in TFLOP/s."""
import json
import sys


def prod_map(m: int, n: int, k: int) -> str:
    tall, longk = m > n, k > 8192
    return "140000008" if tall and longk else "140000000" if tall else "8" if longk else "0"


def main(path: str) -> int:
    rows = json.load(open(path))
    print("| shape | kgs (production) | kgs, C stored non-temporally | hipBLASLt | nt / production | production / hipBLASLt |")
    print("|---|---|---|---|---|---|")
    for r in rows:
        m, n, k = r["shape"]
        f = r.get("kgs_fast_tflops_median")
        nt = r.get(f"kgs_w4pn_{prod_map(m, n, k)}_tflops_median")
        h = r.get("hipblaslt_tflops_median")
        print(f"| {m}x{n}x{k} | {f} | {nt} | {h} | {nt / f:.4f} | {f / h:.4f} |" if nt and f and h else f"| {m}x{n}x{k} | {f} | {nt} | {h} | | |")
    return 0


if __name__ == "__main__":
    raise SystemExit(main(sys.argv[1]))
