#!/usr/bin/env python3
"""Counter-pass driver: the production flash-attention forward and the
one-wave-per-SIMD experiment (attention_w4.h), a few launches each, on the
bench shape (B 4, S 2048, 32 q / 8 kv heads, d 128). Run under
``rocprofv3 --pmc ...`` (scripts/gpu.sh step ``attn_pmc``); the kernels are
told apart by name in the counter CSV."""
from __future__ import annotations

import argparse
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import torch  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--causal", action="store_true")
    a = ap.parse_args()
    from kgs.ops import transformer as T
    from kgs.ops import experiments as ex

    b, s, nh, nkv, hd = 4, 2048, 32, 8, 128
    qkv = torch.randn(b * s, (nh + 2 * nkv) * hd, device="cuda").bfloat16()
    out = torch.empty(b * s, nh * hd, device="cuda", dtype=torch.bfloat16)
    for _ in range(a.iters):
        T.attention_qkv(qkv, b, s, nh, nkv, causal=a.causal, out=out)
        ex.attention_qkv_w4(qkv, b, s, nh, nkv, causal=a.causal, out=out)
    torch.cuda.synchronize()
    print("ok", flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
