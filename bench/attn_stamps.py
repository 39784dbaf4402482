#!/usr/bin/env python3
"""Where a tile's cycles go in the one-wave-per-SIMD attention kernel
(attention_w4.h timing build): per section (A QK^T qb0, B QK^T qb1 + softmax,
the barrier, C P.V qb0 + softmax, D P.V qb1 + K reads + DMA), the median
shader cycles over the steady-state tiles of workgroups 0..63.

    python bench/attn_stamps.py [--causal] [--batch 4 --seq 2048 --heads 32 --kv-heads 8]
"""
import argparse
import json
import statistics as st
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import torch  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--seq", type=int, default=2048)
    ap.add_argument("--heads", type=int, default=32)
    ap.add_argument("--kv-heads", type=int, default=8)
    ap.add_argument("--causal", action="store_true")
    a = ap.parse_args()
    from kgs.ops import experiments as ex

    b, s, nh, nkv, hd = a.batch, a.seq, a.heads, a.kv_heads, 128
    qkv = torch.randn(b * s, (nh + 2 * nkv) * hd, device="cuda").bfloat16()
    st_t = torch.zeros(64, 4, 64, 8, dtype=torch.int64, device="cuda")
    for _ in range(3):
        ex.attention_qkv_w4(qkv, b, s, nh, nkv, causal=a.causal)
    ex.attention_qkv_w4(qkv, b, s, nh, nkv, causal=a.causal, stamps=st_t)
    torch.cuda.synchronize()
    x = st_t.cpu()
    names = ["A_qk0", "B_qk1_sm0", "barrier", "C_pv0_sm1", "D_pv1"]
    d = {n: [] for n in names}
    tile = []
    ntile = s // 64
    for blk in range(64):
        for w in range(4):
            for j in range(2, min(ntile, 63) - 1):
                r = x[blk, w, j]
                nxt = x[blk, w, j + 1]
                if r[0] == 0 or r[5] == 0 or nxt[0] == 0:
                    continue
                for i, n in enumerate(names):
                    d[n].append(int(r[i + 1] - r[i]))
                tile.append(int(nxt[0] - r[0]))
    out = {"causal": a.causal, "tiles": len(tile), "tile_cycles_median": st.median(tile) if tile else None,
           "section_cycles_median": {n: st.median(v) for n, v in d.items() if v},
           "mfma_floor_per_tile": 64 * 32}
    print(json.dumps(out))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
