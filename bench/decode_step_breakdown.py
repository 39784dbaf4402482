#!/usr/bin/env python3
"""Per-kernel breakdown of one decode step from a rocprofv3 kernel trace of
``python -m kgs.serve bench`` (steps are delimited by the sampler's argmax:
torch's reduce or ``kgs::tfm::argmax_rows``).

  python bench/decode_step_breakdown.py gpurun_out/prof_decode/b1/d_kernel_trace.csv [--step -3]
"""
import argparse
import collections
import csv


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--step", type=int, default=-3, help="which argmax-delimited step (python index)")
    ap.add_argument("--gaps", type=int, default=0,
                    help="> 0: over the last N steps, the GPU idle time between one step's token read-back and "
                         "the next step's first kernel (the host's share of the step period)")
    a = ap.parse_args(argv)
    rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if "ArgMax" in r["Kernel_Name"] or "argmax_rows" in r["Kernel_Name"]]
    if a.gaps:
        import statistics

        host, period, gpu = [], [], []
        for j in range(max(1, len(idx) - a.gaps), len(idx)):
            k = idx[j - 1] + 1
            prev_end = int(rows[idx[j - 1]]["End_Timestamp"])
            if "copyBuffer" in rows[k]["Kernel_Name"]:  # the token read-back right behind the argmax
                prev_end = int(rows[k]["End_Timestamp"])
                k += 1
            first = int(rows[k]["Start_Timestamp"])
            host.append((first - prev_end) / 1e3)
            period.append((int(rows[idx[j]]["End_Timestamp"]) - prev_end) / 1e3)
            gpu.append((int(rows[idx[j]]["End_Timestamp"]) - first) / 1e3)
        q = lambda v: f"median {statistics.median(v):.1f} mean {statistics.fmean(v):.1f} max {max(v):.1f}"  # noqa: E731
        print(f"last {len(host)} steps (us): period {q(period)}; read-back -> next step's first kernel {q(host)}; "
              f"first kernel -> argmax {q(gpu)}; host share {100 * sum(host) / sum(period):.1f} %")
        return 0
    s0, s1 = idx[a.step - 1], idx[a.step]
    seg = rows[s0 + 1:s1 + 1]
    agg = collections.defaultdict(lambda: [0, 0])
    for r in seg:
        name = r["Kernel_Name"].split("(")[0][:72]
        agg[name][0] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        agg[name][1] += 1
    busy = sum(v[0] for v in agg.values())
    span = int(seg[-1]["End_Timestamp"]) - int(rows[s0]["End_Timestamp"])
    print(f"step span {span / 1e3:.1f} us, kernels busy {busy / 1e3:.1f} us ({100 * busy / span:.0f} %), "
          f"{len(seg)} kernels, idle between kernels {(span - busy) / 1e3:.1f} us")
    print("| kernel | us / step | share | launches | us / launch |")
    print("|---|---:|---:|---:|---:|")
    for name, (t, c) in sorted(agg.items(), key=lambda kv: -kv[1][0]):
        print(f"| `{name}` | {t / 1e3:.1f} | {100 * t / busy:.1f}% | {c} | {t / c / 1e3:.2f} |")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
