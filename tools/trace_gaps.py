#!/usr/bin/env python3
"""GPU busy / idle timeline of a rocprofv3 kernel trace (MEASUREMENT TOOL).

    python tools/trace_gaps.py run_kernel_trace.csv [--gap-us 50]

Sorts the dispatches by start time, merges overlapping ones, and reports the busy time,
the idle gaps between kernels (the host's share of the critical path: between the
tokens of a decode, between ubatches of a prompt), and the largest gaps with the kernels
on either side. Segments separated by idle gaps longer than --segment-us (default
2000 us) are reported one by one (llama-bench repetitions, warmup)."""
import argparse
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--gap-us", type=float, default=50.0, help="list gaps longer than this")
    ap.add_argument("--segment-us", type=float, default=2000.0)
    ap.add_argument("--top", type=int, default=12)
    a = ap.parse_args()
    rows = []
    for r in csv.DictReader(open(a.trace)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:70]))
    rows.sort()
    segs, cur = [], None
    gaps = []
    for s, e, n in rows:
        if cur is None:
            cur = {"t0": s, "t1": e, "busy": e - s, "idle": 0, "n": 1, "first": n}
            last_n = n
            continue
        gap = s - cur["t1"]
        if gap > a.segment_us * 1000:
            segs.append(cur)
            cur = {"t0": s, "t1": e, "busy": e - s, "idle": 0, "n": 1, "first": n}
            last_n = n
            continue
        if gap > 0:
            cur["idle"] += gap
            gaps.append((gap, last_n, n))
            cur["busy"] += e - s
        else:
            cur["busy"] += max(0, e - cur["t1"])
        cur["t1"] = max(cur["t1"], e)
        cur["n"] += 1
        last_n = n
    if cur:
        segs.append(cur)
    print(f"{'segment':>7s} {'kernels':>8s} {'span_us':>10s} {'busy_us':>10s} {'idle_us':>10s} {'idle%':>6s}  first kernel")
    for i, c in enumerate(segs):
        span = (c["t1"] - c["t0"]) / 1000
        print(f"{i:7d} {c['n']:8d} {span:10.1f} {c['busy'] / 1000:10.1f} {c['idle'] / 1000:10.1f} "
              f"{100 * c['idle'] / max(1, c['t1'] - c['t0']):6.1f}  {c['first']}")
    big = sorted((g for g in gaps if g[0] > a.gap_us * 1000), reverse=True)[:a.top]
    print(f"gaps > {a.gap_us} us: {sum(1 for g in gaps if g[0] > a.gap_us * 1000)} "
          f"(total {sum(g[0] for g in gaps if g[0] > a.gap_us * 1000) / 1000:.1f} us)")
    for g, p, n in big:
        print(f"  {g / 1000:9.1f} us  after {p}  before {n}")


if __name__ == "__main__":
    main()
