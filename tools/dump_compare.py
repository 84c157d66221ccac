#!/usr/bin/env python3
"""Compare two node dumps of oracle/_ref/ref-llama-bench (--dump + --dump-dir): the
reference CPU backend's (-ngl 0) and the MI355X backend's (-ngl 99) values of every f32
graph node, in graph order. Prints per-node NMSE; the first node whose NMSE jumps is
where the backends part. TEST/DEBUG INFRASTRUCTURE.

    python tools/dump_compare.py cpu.txt cpu_dir gpu.txt gpu_dir
"""
import sys

import numpy as np


def names(path):
    out = []
    for ln in open(path):
        t = ln.split()
        # "<name words...> <OP> ne0 ne1 ne2 ne3 sum sumsq v..."
        for i in range(1, len(t)):
            try:
                ne = [int(x) for x in t[i + 1:i + 5]]
                out.append((" ".join(t[:i]), t[i], ne))
                break
            except (ValueError, IndexError):
                continue
    return out


def main():
    ca, da, cb, db = sys.argv[1:5]
    na, nb = names(ca), names(cb)
    detail = sys.argv[5].split(",") if len(sys.argv) > 5 else []
    for i, ((n1, o1, ne), (n2, o2, _)) in enumerate(zip(na, nb)):
        a = np.fromfile(f"{da}/{i:03d}.f32", np.float32).astype(np.float64)
        b = np.fromfile(f"{db}/{i:03d}.f32", np.float32).astype(np.float64)
        if a.shape != b.shape:
            print(f"{i:3d} {n1:40s} {o1:14s} shape mismatch {a.shape} {b.shape}")
            continue
        e = float(np.sum((a - b) ** 2) / max(np.sum(a ** 2), 1e-30))
        mx = float(np.max(np.abs(a - b))) if a.size else 0.0
        print(f"{i:3d} {n1:40s} {o1:14s} n={a.size:9d} nmse={e:.3e} maxabs={mx:.3e}{'  <<<' if e > 1e-4 else ''}")
        if n1 in detail:   # per (ne1, ne2) row NMSE: which tokens / slots differ
            A = a.reshape(ne[3] * ne[2], ne[1], ne[0]); B = b.reshape(A.shape)
            r = np.sum((A - B) ** 2, -1) / np.maximum(np.sum(A ** 2, -1), 1e-30)
            for j in range(A.shape[0]):
                print("      row", j, " ".join(f"{v:.1e}" for v in r[j]))


if __name__ == "__main__":
    main()
