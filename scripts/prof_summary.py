#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel_stats.csv: per-category and top-N kernels, per step."""
import csv
import sys


def cat(n: str) -> str:
    if "damd::bn_" in n:
        return "bn(ours)"
    if "damd::igemm" in n or "damd::stem" in n or "damd::c3v2" in n:
        return "conv(ours)"
    if "damd::" in n:
        return "optim/norm(ours)"
    if "batch_norm" in n:
        return "bn(torch)"
    if "igemm" in n or "conv" in n.lower() or "ck::" in n:
        return "conv(MIOpen)"
    if "Cijk" in n or "gemm" in n.lower():
        return "gemm"
    if "elementwise" in n or "SubTensor" in n or "fillBuffer" in n:
        return "eltwise"
    if "nccl" in n.lower() or "rccl" in n.lower():
        return "rccl"
    return "other"


def main() -> None:
    path = sys.argv[1]
    steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 25
    rows = list(csv.DictReader(open(path)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    cats: dict = {}
    for r in rows:
        c = cat(r["Name"])
        cats.setdefault(c, [0.0, 0])
        cats[c][0] += float(r["TotalDurationNs"])
        cats[c][1] += int(r["Calls"])
    print(f"total kernel time {tot / 1e6 / steps:.2f} ms/step over {steps:g} steps")
    for k, v in sorted(cats.items(), key=lambda x: -x[1][0]):
        print(f"  {k:18s} {v[0] / 1e6 / steps:8.2f} ms/step  {100 * v[0] / tot:5.1f}%  calls/step={v[1] / steps:.0f}")
    print("top kernels:")
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:top]:
        print(f"  {float(r['TotalDurationNs']) / 1e6 / steps:7.2f} ms/step {float(r['Percentage']):5.1f}% "
              f"n/step={int(r['Calls']) / steps:5.0f} avg={float(r['AverageNs']) / 1e3:8.1f}us  {r['Name'][:100]}")


if __name__ == "__main__":
    main()
