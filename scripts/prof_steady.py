#!/usr/bin/env python3
"""Steady-state per-step kernel summary from a rocprofv3 kernel_trace.csv.

Steps are delimited by the fused optimizer launch (one ``damd::sgd_kernel``/``adam_kernel`` per
step); only the last ``--steps`` complete steps are summarised, so warm-up (MIOpen solver
search, first-iteration allocations) is excluded.
"""
import argparse
import csv
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from prof_summary import cat  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("--steps", type=int, default=5)
ap.add_argument("--top", type=int, default=25)
ap.add_argument("--marker", default="damd::sgd_kernel")
ap.add_argument("--seq", default=None, help="also write the last step's launch sequence (with grid sizes) here")
a = ap.parse_args()

rows = list(csv.DictReader(open(a.trace)))
key_start = "Start_Timestamp" if "Start_Timestamp" in rows[0] else "BeginNs"
key_end = "End_Timestamp" if "End_Timestamp" in rows[0] else "EndNs"
name_key = "Kernel_Name" if "Kernel_Name" in rows[0] else "KernelName"
rows.sort(key=lambda r: int(r[key_start]))
marks = [i for i, r in enumerate(rows) if a.marker in r[name_key]]
if len(marks) < a.steps + 1:
    sys.exit(f"only {len(marks)} marker launches found")
lo, hi = marks[-a.steps - 1] + 1, marks[-1] + 1
window = rows[lo:hi]
wall = (int(rows[hi - 1][key_end]) - int(rows[lo][key_start])) / 1e6 / a.steps
busy = sum(int(r[key_end]) - int(r[key_start]) for r in window) / 1e6 / a.steps
per: dict = {}
cats: dict = {}
for r in window:
    d = (int(r[key_end]) - int(r[key_start])) / 1e6 / a.steps
    n = r[name_key]
    per.setdefault(n, [0.0, 0])
    per[n][0] += d
    per[n][1] += 1
    c = cat(n)
    cats.setdefault(c, [0.0, 0])
    cats[c][0] += d
    cats[c][1] += 1
print(f"steady state over {a.steps} steps: wall {wall:.2f} ms/step, kernel busy {busy:.2f} ms/step "
      f"({100 * busy / wall:.1f}%), {len(window) / a.steps:.0f} launches/step")
for k, v in sorted(cats.items(), key=lambda x: -x[1][0]):
    print(f"  {k:18s} {v[0]:8.2f} ms/step {100 * v[0] / busy:5.1f}%  launches/step={v[1] / a.steps:.0f}")
print("top kernels (ms/step, launches/step):")
for n, v in sorted(per.items(), key=lambda x: -x[1][0])[: a.top]:
    print(f"  {v[0]:7.3f} {v[1] / a.steps:5.0f}  {n[:110]}")

if a.seq:
    last = rows[marks[-2] + 1: marks[-1] + 1]
    gk = [k for k in last[0].keys() if "Grid" in k or "Workgroup" in k]
    with open(a.seq, "w") as f:
        prev_end = None
        for r in last:
            d = (int(r[key_end]) - int(r[key_start])) / 1e3
            gap = 0.0 if prev_end is None else (int(r[key_start]) - prev_end) / 1e3
            prev_end = max(prev_end or 0, int(r[key_end]))
            f.write(f"{d:9.1f}us gap {gap:7.1f}us  {' '.join(r[k] for k in gk):24s}  {r[name_key][:100]}\n")
