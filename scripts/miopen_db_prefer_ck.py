#!/usr/bin/env python3
"""Write a variant of the in-tree MIOpen find-db in which, for backward-data problems, the CK
solver is ranked first whenever its recorded time is within --margin of the GTC assembly
solver's.  The GTC backward-data kernels need a separate zero-fill of dX (SubTensorOp) that the
find-db time does not show; CK's do not.  Usage: miopen_db_prefer_ck.py SRC_DIR DST_DIR."""
import argparse
import glob
import os
import shutil

ap = argparse.ArgumentParser()
ap.add_argument("src")
ap.add_argument("dst")
ap.add_argument("--margin", type=float, default=0.10)
ap.add_argument("--dirs", default="B", help="directions to rewrite (F, B, W)")
a = ap.parse_args()
os.makedirs(a.dst, exist_ok=True)
for f in glob.glob(os.path.join(a.src, "*")):
    if not f.endswith(".ufdb.txt"):
        shutil.copy(f, a.dst)
        continue
    out, changed = [], 0
    for line in open(f):
        key, val = line.rstrip("\n").split("=", 1)
        direction = key.split("-")[-1]
        ents = [e.split(":", 1) for e in val.split(";")]
        times = {n: float(v.split(",")[0]) for n, v in ents}
        ck = [n for n in times if n.startswith("ConvHipImplicitGemmGroup")]
        gtc = [n for n in times if n.startswith("ConvAsmImplicitGemmGTCDynamic")]
        if direction in a.dirs and ck and gtc and times[ck[0]] <= times[gtc[0]] * (1 + a.margin) \
                and times[gtc[0]] < times[ck[0]]:
            new_t = times[gtc[0]] * 0.99
            ents = [[n, (f"{new_t:.6g}" + v[v.index(","):]) if n == ck[0] else v] for n, v in ents]
            changed += 1
        out.append(key + "=" + ";".join(f"{n}:{v}" for n, v in ents))
    open(os.path.join(a.dst, os.path.basename(f)), "w").write("\n".join(out) + "\n")
    print(f"{os.path.basename(f)}: {changed} problems now prefer CK")
