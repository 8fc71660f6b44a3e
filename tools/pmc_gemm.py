"""HBM traffic of the library GEMMs of one training step from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE;
MI355X_MICROARCH.md section HBM: FETCH_SIZE counts half the bytes of a wide stream on gfx950, so bytes =
(2 * FETCH_SIZE + WRITE_SIZE) * 1024).  Kernels whose name matches Cijk_ (hipBLASLt / rocBLAS Tensile) are grouped
by (kernel, grid); the groups are printed by total bytes, and the JSON holds the per-step total over `steps` steps
and the largest group's bytes per launch.

    python tools/pmc_gemm.py DIR STEPS OUT.json [NAME_REGEX]   (default Cijk_; e.g. "gemm3" for the in-tree kernels)
"""
import re
import collections
import csv
import glob
import json
import os
import sys


PAT = re.compile(sys.argv[4] if len(sys.argv) > 4 else "Cijk_")


def read(root, sub, counter):
    vals, meta = collections.defaultdict(float), {}
    for f in glob.glob(os.path.join(root, sub, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            name = r.get("Kernel_Name", "")
            if not PAT.search(name) or r.get("Counter_Name") != counter:
                continue
            d = r.get("Dispatch_Id") or r.get("Correlation_Id")
            vals[d] += float(r["Counter_Value"])
            meta[d] = (name[:120], r.get("Grid_Size", "?"))
    return vals, meta


def main():
    root, steps, out = sys.argv[1], int(sys.argv[2]), sys.argv[3]
    fetch, mf = read(root, "fetch", "FETCH_SIZE")
    write, mw = read(root, "write", "WRITE_SIZE")
    groups = collections.defaultdict(lambda: [0, 0.0, 0.0])
    for d, v in fetch.items():
        g = groups[mf[d]]
        g[0] += 1
        g[1] += v
    for d, v in write.items():
        groups[mw[d]][2] += v
    rows = []
    for (name, grid), (n, f, w) in groups.items():
        b = (2 * f + w) * 1024
        rows.append((b, n, name, grid))
    rows.sort(reverse=True)
    total = sum(r[0] for r in rows)
    for b, n, name, grid in rows[:12]:
        print(f"{b / 1e9:9.3f} GB  {n:4d} launches  {b / max(n, 1) / 1e6:9.1f} MB/launch  grid {grid}  {name}")
    res = {"formula": f"(2*FETCH_SIZE + WRITE_SIZE) * 1024 bytes, kernels matching {PAT.pattern!r}", "steps": steps,
           "bytes_per_step": total / max(steps, 1),
           "largest_group": {"kernel": rows[0][2], "grid": rows[0][3], "launches": rows[0][1],
                             "bytes_per_launch": rows[0][0] / max(rows[0][1], 1)} if rows else None}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
