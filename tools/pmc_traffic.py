"""HBM traffic per launch of one kernel from two rocprofv3 --pmc passes (MI355X_MICROARCH.md section HBM):
    rocprofv3 --pmc FETCH_SIZE --kernel-include-regex K --output-format csv -d DIR/fetch -- python bench.py ...
    rocprofv3 --pmc WRITE_SIZE --kernel-include-regex K --output-format csv -d DIR/write -- python bench.py ...
    python tools/pmc_traffic.py DIR KERNEL_SUBSTRING OUT.json [--largest-grid | --large-launches]
FETCH_SIZE and WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE counts half the bytes of a wide (16 B/lane)
stream, so traffic = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 -- the kernels priced here read their value rows
with 16-B loads.  Launches are grouped by grid size (encoder vs decoder calls) and averaged; --largest-grid prices
only the group of the largest grid; --large-launches only the launches whose FETCH_SIZE is at least half the
largest (the encoder's launches of a kernel both call sites launch on the same grid, e.g. the value-gradient
kernel, one workgroup per (video, head, level) for the encoder and the decoder alike)."""
import collections
import csv
import glob
import json
import os
import sys


def read(path_glob, counter, kname):
    vals = collections.defaultdict(float)  # dispatch id -> value
    grid = {}
    for f in glob.glob(path_glob, recursive=True):
        for r in csv.DictReader(open(f)):
            if kname not in r.get("Kernel_Name", "") or r.get("Counter_Name") != counter:
                continue
            d = r.get("Dispatch_Id") or r.get("Correlation_Id")
            vals[d] += float(r["Counter_Value"])
            grid[d] = r.get("Grid_Size", "?")
    return vals, grid


def main():
    root, kname, out = sys.argv[1], sys.argv[2], sys.argv[3]
    fetch, grid_f = read(os.path.join(root, "fetch", "**", "*counter_collection.csv"), "FETCH_SIZE", kname)
    write, grid_w = read(os.path.join(root, "write", "**", "*counter_collection.csv"), "WRITE_SIZE", kname)
    by_grid = collections.defaultdict(lambda: {"fetch_kib": [], "write_kib": []})
    for d, v in fetch.items():
        by_grid[grid_f[d]]["fetch_kib"].append(v)
    for d, v in write.items():
        by_grid[grid_w[d]]["write_kib"].append(v)
    res = {"kernel": kname, "formula": "(2*FETCH_SIZE + WRITE_SIZE) * 1024 bytes per launch", "by_grid": {}}
    total, n = 0.0, 0
    for g, v in sorted(by_grid.items()):
        f = sum(v["fetch_kib"]) / max(len(v["fetch_kib"]), 1)
        w = sum(v["write_kib"]) / max(len(v["write_kib"]), 1)
        b = (2 * f + w) * 1024
        res["by_grid"][g] = {"launches": len(v["fetch_kib"]), "fetch_kib": f, "write_kib": w, "bytes": b}
        total += b * len(v["fetch_kib"])
        n += len(v["fetch_kib"])
    res["avg_bytes_per_launch"] = total / max(n, 1)
    if "--large-launches" in sys.argv and fetch:
        top = max(fetch.values())
        sel = [d for d, v in fetch.items() if v >= 0.5 * top and d in write]
        b = sum((2 * fetch[d] + write[d]) * 1024 for d in sel) / max(len(sel), 1)
        res["large_launches"] = {"launches": len(sel), "bytes": b}
        res["avg_bytes_per_launch"] = b
    if "--largest-grid" in sys.argv and res["by_grid"]:
        g = max(res["by_grid"], key=lambda k: int(k) if str(k).isdigit() else -1)
        res["avg_bytes_per_launch"] = res["by_grid"][g]["bytes"]
        res["priced_grid"] = g
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
