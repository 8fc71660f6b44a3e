"""Per-kernel averages of rocprofv3 --pmc counters from one or more pass directories (diagnostic):
    python tools/pmc_counters.py DIR [KERNEL_SUBSTRING]
Every *counter_collection.csv under DIR is read; counters are summed per dispatch (over dimensions), then
averaged over the dispatches of each (kernel, grid size)."""
import collections
import csv
import glob
import os
import sys


def main():
    root = sys.argv[1]
    ksub = sys.argv[2] if len(sys.argv) > 2 else ""
    per = collections.defaultdict(lambda: collections.defaultdict(float))  # (kernel, grid, dispatch) -> counter
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r.get("Kernel_Name", "")
            if ksub not in k:
                continue
            key = (k.split("(")[0].replace("void ", "")[:60], r.get("Grid_Size", "?"),
                   r.get("Dispatch_Id") or r.get("Correlation_Id"))
            per[key][r["Counter_Name"]] += float(r["Counter_Value"])
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for (k, g, _), cs in per.items():
        for c, v in cs.items():
            agg[(k, g)][c].append(v)
    for (k, g), cs in sorted(agg.items()):
        print(f"{k}  grid={g}")
        for c, vs in sorted(cs.items()):
            print(f"    {c:36s} {sum(vs) / len(vs):16.4g}   (n={len(vs)})")


if __name__ == "__main__":
    main()
