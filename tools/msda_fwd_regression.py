"""Summary of tools/msda_fwd_regression.sh: per arm and kernel, the average duration (kernel trace of the PMC
pass), effective clock GRBM_GUI_ACTIVE / 8 / duration, and the other counters averaged per dispatch.
    python tools/msda_fwd_regression.py gpurun_out/TAG"""
import collections
import csv
import glob
import os
import sys


def arm_stats(d):
    out = collections.defaultdict(lambda: collections.defaultdict(list))
    for p in sorted(glob.glob(os.path.join(d, "p*"))):
        dur = {}
        for f in glob.glob(os.path.join(p, "**", "*kernel_trace.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                dur[r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3  # us
        per = collections.defaultdict(lambda: collections.defaultdict(float))
        names = {}
        for f in glob.glob(os.path.join(p, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                k = r["Kernel_Name"].split("(")[0].replace("void ", "").split("<")[0].split("::")[-1]
                did = r.get("Dispatch_Id")
                names[did] = (k, r.get("Grid_Size"))
                per[did][r["Counter_Name"]] += float(r["Counter_Value"])
        for did, cs in per.items():
            key = names[did]
            if did in dur:
                out[key]["dur_us"].append(dur[did])
                if "GRBM_GUI_ACTIVE" in cs:
                    out[key]["clock_GHz"].append(cs["GRBM_GUI_ACTIVE"] / 8 / (dur[did] * 1e3))
            for c, v in cs.items():
                out[key][c].append(v)
    return out


def main():
    root = sys.argv[1]
    for arm in ("standalone", "step", "step_nog3"):
        d = os.path.join(root, arm)
        if not os.path.isdir(d):
            continue
        print(f"== {arm}")
        for (k, g), cs in sorted(arm_stats(d).items()):
            if not cs.get("dur_us"):
                continue
            print(f"  {k} grid={g}")
            for c in ["dur_us", "clock_GHz"] + sorted(x for x in cs if x not in ("dur_us", "clock_GHz")):
                v = cs.get(c)
                if v:
                    print(f"      {c:36s} {sum(v) / len(v):14.4g}  (n={len(v)})")


if __name__ == "__main__":
    main()
