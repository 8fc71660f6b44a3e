"""Every gemm3 launch of one replayed step, from a rocprofv3 kernel trace of bench.py (diagnostic):
    python tools/g3launches.py RUN_kernel_trace.csv
The trace is cut at the matcher kernel (pdvc::lsap_kernel, once per step) as tools/profsteps.py does; the modal
launch-count windows are the replays; for the median replay window every gemm3 / slab launch is listed with its
template arguments, grid and duration, then totals per template."""
import collections
import csv
import re
import statistics
import sys


def main():
    rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
    wins, cur = [], []
    for r in rows:
        if "lsap_kernel" in r["Kernel_Name"] and cur:
            wins.append(cur)
            cur = []
        cur.append(r)
    counts = collections.Counter(len(w) for w in wins[1:])
    modal = counts.most_common(1)[0][0]
    reps = [w for w in wins[1:] if len(w) == modal]
    tot = [sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in w) for w in reps]
    w = reps[sorted(range(len(reps)), key=lambda i: tot[i])[len(reps) // 2]]
    per = collections.defaultdict(lambda: [0, 0.0])
    print(f"{len(reps)} replay windows of {modal} launches; median window:")
    for r in w:
        n = r["Kernel_Name"]
        if "g3::" not in n:
            continue
        short = re.sub(r"\(.*", "", n).replace("void ", "").replace("pdvc::g3::", "")
        us = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        grid = r.get("Grid_Size_X") or r.get("Grid_Size") or "?"
        print(f"  {us:9.1f} us  grid {grid:>8}  {short}")
        per[short][0] += 1
        per[short][1] += us
    print("per template:")
    for k, (c, us) in sorted(per.items(), key=lambda kv: -kv[1][1]):
        print(f"  {us / 1e3:8.3f} ms  {c:4d} launches  {k}")


if __name__ == "__main__":
    main()
