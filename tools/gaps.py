"""Idle gaps between kernels, per step, from a rocprofv3 kernel trace (eval-line attribution, VERDICT round 5
item 7):  python tools/gaps.py RUN_kernel_trace.csv [CUT_SUBSTRING]
The trace is cut into windows at each launch of CUT_SUBSTRING (default pdvc::lsap_kernel, once per step); per window:
span (first start to last end), summed kernel time, launches, and the largest gap between consecutive kernels with
the kernels on either side."""
import csv
import sys


def main():
    path = [a for a in sys.argv[1:] if not a.startswith("--")][0]
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    cut = args[1] if len(args) > 1 else "lsap_kernel"
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    wins, cur = [], []
    for r in rows:
        if cut in r["Kernel_Name"] and cur:
            wins.append(cur)
            cur = []
        cur.append(r)
    if cur:
        wins.append(cur)
    over1 = 0
    for i, w in enumerate(wins):
        s0, e1 = int(w[0]["Start_Timestamp"]), max(int(r["End_Timestamp"]) for r in w)
        busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in w)
        gap, at, end = 0, 0, int(w[0]["End_Timestamp"])
        n1 = 0
        for j in range(1, len(w)):
            g = int(w[j]["Start_Timestamp"]) - end
            if g > 1_000_000:
                n1 += 1
            if g > gap:
                gap, at = g, j
            end = max(end, int(w[j]["End_Timestamp"]))
        over1 += n1
        if "--all" in sys.argv:
            end = int(w[0]["End_Timestamp"])
            for j in range(1, len(w)):
                g = int(w[j]["Start_Timestamp"]) - end
                if g > 1_000_000:
                    print(f"      gap {g / 1e6:7.2f} ms after launch {j - 1}: "
                          f"{w[j - 1]['Kernel_Name'].split('(')[0][:60]} -> {w[j]['Kernel_Name'].split('(')[0][:60]}")
                end = max(end, int(w[j]["End_Timestamp"]))
        name = lambda r: r["Kernel_Name"].split("(")[0].replace("void ", "")[:70]  # noqa: E731
        print(f"window {i:2d}: span {(e1 - s0) / 1e6:8.2f} ms  kernels {busy / 1e6:8.2f} ms  launches {len(w):5d}  "
              f"largest gap {gap / 1e6:7.2f} ms after launch {at - 1} ({name(w[at - 1]) if at else '-'} -> "
              f"{name(w[at]) if at else '-'})  gaps > 1 ms: {n1}")
    print(f"gaps > 1 ms over all windows: {over1}")


if __name__ == "__main__":
    main()
