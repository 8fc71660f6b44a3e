"""Device time per eval step by kernel, from a rocprofv3 kernel trace of bench.py --mode eval (the trace cut into
steps at the matcher's lsap_kernel, the middle windows averaged; library GEMMs grouped):
    python tools/evalbreak.py RUN_kernel_trace.csv [TOP]"""
import collections
import csv
import sys


def main():
    path = sys.argv[1]
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 25
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    wins, cur = [], []
    for r in rows:
        if "lsap_kernel" in r["Kernel_Name"] and cur:
            wins.append(cur)
            cur = []
        cur.append(r)
    wins.append(cur)
    mid = wins[len(wins) // 3: len(wins) - 1] or wins
    agg = collections.defaultdict(lambda: [0.0, 0.0])
    for w in mid:
        for r in w:
            n = r["Kernel_Name"]
            key = "GEMM (hipBLASLt)" if n.startswith("Cijk") else n.split("(")[0][:90]
            agg[key][0] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 / len(mid)
            agg[key][1] += 1.0 / len(mid)
    print("%d step windows averaged; device time per step %.2f ms" % (len(mid), sum(v[0] for v in agg.values())))
    for k, v in sorted(agg.items(), key=lambda kv: -kv[1][0])[:top]:
        print("%9.3f ms %7.1f launches  %s" % (v[0], v[1], k))


if __name__ == "__main__":
    main()
