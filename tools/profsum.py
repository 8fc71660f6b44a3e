"""Summarise a rocprofv3 --stats kernel_stats.csv per training step:  python tools/profsum.py CSV STEPS [TOP]
STEPS = 0 counts the steps from the matcher kernel (pdvc::lsap_kernel runs once per training step)."""
import collections
import csv
import sys


def main():
    path, steps = sys.argv[1], float(sys.argv[2])
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 25
    rows = list(csv.DictReader(open(path)))
    if steps <= 0:
        steps = float(sum(int(r["Calls"]) for r in rows if "lsap_kernel" in r["Name"]))
        print(f"steps (lsap_kernel launches): {steps:.0f}")
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    n = sum(int(r["Calls"]) for r in rows)
    print(f"GPU time {tot / 1e6 / steps:.2f} ms/step, {n / steps:.0f} launches/step")
    cat = collections.defaultdict(lambda: [0.0, 0])
    for r in rows:
        name = r["Name"]
        if name.startswith("Cijk"):
            k = "GEMM (hipBLASLt)"
        elif "pdvc::" in name:
            k = name.split("(")[0].replace("void ", "").split("<")[0]
        elif "elementwise" in name:
            k = "torch elementwise"
        elif "reduce_kernel" in name:
            k = "torch reduce"
        elif "layer_norm" in name or "GammaBeta" in name:
            k = "torch layernorm"
        elif "rocclr" in name:
            k = "runtime copy/fill"
        else:
            k = "other: " + name[:50]
        cat[k][0] += float(r["TotalDurationNs"]) / 1e6 / steps
        cat[k][1] += int(r["Calls"]) / steps
    for k, (t, c) in sorted(cat.items(), key=lambda x: -x[1][0])[:top]:
        print(f"{t:7.3f} ms/step {c:7.1f} launches/step  {k}")


if __name__ == "__main__":
    main()
