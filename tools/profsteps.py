"""Per-step device time of the REPLAYED steps only, from a rocprofv3 kernel trace of `bench.py`:
    python tools/profsteps.py RUN_kernel_trace.csv [TOP]

tools/profsum.py divides the run's totals by its step count, which mixes the capture's eager warm-up steps and the
eager steps bench.py times its kernels in with the graph replays.  Here the trace is cut at the matcher kernel
(pdvc::lsap_kernel, once per step): each window from one matcher launch to the next is one whole step (its losses
and backward, the eager clip and AdamW, the next step's forward).  The windows of consecutive replays have the
same launch count; the modal count picks them, and the report is the median window by category (the GEMMs,
every other kernel), with the per-kernel breakdown of the median window."""
import collections
import csv
import statistics
import sys


def category(name):
    if name.startswith("Cijk"):
        return "GEMM (hipBLASLt)"
    if "pdvc::" in name:
        return name.split("(")[0].replace("void ", "").split("<")[0]
    if "elementwise" in name:
        return "torch elementwise"
    if "reduce_kernel" in name:
        return "torch reduce"
    if "rocclr" in name:
        return "runtime copy/fill"
    return "other: " + name[:50]


def main():
    path = sys.argv[1]
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 30
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    cuts = [i for i, r in enumerate(rows) if "lsap_kernel" in r["Kernel_Name"]]
    wins = [rows[a:b] for a, b in zip(cuts, cuts[1:])]
    mode = collections.Counter(len(w) for w in wins).most_common(1)[0][0]
    rep = [w for w in wins if len(w) == mode]
    print(f"{len(wins)} step windows; {len(rep)} with the modal {mode} launches (the replays)")

    def dur(r):
        return (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6

    tot, gemm = [], []
    for w in rep:
        tot.append(sum(dur(r) for r in w))
        gemm.append(sum(dur(r) for r in w if r["Kernel_Name"].startswith("Cijk") or "pdvc::g3::" in r["Kernel_Name"]))
    med = statistics.median(tot)
    print(f"device time per replayed step: median {med:.2f} ms (min {min(tot):.2f}, max {max(tot):.2f})")
    print(f"  GEMM (gemm3 + hipBLASLt) {statistics.median(gemm):.2f} ms, non-GEMM {statistics.median([t - g for t, g in zip(tot, gemm)]):.2f} ms")
    w = rep[sorted(range(len(rep)), key=lambda i: tot[i])[len(rep) // 2]]
    cat = collections.defaultdict(lambda: [0.0, 0])
    for r in w:
        k = category(r["Kernel_Name"])
        cat[k][0] += dur(r)
        cat[k][1] += 1
    for k, (t, c) in sorted(cat.items(), key=lambda x: -x[1][0])[:top]:
        print(f"{t:8.3f} ms {c:5d} launches  {k}")


if __name__ == "__main__":
    main()
