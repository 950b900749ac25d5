"""Per-kernel duration statistics of the TIMED steps of a bench.py run under
`rocprofv3 --kernel-trace` (profiles/ evidence).

bench.py runs W warmup steps, K timed steps, then one more step (E = 1) that
reads the result size outside the timed region; with its side legs switched
off (--no-pcie --no-e2e --no-pipelined --no-match --no-cpu-baseline) every
kernel is dispatched the same number of times per step, so the timed steps are
the K x per dispatches before the last E x per, per = (dispatches - E) /
(W + K).  Kernels whose count does not fit that are flagged (not exact).

usage: python tools/kernel_stats.py TRACE_DIR WARMUP STEPS [out.csv] [E]
"""
import csv
import glob
import re
import statistics
import sys
from collections import defaultdict

root, W, K = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
out = sys.argv[4] if len(sys.argv) > 4 else None
E = int(sys.argv[5]) if len(sys.argv) > 5 else 1
rows = []
for path in glob.glob(root + "/**/*kernel_trace.csv", recursive=True):
    rows += list(csv.DictReader(open(path)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
by = defaultdict(list)
for r in rows:
    m = re.findall(r"kmerhip::(?:\(anonymous namespace\)::)?(\w+)", r["Kernel_Name"])
    name = m[0] if m else r["Kernel_Name"].split("(")[0][:60]
    by[name].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)   # us
res = []
for name, d in by.items():
    n = len(d)
    # (bench.py may dispatch a kernel once more before its warmup: e.g. a
    # verification count; the timed steps are still the LAST ones)
    # (bench.py's extra pass after the timed steps -- the result-size read --
    # dispatches E = 1 more step's kernels: the timed window ends before it)
    per = (n - E) // (W + K)
    exact = per > 0 and (n - E) % (W + K) == 0
    take = d[n - E - per * K:n - E] if per else d
    res.append({"kernel": name, "dispatches_total": n, "dispatches_timed": len(take),
                "timed_window_exact": exact, "avg_us": statistics.mean(take), "min_us": min(take),
                "max_us": max(take), "stdev_us": statistics.pstdev(take), "sum_us": sum(take)})
res.sort(key=lambda x: -x["sum_us"])
w = csv.DictWriter(open(out, "w") if out else sys.stdout, fieldnames=list(res[0].keys()))
w.writeheader()
for x in res:
    w.writerow({k: (round(v, 2) if isinstance(v, float) else v) for k, v in x.items()})
