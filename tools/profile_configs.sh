#!/bin/bash
# rocprofv3 evidence for profiles/ (run on the GPU box): kernel traces of the
# timed steps of C2 / C3 / C4 / C5 / C5 in FASTA mode / k = 70 (general path)
# (tools/kernel_stats.py) -- kernel trace only.
# usage: tools/profile_configs.sh TAG [configs...]
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
TAG=$1; shift
O=gpurun_out/$TAG
mkdir -p $O
NOX="--no-cpu-baseline --no-pcie --no-e2e --no-pipelined --no-match"
for cfg in "$@"; do
  case $cfg in
    c2) W=3; K=20; A="--config c2" ;;
    c3) W=1; K=3; A="--config c3" ;;
    c4) W=1; K=5; A="--config c4" ;;
    c5) W=1; K=5; A="--config c5" ;;
    c5fa) W=1; K=5; A="--config c5 --fasta" ;;
    k70) W=1; K=5; A="--k 70" ;;
    k16AT) W=1; K=5; A="--prefix AT" ;;
    k64AT) W=1; K=3; A="--k 64 --prefix AT --reads 2000000" ;;
  esac
  timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/trace_$cfg -o run -- \
      python3 bench.py --steps $K --warmup $W $NOX $A > $O/trace_$cfg.log 2>&1 || exit $?
  python3 tools/kernel_stats.py $O/trace_$cfg $W $K $O/${cfg}_kernel_stats.csv || exit $?
  # the bench line of the SAME run (HIP events) next to rocprof's average of
  # its dominant kernel over the same timed steps
  python3 - $O/trace_$cfg.log $O/${cfg}_kernel_stats.csv $O/${cfg}_check.json <<'PY' || exit $?
import csv, json, sys
line = [l for l in open(sys.argv[1]) if l.startswith("{")][-1]
b = json.loads(line)
kname = b["roofline"]["kernel"].split(" (")[0]
rows = {r["kernel"]: r for r in csv.DictReader(open(sys.argv[2]))}
parts = [k.strip() for k in kname.split(" + ")]
avg = sum(float(rows[k]["avg_us"]) for k in parts if k in rows) / 1e3 if all(k in rows for k in parts) else None
out = {"bench_kernel": kname, "bench_kernel_ms_events": b["roofline"]["kernel_ms"], "rocprof_avg_ms": avg,
       "ratio": (avg / b["roofline"]["kernel_ms"]) if avg else None, "ms_per_step": b["ms_per_step"],
       "algorithmic_bytes_per_launch": b["roofline"]["algorithmic_bytes_per_launch"],
       "frac_events": b["roofline"]["frac"],
       "frac_rocprof": (b["roofline"]["algorithmic_bytes_per_launch"] / (avg * 1e-3) / 1e9 / b["roofline"]["peak"]) if avg else None}
json.dump(out, open(sys.argv[3], "w"), indent=1)
print(out)
PY
  echo "$cfg trace done"
done
