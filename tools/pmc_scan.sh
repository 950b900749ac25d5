#!/bin/bash
# Where the C2 scan kernel's waves spend their time: SQ counter passes (one
# group per pass, kernel trace only).  usage: tools/pmc_scan.sh TAG [bench args]
set -u
cd "$(dirname "$0")/.."
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
for c in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA" \
         "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace --output-format csv -d "$OUT/pmc$i" -o run -- \
      python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-pcie --no-e2e --no-match --no-pipelined "$@" > "$OUT/pmc$i.log" 2>&1
  rc=$?; echo "pmc pass $i rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(out + "/pmc*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r.get("Kernel_Name", "")
        if "scan_planes" not in k and "hit_kernel" not in k:
            continue
        agg[k.split("(")[0][-40:]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    print(k)
    for c, v in sorted(d.items()):
        print("  %-24s %.4g (per dispatch, %d samples)" % (c, sum(v) / max(1, len(v)) * (len(v) / max(1, len(set(v))) if False else 1), len(v)))
PY
