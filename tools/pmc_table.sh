#!/bin/bash
# Where the table-mode kernels' waves spend their time (SQ counter passes, one
# group per pass, kernel trace only).  usage: tools/pmc_table.sh TAG [bench args, e.g. --config c5]
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
  timeout -s KILL 150 rocprofv3 --pmc $c --kernel-trace --output-format csv -d "$OUT/pmc$i" -o run -- \
      python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-pcie --no-e2e --no-match --no-pipelined "$@" > "$OUT/pmc$i.log" 2>&1
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
        if "tab_" not in k:
            continue
        agg[k.split("(")[0][-40:]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    m = {c: sum(x) / len(x) for c, x in d.items()}
    print(k)
    for c in sorted(m):
        print("  %-24s %.4g" % (c, m[c]))
    w = m.get("SQ_WAVES", 0)
    if w and "SQ_INSTS_VALU" in m:
        print("  per wave: VALU %.1f SALU %.1f LDS %.1f VMEM_RD %.1f VMEM_WR %.1f" % (
            m["SQ_INSTS_VALU"] / w, m["SQ_INSTS_SALU"] / w, m["SQ_INSTS_LDS"] / w, m["SQ_INSTS_VMEM_RD"] / w,
            m["SQ_INSTS_VMEM_WR"] / w))
PY
