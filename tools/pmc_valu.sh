#!/bin/bash
# VALU / SALU / LDS instruction counts of the C2 scan kernel (one PMC pass):
# shipping build, then the experiments build with the candidate phase ablated
# (KMERHIP_XFLAG_ABLATE_HITS = --flags 256).  usage: tools/pmc_valu.sh TAG
set -u
cd "$(dirname "$0")/.."
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
C="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"
B="bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-pcie --no-e2e --no-match --no-pipelined"
timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace --output-format csv -d "$OUT/ship" -o run -- python3 $B > "$OUT/ship.log" 2>&1 || exit 1
KMERHIP_LIB_EXPERIMENT=kmerjs_amd/libkmerhip_exp.so timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace --output-format csv \
    -d "$OUT/abl" -o run -- python3 $B --flags 256 > "$OUT/abl.log" 2>&1 || exit 1
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections, json
out = sys.argv[1]
for v in ("ship", "abl"):
    agg = collections.defaultdict(list)
    for f in glob.glob(out + "/%s/**/*counter_collection.csv" % v, recursive=True):
        for r in csv.DictReader(open(f)):
            if "scan_planes_kernel" in r.get("Kernel_Name", ""):
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    d = {c: sum(x) / len(x) for c, x in agg.items()}
    w = d.get("SQ_WAVES", 1)
    print(v, " ".join("%s=%.4g" % (c, d[c]) for c in sorted(d)), "| per wave: VALU %.1f SALU %.1f LDS %.1f" % (
        d["SQ_INSTS_VALU"] / w, d["SQ_INSTS_SALU"] / w, d["SQ_INSTS_LDS"] / w))
for v in ("ship", "abl"):
    j = open(out + "/%s.log" % v).read().strip().splitlines()
    for ln in j:
        if ln.startswith("{"):
            d = json.loads(ln); print(v, "scan_ms %.4f" % d["scan_kernel_ms"])
PY
