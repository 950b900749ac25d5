#!/bin/bash
# One bench line per BASELINE config and per ordered path of the round (1 GPU):
# gpurun_out/TAG/NAME.json (the JSON line) + NAME.log.  Summarised into
# DESIGN.md §8 and copied to profiles/ (rNN_benches.jsonl).
# usage: tools/round_benches.sh TAG
set -u
cd "$(dirname "$0")/.."
TAG=$1
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
run() {
    local name=$1
    shift
    timeout -k 10 400 python bench.py "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    grep '^{' "$OUT/$name.log" > "$OUT/$name.json" || true
    echo "$name rc=$rc"
    [ $rc -eq 0 ] || exit $rc
}
run c2
run c1 --config c1 --steps 5 --warmup 1
run c3 --config c3 --steps 5 --warmup 1
run c4 --config c4 --steps 10 --warmup 2
run c5 --config c5 --steps 10 --warmup 2
run c5_ordered --config c5 --ordered --steps 10 --warmup 2
run c5_fasta --config c5 --fasta --steps 10 --warmup 2
run k40 --k 40 --steps 10 --warmup 2 --no-cpu-baseline
run k64_AT --k 64 --prefix AT --reads 2000000 --steps 3 --warmup 1 --no-cpu-baseline
run k16_AT --prefix AT --steps 5 --warmup 1 --no-cpu-baseline
run k21_noprefix --k 21 --prefix "" --reads 4000000 --steps 5 --warmup 1 --no-cpu-baseline
run k70 --k 70 --steps 10 --warmup 2 --no-cpu-baseline
run k150 --k 150 --steps 10 --warmup 2 --no-cpu-baseline
run k40_noprefix --k 40 --prefix "" --reads 1000000 --steps 3 --warmup 1 --no-cpu-baseline
exit 0
