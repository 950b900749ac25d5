#!/bin/bash
# round-6 final evidence, part 1: GPU suite + smoke + default bench, then kernel traces of C2 / C3 / C5 / C5 FASTA
set -o pipefail
bash tools/round_evidence.sh r06_fin || exit $?
bash tools/profile_configs.sh r06_fin c2 c3 c5 c5fa || exit $?
python3 tools/trace_step.py $(find gpurun_out/r06_fin/trace_c2 -name "*kernel_trace.csv" | head -1) 5 > gpurun_out/r06_fin/c2_step_timeline.txt || exit $?
python3 tools/trace_step.py $(find gpurun_out/r06_fin/trace_c5 -name "*kernel_trace.csv" | head -1) 3 tab_sort_final > gpurun_out/r06_fin/c5_step_timeline.txt || exit $?
