#!/bin/bash
# round-6 rocprof evidence: kernel traces of the timed steps + bench lines of the same runs, C2 step timeline
set -o pipefail
bash tools/profile_configs.sh r06_ev2 c2 c3 c5 c5fa k16AT k64AT || exit $?
python3 tools/trace_step.py $(find gpurun_out/r06_ev2/trace_c2 -name "*kernel_trace.csv" | head -1) 5 > gpurun_out/r06_ev2/c2_step_timeline.txt || exit $?
python3 tools/trace_step.py $(find gpurun_out/r06_ev2/trace_c5 -name "*kernel_trace.csv" | head -1) 3 tab_sort_final > gpurun_out/r06_ev2/c5_step_timeline.txt || exit $?
