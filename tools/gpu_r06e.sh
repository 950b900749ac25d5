#!/bin/bash
# round 6: rocprof kernel statistics on the current code (C2 + step timeline, k16/AT, C5, C3)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06e
mkdir -p $O
bash tools/profile_configs.sh r06e c2 k16AT k64AT c5 c3 > $O/profile.log 2>&1 || exit $?
python3 tools/trace_step.py $(find gpurun_out/r06e/trace_c2 -name "*kernel_trace.csv" | head -1) 5 > $O/c2_step_timeline.txt || exit $?
