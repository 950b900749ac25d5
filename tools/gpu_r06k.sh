#!/bin/bash
# C5 step timeline (kernel trace of the bench), anchored on the sort final
set -o pipefail
O=gpurun_out/r06k
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace_c5 -o tr -- python bench.py --config c5 --steps 6 --warmup 2 --no-cpu-baseline --no-pcie --no-e2e --no-match --no-pipelined > $O/c5.json 2> $O/c5.err || exit $?
python3 tools/trace_step.py $(find $O/trace_c5 -name "*kernel_trace.csv" | head -1) 4 tab_sort_final > $O/c5_step_timeline.txt || exit $?
