#!/bin/bash
# kernel times of the C2 step with deferred verification
set -o pipefail
O=gpurun_out/r06v
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o tr -- python bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-pcie --no-e2e --no-match --no-pipelined > $O/c2.json 2> $O/c2.err || exit $?
python3 tools/trace_step.py $(find $O/tr -name "*kernel_trace.csv" | head -1) 4 > $O/c2_timeline.txt || exit $?
