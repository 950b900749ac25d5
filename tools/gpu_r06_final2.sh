#!/bin/bash
# round-6 final evidence, part 2: PMC traffic of C3 / C5 / C5 FASTA (one counter group per pass), every config's bench line
set -o pipefail
bash tools/pmc_traffic.sh r06f_pmc_c5 --config c5 --no-e2e --no-match --no-pipelined || exit $?
bash tools/pmc_traffic.sh r06f_pmc_c5fa --config c5 --fasta --no-e2e --no-match --no-pipelined || exit $?
bash tools/pmc_traffic.sh r06f_pmc_c3 --config c3 --no-e2e --no-match --no-pipelined || exit $?
bash tools/round_benches.sh r06f_rb || exit $?
