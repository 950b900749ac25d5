#!/bin/bash
# round-6 PMC traffic (one counter group per pass, kernel trace only) of C2, C3, C5, C5 FASTA
set -o pipefail
bash tools/pmc_traffic.sh r06_pmc_c2 --config c2 || exit $?
bash tools/pmc_traffic.sh r06_pmc_c5 --config c5 --no-e2e --no-match --no-pipelined || exit $?
bash tools/pmc_traffic.sh r06_pmc_c5fa --config c5 --fasta --no-e2e --no-match --no-pipelined || exit $?
bash tools/pmc_traffic.sh r06_pmc_c3 --config c3 --no-e2e --no-match --no-pipelined || exit $?
