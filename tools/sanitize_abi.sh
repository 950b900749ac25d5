#!/bin/bash
# Host-side ASan + UBSan run of the C-ABI on the GPU box:
# tools/sanitize/build/abi_driver over the golden inputs -- one context, a
# 3-way device group (threads), and kmer_count_file in small batches must give
# equal results with no sanitizer report.  Build first (here, on the CPU):
#   make -j4 -C tools/sanitize
set -o pipefail
cd "$(dirname "$0")/.."
export ASAN_OPTIONS=detect_leaks=0:abort_on_error=1:verify_asan_link_order=0
export UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1
timeout -k 10 600 tools/sanitize/build/abi_driver tests/golden/inputs/*.fastq tests/golden/inputs/*.fsa
