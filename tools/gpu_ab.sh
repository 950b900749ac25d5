# A/B: the in-tree library vs ab/<variant>.so on a bench config, each variant
# first checked on the golden / synthetic / realistic parity tests;
# extra bench arguments in $BENCH_ARGS, the test selection in $AB_TESTS
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1; shift
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-pcie $BENCH_ARGS > gpurun_out/ab_${TAG}_base.log 2>&1 || exit $?
for v in "$@"; do
  cp ab/$v.so kmerjs_amd/libkmerhip.so && \
  timeout -k 10 400 python -u -m pytest ${AB_TESTS:-tests/test_gpu_parity.py -k "every_golden or synthetic_vs_oracle or realistic or full_size_properties"} \
      -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/ab_${TAG}_${v}_pytest.log 2>&1 && \
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-pcie $BENCH_ARGS > gpurun_out/ab_${TAG}_$v.log 2>&1 || exit $?
done
