# A/B of SQ instruction counters (one PMC pass each): in-tree library vs exp/<variant>.so
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1; shift
cp kmerjs_amd/libkmerhip.so exp/_base.so
for v in _base "$@"; do
  cp exp/$v.so kmerjs_amd/libkmerhip.so && \
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-pcie > gpurun_out/ab_${TAG}_$v.log 2>&1 && \
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_SMEM --kernel-trace --output-format csv -d gpurun_out/pmc_${TAG}_$v -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-pcie > gpurun_out/pmc_${TAG}_$v.log 2>&1 || exit $?
done
