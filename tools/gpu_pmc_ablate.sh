set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for f in 0 256 1024; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_SMEM --kernel-trace --output-format csv -d gpurun_out/pmcab_$f -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-pcie --flags $f > gpurun_out/pmcab_$f.log 2>&1 || exit $?
done
