# Everything the committed profiles/ come from, in two GPU calls:
#   part a: tests, the default bench line (with CPU baseline + PCIe-inclusive
#           rate), a kernel-trace profile of the same command, PMC
#           traffic / instruction passes (pmc1..3: tools/pmc_traffic.py);
#   part b: the other BASELINE configs (C1, C3 + its kernel trace, C5), two
#           sessions in rotation, and a two-rank rehearsal on one device.
# usage: bash tools/round_evidence.sh TAG a|b
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-round}
P=${2:-a}
O=gpurun_out/$T
mkdir -p $O
if [ "$P" = a ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -u bench.py > $O/bench.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-pcie > $O/prof.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmc/pmc1 -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-pcie > $O/pmc1.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/pmc/pmc2 -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-pcie > $O/pmc2.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD --kernel-trace --output-format csv -d $O/pmc/pmc3 -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-pcie > $O/pmc3.log 2>&1
else
timeout -k 10 300 python -u bench.py --config c1 --steps 50 --warmup 5 > $O/c1.log 2>&1 && \
timeout -k 10 300 python -u bench.py --config c3 --steps 3 --warmup 1 > $O/c3.log 2>&1 && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c3prof -o run -- python3 bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline > $O/c3prof.log 2>&1 && \
timeout -k 10 300 python -u bench.py --config c5 --steps 5 --warmup 1 > $O/c5.log 2>&1 && \
timeout -k 10 300 python -u bench.py --pipeline 2 --no-cpu-baseline --no-pcie > $O/pipe2.log 2>&1 && \
KMERHIP_ONE_DEVICE=1 KMERHIP_DIST_BACKEND=gloo KMERHIP_BENCH_VERIFY=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --reads 1000000 --steps 5 --warmup 1 > $O/rehearse2.log 2>&1
fi
