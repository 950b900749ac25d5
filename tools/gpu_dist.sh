set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/exp_dist.py > gpurun_out/exp_dist.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_dist -o run -- python -u tools/exp_dist.py --steps 5 > gpurun_out/prof_dist.log 2>&1
