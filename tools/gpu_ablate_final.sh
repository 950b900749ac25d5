set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-abl}
mkdir -p $O
for a in 0 1 2 3; do
  KMERHIP_TAB_ABLATE=$a timeout -k 10 200 python -u bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline --no-pcie > $O/c5_a$a.log 2>&1 || exit $?
  KMERHIP_TAB_ABLATE=$a timeout -k 10 200 python -u bench.py --config c3 --reads 25000000 --steps 2 --warmup 1 --no-cpu-baseline --no-pcie --no-e2e > $O/c3_a$a.log 2>&1 || exit $?
  echo "ablate $a done"
done
