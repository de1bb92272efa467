# A/B of lib/variants/*.so on one config. Usage: bash tools/gpu/r03_variants.sh TAG CFG "names..."
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=$1; CFG=${2:-c2}; shift 2
mkdir -p gpurun_out/var
RV_CFG=$CFG RV_RECUR=${RV_RECUR:-1} timeout -k 10 900 python -u tools/run_variants.py $@ 2>&1 | tee gpurun_out/var/$TAG.txt
