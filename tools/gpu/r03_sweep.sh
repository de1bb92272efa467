# Randomized parity sweep of the final kernels (one-wave blocks): plain, and variants + adaptive order.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-sweep}
mkdir -p gpurun_out/$TAG
timeout -k 10 500 python -u tools/parity_sweep.py 300 30000 > gpurun_out/$TAG/sweep_300_plain.txt 2>&1 || { tail -5 gpurun_out/$TAG/sweep_300_plain.txt; exit 1; }
tail -2 gpurun_out/$TAG/sweep_300_plain.txt
timeout -k 10 500 python -u tools/parity_sweep.py 300 31000 variants,adaptive > gpurun_out/$TAG/sweep_300_var_adaptive.txt 2>&1 || { tail -5 gpurun_out/$TAG/sweep_300_var_adaptive.txt; exit 1; }
tail -2 gpurun_out/$TAG/sweep_300_var_adaptive.txt
