# Larger randomized parity sweeps of the final kernels: 1500 plain cases + 1500 with the trace variants and the adaptive order.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-sweepbig}
mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -u tools/parity_sweep.py 1500 40000 > gpurun_out/$TAG/sweep_1500_plain.txt 2>&1 || { tail -5 gpurun_out/$TAG/sweep_1500_plain.txt; exit 1; }
tail -1 gpurun_out/$TAG/sweep_1500_plain.txt
timeout -k 10 600 python -u tools/parity_sweep.py 1500 42000 variants,adaptive > gpurun_out/$TAG/sweep_1500_var_adaptive.txt 2>&1 || { tail -5 gpurun_out/$TAG/sweep_1500_var_adaptive.txt; exit 1; }
tail -1 gpurun_out/$TAG/sweep_1500_var_adaptive.txt
