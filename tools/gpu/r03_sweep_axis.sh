# Randomized parity sweep with degenerate directions (parity_sweep.py "axis" mode): plain and with the
# trace variants + adaptive order. Usage: bash tools/gpu/r03_sweep_axis.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-sweep_axis}
mkdir -p gpurun_out/$TAG
timeout -k 10 700 python -u tools/parity_sweep.py ${N:-300} 40000 axis > gpurun_out/$TAG/sweep_${N:-300}_axis.txt 2>&1 || { tail -5 gpurun_out/$TAG/sweep_${N:-300}_axis.txt; exit 1; }
tail -1 gpurun_out/$TAG/sweep_${N:-300}_axis.txt
timeout -k 10 700 python -u tools/parity_sweep.py ${N:-300} 50000 axis,variants,adaptive > gpurun_out/$TAG/sweep_${N:-300}_axis_var_adaptive.txt 2>&1 || { tail -5 gpurun_out/$TAG/sweep_${N:-300}_axis_var_adaptive.txt; exit 1; }
tail -1 gpurun_out/$TAG/sweep_${N:-300}_axis_var_adaptive.txt
