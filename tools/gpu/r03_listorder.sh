# tools/exp_c5_list_order.py on C5, C4, C2. Usage: bash tools/gpu/r03_listorder.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-lo}
mkdir -p gpurun_out/$TAG
for c in c5 c4 c2; do
  timeout -k 10 300 python -u tools/exp_c5_list_order.py --config $c > gpurun_out/$TAG/$c.json 2> gpurun_out/$TAG/$c.err || { tail -20 gpurun_out/$TAG/$c.err; exit 1; }
  cat gpurun_out/$TAG/$c.json
done
