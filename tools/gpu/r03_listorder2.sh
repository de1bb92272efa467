# C5 one-launch time in a fresh process vs after other scenes were uploaded and traced on the same
# engine first (bench.py's aux order). Usage: bash tools/gpu/r03_listorder2.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-lo}
mkdir -p gpurun_out/$TAG
for pre in "" c4 c2,c4; do
  n=pre_${pre//,/_}
  timeout -k 10 300 python -u tools/exp_c5_list_order.py --config c5 --before "$pre" --only swizzle,swizzle_info,tile64 > gpurun_out/$TAG/$n.json 2> gpurun_out/$TAG/$n.err || { tail -20 gpurun_out/$TAG/$n.err; exit 1; }
  cat gpurun_out/$TAG/$n.json
done
