# C5 one launch with Generate's MaxBounce 0 / 1 / 2 (the jitter hash seed). Usage: bash tools/gpu/r03_c5mb.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-c5mb}
mkdir -p gpurun_out/$TAG
for mb in 0 1 2; do
  timeout -k 10 300 python -u tools/exp_c5_list_order.py --config c5 --max-bounce $mb --only swizzle,swizzle_info > gpurun_out/$TAG/mb$mb.json 2> gpurun_out/$TAG/mb$mb.err || { tail -20 gpurun_out/$TAG/mb$mb.err; exit 1; }
  echo "mb=$mb $(cat gpurun_out/$TAG/mb$mb.json)"
done
