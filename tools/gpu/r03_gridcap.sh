# Two-part C2 step vs the persistent grid's blocks per CU (TT_BLOCKS_PER_CU; one-wave blocks: 20 = 5 waves/SIMD).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-gridcap}
mkdir -p gpurun_out/$TAG
for cap in 20 18 16 12 20; do
  TT_BLOCKS_PER_CU=$cap timeout -k 10 300 python -u tools/exp_order.py --config c2 --parts 2 --rounds 2 > gpurun_out/$TAG/p2_cap$cap.json 2> gpurun_out/$TAG/p2_cap$cap.err || { tail -5 gpurun_out/$TAG/p2_cap$cap.err; exit 1; }
  echo "== cap $cap"; grep -v amdgpu.ids gpurun_out/$TAG/p2_cap$cap.err
done
for cap in 20 16; do
  TT_BLOCKS_PER_CU=$cap timeout -k 10 300 python -u tools/exp_order.py --config c2 --parts 3 --rounds 2 > gpurun_out/$TAG/p3_cap$cap.json 2> gpurun_out/$TAG/p3_cap$cap.err || { tail -5 gpurun_out/$TAG/p3_cap$cap.err; exit 1; }
  echo "== 3 parts cap $cap"; grep -v amdgpu.ids gpurun_out/$TAG/p3_cap$cap.err
done
