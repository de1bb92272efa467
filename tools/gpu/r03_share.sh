# Scene sharing between the part contexts (tt_ctx_share_scene): the two-part step with one scene copy vs one per part.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-share}
mkdir -p gpurun_out/$TAG
for cfg in c2 c4 c2 c4; do
  for sh in "" "--share"; do
    timeout -k 10 300 python -u tools/exp_order.py --config $cfg --parts 2 --rounds 1 --steps 40 $sh --primary-only > gpurun_out/$TAG/p2_${cfg}${sh}.json 2> gpurun_out/$TAG/p2_${cfg}${sh}.err || { tail -5 gpurun_out/$TAG/p2_${cfg}${sh}.err; exit 1; }
    echo "== $cfg parts 2 $sh $(grep -v amdgpu.ids gpurun_out/$TAG/p2_${cfg}${sh}.err)"
  done
done
timeout -k 10 300 python -u tools/exp_order.py --config c5 --parts 2 --rounds 1 --steps 20 > gpurun_out/$TAG/p2_c5.json 2> gpurun_out/$TAG/p2_c5.err && echo "== c5 $(grep -v amdgpu.ids gpurun_out/$TAG/p2_c5.err)"
timeout -k 10 300 python -u tools/exp_order.py --config c5 --parts 2 --rounds 1 --steps 20 --share > gpurun_out/$TAG/p2_c5s.json 2> gpurun_out/$TAG/p2_c5s.err && echo "== c5 share $(grep -v amdgpu.ids gpurun_out/$TAG/p2_c5s.err)"
