# Part-split tile edge for the two-part layout (C2, C4 adaptive-off): 32 / 64 / 128, interleaved.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-tile}
mkdir -p gpurun_out/$TAG
for r in 1 2; do for cfg in c2 c4; do for t in 32 64 128; do
  timeout -k 10 300 python -u tools/exp_order.py --config $cfg --parts 2 --rounds 1 --steps 60 --share --tile $t > gpurun_out/$TAG/${cfg}_t${t}_r$r.json 2> gpurun_out/$TAG/${cfg}_t${t}_r$r.err || { tail -5 gpurun_out/$TAG/${cfg}_t${t}_r$r.err; exit 1; }
  echo "== $cfg tile $t round $r $(grep -v amdgpu.ids gpurun_out/$TAG/${cfg}_t${t}_r$r.err | tail -1)"
done; done; done
