# Scheduler knobs under the two-part layout with one-wave blocks: the C2 two-part step per variant (x2, interleaved).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=$1; shift
mkdir -p gpurun_out/$TAG
V=truetrace-unity-pathtracer_amd/lib/variants
for v in "$@" "$@"; do
  TT_HIP_LIB=$PWD/$V/libtruetrace_hip_$v.so timeout -k 10 300 python -u tools/exp_order.py --config c2 --parts 2 --rounds 1 --steps 60 > gpurun_out/$TAG/p2_$v.json 2> gpurun_out/$TAG/p2_$v.err || { tail -5 gpurun_out/$TAG/p2_$v.err; exit 1; }
  echo "== c2 parts 2 $v $(grep -v amdgpu.ids gpurun_out/$TAG/p2_$v.err)"
done
