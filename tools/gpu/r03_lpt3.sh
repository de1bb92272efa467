# Bounce chunk orders predicted from the same frame's primary tile costs (C4, C2).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-lpt3}
mkdir -p gpurun_out/$TAG
timeout -k 10 500 python -u tools/exp_lpt.py --config c4 > gpurun_out/$TAG/lpt_c4.json 2> gpurun_out/$TAG/lpt_c4.err || { tail -5 gpurun_out/$TAG/lpt_c4.err; exit 1; }
grep -v amdgpu.ids gpurun_out/$TAG/lpt_c4.err
timeout -k 10 300 python -u tools/exp_lpt.py --config c2 > gpurun_out/$TAG/lpt_c2.json 2> gpurun_out/$TAG/lpt_c2.err || { tail -5 gpurun_out/$TAG/lpt_c2.err; exit 1; }
grep -v amdgpu.ids gpurun_out/$TAG/lpt_c2.err
