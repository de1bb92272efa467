# The driver's round-end commands (GPU suite, smoke, bench W=5 K=20 at N = 1) + the multi-rank rehearsals.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-drv}
mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -m pytest tests/ -x -q -m gpu > gpurun_out/$TAG/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 gpurun_out/$TAG/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$TAG/smoke.log 2>&1 || exit $?
tail -1 gpurun_out/$TAG/smoke.log
for i in 1 2; do
  timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/$TAG/bench$i.json 2> gpurun_out/$TAG/bench$i.err || exit $?
  python -c "
import json; d=json.loads(open('gpurun_out/$TAG/bench$i.json').read().strip().splitlines()[-1]); print('bench', d['value'], d['ms_per_step'], d['config']['steady_state']['mrays_s'], d['roofline']['frac'])"
done
bash tools/gpu/r03_rehearse.sh $TAG || exit $?
