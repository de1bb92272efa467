set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-sharechk}
mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -m pytest tests/ -x -q -m gpu > gpurun_out/$TAG/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/$TAG/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err || exit $?
python -c "
import json; d=json.loads(open('gpurun_out/$TAG/bench.json').read().strip().splitlines()[-1]); print('bench', d['value'], d['ms_per_step'], d['config']['steady_state']['mrays_s'], d['config']['parts_share_one_scene_copy']); a=d['config']['aux_configs']; print({k:(v.get('two_parts_two_streams'),v.get('adaptive_order',{}).get('two_parts_two_streams')) for k,v in a.items() if 'rays' in v})"
bash tools/gpu/r03_rehearse.sh $TAG || exit $?
