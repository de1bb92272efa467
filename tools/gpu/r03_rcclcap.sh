# RCCL size-1 tile path (the N > 1 step with a real gather on one GPU) vs the trace grid's blocks per CU:
# room left on every SIMD lets RCCL's copy kernel run beside the persistent waves.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-rcclcap}
mkdir -p gpurun_out/$TAG
i=0
for cap in 20 16 18 20 16; do
  i=$((i+1))
  RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=$((29540+i)) TT_BENCH_RCCL_WORLD1=1 TT_BLOCKS_PER_CU=$cap timeout -k 10 300 python -u bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-shadow --steady-steps 0 --aux '' --no-recur > gpurun_out/$TAG/rccl1_cap$cap.$i.json 2> gpurun_out/$TAG/rccl1_cap$cap.$i.err || { tail -5 gpurun_out/$TAG/rccl1_cap$cap.$i.err; exit 1; }
  python -c "
import json; d=json.loads([l for l in open('gpurun_out/$TAG/rccl1_cap$cap.$i.json') if l.startswith('{')][-1]); print('rccl1 cap $cap', d['value'], d['ms_per_step'], d['config']['gather_identical_to_1gpu'])"
  TT_BLOCKS_PER_CU=$cap timeout -k 10 300 python -u bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-shadow --steady-steps 0 --aux '' --no-recur --no-single > gpurun_out/$TAG/n1_cap$cap.$i.json 2> gpurun_out/$TAG/n1_cap$cap.$i.err || { tail -5 gpurun_out/$TAG/n1_cap$cap.$i.err; exit 1; }
  python -c "
import json; d=json.loads([l for l in open('gpurun_out/$TAG/n1_cap$cap.$i.json') if l.startswith('{')][-1]); print('n1    cap $cap', d['value'], d['ms_per_step'])"
done
