set -o pipefail
cd $GRAFT_REPO_ROOT
nproc; cat /sys/fs/cgroup/cpu.max 2>/dev/null; python -c "import os; print(len(os.sched_getaffinity(0)), os.cpu_count())"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02_gputests.log 2>&1 && echo TESTS_OK &&
timeout -k 10 400 python -u bench.py --steps 20 --warmup 3 > gpurun_out/r02_bench.json 2> gpurun_out/r02_bench.err && echo BENCH_OK &&
timeout -k 10 300 python -u tools/ray_count_sweep.py > gpurun_out/r02_sweep.json 2> gpurun_out/r02_sweep.err && echo SWEEP_OK
