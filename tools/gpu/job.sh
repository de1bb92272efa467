#!/bin/bash
# One parameterised GPU job for gpurun (replaces the per-experiment r0x_*.sh scripts of rounds 1-3):
#   bash tools/gpu/job.sh TAG STAGE [STAGE ...]
# Stages run in order, each under its own time limit, outputs in gpurun_out/TAG/; the job stops at
# the first failing stage (no GPU step runs after a failure). Stages:
#   tests      pytest -m gpu (the parity suite)
#   bench      the driver's command: python bench.py --gpus 1 --steps 20 --warmup 5
#   group      the multi-GPU group (tt_group_*), batched-frame oracle and lifecycle GPU tests
#   groupbench the bench headline + aux_group_tiles (the library's group path) + interactive, no other aux legs
#   smoke      __graft_entry__.smoke() (the driver runs it before the bench)
#   blocks     the headline per persistent-grid size: BLOCKS="20 16 12" blocks per CU (TT_BLOCKS_PER_CU), REPS
#   quick      bench without aux configs / CPU baseline (layout and headline only)
#   dyn        bench headline + the C4 dynamic frame legs (aux dyn), per TT_BLOCKS_PER_CU in BLOCKS (0 = default)
#   dyndiag    the C4 dynamic frame with per-frame calls left out (DIAGS="none noupdate nogen noupdate,nogen")
#   slots2     quick with 2 frame slots (frame k + 1's primaries overlap frame k's bounce-1 launches)
#   layouts    the N = 1 headline per parts x slots layout: LAYOUTS="2x1 2x2 1x3", REPS=2 (profiles/r04/ab/r04k_*)
#   testlib    the GPU suite with a variant library: LIB=name (lib/variants/libtruetrace_hip_NAME.so)
#   newtests   the GPU tests of the layouts, shared scenes and hit streams only
#   prof       rocprofv3 --kernel-trace --stats of the bench + the FETCH_SIZE / WRITE_SIZE passes
#              (tools/profile_round.sh -> traffic JSON; profiles/traffic_latest.json is fed from it)
#   pmcu       the PMC unit passes behind roofline (tools/pmc_units.sh -> profiles/units_latest.json)
#   diag       per-block execution counts (TT_DIAG_BLOCKS build, tools/diag_blocks.py)
#   replay     strong-scaling replay of every rank's N-GPU shard on this GPU (tools/strong_replay.py; REPLAY_ARGS)
#   replaykt   the same replay under rocprofv3 --kernel-trace (REPLAY_ARGS; per-rank launch overlap)
#   lifecycle  the GPU tests of stream teardown (rocprofv3 leg included), root-leaf bookkeeping and the timed kernels' jittered parity
#   gloo2      the 2-rank bench rehearsal on this GPU (gloo collectives, C5 tiles included)
#   gloo4      the same with 4 ranks
#   groupscale the library group at world 1 on 1, 1/4, 1/8 of a 1080p frame x 2/4/8 slots (tools/group_scale.py)
#   rccl1      one rank through the N > 1 tile path with a real RCCL communicator of size 1 (+ the group leg)
#   longray    the C5 frame's degenerate ray: its chain alone and under load (tools/long_ray_chain.py)
#   c4loc      C4 one-launch time, TCC hit / miss and FETCH_SIZE per variant (AB_LIBS, default "cur n128")
#   l2loc      C2 per variant (AB_ORDER, AB_LIBS; default cur vs trint = non-temporal triangle loads): launch
#              times, then TCC hit / miss / EA read requests and TCP / TD counters of the same launches
#   order      tools/exp_order.py per TT_ORDER_HOT threshold (ORDER_HOT, ORDER_CFGS, ORDER_ARGS)
#   sweep      randomized parity sweep (tools/parity_sweep.py): SWEEP_N plain + SWEEP_N variants/adaptive + SWEEP_N
#              degenerate-direction cases + SWEEP_N frame-slot cases from seed SWEEP_SEED
#   sweepgroup the multi-GPU group sweep (random members / tiles / slots, copy gather on one GPU): SWEEP_N, SWEEP_SEED
#   sweepslots the frame-slot sweep alone (SWEEP_MODES, default "slots": instanced cases also traced by a moved slot)
#   ordercheck the shared-scene ordering tests on the no-ordering variant (expected to fail)
#   variants   A/B of the library variants in lib/variants (tools/run_variants.py)
#   ab         the bench headline per variant: AB_LIBS="product n128 ..." (lib/variants/libtruetrace_hip_NAME.so),
#              AB_ARGS extra bench.py flags, REPS rounds of the list in turn
#   abcfg      one-launch C4 and C5 per variant (tools/run_variants.py; AB_LIBS names lib/variants entries)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$PWD}"
TAG=$1
shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
run() {  # run NAME SECONDS CMD...: one GPU step, its own limit, output to $OUT/NAME.{out,err}
    local name=$1 secs=$2
    shift 2
    echo "[job] $name: $*" >&2
    local t0=$SECONDS
    timeout -k 10 "$secs" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
    local rc=$?
    echo "[job] $name rc=$rc ($((SECONDS - t0)) s)" >&2
    tail -c 400 "$OUT/$name.out" >&2
    return $rc
}
for stage in "$@"; do
    case $stage in
    tests) run tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread || exit $? ;;
    blocks) for i in $(seq ${REPS:-1}); do for b in ${BLOCKS:-20 16}; do  # persistent grid blocks per CU (env knob)
                run "blocks_${b}_$i" 300 env TT_BLOCKS_PER_CU=$b python -u bench.py --steps 20 --warmup 5 --aux "" \
                    --no-cpu-baseline --no-recur --no-shadow || exit $?
            done; done ;;
    group) run group 900 env TT_TEST_ROCPROF=1 python -u -m pytest -x -v --timeout 400 --timeout-method thread \
               tests/test_gpu_group.py tests/test_gpu_batch_oracle.py tests/test_gpu_lifecycle.py -m gpu || exit $? ;;
    groupbench) run groupbench 400 python -u bench.py --steps 20 --warmup 5 --aux "" --no-cpu-baseline --no-recur \
                    --no-shadow --no-single ${GB_ARGS:-} || exit $? ;;
    smoke) run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" || exit $? ;;
    bench) run bench 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 || exit $? ;;
    quick) run quick 300 python -u bench.py --steps 20 --warmup 5 --aux "" --cpu-seconds 2 || exit $? ;;
    dyn) for b in ${BLOCKS:-0}; do  # the headline + the C4 dynamic frame (one launch and frame slots) per grid cap
             run "dyn_b$b" 400 env TT_BLOCKS_PER_CU=$b python -u bench.py --steps 20 --warmup 5 --aux dyn \
                 --no-cpu-baseline --no-recur --no-shadow ${DYN_ARGS:-} || exit $?
         done ;;
    dyndiag) for d in ${DIAGS:-none noupdate nogen noupdate,nogen}; do  # the C4 dynamic frame without one per-frame call
                 run "dyndiag_$d" 400 python -u bench.py --steps 20 --warmup 5 --aux dyn --no-cpu-baseline --no-recur \
                     --no-shadow --no-oracle-check --dyn-diag "$d" ${DYN_ARGS:-} || exit $?
             done ;;
    slots2) run slots2 300 python -u bench.py --steps 20 --warmup 5 --aux "" --no-cpu-baseline --slots 2 || exit $? ;;
    layouts) for i in $(seq ${REPS:-2}); do for l in ${LAYOUTS:-2x1 2x2 1x3}; do  # N = 1 headline per parts x slots
                 run "n1_${l}_$i" 300 python -u bench.py --steps 20 --warmup 5 --aux "" --no-cpu-baseline --no-recur \
                     --no-shadow --parts ${l%x*} --slots ${l#*x} || exit $?
             done; done ;;
    testlib) lib=$PWD/truetrace-unity-pathtracer_amd/lib/variants/libtruetrace_hip_${LIB:?set LIB=variant name}.so
             run "tests_$LIB" 600 env TT_HIP_LIB=$lib python -u -m pytest tests -m gpu -x -q --timeout 300 \
                 --timeout-method thread || exit $? ;;
    newtests) run newtests 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parts.py \
                  tests/test_gpu_order.py tests/test_bench_launch.py -m gpu || exit $? ;;
    prof) run prof 900 bash tools/profile_round.sh "$TAG" || exit $? ;;
    pmcu) run pmcu 900 bash tools/pmc_units.sh "$OUT/pmcu" || exit $? ;;
    diag) run diag 200 env TT_HIP_LIB=truetrace-unity-pathtracer_amd/lib/variants/libtruetrace_hip_diag.so \
              python -u tools/diag_blocks.py c2 || exit $? ;;
    replay) run replay 900 python -u tools/strong_replay.py --configs c2,c5 ${REPLAY_ARGS:-} || exit $? ;;
    replaykt) export TMPDIR=/tmp
              run replaykt 600 rocprofv3 --kernel-trace --output-format csv -d "$OUT/kt" -o kt -- \
                  python -u tools/strong_replay.py --configs c2 ${REPLAY_ARGS:---ns 8 --layouts 1x6} || exit $? ;;
    lifecycle) run lifecycle 600 env TT_TEST_ROCPROF=1 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
                   tests/test_gpu_lifecycle.py "tests/test_gpu_parity.py::test_sponza_1080p_jittered_frames_through_the_timed_kernels" \
                   -m gpu || exit $? ;;
    longray) run longray 300 python -u tools/long_ray_chain.py || exit $? ;;
    c4loc) export TMPDIR=/tmp
           for v in ${AB_LIBS:-cur n128}; do  # C4 one-launch time + L2 hit / miss and fabric reads per variant
               run "c4loc_time_$v" 400 env RV_CFG=c4 python -u tools/run_variants.py "$v" || exit $?
               export TT_HIP_LIB=truetrace-unity-pathtracer_amd/lib/variants/libtruetrace_hip_$v.so
               run "c4loc_tcc_$v" 400 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d "$OUT/c4loc_tcc_$v" -o tcc \
                   --output-format csv -- python tools/prof_config.py c4 --reps 2 || exit $?
               run "c4loc_fetch_$v" 400 rocprofv3 --pmc FETCH_SIZE -d "$OUT/c4loc_fetch_$v" -o fetch \
                   --output-format csv -- python tools/prof_config.py c4 --reps 2 || exit $?
               unset TT_HIP_LIB
           done ;;
    l2loc) export TMPDIR=/tmp  # C2 one launch at a time per variant (AB_ORDER), then per variant (AB_LIBS) the
           # L2 side (TCC hit / miss / fabric read requests) and the L1 / TD side of the same launches
           run l2loc_time 600 python -u tools/run_variants.py ${AB_ORDER:-cur trint cur trint cur trint} || exit $?
           for v in ${AB_LIBS:-cur trint}; do
               export TT_HIP_LIB=truetrace-unity-pathtracer_amd/lib/variants/libtruetrace_hip_$v.so
               run "l2loc_tcc_$v" 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum \
                   -d "$OUT/l2loc_tcc_$v" -o tcc --output-format csv -- python tools/prof_config.py c2 --reps 2 || exit $?
               run "l2loc_tcp_$v" 300 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TD_TD_BUSY_sum \
                   GRBM_GUI_ACTIVE -d "$OUT/l2loc_tcp_$v" -o tcp --output-format csv -- python tools/prof_config.py c2 \
                   --reps 2 || exit $?
               unset TT_HIP_LIB
           done ;;
    order) for h in ${ORDER_HOT:-0 128}; do  # adaptive order, hoisting only chunks costing >= h node steps (0: full sort)
               for cfg in ${ORDER_CFGS:-c4 c5}; do
                   run "order_${cfg}_hot$h" 400 env TT_ORDER_HOT=$h python -u tools/exp_order.py --config $cfg \
                       --primary-only ${ORDER_ARGS:-} || exit $?
               done
           done ;;
    gloo2) run gloo2 600 env TT_BENCH_DIST_BACKEND=gloo python -u bench.py --gpus 2 --steps 4 --warmup 1 \
               --no-cpu-baseline --no-shadow --steady-steps 0 || exit $? ;;
    groupscale) run groupscale 600 python -u tools/group_scale.py ${GS_FRAMES:-200} || exit $? ;;
    rccl1) run rccl1 600 env TT_BENCH_RCCL_WORLD1=1 RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29611 python -u bench.py --steps 4 --warmup 1 --no-cpu-baseline \
               --no-shadow --steady-steps 0 --aux "" || exit $? ;;
    gloo4) run gloo4 600 env TT_BENCH_DIST_BACKEND=gloo python -u bench.py --gpus 4 --steps 4 --warmup 1 \
               --no-cpu-baseline --no-shadow --steady-steps 0 || exit $? ;;
    sweep) n=${SWEEP_N:-300}; s0=${SWEEP_SEED:-40000}  # plain; trace variants + adaptive order; + degenerate directions
           run sweep_plain 900 python -u tools/parity_sweep.py $n $s0 || exit $?
           run sweep_var 900 python -u tools/parity_sweep.py $n $((s0 + 1000)) variants,adaptive || exit $?
           run sweep_axis 900 python -u tools/parity_sweep.py $n $((s0 + 2000)) axis,variants,adaptive || exit $?
           run sweep_slots 900 python -u tools/parity_sweep.py $n $((s0 + 3000)) slots,adaptive || exit $? ;;
    sweepgroup) run sweep_group 900 python -u tools/parity_sweep.py ${SWEEP_N:-200} ${SWEEP_SEED:-60000} \
                    ${SWEEP_MODES:-group,variants} || exit $? ;;
    sweepslots) run sweep_slots 900 python -u tools/parity_sweep.py ${SWEEP_N:-300} ${SWEEP_SEED:-43000} \
               ${SWEEP_MODES:-slots} || exit $? ;;
    ordercheck) # the shared-scene ordering tests against the variant whose sections order nothing (make variant
                # NAME=noorder VFLAGS=-DTT_NO_SCENE_ORDER): they must FAIL there (the job goes on either way)
                run ordercheck 300 env TT_HIP_LIB=truetrace-unity-pathtracer_amd/lib/variants/libtruetrace_hip_noorder.so \
                    python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_gpu_parts.py \
                    -k "ordered or sections" -m gpu
                echo "[job] ordercheck rc=$? (expected non-zero)" >&2 ;;
    variants) run variants 900 python -u tools/run_variants.py || exit $? ;;
    ab) for i in $(seq ${REPS:-1}); do for v in ${AB_LIBS:-product}; do  # the bench headline per library variant, in turn
            lib=truetrace-unity-pathtracer_amd/lib/variants/libtruetrace_hip_$v.so
            [ "$v" = product ] && lib=truetrace-unity-pathtracer_amd/lib/libtruetrace_hip.so
            run "ab_${v}_$i" 300 env TT_HIP_LIB=$lib python -u bench.py --steps 20 --warmup 5 --aux "" --no-cpu-baseline \
                --no-recur --no-shadow ${AB_ARGS:-} || exit $?
        done; done ;;
    abcfg) for v in ${AB_LIBS:-product}; do  # one-launch C4 / C5 per variant (tools/run_variants.py)
            for cfg in c4 c5; do run "abcfg_${v}_$cfg" 400 env RV_CFG=$cfg python -u tools/run_variants.py "$v" || exit $?; done
        done ;;
    *) echo "unknown stage $stage" >&2; exit 2 ;;
    esac
done
echo "[job] $TAG done" >&2
