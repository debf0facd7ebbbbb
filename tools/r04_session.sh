#!/bin/bash
# Round-4 GPU session: each GPU step under its own time limit; a crash / timeout ends the session
# (a plain test failure, exit 1, does not).  STEPS picks the steps; logs under gpurun_out/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
TAG=${TAG:-r04}
run() { local name=$1 to=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?
        echo "$name rc=$rc"; tail -4 "gpurun_out/$name.log"; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
for step in ${STEPS:-pytest smoke bench}; do
  case $step in
    pytest) run pytest_gpu 1100 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ;;
    pyfiles) run pytest_files 1100 python3 -u -m pytest ${FILES} -x -v --timeout 120 --timeout-method thread ;;
    smoke) run smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 300 python3 bench.py ;;
    secondary)
      : > gpurun_out/secondary.jsonl
      for wl in ${WL:-sign sign256 qsgd terngrad powersgd}; do
        st=20; case $wl in sign|powersgd|ddp_segmented|qsgd|terngrad|qsgd_step|terngrad_step) st=200;; esac
        run "bench_$wl" 300 python3 bench.py --workload $wl --steps $st --no-cpu-baseline
        grep '^{' "gpurun_out/bench_$wl.log" | tail -1 >> gpurun_out/secondary.jsonl
      done ;;
    prof) # the headline, single stream (no two-stream leg), no in-bench probes: every traced launch
          # is a steady-state, one-stream launch of the step (tools/prof_steady.py drops the first steps)
          GRACE_BENCH_NO_PROBE=1 run prof_topk 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG}_topk -o run \
            -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-overlap ;;
    profwl) for wl in ${PROF_WL:-powersgd terngrad qsgd sign}; do
              st=20; run "prof_$wl" 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG}_$wl -o run \
                -- python3 bench.py --workload $wl --steps $st --warmup 5 --no-cpu-baseline
            done ;;
    exp) run exp 600 python3 ${EXP} ;;
    exps) for e in ${EXPS}; do b=$(basename $e .py); run $b 300 python3 $e; grep -v amdgpu.ids gpurun_out/$b.log | tail -4; done ;;
    ternab) # TernGrad: does the encoder's re-read of x hit the Infinity Cache?  The same bench with a
            # 512 MiB write stream between the statistics pass and the encoder (ternflush build)
            for lib in libgrace_hip libgrace_hip_ternflush libgrace_hip_ternnt; do
              GRACE_HIP_LIB=grace_amd/lib/$lib.so GRACE_BENCH_NO_PROBE=1 run prof_tern_$lib 300 rocprofv3 --kernel-trace \
                --stats --output-format csv -d gpurun_out/prof_${TAG}_tern_$lib -o run \
                -- python3 bench.py --workload terngrad --steps 50 --warmup 5 --no-cpu-baseline
            done ;;
    rehearse) # 2 ranks on cuda:0 over gloo: the default N > 1 line, then with an injected sharded-leg
              # failure on every rank (agreed, recorded) and on rank 1 only (watchdog)
              for inj in none all 1; do
                run w2_$inj 240 env GRACE_BENCH_INJECT_SHARDED_FAILURE=$inj GRACE_BENCH_SHARDED_LIMIT=60 \
                  GRACE_BENCH_ONE_DEVICE=1 GRACE_BENCH_BACKEND=gloo python3 -m torch.distributed.run --nnodes=1 \
                  --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29521 bench.py --gpus 2 --steps 5 --warmup 2
                grep '^{' gpurun_out/w2_$inj.log | tail -1
              done ;;
  esac
done
