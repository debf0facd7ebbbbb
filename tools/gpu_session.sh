#!/bin/bash
# GPU-box session runner: each GPU step under its own timeout; stop at the first crash / timeout
# (a plain test failure, exit 1, does not stop the session).  Logs under gpurun_out/.
# usage: tools/gpu_session.sh STEP [STEP ...]   (steps: smoke pytest bench prof pmc)
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
TAG="${SESSION_TAG:-r01}"

run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  tail -n 15 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "STOP: $name exited with $rc"; exit $rc
  fi
  return 0
}

for step in "$@"; do
  case "$step" in
    smoke)  run smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()" ;;
    pytest) run pytest_gpu 1200 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ;;
    pytopk) run pytest_topk 900 python3 -m pytest tests/test_gpu_topk.py -x -q ;;
    pytestall) run pytest_gpu_all 1200 python3 -m pytest tests -m gpu -q ;;
    bench)  run bench 600 python3 bench.py ;;
    benchall) for wl in ${BENCH_WL:-sign sign256 qsgd terngrad powersgd topk_e2e topk_sharded ddp_params ddp_bucket}; do run "bench_$wl" 300 python3 bench.py --workload $wl; done ;;
    prof)   run prof 600 rocprofv3 --kernel-trace --stats --output-format csv \
                -d "$ROOT/gpurun_out/prof_$TAG" -o bench -- python3 "$ROOT/bench.py" --steps 10 --warmup 3 --no-cpu-baseline ;;
    profwl) for wl in ${PROF_WL:-sign qsgd terngrad powersgd}; do
              run "prof_$wl" 300 rocprofv3 --kernel-trace --stats --output-format csv \
                  -d "$ROOT/gpurun_out/prof_${TAG}_$wl" -o bench -- python3 "$ROOT/bench.py" --workload $wl --steps 10 --warmup 3
            done ;;
    pmcmem) for c in FETCH_SIZE WRITE_SIZE; do
              run "pmc_$c" 600 rocprofv3 --pmc $c --output-format csv -d "$ROOT/gpurun_out/pmc_${TAG}_$c" -o pmc \
                  -- python3 "$ROOT/bench.py" --steps 3 --warmup 3 --no-cpu-baseline
            done ;;
    probe)  run hbm_probe 300 tools/hbm_probe ;;
    ab)     run ab 600 python3 tools/ab_topk.py ${AB_LIBS} ;;
    pmc)    for c in FETCH_SIZE WRITE_SIZE "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT"; do
              tag=$(echo $c | cut -d' ' -f1)
              run "pmc_$tag" 600 rocprofv3 --pmc $c --output-format csv -d "$ROOT/gpurun_out/pmc_${TAG}_$tag" -o pmc \
                  -- python3 "$ROOT/bench.py" --steps 3 --warmup 3 --no-cpu-baseline
            done ;;
    stamps) run stamps 300 env GRACE_HIP_LIB=grace_amd/lib/libgrace_hip_stamps.so python3 tools/exp_stamps.py ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
