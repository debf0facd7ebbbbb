#!/bin/bash
# r05 GPU measurement session: tools/r05_session.sh STEP...  (each step under its own timeout;
# outputs under gpurun_out/r05/).  Steps:
#   fallback   tools/exp_fallback.py (degenerate buckets through the claimed-slice exact fallback)
#   stamps     phase stamps of the local top-k at configs[4] (m = 2^23, k = 67,108, residual only)
#              and of the W > 1 DP local step (2^26, k = 671,088, residual only)
#   shard      tools/exp_shard_local.py 8
#   wn         tools/exp_wn_local.py (DP-replica per-rank device time at W = 8)
#   sq         SQ / GRBM counter passes over the headline bench (topk_main and its stream skeleton)
#   bench      the default bench line
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05; mkdir -p $O
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
run() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?
        echo "$name rc=$rc"; tail -4 "$O/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
for s in "$@"; do
  case $s in
    fallback) run fallback 180 python3 tools/exp_fallback.py ;;
    stamps)
      GRACE_HIP_LIB=grace_amd/lib/libgrace_hip_stamps.so N=8388608 K=67108 RES_ONLY=1 PATH_KIND=plain \
        run stamps_shard_local 120 python3 tools/exp_stamps.py
      GRACE_HIP_LIB=grace_amd/lib/libgrace_hip_stamps.so RES_ONLY=1 PATH_KIND=plain \
        run stamps_wn_local 120 python3 tools/exp_stamps.py ;;
    shard) run shard_local 180 python3 tools/exp_shard_local.py 8 ;;
    shardstamps) GRACE_HIP_LIB=grace_amd/lib/libgrace_hip_stamps.so run shard_local_stamps 180 python3 tools/exp_shard_local.py 8 ;;
    wn) run wn_local 180 python3 tools/exp_wn_local.py ;;
    decab)   # the decode: one workgroup per chunk (decnopipe) vs the persistent pipelined form (4 / 5 / 8 per CU)
      for i in 1 2; do
        for v in decnopipe decpipe4 "" decpipe8; do
          lib=grace_amd/lib/libgrace_hip${v:+_$v}.so
          GRACE_HIP_LIB=$lib run wn_${v:-decpipe5}_$i 180 python3 tools/exp_wn_local.py
        done
      done ;;
    quanttests) run quanttests 900 python3 -u -m pytest tests/test_gpu_sharded_powersgd.py tests/test_gpu_sharded_randomk.py \
        -q -x --timeout 300 --timeout-method thread ;;
    sparsetests) run sparsetests 600 python3 -u -m pytest tests/test_gpu_sparse.py tests/test_gpu_world2.py \
        tests/test_gpu_w8.py -q -x --timeout 300 --timeout-method thread ;;
    sq)
      i=0
      for c in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT" \
               "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU"; do
        i=$((i + 1))
        run sq_head_$i 120 rocprofv3 --pmc $c --output-format csv -d $O/sq_head_$i -o pmc \
            -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-overlap
      done
      run sq_head_kt 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/sq_head_kt -o run \
          -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-overlap
      python3 tools/pmc_sq_summary.py $O/sq_head > $O/sq_head_summary.json; echo "sq summary rc=$?" ;;
    bench) run bench 300 python3 bench.py ;;
    prof) # the headline, single stream, no in-bench probes (tools/prof_steady.py keeps the timed launches)
          GRACE_BENCH_NO_PROBE=1 run prof_topk 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_topk -o run \
            -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-overlap
          python3 tools/prof_steady.py $O/prof_topk --last 20 --out $O/prof_topk_steady.json; echo "steady rc=$?" ;;
    profwl) for wl in ${PROF_WL:-powersgd terngrad qsgd sign}; do
              run "prof_$wl" 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$wl -o run \
                -- python3 bench.py --workload $wl --steps 20 --warmup 5 --no-cpu-baseline
            done ;;
    pytest) run pytest_gpu 1100 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread ;;
    secondary)
      : > $O/secondary.jsonl
      for wl in ${WL:-topk_sharded ddp_segmented sign sign256 qsgd qsgd_step terngrad terngrad_step powersgd randomk threshold dgc topk_nomem}; do
        st=20; case $wl in sign) st=200 ;; esac
        run "bench_$wl" 300 python3 bench.py --workload $wl --steps $st --no-cpu-baseline
        grep '^{' "$O/bench_$wl.log" | tail -1 >> $O/secondary.jsonl
      done ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
