#!/bin/bash
# r06 GPU measurement session: tools/r06_session.sh STEP...  (each step under its own timeout;
# outputs under gpurun_out/r06/).  Steps:
#   scatter    tools/scatter_probe (read + sparse-write granules, clear lists)
#   nomemkt    kernel trace of the no-memory top-k bench (bench.py --workload topk_nomem)
#   nomemsq    SQ + FETCH / WRITE counter passes of the no-memory top-k (tools/pmc_sq.sh)
#   headsq     SQ counter passes of the headline (the bimodality record)
#   prof       the headline, single stream, steady composition (tools/prof_steady.py)
#   bench      the default bench line
#   wl:NAME    one secondary bench line (bench.py --workload NAME)
#   pytest     the whole -m gpu suite
#   t:PATH     one GPU test file
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r06; mkdir -p $O
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
run() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?
        echo "$name rc=$rc"; tail -4 "$O/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
sqpasses() {   # $1 tag, rest: the program
  local tag=$1; shift
  local i=0
  for c in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT" \
           "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_BRANCH" \
           "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i + 1))
    run ${tag}_$i 120 rocprofv3 --pmc $c --output-format csv -d $O/${tag}_$i -o pmc -- "$@"
  done
}
for s in "$@"; do
  case $s in
    scatter) run scatter 120 ./tools/scatter_probe ;;
    nomemkt) GRACE_BENCH_NO_UNFUSED=1 run nomem_kt 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/sq_nomem_kt -o run \
               -- python3 bench.py --workload topk_nomem --steps 20 --warmup 5 --no-cpu-baseline ;;
    nomemsq) GRACE_BENCH_NO_UNFUSED=1 sqpasses sq_nomem python3 bench.py --workload topk_nomem --steps 5 --warmup 2 --no-cpu-baseline
             python3 tools/pmc_sq_summary.py $O/sq_nomem > $O/sq_nomem_summary.json; echo "sq summary rc=$?" ;;
    headsq) # the headline's main pass AND its streaming skeleton (the in-bench probe launches), one box
            tag=sq_head_${BOXTAG:-a}
            sqpasses $tag python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-overlap
            run ${tag}_kt 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${tag}_kt -o run \
              -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-overlap
            python3 tools/pmc_sq_summary.py $O/$tag > $O/${tag}_summary.json; echo "sq summary rc=$?"
            grep -h '^{' $O/${tag}_kt.log | tail -1 > $O/${tag}_line.json ;;
    prof) GRACE_BENCH_NO_PROBE=1 run prof_topk 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_topk -o run \
            -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-overlap
          python3 tools/prof_steady.py $O/prof_topk --last 20 --out $O/prof_topk_steady.json; echo "steady rc=$?" ;;
    bench) run bench 300 python3 bench.py ;;
    secondary)
      : > $O/secondary.jsonl
      for wl in ${WL:-topk_nomem topk_sharded ddp_segmented sign sign256 qsgd qsgd_step terngrad terngrad_step powersgd randomk threshold dgc natural cnat fp16 sign_bits}; do
        st=20; case $wl in sign) st=200 ;; esac
        run "bench_$wl" 300 python3 bench.py --workload $wl --steps $st --no-cpu-baseline
        grep '^{' "$O/bench_$wl.log" | tail -1 >> $O/secondary.jsonl
      done ;;
    pmc) # FETCH_SIZE / WRITE_SIZE passes (one counter per run) of the headline and every secondary
         # workload -> $O/pmc_topk_main.json and $O/r06_pmc_secondary.json (bench.py reads both from profiles/)
         export GRACE_BENCH_NO_PROBE=1 GRACE_BENCH_NO_UNFUSED=1
         for c in FETCH_SIZE WRITE_SIZE; do
           run pmc_head_$c 120 rocprofv3 --pmc $c --output-format csv -d $O/pmc_head_$c -o pmc \
               -- python3 bench.py --steps 3 --warmup 3 --no-cpu-baseline --no-overlap
         done
         python3 tools/pmc_summary.py $O/pmc_head_FETCH_SIZE $O/pmc_head_WRITE_SIZE "topk_main<true" 67108864 1 \
             $O/pmc_topk_main.json; echo "head summary rc=$?"
         args=""
         for wl in ${PMC_WL:-topk_nomem topk_sharded randomk qsgd terngrad powersgd sign sign256 qsgd_step terngrad_step ddp_segmented threshold dgc natural cnat fp16 sign_bits}; do
           for c in FETCH_SIZE WRITE_SIZE; do
             run pmc_${wl}_$c 120 rocprofv3 --pmc $c --output-format csv -d $O/pmc_${wl}_$c -o pmc \
                 -- python3 bench.py --workload $wl --steps 3 --warmup 1 --no-cpu-baseline
           done
           args="$args $wl=$O/pmc_${wl}_FETCH_SIZE,$O/pmc_${wl}_WRITE_SIZE"
         done
         # the output modes these passes ran in (the default: recycled outputs at world 1)
         python3 tools/pmc_all.py $O/r06_pmc_secondary.json --last 3 --mode topk_nomem=recycled \
             --mode topk_sharded=recycled --mode randomk=recycled --exclude "threshold:<1>" --exclude "randomk:<false>" \
             --exclude "dgc:spec_kernel<false>" --exclude "ddp_segmented:seg_main_kernel<false|seg_prep_kernel<false" \
             --exclude "topk_sharded:topk_main<false|topk_bracket<false|stream_kernel" $args; echo "pmc_all rc=$?" ;;
    shardlocal) run shard_local 180 python3 tools/exp_shard_local.py 8 ;;
    shardstamps) GRACE_HIP_LIB=grace_amd/lib/libgrace_hip_stamps.so run shard_local_stamps 180 python3 tools/exp_shard_local.py 8 ;;
    abshard) for i in 1 2; do
               GRACE_HIP_LIB=grace_amd/lib/libgrace_hip_shold.so run shard_old_$i 180 python3 tools/exp_shard_local.py 8
               GRACE_HIP_LIB=grace_amd/lib/libgrace_hip_shpre.so run shard_pre_$i 180 python3 tools/exp_shard_local.py 8
               run shard_new_$i 180 python3 tools/exp_shard_local.py 8
             done ;;
    absample) for i in 1 2; do
                for v in "" _s64k _s32k _c8; do
                  GRACE_HIP_LIB=grace_amd/lib/libgrace_hip$v.so run shard_smp${v}_$i 180 python3 tools/exp_shard_local.py 8
                done
              done
              AB_MODES=fused,swap,nomem_rec run ab_sample 400 python3 tools/ab_v3.py grace_amd/lib/libgrace_hip.so \
                grace_amd/lib/libgrace_hip_s64k.so grace_amd/lib/libgrace_hip_s32k.so grace_amd/lib/libgrace_hip_c8.so ;;
    smpcheck) for i in 1 2; do run shard_half_$i 180 python3 tools/exp_shard_local.py 8; done
              AB_MODES=fused,swap,nomem_rec run ab_half 400 python3 tools/ab_v3.py grace_amd/lib/libgrace_hip.so ;;
    localstamps) GRACE_HIP_LIB=grace_amd/lib/libgrace_hip_stamps.so N=8388608 K=67108 RES_ONLY=1 PATH_KIND=plain \
                   run stamps_local 120 python3 tools/exp_stamps.py
                 GRACE_HIP_LIB=grace_amd/lib/libgrace_hip_stamps.so run stamps_head 120 python3 tools/exp_stamps.py ;;
    abfin) for i in 1 2; do
             GRACE_HIP_LIB=grace_amd/lib/libgrace_hip_prefin.so run shard_prefin_$i 180 python3 tools/exp_shard_local.py 8
             run shard_fin_$i 180 python3 tools/exp_shard_local.py 8
           done
           AB_MODES=fused,swap,nomem_rec run ab_fin 400 python3 tools/ab_v3.py grace_amd/lib/libgrace_hip_prefin.so grace_amd/lib/libgrace_hip.so ;;
    abplace2) run ab_place2 400 python3 tools/ab_place2.py grace_amd/lib/libgrace_hip.so 8 ;;
    abgrid) AB_MODES=fused run ab_grid 500 python3 tools/ab_v3.py grace_amd/lib/libgrace_hip.so grace_amd/lib/libgrace_hip_v16c1k.so \
              grace_amd/lib/libgrace_hip_v8c1k.so grace_amd/lib/libgrace_hip_v12c1k.so grace_amd/lib/libgrace_hip_v16c2k.so ;;
    abgrid2) AB_MODES=fused,swap run ab_grid2a 500 python3 tools/ab_v3.py grace_amd/lib/libgrace_hip_v16c1k.so grace_amd/lib/libgrace_hip.so
             AB_MODES=fused,swap run ab_grid2b 500 python3 tools/ab_v3.py grace_amd/lib/libgrace_hip.so grace_amd/lib/libgrace_hip_v16c1k.so
             for i in 1 2; do
               GRACE_HIP_LIB=grace_amd/lib/libgrace_hip_v16c1k.so run bench_v16c1k_$i 300 python3 bench.py --no-cpu-baseline
               run bench_base_$i 300 python3 bench.py --no-cpu-baseline
             done ;;
    abplace3) run ab_place3 500 python3 tools/ab_place3.py grace_amd/lib/libgrace_hip.so 12 ;;
    abcontig) run ab_contig 500 python3 tools/ab_contig.py grace_amd/lib/libgrace_hip.so 4 ;;
    abplace4) run ab_place4 600 python3 tools/ab_place4.py grace_amd/lib/libgrace_hip.so 12 ;;
    abplace5) run ab_place5 600 python3 tools/ab_place5.py grace_amd/lib/libgrace_hip.so 12 ;;
    abpb) for i in 1 2 3; do
            run bench_place_$i 300 python3 bench.py --no-cpu-baseline
            GRACE_PLACE_PROBE=0 run bench_noplace_$i 300 python3 bench.py --no-cpu-baseline
          done ;;
    abthr) for i in 1 2 3; do
             run bench_thr_place_$i 300 python3 bench.py --workload threshold --steps 20 --no-cpu-baseline
             GRACE_PLACE_PROBE=0 run bench_thr_noplace_$i 300 python3 bench.py --workload threshold --steps 20 --no-cpu-baseline
           done ;;
    abspacer) run ab_spacer 500 python3 tools/ab_spacer.py ;;
    abpb2) for i in 1 2; do
             run bench_sp_$i 300 python3 bench.py --no-cpu-baseline
             GRACE_PLACE_SPACER_GIB=0 GRACE_PLACE_SPACER_STEP_GIB=0 run bench_nosp_$i 300 python3 bench.py --no-cpu-baseline
             GRACE_PLACE_PROBE=0 run bench_off_$i 300 python3 bench.py --no-cpu-baseline
             run bench_thr_sp_$i 300 python3 bench.py --workload threshold --steps 20 --no-cpu-baseline
           done ;;
    abpb3) for i in 1 2 3; do
             run bench_p43_$i 300 python3 bench.py --no-cpu-baseline --no-overlap
             GRACE_PLACE_RES=6 GRACE_PLACE_OUT=4 GRACE_PLACE_SPACER_STEP_GIB=1 run bench_p64_$i 300 python3 bench.py --no-cpu-baseline --no-overlap
           done ;;
    aboutplace) run ab_out_place 400 python3 tools/ab_out_place.py ;;
    bench2) for i in 1 2; do run bench_r$i 300 python3 bench.py --no-cpu-baseline --no-overlap; done ;;
    abspacerw) python3 -c "import torch; print(torch.cuda.get_device_properties(0).pci_bus_id if hasattr(torch.cuda.get_device_properties(0), 'pci_bus_id') else '')" > $O/spacer_wide_pci.txt 2>&1
               run ab_spacer_wide 600 python3 tools/ab_spacer_wide.py ;;
    shardtk) run shardtk 900 python3 -u -m pytest tests/test_gpu_sharded.py "tests/test_gpu_configs.py::test_sharded_topk_w8_one_device" \
               -q -x --timeout 300 --timeout-method thread ;;
    wnlocal) run wn_local 180 python3 tools/exp_wn_local.py ;;
    abvec2) AB_MODES=fused,swap run ab_vec2 400 python3 tools/ab_v3.py grace_amd/lib/libgrace_hip.so \
            grace_amd/lib/libgrace_hip_vec8.so grace_amd/lib/libgrace_hip_vec4.so ;;
    abpick) AB_MODES=nomem_rec,nomem_dense,fused run ab_pick 400 python3 tools/ab_v3.py grace_amd/lib/libgrace_hip_pickmain.so \
              grace_amd/lib/libgrace_hip.so ;;
    abplace) run ab_place 300 python3 tools/ab_place.py grace_amd/lib/libgrace_hip.so 6 ;;
    abpick2) AB_MODES=fused,nomem_rec run ab_pick2 400 python3 tools/ab_v3.py grace_amd/lib/libgrace_hip.so \
              grace_amd/lib/libgrace_hip_pickmain.so ;;
    abtile) run ab_tile 300 python3 tools/ab_decode.py grace_amd/lib/libgrace_hip.so grace_amd/lib/libgrace_hip_tile1.so \
              grace_amd/lib/libgrace_hip_tile2.so grace_amd/lib/libgrace_hip_tile4.so ;;
    abdec1) run ab_decode1 300 python3 tools/ab_decode.py grace_amd/lib/libgrace_hip.so ;;
    abdec) run ab_decode 300 python3 tools/ab_decode.py grace_amd/lib/libgrace_hip.so grace_amd/lib/libgrace_hip_qnb1g8k.so \
             grace_amd/lib/libgrace_hip_qnb1g32k.so grace_amd/lib/libgrace_hip_qnb2g16k.so ;;
    psgdab) run psgd_ab 300 python3 tools/ab_psgd.py grace_amd/lib/libgrace_hip_psgd_r04.so \
              grace_amd/lib/libgrace_hip_psgd_r05.so grace_amd/lib/libgrace_hip.so ;;
    ternsq) sqpasses sq_tern python3 bench.py --workload terngrad --steps 5 --warmup 2 --no-cpu-baseline
            run sq_tern_kt 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/sq_tern_kt -o run \
              -- python3 bench.py --workload terngrad --steps 20 --warmup 5 --no-cpu-baseline
            python3 tools/pmc_sq_summary.py $O/sq_tern > $O/sq_tern_summary.json; echo "sq summary rc=$?" ;;
    shardcodecs) run shard_codecs 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/shard_codecs -o run \
                   -- python3 tools/exp_shard_codecs.py 8
                 python3 tools/shard_codecs_summary.py $O/shard_codecs 8 > $O/shard_codecs_summary.txt; echo "summary rc=$?"
                 cat $O/shard_codecs_summary.txt ;;
    shardtests) run shardtests 900 python3 -u -m pytest tests/test_gpu_sharded_quant.py tests/test_gpu_sharded_terngrad.py \
        tests/test_gpu_sharded_powersgd.py tests/test_gpu_sharded_randomk.py -q -x --timeout 300 --timeout-method thread ;;
    abnv) AB_MODES=nomem_rec,nomem_dense run ab_nv 400 python3 tools/ab_v3.py grace_amd/lib/libgrace_hip.so \
            grace_amd/lib/libgrace_hip_nv16.so grace_amd/lib/libgrace_hip_nv24.so grace_amd/lib/libgrace_hip_nv40.so \
            grace_amd/lib/libgrace_hip_nv48.so grace_amd/lib/libgrace_hip_nv64.so ;;
    abnv2) AB_MODES=nomem_rec,nomem_dense run ab_nv2 400 python3 tools/ab_v3.py grace_amd/lib/libgrace_hip_nv64.so \
            grace_amd/lib/libgrace_hip_nv80.so grace_amd/lib/libgrace_hip_nv96.so grace_amd/lib/libgrace_hip_nv128.so ;;
    abvec) AB_MODES=fused run ab_vec 400 python3 tools/ab_v3.py grace_amd/lib/libgrace_hip.so \
            grace_amd/lib/libgrace_hip_vec16.so grace_amd/lib/libgrace_hip_vec20.so grace_amd/lib/libgrace_hip_vec24.so ;;
    ab12b) AB_MODES=swap run ab_12b 400 python3 tools/ab_v3.py grace_amd/lib/libgrace_hip.so \
            grace_amd/lib/libgrace_hip_v12b28.so grace_amd/lib/libgrace_hip_v12b32.so grace_amd/lib/libgrace_hip_v12b40.so ;;
    abv3) run ab_v3 300 python3 tools/ab_v3.py grace_amd/lib/libgrace_hip_main_v2.so grace_amd/lib/libgrace_hip.so ;;
    topktests) run topktests 900 python3 -u -m pytest tests/test_gpu_topk.py tests/test_gpu_topk_recycle.py \
        tests/test_gpu_topk_carry.py tests/test_gpu_harness.py tests/test_gpu_sparse.py -q -x --timeout 300 --timeout-method thread ;;
    wl:*) w=${s#wl:}; run "bench_$w" 300 python3 bench.py --workload $w --steps 20 --no-cpu-baseline ;;
    pytest) run pytest_gpu 1100 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread ;;
    t:*) f=${s#t:}; b=$(basename $f .py); run "pytest_$b" 600 python3 -u -m pytest $f -q -x --timeout 300 --timeout-method thread ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
