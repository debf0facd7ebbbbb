#!/bin/bash
# SQ counter passes (one rocprofv3 --pmc run each, <= 8 SQ counters) over one bench workload, plus
# a kernel-trace pass: tools/pmc_sq.sh WORKLOAD [STEPS]  -> gpurun_out/sq_<wl>_<pass>/ and a
# per-kernel summary (tools/pmc_sq_summary.py) on stdout.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
wl=$1; st=${2:-5}
i=0
for c in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT" \
         "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_ANY" \
         "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i + 1))
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d gpurun_out/sq_${wl}_$i -o pmc \
      -- python3 bench.py --workload "$wl" --steps "$st" --warmup 2 --no-cpu-baseline > gpurun_out/sq_${wl}_$i.log 2>&1
  rc=$?
  echo "pass $i rc=$rc"
  if [ $rc -ne 0 ]; then tail -3 gpurun_out/sq_${wl}_$i.log; exit $rc; fi
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sq_${wl}_kt -o run \
    -- python3 bench.py --workload "$wl" --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/sq_${wl}_kt.log 2>&1
echo "kt rc=$?"
python3 tools/pmc_sq_summary.py gpurun_out/sq_${wl}
