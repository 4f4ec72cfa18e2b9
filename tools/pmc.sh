#!/bin/bash
# PMC passes for the bench workload (one counter group per rocprofv3 run, as the gfx950
# guide prescribes; no trace domains combined with --pmc).  Output under gpurun_out/pmc_$TAG.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r01}
OUT=gpurun_out/pmc_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
ARGS="--steps 3 --warmup 1 --no-cpu-baseline --host-steps 0"
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU" "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o pmc -- python3 bench.py $ARGS > $OUT/p$i.log 2>&1 || { echo "pmc pass $i ($grp) failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python3 tools/parse_pmc.py $OUT $OUT/pmc_traffic.json > $OUT/summary.json && cat $OUT/pmc_traffic.json
