#!/bin/bash
# PMC passes over the bench workload (round 3): one counter group per rocprofv3 run and no trace
# domain next to --pmc (MI355X_MICROARCH.md, HBM / rocprofv3 section), each pass under its own
# time limit; the first failure ends the script.  Groups come from PMC_GROUPS (';'-separated),
# defaulting to HBM traffic, instruction mix, wave states and the clock; PMC_SCRIPT / PMC_ARGS
# choose another workload (e.g. tools/bench_extra.py --workload c4).
#   TAG=x bash tools/pmc_r03.sh           -> gpurun_out/pmc_x/p<i>/..., summary via parse_pmc.py
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r03}
OUT=gpurun_out/pmc_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
ARGS=${PMC_ARGS:-"--steps 3 --warmup 1 --no-cpu-baseline --host-steps 0"}
GROUPS_DEFAULT="FETCH_SIZE;WRITE_SIZE;SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD;SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU;GRBM_GUI_ACTIVE GRBM_COUNT"
IFS=';' read -ra GRPS <<< "${PMC_GROUPS:-$GROUPS_DEFAULT}"
i=0
for grp in "${GRPS[@]}"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o pmc -- python3 ${PMC_SCRIPT:-bench.py} $ARGS > $OUT/p$i.log 2>&1 \
      || { echo "pmc pass $i ($grp) failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python3 tools/parse_pmc.py $OUT $OUT/pmc_traffic.json > $OUT/summary.json || exit 1
# (the traffic file exists for the headline workload only)
[ ! -f $OUT/pmc_traffic.json ] || cat $OUT/pmc_traffic.json
