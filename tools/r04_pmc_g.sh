#!/bin/bash
# PMC passes of the RS8(200,55) 16-erasure repair on the runtime-coefficient kernel with one wave
# per item group (NFEC_RT_GPB=1) against two (=2): instruction mix, waits and cycles per
# launch (diagnostic library; tools/pmc_r03.sh, one counter group per pass).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export NFEC_LIBRARY=$(pwd)/norm_amd/_lib/libnfec_diag.so
export PMC_SCRIPT=tools/bench_extra.py
export PMC_ARGS="--workload rs8 --k 200 --m 55 --erasures 16 --blocks 16384 --steps 1 --warmup 1"
export PMC_GROUPS="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_BUSY_CYCLES;SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT;GRBM_GUI_ACTIVE GRBM_COUNT"
for g in ${GLIST:-1 2}; do
    NFEC_RT_GPB=$g TAG=g$g bash tools/pmc_r03.sh > /dev/null; [ -s gpurun_out/pmc_g$g/summary.json ] || exit 1
done
