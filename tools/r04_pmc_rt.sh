#!/bin/bash
# PMC passes of the runtime-coefficient repair (per-block launches): RS8(64,32) 16-erasure
# repair on the rt kernel (NFEC_RT_DEC=1, diagnostic library) and the MDP(64,32) repair, one
# counter group per rocprofv3 pass (tools/pmc_r03.sh).  -> gpurun_out/pmc_<tag>/summary.json
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export NFEC_LIBRARY=$(pwd)/norm_amd/_lib/libnfec_diag.so
export PMC_SCRIPT=tools/bench_extra.py
export PMC_GROUPS="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_BUSY_CYCLES;SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_SMEM;GRBM_GUI_ACTIVE GRBM_COUNT;FETCH_SIZE;WRITE_SIZE"
NFEC_RT_DEC=1 PMC_ARGS="--workload rs8 --k 64 --m 32 --erasures 16 --steps 1 --warmup 1" TAG=rt6432 bash tools/pmc_r03.sh > /dev/null
[ -s gpurun_out/pmc_rt6432/summary.json ] || exit 1
PMC_ARGS="--workload mdp --steps 1 --warmup 1" TAG=rtmdp bash tools/pmc_r03.sh > /dev/null
[ -s gpurun_out/pmc_rtmdp/summary.json ] || exit 1
