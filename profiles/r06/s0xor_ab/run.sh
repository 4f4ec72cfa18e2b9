# level-2 s_0 read as the XOR of two pair-sum columns (product library) against the previous tree
# (knob library with NFEC_TMVP_POLICY=1 = the previous product), alternating on one box
set -o pipefail
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  -k "tmvp or rs16 or c4 or shortened or tw" > gpurun_out/r06n_pytest.log 2>&1 || { tail -20 gpurun_out/r06n_pytest.log; exit 1; }
tail -2 gpurun_out/r06n_pytest.log
for rep in 1 2; do
  for w in "rs16 --erasures 0 --steps 10" "c4 --erasures 0 --steps 3"; do
    n=$(echo $w | cut -d' ' -f1)
    TAG=r06n/${n}_new_$rep AB_REPS=1 AB_LIB=norm_amd/_lib/libnfec.so AB_ENVS="X=new" AB_ARGS="--workload $w" bash tools/ab_env.sh || exit 1
    TAG=r06n/${n}_old_$rep AB_REPS=1 AB_LIB=norm_amd/_lib/libnfec_knobs.so AB_ENVS="NFEC_TMVP_POLICY=1" AB_ARGS="--workload $w" bash tools/ab_env.sh || exit 1
  done
done
