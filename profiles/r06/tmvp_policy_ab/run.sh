set -o pipefail
K=norm_amd/_lib/libnfec_knobs.so; N=norm_amd/_lib/libnfec_twnt.so
for rep in 1 2; do
TAG=r06j/rs16_k$rep AB_REPS=1 AB_LIB=$K AB_ENVS="NFEC_TMVP_POLICY=0;NFEC_TMVP_POLICY=1" AB_ARGS="--workload rs16 --erasures 50 --steps 10" bash tools/ab_env.sh || exit 1
TAG=r06j/rs16_n$rep AB_REPS=1 AB_LIB=$N AB_ENVS="NFEC_TMVP_POLICY=0;NFEC_TMVP_POLICY=1" AB_ARGS="--workload rs16 --erasures 50 --steps 10" bash tools/ab_env.sh || exit 1
TAG=r06j/c4_k$rep AB_REPS=1 AB_LIB=$K AB_ENVS="NFEC_TMVP_POLICY=0;NFEC_TMVP_POLICY=1" AB_ARGS="--workload c4 --erasures 0 --steps 3" bash tools/ab_env.sh || exit 1
TAG=r06j/c4_n$rep AB_REPS=1 AB_LIB=$N AB_ENVS="NFEC_TMVP_POLICY=1" AB_ARGS="--workload c4 --erasures 0 --steps 3" bash tools/ab_env.sh || exit 1
done
