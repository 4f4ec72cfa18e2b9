# fused RS8 repair with non-temporal stores / loads (tools/ab_build.sh AB_GEN=fdec_asm --nt-stores |
# --nt-loads) against the product library, alternating three times on one box
set -o pipefail
for rep in 1 2 3; do
  for L in libnfec libnfec_fdnts libnfec_fdntl; do
    TAG=r06k/${L}_$rep AB_REPS=1 AB_LIB=norm_amd/_lib/$L.so AB_ENVS="NFEC_AB=$L" \
      AB_ARGS="--workload rs8 --erasures 16 --steps 20" bash tools/ab_env.sh || exit 1
  done
done
