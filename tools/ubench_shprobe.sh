cd $GRAFT_REPO_ROOT
O=gpurun_out/r06h; mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2; do
for v in full product shnomask shnofetch; do
  lib=norm_amd/_lib/libnfec.so; args="--workload rs8 --erasures 0 --steps 10 --shortened --nd-dist rfc"
  [ $v = full ] && args="--workload rs8 --erasures 0 --steps 10"
  [ $v = shnomask ] && lib=norm_amd/_lib/libnfec_shnomask.so
  [ $v = shnofetch ] && lib=norm_amd/_lib/libnfec_shnofetch.so
  (cd /tmp && NFEC_LIBRARY=$GRAFT_REPO_ROOT/$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/p_${v}_$rep -o x -- python3 $GRAFT_REPO_ROOT/tools/bench_extra.py $args) > $O/${v}_${rep}.json 2>/dev/null || exit 1
  f=$(find $O/p_${v}_$rep -name "x_kernel_stats.csv" -print -quit)
  python3 -c "
import csv,sys
for r in csv.DictReader(open('$f')):
    if 'q4' in r['Name']: print('$v', $rep, r['Name'][23:50], round(float(r['AverageNs'])/1e3,1), r['Calls'])"
done; done
