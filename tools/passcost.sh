cd $GRAFT_REPO_ROOT
for m in 20 44 64 88; do
  NFEC_RS16_TMVP=0 timeout -k 10 200 python3 tools/bench_extra.py --workload c4 --k 4096 --m $m --vec 1400 --blocks 1024 --erasures 0 --steps 3 2>&1 | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print($m, d['encode_ms'])" || exit 1
done
