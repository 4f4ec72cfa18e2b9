#!/bin/bash
# A/B of the tower kernel's rows per wave: product (11 rows, 2 waves/SIMD) vs 6 rows (3 waves/SIMD)
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/r05d; mkdir -p $O
R6=$(pwd)/norm_amd/_lib/libnfec_r6.so
NFEC_LIBRARY=$R6 timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gpu_rs16_tw.py tests/test_gpu_rs16_kernels.py tests/test_c4_c5.py -m gpu > $O/pytest_r6.log 2>&1 || { tail -20 $O/pytest_r6.log; exit 1; }
tail -2 $O/pytest_r6.log
for i in 1 2; do
  timeout -k 10 300 python3 tools/bench_extra.py --workload rs16 > $O/rs16_r11_$i.json || exit 1
  NFEC_LIBRARY=$R6 timeout -k 10 300 python3 tools/bench_extra.py --workload rs16 > $O/rs16_r6_$i.json || exit 1
  timeout -k 10 300 python3 tools/bench_extra.py --workload c4 > $O/c4_r11_$i.json || exit 1
  NFEC_LIBRARY=$R6 timeout -k 10 300 python3 tools/bench_extra.py --workload c4 > $O/c4_r6_$i.json || exit 1
done
for f in $O/*.json; do python3 -c "import json,sys; d=json.load(open('$f')); print('$f', d.get('encode_ms'), d.get('decode_ms'), d.get('verified'))"; done
