cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 ./tools/diag/stream_depth > gpurun_out/stream_depth.jsonl 2>&1 || exit 1
cat gpurun_out/stream_depth.jsonl
VARIANTS="NFEC_Q4_VARIANT=0 NFEC_Q4_VARIANT=5 NFEC_Q4_VARIANT=6 NFEC_Q4_VARIANT=7 NFEC_FDEC_VARIANT=4 NFEC_Q4_VARIANT=0,NFEC_FDEC_VARIANT=0" timeout -k 10 400 bash tools/ab_bench.sh || exit 2
NFEC_FDEC_VARIANT=4 timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "fused or unfused" > gpurun_out/fdec_v4_tests.log 2>&1; tail -3 gpurun_out/fdec_v4_tests.log
