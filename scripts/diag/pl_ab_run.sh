set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gas_gpu.py tests/test_gas_commit.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pl_tests.log 2>&1 && tail -3 gpurun_out/pl_tests.log &&
timeout -k 10 500 scripts/diag/bench_ab.sh "--workload gas --steps 20 --warmup 3" 2 lib_ab/npl.so lib_ab/pl_nt32.so lib_ab/pl_g1nt32.so > gpurun_out/pl_ab_50000.log 2>&1 && cat gpurun_out/pl_ab_50000.log &&
timeout -k 10 500 scripts/diag/bench_ab.sh "--workload gas --steps 20 --warmup 3 --nodes 50048" 2 lib_ab/npl.so lib_ab/pl_nt32.so lib_ab/pl_g1nt32.so > gpurun_out/pl_ab_50048.log 2>&1 && cat gpurun_out/pl_ab_50048.log
