set -u
cd /root/repo
timeout -k 10 400 bash scripts/diag/bench_ab.sh "--workload tas --steps 20 --warmup 3 --no-pipelined" 3 lib_ab/prep_ab1.so lib_ab/prep_ab2.so > gpurun_out/tas_ab.log 2>&1
rc=$?; cat gpurun_out/tas_ab.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do PAS_EVAL_NOGROUP=1 timeout -k 10 150 python3 bench.py --workload tas --steps 20 --warmup 3 --no-pipelined --no-cpu-baseline --no-request-latency | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('nogroup', round(d['ms_per_step'],4), d['config']['kernel_ms_per_step'])"; done
