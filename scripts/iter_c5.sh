#!/bin/bash
# One GPU iteration on the C5 combined kernel: its parity tests, then an alternating A/B of
# bench.py --workload c5 (in-tree library against lib_ab/*.so).  usage: iter_c5.sh [lib ...]
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  -m gpu tests/test_shard.py tests/test_configs_full.py -k "tas_gas or c5 or topk" \
  > gpurun_out/iter_c5_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|error" gpurun_out/iter_c5_tests.log | tail -3
[ $rc -ne 0 ] && { tail -40 gpurun_out/iter_c5_tests.log; exit $rc; }
T=("$PWD")
for L in "$@"; do
  D="/tmp/ab_$(basename "$L" .so)"; rm -rf "$D"; mkdir -p "$D"
  cp -r bench.py platform-aware-scheduling_amd oracle "$D/"; cp "$L" "$D/platform-aware-scheduling_amd/lib/libpas.so"; T+=("$D")
done
for i in 1 2 3; do
  for D in "${T[@]}"; do
    timeout -k 10 300 python3 "$D/bench.py" --workload c5 --steps 10 --warmup 2 --no-cpu-baseline \
      > /tmp/c5.json 2>/tmp/c5.err || { tail /tmp/c5.err; exit 1; }
    tail -1 /tmp/c5.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print('$(basename $D)', round(d['ms_per_step'],4), 'kernel', round(c['topk_kernel_ms'],4), 'len', round(c['mean_list_len'],2))"
  done
done
