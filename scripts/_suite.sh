# GPU box: the whole GPU suite, then (optional) bench lines of $WLS.  Each GPU step time-limited.
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/suite
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread \
    > gpurun_out/suite/pytest.log 2>&1; rc=$?
tail -5 gpurun_out/suite/pytest.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/suite/pytest.log | head -20; exit 1; }
for w in ${WLS:-}; do
  timeout -k 10 300 python -u bench.py --workload "$w" --steps ${STEPS:-30} --warmup 3 --no-cpu-baseline --no-e2e \
      --no-pipelined --no-cells-line > gpurun_out/suite/bench_$w.log 2>&1 || { tail -5 gpurun_out/suite/bench_$w.log; exit 2; }
  grep '^{' gpurun_out/suite/bench_$w.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$w', round(d['ms_per_step'],4), round(r['avg_kernel_us'],1), round(r['frac'],3))"
done
