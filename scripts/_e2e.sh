# GPU box: chunked-staging tests, the C2 bench line with its e2e object, and a kernel trace
# of the host-window path (copy / compute overlap).
set -e
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -k "staging or knn" > gpurun_out/pytest_e2e.log 2>&1
tail -1 gpurun_out/pytest_e2e.log
timeout -k 10 300 python -u bench.py --workload knn --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/bench_knn_e2e.log 2>&1
grep '^{' gpurun_out/bench_knn_e2e.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['frac'], json.dumps(d.get('e2e')))"
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/prof -o e2e -- python3 scripts/e2e_trace.py > gpurun_out/prof/e2e.log 2>&1
ls gpurun_out/prof | grep e2e
