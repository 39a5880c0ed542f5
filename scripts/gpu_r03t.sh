#!/bin/bash
# Round 3 at HEAD: the whole -m gpu suite, smoke(), the default bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v \
  --timeout 300 --timeout-method thread > gpurun_out/pytest_t.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 3 gpurun_out/pytest_t.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_t.log 2>&1 || { tail -5 gpurun_out/smoke_t.log; exit 1; }
tail -n 1 gpurun_out/smoke_t.log
timeout -k 10 300 python bench.py > gpurun_out/bench_t.json 2> gpurun_out/bench_t.err || exit $?
cut -c1-700 gpurun_out/bench_t.json
for cfg in s1 s3; do
  timeout -k 10 300 python bench.py --config $cfg --no-cpu-baseline > gpurun_out/bench_t_$cfg.json 2> gpurun_out/bench_t_$cfg.err || exit $?
  cut -c1-200 gpurun_out/bench_t_$cfg.json
done
