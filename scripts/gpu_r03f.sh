#!/bin/bash
# Round 3: the 2-D build against the reference's 2-D golden vectors, the
# one-workgroup direct solve on an 8^3 level-1 grid, bench lines s1 / s3.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_2d.py tests/test_fusions.py -m gpu -v -s \
  --timeout 300 --timeout-method thread -k "2d or direct" > gpurun_out/pytest_f.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E 'PASS|FAIL|Error|error|uni2d|amr2d' gpurun_out/pytest_f.log | cut -c1-3000 | head -40
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for cfg in s1 s3; do
  timeout -k 10 300 python bench.py --config $cfg --no-cpu-baseline > gpurun_out/bench_f_$cfg.json 2> gpurun_out/bench_f_$cfg.err || exit $?
  cut -c1-300 gpurun_out/bench_f_$cfg.json
done
timeout -k 10 300 python bench.py --config 2d > gpurun_out/bench_f_2d.json 2> gpurun_out/bench_f_2d.err || { tail -5 gpurun_out/bench_f_2d.err; exit 1; }
cut -c1-400 gpurun_out/bench_f_2d.json
