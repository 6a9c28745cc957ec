#!/bin/bash
# GPU box, development: kbench A/B of the given libraries, then the given GPU
# test files, then one bench line.  usage: bash scripts/ab_and_tests.sh "libs" tests...
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
bash scripts/ab_kbench.sh "-n 100 -r 5" $1 || exit $?
shift
timeout -k 10 800 python -u -m pytest "$@" -m gpu -x -q -p no:cacheprovider --timeout 400 --timeout-method thread > gpurun_out/tests_ab.log 2>&1
rc=$?; tail -2 gpurun_out/tests_ab.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_ab.log 2>&1 || exit $?
tail -1 gpurun_out/bench_ab.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('kernel_ms', d['roofline']['kernel_ms'], 'frac', d['roofline']['frac'], 'cold', d['cold_batch'])"
