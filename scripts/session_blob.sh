#!/bin/bash
# GPU box: blob parity tests, then the blob A/B (first lib = baseline).
# usage: bash scripts/session_blob.sh TAG lib1 [lib2 ...]
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/blob; mkdir -p $OUT; TAG="$1"; shift
timeout -k 10 600 python -u -m pytest tests/test_gpu_blob.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/tests_$TAG.log 2>&1
rc=$?; tail -3 $OUT/tests_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python scripts/blob_ab.py "$@" > $OUT/ab_$TAG.txt 2>&1; rc=$?; cat $OUT/ab_$TAG.txt; exit $rc
