#!/bin/bash
# GPU box: the whole GPU suite, the C3/C3-driver/C4 bench lines, kernel stats of
# the C3 bench, then the PMC passes of the C3 bench (one counter group per run).
#   bash scripts/session_final.sh TAG
set -u
cd "$GRAFT_REPO_ROOT"; TAG="$1"
bash scripts/session_round.sh "$TAG" tests/ || exit $?
bash scripts/pmc_session.sh "pmc_$TAG" || exit $?
python3 scripts/pmc_summary.py "gpurun_out/pmc_$TAG" "chroma_kernel<0, 4, false>" 2516582400 "gpurun_out/pmc_$TAG/summary.json" \
  > "gpurun_out/pmc_$TAG/summary.log" 2>&1 || { cat "gpurun_out/pmc_$TAG/summary.log"; exit 5; }
tail -5 "gpurun_out/pmc_$TAG/summary.log"
