#!/bin/bash
# PMC passes (scripts/pmc_groups.txt) for a library variant's chroma kernel.
# usage: bash scripts/pmc_chroma.sh TAG LIB(relative to trik-media-sensors-dsp_amd/) [bench args]
set -u
cd "$GRAFT_REPO_ROOT"; TAG=$1; LIB=$2; shift 2
export TRIK_HSV_LIB="$GRAFT_REPO_ROOT/trik-media-sensors-dsp_amd/$LIB"
bash scripts/pmc_session.sh "$TAG" --steps 3 --warmup 1 --no-cpu-baseline --hot chroma "$@"
