#!/bin/bash
# GPU-box helper: drop-in GBA call timing (scripts/e2e_timing.py) for library
# builds, interleaved, REPS calls each (median printed).
# usage: bash scripts/e2e_ab.sh lib1.so lib2.so ...
cd "$GRAFT_REPO_ROOT" || exit 1
for rep in 1 2; do
  for lib in "$@"; do
    echo "== $lib"
    SQLM_LIB_PATH=$PWD/sqrtlm-slam_amd/sqrtlm/$lib REPS=${REPS:-6} timeout -k 5 240 python scripts/e2e_timing.py 2>&1 \
      | grep -E "^median" || exit 1
  done
done
