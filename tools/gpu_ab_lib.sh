#!/bin/bash
# A/B of two library builds on one box: lasp_amd/liblaspj_base.so (LASPJ_LIB) against
# lasp_amd/liblaspj.so (or $NEW_LIB), interleaved, running the command in $AB_CMD.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
: > gpurun_out/ab.log
for round in 1 2; do
  for v in base new; do
    if [ $v = base ]; then export LASPJ_LIB=$PWD/lasp_amd/liblaspj_base.so
    elif [ -n "${NEW_LIB:-}" ]; then export LASPJ_LIB=$PWD/$NEW_LIB
    else unset LASPJ_LIB; fi
    echo "== $v round $round" >> gpurun_out/ab.log
    timeout -k 10 200 python -u $AB_CMD >> gpurun_out/ab.log 2>&1 || exit $?
  done
done
cat gpurun_out/ab.log
