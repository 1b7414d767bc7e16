#!/bin/bash
# The whole GPU test suite (one process, per-test timeout), then an interleaved step A/B of the variants
# in $AB (scripts/step_ab.py) when given; stops at the first failure.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r4full}
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/gputests_$TAG.log 2>&1
rc=$?; tail -4 gpurun_out/gputests_$TAG.log; [ $rc -eq 0 ] || exit $rc
[ -n "${AB:-}" ] || exit 0
timeout -k 10 600 python -u scripts/step_ab.py ${ROUNDS:-3} $AB > gpurun_out/ab_$TAG.log 2>&1
rc=$?; tail -6 gpurun_out/ab_$TAG.log; exit $rc
