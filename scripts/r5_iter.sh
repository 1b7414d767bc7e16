#!/bin/bash
# One GPU iteration (through gpurun), each step under its own time limit and chained so that a fault or
# timeout ends the call:
#   1. focused parity tests ($K: a pytest -k expression over $FILES),
#   2. an interleaved step A/B of ab_base/ (scripts/build_base_tree.sh REV) against the working tree
#      ($ROUNDS rounds; skipped when ROUNDS=0),
#   3. a kernel trace of the working tree's step and its per-kernel breakdown (skipped when TRACE=0), and
#      with TRACE_BASE=1 the same of ab_base's step,
#   4. $EXTRA (a shell command, e.g. a trace build's phase-stamp script).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r5}
ROOT=$(pwd)
FILES=${FILES:-"tests/test_gpu_kernels.py tests/test_gpu_model.py"}
if [ -n "${K:-}" ]; then
  timeout -k 10 900 python -u -m pytest $FILES -q -m gpu -x -k "$K" --timeout 300 --timeout-method thread \
    > gpurun_out/t_$TAG.log 2>&1
  rc=$?; tail -3 gpurun_out/t_$TAG.log; [ $rc -eq 0 ] || exit $rc
fi
if [ "${ROUNDS:-3}" != "0" ]; then
  timeout -k 10 900 python -u scripts/step_ab.py ${ROUNDS:-3} base=AB_ROOT=ab_base new= ${AB_EXTRA:-} > gpurun_out/ab_$TAG.log 2>&1
  rc=$?; tail -3 gpurun_out/ab_$TAG.log; [ $rc -eq 0 ] || exit $rc
fi
if [ "${TRACE:-1}" != "0" ]; then
  cd /tmp
  timeout -k 10 300 rocprofv3 --kernel-trace -d $ROOT/gpurun_out/prof_$TAG -o run --output-format csv \
    -- python3 $ROOT/bench.py --step-only --steps 30 --warmup 5 > $ROOT/gpurun_out/prof_$TAG.log 2>&1
  rc=$?; [ $rc -eq 0 ] || exit $rc
  cd $ROOT
  python scripts/step_breakdown.py $(ls gpurun_out/prof_$TAG/*/run_kernel_trace.csv gpurun_out/prof_$TAG/run_kernel_trace.csv 2>/dev/null | head -1) \
    > gpurun_out/steps_$TAG.txt 2>&1
  head -16 gpurun_out/steps_$TAG.txt; tail -1 gpurun_out/steps_$TAG.txt
fi
if [ "${TRACE_BASE:-0}" != "0" ]; then  # the same trace of ab_base's step (per-kernel A/B on this box)
  cd /tmp
  timeout -k 10 300 rocprofv3 --kernel-trace -d $ROOT/gpurun_out/profb_$TAG -o run --output-format csv \
    -- python3 $ROOT/ab_base/bench.py --step-only --steps 30 --warmup 5 > $ROOT/gpurun_out/profb_$TAG.log 2>&1
  rc=$?; [ $rc -eq 0 ] || exit $rc
  cd $ROOT
  python scripts/step_breakdown.py $(ls gpurun_out/profb_$TAG/*/run_kernel_trace.csv gpurun_out/profb_$TAG/run_kernel_trace.csv 2>/dev/null | head -1) \
    > gpurun_out/stepsb_$TAG.txt 2>&1
  head -8 gpurun_out/stepsb_$TAG.txt; tail -1 gpurun_out/stepsb_$TAG.txt
fi
if [ -n "${EXTRA:-}" ]; then  # extra diagnostics (a trace build's script), its output under gpurun_out/
  timeout -k 10 300 bash -c "$EXTRA" > gpurun_out/extra_$TAG.log 2>&1
  rc=$?; tail -30 gpurun_out/extra_$TAG.log; [ $rc -eq 0 ] || exit $rc
fi
exit 0
