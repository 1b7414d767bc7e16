#!/bin/bash
# One GPU iteration (through gpurun): focused parity tests, the bench line (probes), a kernel trace
# of the step, then optional extras ($EXTRA: loss | pmc).  Each step under its own time limit,
# chained so that a fault or timeout ends the call.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r4x}
ROOT=$(pwd)
K=${K:-"conv or attention or model_energies or trainer or factorised or config2 or fused_variants or transpose or symmetric"}
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -q -m gpu -x -k "$K" \
  --timeout 300 --timeout-method thread > gpurun_out/t_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/t_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_$TAG.log 2>&1
rc=$?; tail -c 600 gpurun_out/bench_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv \
  -- python "$ROOT/bench.py" --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/prof_$TAG.log 2>&1
rc=$?; [ $rc -eq 0 ] || exit $rc
python scripts/step_breakdown.py gpurun_out/prof_$TAG/run_kernel_trace.csv > gpurun_out/steps_$TAG.txt 2>&1
head -14 gpurun_out/steps_$TAG.txt; tail -1 gpurun_out/steps_$TAG.txt
for x in ${EXTRA:-}; do
  case $x in
    loss) timeout -k 10 400 python -u scripts/loss_check.py 225 > gpurun_out/loss_$TAG.txt 2>&1; rc=$?; cat gpurun_out/loss_$TAG.txt | tail -12; [ $rc -eq 0 ] || exit $rc ;;
    pmc) TAG=$TAG bash scripts/pmc_sq.sh list; rc=$?; [ $rc -eq 0 ] || exit $rc ;;
  esac
done
