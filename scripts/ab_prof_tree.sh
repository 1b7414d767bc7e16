#!/bin/bash
# Per-kernel in-step durations of two whole trees on one box: ab_base/ (scripts/build_base_tree.sh REV)
# and the working tree, each bench.py --step-only under rocprofv3 --kernel-trace, then the step
# breakdown of each (scripts/step_breakdown.py).  ROUNDS alternations (default 1).
set -u
mkdir -p gpurun_out
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
TAG=${TAG:-abtree}
for r in $(seq 1 ${ROUNDS:-1}); do
  for v in base new; do
    if [ $v = base ]; then B=$R/ab_base/bench.py; else B=$R/bench.py; fi
    D=$R/gpurun_out/prof_${TAG}_${v}_$r
    timeout -k 10 300 rocprofv3 --kernel-trace -d $D -o run --output-format csv -- python3 $B --step-only \
      --steps 30 --warmup 5 > $R/gpurun_out/prof_${TAG}_${v}_$r.log 2>&1 || exit $?
    python3 $R/scripts/step_breakdown.py $(ls $D/*/run_kernel_trace.csv $D/run_kernel_trace.csv 2>/dev/null | head -1) \
      > $R/gpurun_out/steps_${TAG}_${v}_$r.txt || exit $?
    tail -1 $R/gpurun_out/steps_${TAG}_${v}_$r.txt
  done
done
