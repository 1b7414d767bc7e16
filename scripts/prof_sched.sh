#!/bin/bash
# rocprofv3 kernel stats of the step with collate's host schedule vs the device-made one (configs 2 and 5)
mkdir -p gpurun_out
export TMPDIR=/tmp
ROOT=$(pwd)
for wl in c2 c5; do
  if [ $wl = c5 ]; then W="--workload aid_infer"; else W=""; fi
  for v in host dev; do
    if [ $v = dev ]; then D="--device-schedule"; else D=""; fi
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_sched_${wl}_$v -o run --output-format csv \
      -- python "$ROOT/bench.py" --step-only --steps 20 --warmup 3 $W $D > gpurun_out/prof_sched_${wl}_$v.log 2>&1 || exit $?
    tail -n 1 gpurun_out/prof_sched_${wl}_$v.log
  done
done
