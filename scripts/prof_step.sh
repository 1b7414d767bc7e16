#!/bin/bash
# rocprofv3 kernel stats of 20 graph-replayed config-2 steps (bench.py --step-only): TAG, then extra bench args
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=$1; shift
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_step_$TAG -o run --output-format csv \
  -- python "$(pwd)/bench.py" --step-only --steps 20 --warmup 3 "$@" > gpurun_out/prof_step_$TAG.log 2>&1
