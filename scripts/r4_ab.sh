#!/bin/bash
# Step A/B on one box (through gpurun): quick parity tests of the default build, then interleaved
# whole-step timings of the variants named in $AB (NAME=ENV;... specs, scripts/step_ab.py).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r4ab}
K=${K:-"featurize or model_energies or config2_trainer or chain or conv_proj or flat"}
timeout -k 10 600 python -u -m pytest ${FILES:-tests/test_gpu_kernels.py tests/test_gpu_model.py} -q -m gpu -x -k "$K" \
  --timeout 300 --timeout-method thread > gpurun_out/t_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/t_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 1200 python -u scripts/step_ab.py ${ROUNDS:-3} $AB > gpurun_out/ab_$TAG.log 2>&1
rc=$?; tail -8 gpurun_out/ab_$TAG.log; exit $rc
