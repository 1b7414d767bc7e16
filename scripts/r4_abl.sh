#!/bin/bash
# Ablation timings (through gpurun): the chain kernels (scripts/chain_time.py) and the flat weight
# gradient (scripts/flat_time.py) for the A/B builds named in $CT / $FT (lib/ab/libx2g_NAME.so),
# alternating twice; every run under its own time limit.  Ablation builds give wrong numbers by design.
set -u
mkdir -p gpurun_out
TAG=${TAG:-r4abl}
L=$(pwd)/x2-gnn_amd/lib/ab
for rep in 1 2; do
  for v in ${CT:-}; do
    X2G_LIB=$L/libx2g_$v.so timeout -k 10 120 python scripts/chain_time.py >> gpurun_out/abl_chain_$TAG.txt 2>&1 || exit $?
  done
  for v in ${FT:-}; do
    X2G_LIB=$L/libx2g_$v.so timeout -k 10 120 python scripts/flat_time.py >> gpurun_out/abl_flat_$TAG.txt 2>&1 || exit $?
  done
done
if [ -n "${FEAT_TRACE:-}" ]; then
  X2G_LIB=$L/libx2g_ftrace.so timeout -k 10 120 python scripts/trace_feat.py > gpurun_out/trace_feat_$TAG.txt 2>&1 || exit $?
  cat gpurun_out/trace_feat_$TAG.txt
fi
grep -h "libx2g" gpurun_out/abl_chain_$TAG.txt gpurun_out/abl_flat_$TAG.txt 2>/dev/null
exit 0
