#!/bin/bash
# Phase stamps of the chain forward / backward and the flat weight gradient (trace build: make -C
# x2-gnn_amd ab AB_NAME=trace AB_FLAGS=-DX2G_TRACE), each under its own time limit.
set -u
mkdir -p gpurun_out
TAG=${TAG:-r4t}
L=$(pwd)/x2-gnn_amd/lib/ab/libx2g_trace.so
X2G_LIB=$L timeout -k 10 180 python scripts/trace_chain.py 21120 fwd > gpurun_out/trace_chain_fwd_$TAG.txt 2>&1 || exit $?
X2G_LIB=$L timeout -k 10 180 python scripts/trace_chain.py 21120 > gpurun_out/trace_chain_bwd_$TAG.txt 2>&1 || exit $?
X2G_LIB=$L timeout -k 10 180 python scripts/trace_flat.py > gpurun_out/trace_flat_$TAG.txt 2>&1 || exit $?
cat gpurun_out/trace_chain_fwd_$TAG.txt gpurun_out/trace_chain_bwd_$TAG.txt gpurun_out/trace_flat_$TAG.txt
# chain kernel times of A/B builds named in $CT (lib/ab/libx2g_NAME.so), alternating twice
for rep in 1 2; do
  for v in ${CT:-}; do
    X2G_LIB=$(pwd)/x2-gnn_amd/lib/ab/libx2g_$v.so timeout -k 10 120 python scripts/chain_time.py >> gpurun_out/chain_time_$TAG.txt 2>&1 || exit $?
  done
done
cat gpurun_out/chain_time_$TAG.txt 2>/dev/null
exit 0
