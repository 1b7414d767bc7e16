#!/bin/bash
# Featurisation A/B (through gpurun): parity of the candidate build, then alternating kernel timings
# of the builds named in $FV (lib/ab/libx2g_NAME.so), then the SCLK of the chain / flat kernels (trace
# build); every GPU step under its own time limit, stopping at the first failure.
set -u
mkdir -p gpurun_out
TAG=${TAG:-r4f}
L=$(pwd)/x2-gnn_amd/lib/ab
X2G_LIB=$L/libx2g_${CAND:-fnew}.so timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -q -m gpu -x \
  -k "featurize" --timeout 120 --timeout-method thread > gpurun_out/t_$TAG.log 2>&1 || { tail -20 gpurun_out/t_$TAG.log; exit 1; }
tail -2 gpurun_out/t_$TAG.log
for rep in 1 2 3; do
  for v in ${FV:-}; do
    X2G_LIB=$L/libx2g_$v.so timeout -k 10 120 python scripts/feat_time.py >> gpurun_out/feat_$TAG.txt 2>&1 || exit $?
  done
done
grep -h libx2g gpurun_out/feat_$TAG.txt
[ -f $L/libx2g_trace.so ] || exit 0
X2G_LIB=$L/libx2g_trace.so timeout -k 10 120 python scripts/trace_chain.py 21120 fwd > gpurun_out/clk_$TAG.txt 2>&1 || exit $?
X2G_LIB=$L/libx2g_trace.so timeout -k 10 120 python scripts/trace_chain.py 21120 >> gpurun_out/clk_$TAG.txt 2>&1 || exit $?
X2G_LIB=$L/libx2g_trace.so timeout -k 10 120 python scripts/trace_flat.py >> gpurun_out/clk_$TAG.txt 2>&1 || exit $?
grep -h "SCLK\|event\|per launch" gpurun_out/clk_$TAG.txt
