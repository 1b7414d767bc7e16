# dW_sbf (sbf_radial_wgrad) variants: parity under each lib/ab/libx2g_$v.so, per-kernel durations
# (rocprofv3 kernel stats of a short step run), then an interleaved whole-step A/B against the default build.
#   VARS="base v8" bash scripts/rad_ab.sh TAG      (variants built with make ab AB_UNIT=attention AB_FLAGS=-DX2G_RAD_...)
mkdir -p gpurun_out
TAG=${1:-rad}
R=$(pwd)
for v in cur $VARS; do
  if [ $v = cur ]; then unset X2G_LIB; else export X2G_LIB=$R/x2-gnn_amd/lib/ab/libx2g_$v.so; fi
  timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -q -m gpu \
    -k "radial or energies or bucket" --timeout 120 --timeout-method thread \
    > gpurun_out/t_${v}_$TAG.log 2>&1 || { tail -20 gpurun_out/t_${v}_$TAG.log; exit 1; }
  tail -n 1 gpurun_out/t_${v}_$TAG.log
done
export TMPDIR=/tmp
for v in cur $VARS; do
  if [ $v = cur ]; then unset X2G_LIB; else export X2G_LIB=$R/x2-gnn_amd/lib/ab/libx2g_$v.so; fi
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_${v}_$TAG -o run \
    --output-format csv -- python3 $R/bench.py --step-only --steps 50 --warmup 5 > $R/gpurun_out/prof_${v}_$TAG.log 2>&1) || exit $?
done
unset X2G_LIB
args=""
for v in $VARS; do args="$args $v=X2G_LIB=$R/x2-gnn_amd/lib/ab/libx2g_$v.so"; done
timeout -k 10 900 python -u scripts/step_ab.py ${AB_ROUNDS:-4} cur= $args > gpurun_out/ab_$TAG.log 2>&1
rc=$?; tail -n $((1 + $(echo $VARS | wc -w))) gpurun_out/ab_$TAG.log; exit $rc
