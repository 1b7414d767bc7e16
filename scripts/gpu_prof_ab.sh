# A/B of library builds (AB_VARIANTS as scripts/step_ab.py, e.g. 'base= noext=X2G_LIB=...'), then a
# rocprofv3 kernel trace of the default build's graph-replayed step -> gpurun_out/prof_step/
mkdir -p gpurun_out
R=$(pwd)
timeout -k 10 800 python -u scripts/step_ab.py ${AB_ROUNDS:-3} $AB_VARIANTS > gpurun_out/ab.log 2>&1
rc=$?; tail -6 gpurun_out/ab.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_step -o run --output-format csv -- python3 $R/bench.py --step-only --steps 50 --warmup 5 > $R/gpurun_out/prof_step.log 2>&1
rc=$?; tail -2 $R/gpurun_out/prof_step.log; exit $rc
