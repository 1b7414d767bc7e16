# GPU tests, an interleaved whole-step A/B (AB_VARIANTS as scripts/step_ab.py), and a rocprofv3
# kernel trace of the default build's graph-replayed step (gpurun_out/prof_step/)
bash scripts/gpu_ab_env.sh || exit $?
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_step -o run --output-format csv -- python3 $R/bench.py --step-only --steps 50 --warmup 5 > $R/gpurun_out/prof_step.log 2>&1
rc=$?; tail -1 $R/gpurun_out/prof_step.log; exit $rc
