# GPU tests, an interleaved whole-step A/B (AB_VARIANTS as scripts/step_ab.py), then the default bench
bash scripts/gpu_ab_env.sh || exit $?
timeout -k 10 420 python bench.py > gpurun_out/bench.log 2>&1
rc=$?; tail -c 600 gpurun_out/bench.log; exit $rc
