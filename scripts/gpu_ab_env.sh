# GPU tests, then an interleaved whole-step A/B of environment variants on one box:
#   AB_VARIANTS='name=ENV=V;ENV2=V2 name2=...' bash scripts/gpu_ab_env.sh   (AB_ROUNDS, default 3)
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -q -m gpu -x -rf --timeout 120 --timeout-method thread > gpurun_out/t_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/t_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 800 python -u scripts/step_ab.py ${AB_ROUNDS:-3} $AB_VARIANTS > gpurun_out/ab.log 2>&1
rc=$?; tail -6 gpurun_out/ab.log; exit $rc
