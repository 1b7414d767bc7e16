# A/B of the projection kernels on one box: the GPU parity tests that cover them under the
# default build, then interleaved whole-step timings of the default build vs lib/ab/libx2g_base.so
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -q -m gpu -k "${AB_TESTS:-conv_proj or fan_in or bucket or model_energies}" --timeout 120 --timeout-method thread > gpurun_out/t_new.log 2>&1
rc=$?; tail -3 gpurun_out/t_new.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u scripts/step_ab.py 3 base=X2G_LIB=$PWD/x2-gnn_amd/lib/ab/libx2g_base.so new= > gpurun_out/ab.log 2>&1
rc=$?; tail -4 gpurun_out/ab.log; [ $rc -eq 0 ] || exit $rc
