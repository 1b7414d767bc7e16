# parity tests under lib/ab/libx2g_$VAR.so, then an interleaved step A/B of the default build vs it
mkdir -p gpurun_out
X2G_LIB=$PWD/x2-gnn_amd/lib/ab/libx2g_$VAR.so timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -q -m gpu -k "${AB_TESTS:-energies or bucket}" --timeout 120 --timeout-method thread > gpurun_out/t_$VAR.log 2>&1
rc=$?; tail -2 gpurun_out/t_$VAR.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u scripts/step_ab.py ${AB_ROUNDS:-3} cur= $VAR=X2G_LIB=$PWD/x2-gnn_amd/lib/ab/libx2g_$VAR.so > gpurun_out/ab.log 2>&1
rc=$?; tail -2 gpurun_out/ab.log; exit $rc
