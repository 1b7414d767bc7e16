mkdir -p gpurun_out
for v in nb3wt3 nb2wt4; do
  X2G_LIB=$PWD/x2-gnn_amd/lib/ab/libx2g_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -q -m gpu -k "flat or bucket or wgrad or energies" --timeout 120 --timeout-method thread > gpurun_out/t_$v.log 2>&1 || { tail -20 gpurun_out/t_$v.log; exit 1; }
  tail -1 gpurun_out/t_$v.log
done
timeout -k 10 900 python -u scripts/step_ab.py 3 cur= nb3wt3=X2G_LIB=$PWD/x2-gnn_amd/lib/ab/libx2g_nb3wt3.so nb2wt4=X2G_LIB=$PWD/x2-gnn_amd/lib/ab/libx2g_nb2wt4.so > gpurun_out/ab.log 2>&1
rc=$?; tail -3 gpurun_out/ab.log; exit $rc
