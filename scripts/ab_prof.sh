# Per-kernel durations of the default build vs lib/ab/libx2g_base.so (rocprofv3 kernel stats)
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for v in base new; do
  if [ $v = base ]; then export X2G_LIB=$R/x2-gnn_amd/lib/ab/libx2g_base.so; else unset X2G_LIB; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$v -o run --output-format csv -- python3 $R/bench.py --step-only --steps 50 --warmup 5 > $R/gpurun_out/prof_$v.log 2>&1 || exit $?
done
