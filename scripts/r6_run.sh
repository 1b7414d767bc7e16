#!/bin/bash
# Round-6 GPU pass (through gpurun): named steps, each under its own time limit, stop at the first
# step that ends in anything but pass / fail.  bash scripts/r6_run.sh TAG step...
#   kc: center-attention kernel tests  model: model tests  gpu: the whole GPU suite  smoke
#   c2 / s5a / c3 / c5: bench lines (no CPU baseline)  c2full: bench with the CPU baseline
#   prof_c2 / prof_c5: rocprofv3 --kernel-trace --stats of the bench command
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=$1; shift
ROOT=$(pwd)
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "=== $name: $*" | tee -a gpurun_out/steps_$TAG.log
  timeout -k 10 "$secs" "$@" > "gpurun_out/${name}_$TAG.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/steps_$TAG.log
  tail -n 3 "gpurun_out/${name}_$TAG.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
PT="python -u -m pytest -q -rf --timeout 300 --timeout-method thread -m gpu"
for s in "$@"; do
  case $s in
    kc) step kc 400 $PT tests/test_gpu_kernels.py -k "center" ;;
    opt) step opt 300 $PT tests/test_gpu_kernels.py -k "flat_adam" ;;
    ktab) step ktab 300 $PT tests/test_gpu_kernels.py -k "table" ;;
    kch) step kch 400 $PT tests/test_gpu_kernels.py -k "chain or tiled or wgrad or schedule" ;;
    model) step model 600 $PT tests/test_gpu_model.py ;;
    dist) step dist 600 $PT tests/test_dist_gpu.py tests/test_rccl_gpu.py ;;
    gpu) step gputests 1000 $PT tests ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    c2) step bench_c2 300 python bench.py --no-cpu-baseline ;;
    c2full) step bench_c2full 420 python bench.py ;;
    c2dev) step bench_c2dev 300 python bench.py --no-cpu-baseline --device-schedule ;;
    s5a) step bench_s5a 300 python bench.py --shape S5A --no-cpu-baseline ;;
    c3) step bench_c3 300 python bench.py --workload qm9_allprop --target 0 --no-cpu-baseline ;;
    c5) step bench_c5 300 python bench.py --workload aid_infer --steps 50 --warmup 5 --no-cpu-baseline ;;
    prof_c2) step prof_c2 420 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c2_$TAG -o run --output-format csv \
            -- python "$ROOT/bench.py" --steps 50 --warmup 3 --no-cpu-baseline ;;
    prof_c5) step prof_c5 420 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c5_$TAG -o run --output-format csv \
            -- python "$ROOT/bench.py" --workload aid_infer --steps 10 --warmup 2 --no-cpu-baseline ;;
    ab) step ab 900 python -u scripts/step_ab.py ${AB_ROUNDS:-3} $AB_VARIANTS ;;
    ab_c5) step ab_c5 900 python -u scripts/step_ab.py ${AB_ROUNDS:-3} $AB_VARIANTS ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
