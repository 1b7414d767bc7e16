#!/bin/bash
# GPU validation/profiling run (used through gpurun): each step under its own time limit; stop
# at the first step that ends in anything but pass/fail (fault, abort, timeout).
#   bash scripts/gpu_check.sh [kernels] [model] [proj] [gpu] [ab: AB_VARIANTS='name=ENV ...'] [smoke] [bench] [dist2] [bench_c3] [bench_c3a] [bench_c5] [prof] [prof_c5] [pmc]
mkdir -p gpurun_out
export TMPDIR=/tmp
ROOT=$(pwd)
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "=== $name: $*" | tee -a gpurun_out/steps.log
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/steps.log
  tail -n 4 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
TAG=${TAG:-r1}
for s in "$@"; do
  case $s in
    kernels) step kernels 420 python -m pytest tests/test_gpu_kernels.py -q -m gpu -rf ;;
    model) step model 420 python -m pytest tests/test_gpu_model.py -q -m gpu -rf ;;
    proj) step proj 300 python -u -m pytest tests/test_gpu_kernels.py -q -m gpu -rf -k "conv_proj or pool or layernorm or readout or flat or smooth_l1" --timeout 120 --timeout-method thread ;;
    ab) step ab 900 python -u scripts/step_ab.py ${AB_ROUNDS:-3} $AB_VARIANTS ;;
    gpu) step gputests 900 python -u -m pytest tests -q -m gpu -rf --timeout 600 --timeout-method thread ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) step bench 420 python bench.py ;;
    dist2) step dist2 420 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
            --master-port 29517 bench.py --gpus 2 --steps 10 --warmup 3 --dist-backend gloo --no-cpu-baseline ;;
    bench_c3) step bench_c3 420 python bench.py --workload qm9_allprop --target 0 ;;
    bench_c3a) step bench_c3a 420 python bench.py --workload qm9_allprop --target 7 --no-cpu-baseline ;;
    bench_c5) step bench_c5 420 python bench.py --workload aid_infer --steps 50 --warmup 5 ;;
    prof_c5) step prof_c5 420 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c5_$TAG -o run --output-format csv \
            -- python "$ROOT/bench.py" --workload aid_infer --steps 5 --warmup 2 --no-cpu-baseline ;;
    prof) step prof 420 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv \
            -- python "$ROOT/bench.py" --steps 20 --warmup 3 --no-cpu-baseline ;;
    pmc) step pmc 420 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc_fetch_$TAG -o run \
            --output-format csv -- python "$ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --kernel-reps 3 &&
         step pmc2 420 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmc_write_$TAG -o run \
            --output-format csv -- python "$ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --kernel-reps 3 ;;
    pmc_c5) step pmc_c5 420 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc_fetch_c5_$TAG -o run \
            --output-format csv -- python "$ROOT/bench.py" --workload aid_infer --steps 2 --warmup 1 --no-cpu-baseline --kernel-reps 3 &&
         step pmc_c5w 420 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmc_write_c5_$TAG -o run \
            --output-format csv -- python "$ROOT/bench.py" --workload aid_infer --steps 2 --warmup 1 --no-cpu-baseline --kernel-reps 3 ;;
  esac
done
