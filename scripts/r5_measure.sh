#!/bin/bash
# Measurement pass (through gpurun): PMC HBM summaries for every bench line at its own workload and
# shape (FETCH_SIZE and WRITE_SIZE in separate passes), the config-2 step's per-kernel work table behind
# step_roofline, then the bench lines themselves (config 2 S160 and S5A, config 3, config 5).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r5m}
R=${R:-r5}  # the round prefix of the installed summaries
ROOT=$(pwd)
run() {  # run <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$secs" "$@" > "gpurun_out/${name}_$TAG.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 2 "gpurun_out/${name}_$TAG.log"
  [ $rc -eq 0 ] || exit $rc
}
pmc2() {  # pmc2 <name> <bench args...>: FETCH_SIZE pass, WRITE_SIZE pass, summary json
  local name=$1; shift
  run pmcf_$name 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmcf_${name}_$TAG -o run --output-format csv -- python "$ROOT/bench.py" "$@"
  run pmcw_$name 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmcw_${name}_$TAG -o run --output-format csv -- python "$ROOT/bench.py" "$@"
  run sum_$name 120 python scripts/pmc_traffic.py gpurun_out/pmcf_${name}_$TAG gpurun_out/pmcw_${name}_$TAG gpurun_out/pmc_traffic_${name}_$TAG.json
}
# PARTS selects the stages (a call is capped at 20 min): tests (the whole GPU suite), pmc (the four PMC
# summaries), work (step table), bench (the four bench lines), prof (config 2's bench command under
# rocprofv3 --kernel-trace --stats).  X2G_COMMIT (the caller's git HEAD: .git does not travel) stamps the
# summaries.
PARTS=${PARTS:-pmc work bench}
has() { [[ " $PARTS " == *" $1 "* ]]; }
if has tests; then
run gputests 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
fi
P="--steps 2 --warmup 1 --no-cpu-baseline --kernel-reps 3"
if has pmc; then
pmc2 c2 $P
pmc2 s5a $P --shape S5A
pmc2 c3 $P --workload qm9_allprop --target 0
pmc2 c5 $P --workload aid_infer
cp gpurun_out/pmc_traffic_c2_$TAG.json profiles/${R}_pmc_traffic.json
cp gpurun_out/pmc_traffic_s5a_$TAG.json profiles/${R}_pmc_traffic_s5a.json
cp gpurun_out/pmc_traffic_c3_$TAG.json profiles/${R}_pmc_traffic_c3.json
cp gpurun_out/pmc_traffic_c5_$TAG.json profiles/${R}_pmc_traffic_c5.json
fi
if has work; then
# the step's work table: PMC over eager steps, kernel trace over graph-replayed steps
run pmcf_step 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmcf_step_$TAG -o run --output-format csv -- python "$ROOT/bench.py" --step-only --eager --steps 3 --warmup 1
run pmcw_step 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmcw_step_$TAG -o run --output-format csv -- python "$ROOT/bench.py" --step-only --eager --steps 3 --warmup 1
run trace_step 300 rocprofv3 --kernel-trace --stats -d gpurun_out/trace_step_$TAG -o run --output-format csv -- python "$ROOT/bench.py" --step-only --steps 20 --warmup 3
run work 300 python scripts/step_work.py gpurun_out/pmcf_step_$TAG gpurun_out/pmcw_step_$TAG gpurun_out/trace_step_$TAG gpurun_out/step_work_$TAG.json
cp gpurun_out/step_work_$TAG.json profiles/${R}_step_work.json
fi
# the bench lines read the summaries installed above (on this box; the caller copies them into profiles/)
has bench || exit 0
run bench_c2 420 python bench.py
# the same command under rocprofv3 (kernel stats: the roofline kernel's average launch must agree)
if has prof; then
run prof_c2 420 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c2_$TAG -o run --output-format csv -- python "$ROOT/bench.py" --no-cpu-baseline
fi
run bench_s5a 420 python bench.py --shape S5A --no-cpu-baseline
run bench_c3 420 python bench.py --workload qm9_allprop --target 0
run bench_c5 420 python bench.py --workload aid_infer --steps 50 --warmup 5
