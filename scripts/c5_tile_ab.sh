mkdir -p gpurun_out
for t in 1073741824 524288 131072 65536; do
  X2G_INFER_TILE=$t timeout -k 10 400 python bench.py --workload aid_infer --steps 30 --warmup 3 --no-cpu-baseline --step-only > gpurun_out/c5_$t.log 2>&1 || exit $?
  python -c "import json,sys; d=[json.loads(l) for l in open('gpurun_out/c5_$t.log') if l.startswith('{')][-1]; print($t, d['value'], d['ms_per_step'])"
done
