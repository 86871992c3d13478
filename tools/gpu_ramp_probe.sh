set -o pipefail
mkdir -p gpurun_out/ramp
X="--steps 20 --warmup 5 --no-cpu-baseline --no-superbatch --no-kernel-timer --no-finetune"
for cfg in "0" "200" "0" "200"; do
  if [ "$cfg" = 0 ]; then E=""; else E="SCGIB_PRELOAD_MS=$cfg"; fi
  env $E SCGIB_STEP_PROBE=1 timeout -k 10 200 python bench.py $X > gpurun_out/ramp/r.log 2>&1 || { tail -5 gpurun_out/ramp/r.log; exit 1; }
  echo "== preload $cfg ms: $(grep 'timed:' gpurun_out/ramp/r.log | sed 's/.*timed: //')"
  grep "step probe" gpurun_out/ramp/r.log | sed 's/.*step probe (ms): //' | cut -d' ' -f1-12
done
