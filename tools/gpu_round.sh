#!/bin/bash
# Round measurement: GPU tests, smoke, the PMC traffic passes, a rocprofv3
# kernel trace of the bench (replayed steps + kernel-timer pass: the replay
# file), the same three for the fine-tune step (configs[4]) plus its stamped
# critical-path run, then the full bench line (its roofline.traffic from this
# run's PMC summaries, roofline.replay_* from this run's traces, the
# fine-tune's critical_path_us from the stamped run).  Every GPU step has its
# own limit and the first failure ends the script.
# Usage: bash tools/gpu_round.sh TAG [--no-tests]
set -o pipefail
TAG=${1:-round}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG; mkdir -p $O
python -c "import __graft_entry__ as g; g.build()" > $O/build.log 2>&1 || { echo build failed; exit 3; }
if [ "$2" != "--no-tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 180 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
  echo "pytest rc=$rc"; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail -5 $O/smoke.log; exit 1; }
  tail -1 $O/smoke.log
fi
# (--no-finetune: the N = 1 line's fine-tune leg would mix its B = 32 launches into the averages)
ARGS="--steps 5 --warmup 2 --no-cpu-baseline --no-superbatch --no-kernel-timer --no-finetune"
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $C --output-format csv -d "$O/pmc/$C" -o pmc \
    -- python bench.py $ARGS > "$O/pmc_$C.log" 2>&1 || { echo "pmc $C failed"; exit 1; }
done
python tools/pmc_summary.py "$O/pmc" qm9,512,1 > "$O/traffic.json" && echo traffic ok
# the bench with its kernel-timer pass: kernel_instances.py --split separates
# the replayed steps from the timer pass (the launches the timer averages)
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_kt -o kt \
  -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-superbatch --no-finetune > $O/prof_bench.log 2>&1 || { echo rocprof failed; exit 1; }
python tools/kernel_instances.py $O/prof_kt --split adam_step_k,adam_reduce_k --json $O/replay.json --config qm9,512,1 > $O/kernel_instances.txt 2>&1 && echo replay ok
# the fine-tune step (bench.py --finetune molhiv): PMC passes, kernel trace, stamps
FARGS="--finetune molhiv --steps 5 --warmup 2 --no-cpu-baseline --no-kernel-timer"
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $C --output-format csv -d "$O/ft_pmc/$C" -o pmc \
    -- python bench.py $FARGS > "$O/ft_pmc_$C.log" 2>&1 || { echo "ft pmc $C failed"; exit 1; }
done
python tools/pmc_summary.py "$O/ft_pmc" molhiv-finetune,32,1 > "$O/traffic_finetune.json" && echo ft traffic ok
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ft_prof_kt -o kt \
  -- python bench.py --finetune molhiv --steps 20 --warmup 5 --no-cpu-baseline > $O/ft_prof_bench.log 2>&1 || { echo ft rocprof failed; exit 1; }
python tools/kernel_instances.py $O/ft_prof_kt --split adam_step_k --json $O/replay_finetune.json --config molhiv-finetune,32,1 > $O/ft_kernel_instances.txt 2>&1 && echo ft replay ok
SCGIB_STAMPS=1 SCGIB_STAMPS_JSON=$O/ft_stamps.json timeout -k 10 200 python bench.py --finetune molhiv \
  --steps 100 --warmup 10 --no-cpu-baseline --no-kernel-timer > $O/ft_stamps.log 2>&1 || { echo ft stamps failed; exit 1; }
echo ft stamps ok
SCGIB_TRAFFIC_FILE=$O/traffic.json SCGIB_REPLAY_FILE=$O/replay.json \
SCGIB_FT_TRAFFIC_FILE=$O/traffic_finetune.json SCGIB_FT_REPLAY_FILE=$O/replay_finetune.json \
SCGIB_FT_STAMPS_FILE=$O/ft_stamps.json \
  timeout -k 10 600 python bench.py --steps 300 --warmup 20 --cpu-seconds 20 > $O/bench.log 2>&1 || { echo bench failed; tail -5 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-400
# the driver's own command (K = 20 after 5 warm-up), same evidence files
SCGIB_TRAFFIC_FILE=$O/traffic.json SCGIB_REPLAY_FILE=$O/replay.json \
SCGIB_FT_TRAFFIC_FILE=$O/traffic_finetune.json SCGIB_FT_REPLAY_FILE=$O/replay_finetune.json \
SCGIB_FT_STAMPS_FILE=$O/ft_stamps.json \
  timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.log 2>&1 || { echo driver bench failed; tail -5 $O/bench_driver.log; exit 1; }
tail -1 $O/bench_driver.log | cut -c1-300
echo done
