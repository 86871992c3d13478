#!/bin/bash
# Round measurement: GPU tests, smoke, the PMC traffic passes, a rocprofv3
# kernel trace of the bench (replayed steps + kernel-timer pass: the replay
# file), then the full bench line (its roofline.traffic from this run's PMC
# summary, roofline.replay_* from this run's trace).  Every GPU step has its
# own limit and the first failure ends the script.  Usage: bash tools/gpu_round.sh TAG
set -o pipefail
TAG=${1:-round}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG; mkdir -p $O
python -c "import __graft_entry__ as g; g.build()" > $O/build.log 2>&1 || { echo build failed; exit 3; }
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
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
python tools/kernel_instances.py $O/prof_kt --split adam_step_k --json $O/replay.json --config qm9,512,1 > $O/kernel_instances.txt 2>&1 && echo replay ok
SCGIB_TRAFFIC_FILE=$O/traffic.json SCGIB_REPLAY_FILE=$O/replay.json timeout -k 10 600 python bench.py --steps 300 --warmup 20 --cpu-seconds 20 > $O/bench.log 2>&1 || { echo bench failed; tail -5 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-400
echo done
