#!/bin/bash
# Fine-tune path check: Set2Set / fine-tune / domain-adaptation parity tests,
# the fine-tune bench line, and a kernel trace of its replayed steps with one
# step's timeline.  Usage: bash tools/gpu_ft.sh TAG
set -o pipefail
TAG=${1:-ft}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 400 python -u -m pytest -q -p no:cacheprovider --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "set2set or finetune or domain" > $O/pytest.log 2>&1; rc=$?
tail -1 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --finetune molhiv --steps 200 --warmup 20 ${FT_ARGS:---no-cpu-baseline} > $O/ft_bench.log 2>&1 || { echo bench failed; tail -5 $O/ft_bench.log; exit 1; }
tail -1 $O/ft_bench.log | cut -c1-330
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_kt -o kt -- python bench.py --finetune molhiv --steps 30 --warmup 5 --no-cpu-baseline --no-kernel-timer > $O/prof_bench.log 2>&1 || { echo rocprof failed; exit 1; }
python tools/prof_step.py $O/prof_kt/kt_kernel_trace.csv 20 > $O/step_timeline.txt
grep -E "set2set|Fill|span" $O/step_timeline.txt | cut -c1-120
