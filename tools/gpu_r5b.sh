#!/bin/bash
# round-5 batch: tests, stamped timeline, library A/Bs (NT saved stores, layer-0
# backward grid cap), this tree vs ab_tree (pretrain + fine-tune)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  -k "interaction or capacity or finetune_config or noise or layer0 or transfer" > gpurun_out/r5b_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/r5b_pytest.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_stamps.sh r05_stamps || exit 1
ROUNDS=3 timeout -k 10 600 bash tools/ab_bench.sh --no-finetune "DIR=ab_tree" > gpurun_out/r5b_int_ab.txt 2>&1; rc=$?
cat gpurun_out/r5b_int_ab.txt; [ $rc -eq 0 ] || exit $rc
NO_TESTS=1 NO_FULL=1 bash tools/gpu_ft_ab.sh r05_int_ft "" "DIR=ab_tree" || exit 1
bash tools/gpu_lib_ab.sh r05_b0 libscgib_b0.so || exit 1
bash tools/gpu_lib_ab.sh r05_nt libscgib_nt.so
