cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r02_b1 && \
timeout -k 10 600 python -u -m pytest tests/test_gpu_optim.py -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r02_b1/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r02_b1/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --steps 200 --warmup 20 --cpu-seconds 15 > gpurun_out/r02_b1/bench.log 2>&1 || { tail -20 gpurun_out/r02_b1/bench.log; exit 1; }
tail -1 gpurun_out/r02_b1/bench.log
