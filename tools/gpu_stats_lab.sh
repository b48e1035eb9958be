set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONPATH=.
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_quantile.py tests/test_stats_kernels_gpu.py tests/test_stats_stream.py -m gpu > gpurun_out/q_tests.log 2>&1 && \
timeout -k 10 400 python -u tools/qlab.py > gpurun_out/qlab.log 2>&1 && \
timeout -k 10 400 python -u bench.py --model stats --steps 2 --warmup 1 > gpurun_out/q_bench100m.log 2>&1
echo EXIT $?
