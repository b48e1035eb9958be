set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONPATH=.
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/gpu_tests_full.log 2>&1 && \
timeout -k 10 600 python -u bench.py > gpurun_out/bench_default.log 2>&1
echo EXIT $?
