# full GPU suite + smoke + default bench + tree-scoring bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONPATH=.
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/gpu_tests_full.log 2>&1 || { echo TESTS_FAILED; exit 1; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAILED; exit 1; }
timeout -k 10 600 python -u bench.py > gpurun_out/bench_default.log 2>&1 || { echo BENCH_FAILED; exit 1; }
timeout -k 10 300 python -u bench.py --model treeinfer --steps 3 --warmup 1 > gpurun_out/treeinfer.json 2> gpurun_out/treeinfer.err
echo EXIT $?
