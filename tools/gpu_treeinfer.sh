# K13 tree inference: GPU tests + bench + kernel trace
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONPATH=.
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_scoring_kernels.py > gpurun_out/t_ti.log 2>&1 || { echo TESTS_FAILED; exit 1; }
timeout -k 10 300 python -u bench.py --model treeinfer --steps 3 --warmup 1 > gpurun_out/treeinfer.json 2> gpurun_out/treeinfer.err || { echo BENCH_FAILED; exit 1; }
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/tiprof -o tiprof -- python -u bench.py --model treeinfer --rows 5000000 --steps 2 --warmup 1 > gpurun_out/ti_prof.log 2>&1
echo EXIT $?
