set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONPATH=.
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gbdt.py tests/test_pipeline_gpu.py > gpurun_out/t_gbdt.log 2>&1 || { echo TESTS_FAILED; exit 1; }
timeout -k 10 300 python -u bench.py --model gbdt --steps 5 --warmup 1 > gpurun_out/gbdt_pf4.json 2> gpurun_out/gbdt_pf4.err || { echo GBDT_FAILED; exit 1; }
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/gprof -o gprof -- python -u bench.py --model gbdt --rows 20000000 --steps 3 --warmup 1 > gpurun_out/g_prof.log 2>&1
echo EXIT $?
