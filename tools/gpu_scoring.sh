# Round-2 late: K13/K17/K18 + GBDT u32 root histogram: GPU tests, A/B benches, kernel traces
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONPATH=.
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_scoring_kernels.py tests/test_pipeline_gpu.py tests/test_gbdt.py > gpurun_out/t_scoring.log 2>&1 || { echo TESTS_FAILED; exit 1; }
echo TESTS_OK
timeout -k 10 300 python -u bench.py --model gbdt --steps 5 --warmup 1 > gpurun_out/gbdt_u32.json 2> gpurun_out/gbdt_u32.err || { echo GBDT_FAILED; exit 1; }
SHIFU_GBDT_ROOT_U32=0 timeout -k 10 300 python -u bench.py --model gbdt --steps 5 --warmup 1 > gpurun_out/gbdt_u64.json 2> gpurun_out/gbdt_u64.err || { echo GBDT64_FAILED; exit 1; }
timeout -k 10 300 python -u bench.py --model treeinfer --steps 3 --warmup 1 > gpurun_out/treeinfer.json 2> gpurun_out/treeinfer.err || { echo BENCH_FAILED; exit 1; }
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/tiprof -o tiprof -- python -u bench.py --model treeinfer --rows 5000000 --steps 2 --warmup 1 > gpurun_out/ti_prof.log 2>&1 || { echo PROF1_FAILED; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/gprof -o gprof -- python -u bench.py --model gbdt --rows 20000000 --steps 3 --warmup 1 > gpurun_out/g_prof.log 2>&1
echo EXIT $?
