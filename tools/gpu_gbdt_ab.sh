# GBDT tests + bench (root u32 with two LDS copies) + u64 A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONPATH=.
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gbdt.py > gpurun_out/t_gbdt.log 2>&1 || { echo TESTS_FAILED; exit 1; }
timeout -k 10 300 python -u bench.py --model gbdt --steps 5 --warmup 1 > gpurun_out/gbdt_u32x2.json 2> gpurun_out/gbdt_u32x2.err || { echo GBDT_FAILED; exit 1; }
SHIFU_GBDT_ROOT_U32=0 timeout -k 10 300 python -u bench.py --model gbdt --steps 5 --warmup 1 > gpurun_out/gbdt_u64.json 2> gpurun_out/gbdt_u64.err
echo EXIT $?
