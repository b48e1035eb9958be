# MLP GPU tests (incl. bitwise reproducibility of the bench-path gradient) + default bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONPATH=.
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_mlp_gpu.py > gpurun_out/t_mlp.log 2>&1 || { echo TESTS_FAILED; exit 1; }
timeout -k 10 600 python -u bench.py --gbdt-steps 0 > gpurun_out/bench_mlp.log 2>&1
echo EXIT $?
