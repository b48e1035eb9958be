set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONPATH=.
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_mlp_gpu.py > gpurun_out/lanes_tests.log 2>&1 && \
SHIFU_CHUNK_LANES=1 timeout -k 10 300 python -u bench.py --gbdt-steps 0 > gpurun_out/lanes1.log 2>&1 && \
SHIFU_CHUNK_LANES=2 SHIFU_CHUNK_STAGGER=0 timeout -k 10 300 python -u bench.py --gbdt-steps 0 > gpurun_out/lanes2.log 2>&1 && \
SHIFU_CHUNK_LANES=2 timeout -k 10 300 python -u bench.py --gbdt-steps 0 > gpurun_out/lanes2s.log 2>&1
echo EXIT $?
