set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONPATH=.
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py --gbdt-steps 0 > gpurun_out/chunk2M.log 2>&1 || { echo A_FAILED; exit 1; }
timeout -k 10 400 python -u bench.py --gbdt-steps 0 --chunk-rows 4194304 > gpurun_out/chunk4M.log 2>&1 || { echo B_FAILED; exit 1; }
timeout -k 10 400 python -u bench.py --gbdt-steps 0 > gpurun_out/chunk2M_b.log 2>&1
echo EXIT $?
