set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONPATH=.
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/gprof -o gprof -- python -u bench.py --model gbdt --rows 20000000 --steps 3 --warmup 1 > gpurun_out/g_prof.log 2>&1
echo EXIT $?
