set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONPATH=.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/qprof -o qprof -- python -u bench.py --model stats --steps 1 --warmup 0 > gpurun_out/q_prof.log 2>&1
echo EXIT $?
