set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONPATH=.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/mprof -o mprof -- python -u bench.py --rows 20000000 --steps 3 --warmup 1 --gbdt-steps 0 > gpurun_out/m_prof.log 2>&1
echo EXIT $?
