set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONPATH=.

timeout -k 10 500 python -u bench.py --model varsel --stream --rows 20971520 --host-rows 2097152 --chunk-rows 131072 --steps 2 --warmup 1 > gpurun_out/se_stream_bench.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && \
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/seprof -o seprof -- python -u bench.py --model varsel --stream --rows 4194304 --host-rows 2097152 --chunk-rows 131072 --steps 1 --warmup 0 > gpurun_out/se_prof.log 2>&1
echo EXIT $?
