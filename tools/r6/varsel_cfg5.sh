set -o pipefail
mkdir -p gpurun_out/r6
timeout -k 10 400 python -u bench.py --model varsel --rows 2000000 --cols 10000 --steps 3 --warmup 1 > gpurun_out/r6/varsel_2Mx10k.json 2> gpurun_out/r6/varsel_2Mx10k.err &&
cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r6/prof_varsel -o run -- python3 $GRAFT_REPO_ROOT/bench.py --model varsel --rows 2000000 --cols 10000 --steps 2 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/r6/varsel_prof.log 2>&1
