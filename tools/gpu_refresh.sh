# refresh the secondary benches on the final tree
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONPATH=.
mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py --model stats --steps 2 --warmup 1 > gpurun_out/bench_stats.json 2> gpurun_out/bench_stats.err || { echo STATS_FAILED; exit 1; }
timeout -k 10 600 python -u bench.py --model varsel --steps 2 --warmup 1 > gpurun_out/bench_varsel.json 2> gpurun_out/bench_varsel.err || { echo VARSEL_FAILED; exit 1; }
echo EXIT 0
