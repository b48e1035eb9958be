set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONPATH=.
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gbdt.py -m gpu > gpurun_out/tree_tests.log 2>&1
echo EXIT $?
