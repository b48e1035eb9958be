# One parameterised GPU-box runner (replaces the per-experiment gpu_*.sh one-offs).
#   gpurun --timeout 1200 -- bash tools/gpu_run.sh TAG step [step ...]
# Steps (each under its own timeout; the first failure ends the run):
#   tests            full `pytest -m gpu` suite
#   tests:<k-expr>   GPU tests matching a -k expression ("=" stands for a space: tests:a=or=b)
#   smoke            __graft_entry__.smoke()
#   bench            default bench line (MLP + GBDT halves)
#   bench:<args>     bench.py with extra args, e.g. bench:--model=gbdt (use '=' not spaces)
#   prof:<args>      rocprofv3 --kernel-trace --stats around bench.py <args>
#   pmc:<ctrs>:<args> rocprofv3 --pmc <ctrs> (comma list) around bench.py <args>
#   py:<file>        python <file> (a lab script)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONPATH=.
export TMPDIR=/tmp
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
n=0
for step in "$@"; do
  n=$((n + 1))
  kind=${step%%:*}
  arg=${step#*:}
  [ "$arg" = "$step" ] && arg=""
  args=${arg//=/ }
  log="$OUT/$n-$kind.log"
  echo "[gpu_run] step $n: $step -> $log"
  case $kind in
    tests)
      if [ -n "$arg" ]; then
        timeout -k 10 900 python -u -m pytest -x -v -rA --timeout 300 --timeout-method thread tests -m gpu -k "$args" > "$log" 2>&1
      else
        timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > "$log" 2>&1
      fi ;;
    smoke) timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$log" 2>&1 ;;
    bench) timeout -k 10 900 python -u bench.py $args > "$OUT/$n-bench.json" 2> "$log" ;;
    prof)
      timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof$n" -o run -- python3 -u bench.py $args > "$log" 2>&1 ;;
    pmc)
      ctrs=${arg%%:*}; pargs=${arg#*:}; pargs=${pargs//=/ }
      timeout -s KILL 300 rocprofv3 --kernel-trace --pmc ${ctrs//,/ } --output-format csv -d "$OUT/pmc$n" -o run -- python3 -u bench.py $pargs > "$log" 2>&1 ;;
    py) timeout -k 10 900 python -u $args > "$log" 2>&1 ;;
    *) echo "unknown step $kind"; exit 2 ;;
  esac
  rc=$?
  echo "[gpu_run] step $n rc=$rc"
  tail -3 "$log"
  if [ $rc -ne 0 ]; then echo "STEP_FAILED $n $step rc=$rc"; exit $rc; fi
done
echo "[gpu_run] all steps ok"
