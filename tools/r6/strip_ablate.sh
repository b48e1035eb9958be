# strip forward LAB ablations (timing only): dbg bits 1 no epilogue, 4 no MFMAs, 8 no B DMA, 16 no A loads
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONPATH=. TMPDIR=/tmp
mkdir -p gpurun_out/r6
timeout -k 10 300 python -u tools/strip_lab.py --rounds 2 --dbg 1 4 5 13 21 29 8 16 > gpurun_out/r6/strip_ablate_$1.jsonl 2> gpurun_out/r6/strip_ablate_$1.err || { tail -20 gpurun_out/r6/strip_ablate_$1.err; exit 1; }
grep -h "variant" gpurun_out/r6/strip_ablate_$1.jsonl | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l)
    if 'ms_median' in d: print(d['variant'], d['round'], d['ms_median'])"
