set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r1h; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_fusion.py -x -q --timeout 120 --timeout-method thread > $O/fusion_tests.log 2>&1 || { tail -20 $O/fusion_tests.log; exit 1; }
tail -2 $O/fusion_tests.log
QDC_RQ_STATS=1 timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-gate-sample > $O/stats1.log 2> $O/stats1.err || exit $?
QDC_RQ_MAXCL=0 QDC_RQ_STATS=1 timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-gate-sample > $O/stats0.log 2> $O/stats0.err || exit $?
for r in 1 2; do
for m in 0 1; do
QDC_RQ_MAXCL=$m timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-gate-sample > $O/ab_${m}_$r.log 2>&1 || exit $?
echo "maxcl=$m run $r: $(grep -o '"value": [0-9.]*' $O/ab_${m}_$r.log | head -1)"
done; done
