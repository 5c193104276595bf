set -o pipefail
cd "${GRAFT_REPO_ROOT}"
OUT=gpurun_out/r2m; mkdir -p $OUT; export TMPDIR=/tmp
echo "== tests TILE_FAR=3 $(date +%T)"
QDC_TILE_FAR=3 timeout -k 10 300 python -u -m pytest tests/test_gpu_primitives.py tests/test_gpu_golden.py tests/test_gpu_layout.py -x -q --timeout 120 --timeout-method thread > $OUT/tests_tf3.log 2>&1 || { tail -30 $OUT/tests_tf3.log; exit 1; }
tail -1 $OUT/tests_tf3.log
for v in 0 3 1; do
  echo "== micro TILE_FAR=$v $(date +%T)"
  QDC_TILE_FAR=$v timeout -k 10 400 python -u bench.py --micro > $OUT/micro_tf$v.log 2>&1 || { tail -20 $OUT/micro_tf$v.log; exit 1; }
  python3 tools/micro_table.py $OUT/micro_tf$v.log > $OUT/micro_table_tf$v.txt
done
echo "== done $(date +%T)"
