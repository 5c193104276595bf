set -o pipefail
mkdir -p gpurun_out/r4w
export QDC_LIB_DIR=$PWD/qkx
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_dense.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r4w/tests.log 2>&1 || { tail -30 gpurun_out/r4w/tests.log; exit 1; }
tail -2 gpurun_out/r4w/tests.log
for v in 0 1 2; do
  echo "QDC_QK_LDS=$v" >> gpurun_out/r4w/pos.log
  QDC_QK_LDS=$v timeout -k 10 240 python3 tools/qk_pos_probe.py >> gpurun_out/r4w/pos.log 2>&1 || exit $?
done
cat gpurun_out/r4w/pos.log
