set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k gemm_fused -x -q --timeout 120 --timeout-method thread > gpurun_out/fg_test.log 2>&1; rc=$?
tail -15 gpurun_out/fg_test.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench/micro.py fgemm 65536 > gpurun_out/fg_micro.log 2>&1
cat gpurun_out/fg_micro.log
