set -o pipefail
export LLMTRAIN_WGRAD_KERNEL=pp
mkdir -p gpurun_out/wpp
timeout -k 10 200 python -u bench/wgrad_pp.py check > gpurun_out/wpp/check.log 2>&1; echo "check rc=$?"; tail -2 gpurun_out/wpp/check.log
timeout -k 10 200 python -u bench/wgrad_pp.py time --tokens 131072 > gpurun_out/wpp/time_124m_131k.log 2>&1 || exit 1
timeout -k 10 200 python -u bench/wgrad_pp.py time --tokens 32768 > gpurun_out/wpp/time_124m_32k.log 2>&1 || exit 1
timeout -k 10 200 python -u bench/wgrad_pp.py time --model head --tokens 131072 > gpurun_out/wpp/time_head.log 2>&1 || exit 1
timeout -k 10 500 python -u -m pytest tests/test_kernels_gpu.py -k "wgrad_gemm_pp or layernorm_bwd or attn_dx_delta" -x -q --timeout 200 --timeout-method thread > gpurun_out/wpp/tests_kern.log 2>&1; echo "kern tests rc=$?"; tail -2 gpurun_out/wpp/tests_kern.log
timeout -k 10 500 python -u -m pytest tests/test_parity_gpu.py tests/test_engine_gpu.py::test_fused_step_at_benchmark_shape -x -v -s --timeout 300 --timeout-method thread > gpurun_out/wpp/tests.log 2>&1; echo "engine tests rc=$?"; tail -3 gpurun_out/wpp/tests.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/wpp/bench128.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --micro-batch 32 > gpurun_out/wpp/bench32.log 2>&1 || exit 1
tail -1 gpurun_out/wpp/bench128.log | cut -c1-200; tail -1 gpurun_out/wpp/bench32.log | cut -c1-200
