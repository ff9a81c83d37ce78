set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python3 tools/gemm_var.py > gpurun_out/r04_base_gemm.log 2>&1 && \
timeout -k 10 200 python3 tools/gemm_var.py >> gpurun_out/r04_base_gemm.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 40 --warmup 5 --cpu-baseline-seconds 0 > gpurun_out/r04_base_bench.log 2>&1
rc=$?; cat gpurun_out/r04_base_gemm.log; tail -1 gpurun_out/r04_base_bench.log | cut -c1-400; exit $rc
