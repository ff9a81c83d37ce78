#!/bin/bash
# Full GPU check + committed-profile refresh: pytest -m gpu, the rocprofv3 passes of
# tools/profile_bench.sh (kernel trace, FETCH / WRITE, MFMA busy), then the default bench line
# from the same build. Usage: bash tools/gpu/round_profile.sh <tag>
set -o pipefail
TAG=${1:-r02}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || { tail -30 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -2 gpurun_out/${TAG}_pytest.log
bash tools/profile_bench.sh $TAG > gpurun_out/${TAG}_profile.log 2>&1 || { tail -30 gpurun_out/${TAG}_profile.log; exit 1; }
cat gpurun_out/prof_$TAG/summary.txt
timeout -k 10 400 python bench.py > gpurun_out/${TAG}_bench.log 2>&1 || { tail -20 gpurun_out/${TAG}_bench.log; exit 1; }
tail -1 gpurun_out/${TAG}_bench.log | cut -c1-300
