set -o pipefail
O=gpurun_out/r05f; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_graphs.py tests/test_gpu_train.py tests/test_gpu_kernels.py tests/test_gpu_retrieval.py tests/test_gpu_model.py -k "dp_step or cls_last_layer_training or colsum or shard_rank_matches or dgelu or four_wave or c2_finetune or c2_bench_mode or 12l_768 or catalog_batch" -v --timeout 200 --timeout-method thread > $O/t.log 2>&1
grep -E "PASSED|FAILED|^E  " $O/t.log | cut -c1-300 | grep -v PASSED | head -20; grep -cE "PASSED" $O/t.log
grep -q "illegal memory\|Fatal Python\|core dumped" $O/t.log && exit 1
bash tools/gpu/run.sh torchops r05f_ops > /dev/null; head -90 gpurun_out/r05f_ops/torchops.txt; timeout -k 10 300 python tools/torch_ops_trace.py --infer > $O/torchops_infer.txt 2>&1; head -70 $O/torchops_infer.txt
timeout -k 10 500 python tools/retrieval_bench.py --items 1000000 --growth 2,4,8 --family w16,w32 > $O/c5ab.log 2>&1; grep items $O/c5ab.log
timeout -k 10 300 python bench.py --gpus 2 --steps 10 --warmup 3 --cpu-baseline-seconds 0 --no-kernel-timing > $O/rehearsal.log 2>&1; tail -1 $O/rehearsal.log | cut -c1-400
timeout -k 10 300 python tools/train_bench.py --graph --steps 8 --warmup 2 > $O/c3.log 2>&1; tail -1 $O/c3.log | cut -c1-400
