set -o pipefail
O=gpurun_out/r05e; mkdir -p $O
AMD_SERIALIZE_KERNEL=3 timeout -k 10 200 python -u tools/probe/mailbox_probe2.py on > $O/probe2_on.log 2>&1 || { echo "probe2 on failed"; tail -4 $O/probe2_on.log; exit 1; }
tail -1 $O/probe2_on.log
bash tools/gpu/run.sh suite r05e || exit 1
BENCH_ARGS="--cpu-baseline-seconds 0" bash tools/gpu/run.sh bench r05e
