set -o pipefail
O=gpurun_out/r05c; mkdir -p $O
for mode in off sep; do
  AMD_SERIALIZE_KERNEL=3 timeout -k 10 200 python -u tools/probe/mailbox_probe.py $mode > $O/probe_$mode.log 2>&1 || { echo "probe $mode failed"; tail -5 $O/probe_$mode.log; exit 1; }
  tail -1 $O/probe_$mode.log
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o g -- python3 tools/gemm_pmc.py 30 ffn1,ffn1b > $O/gelu.log 2>&1 || { tail -5 $O/gelu.log; exit 1; }
python3 tools/summarize_pmc.py $O ffn1,ffn1b | grep -E '"(ffn1|ffn1b)"|median_us' 
AB="knob:gemm_gn=12,6 knob:gemm_gn=3,6" bash tools/gpu/run.sh abc2 r05c_gn || exit 1
AMD_SERIALIZE_KERNEL=3 timeout -k 10 200 python -u tools/probe/mailbox_probe.py on > $O/probe_on.log 2>&1; tail -3 $O/probe_on.log
