# diagnostic: band attention time with the normal and RF_BAND_DIAG builds (1 no compute, 2 no stores, 3 neither)
set -e
cd "$GRAFT_REPO_ROOT"
timeout -k 10 120 python3 tools/kbench.py attn
for d in 1 2 3; do
  echo "diag $d"; RF_HIP_LIB=$GRAFT_REPO_ROOT/recformer_amd/csrc/build/libbdiag$d.so timeout -k 10 120 python3 tools/kbench.py attn
done
