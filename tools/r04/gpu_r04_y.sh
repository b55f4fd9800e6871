# Round 4: the round kernels' block stores as nt (a study build, build/libomr_nt.so via OMR_LIB) against the
# product's write-through sc0 sc1, interleaved as whole runs of tools/tune_round_r03.py, 3 each.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4y
mkdir -p $O
for r in 1 2 3; do
  timeout -k 10 200 python3 -u tools/tune_round_r03.py > $O/wt_$r.log 2>&1
  OMR_LIB=$GRAFT_REPO_ROOT/build/libomr_nt.so timeout -k 10 200 python3 -u tools/tune_round_r03.py > $O/nt_$r.log 2>&1
done
