# Round 4: the round-gap study with stream write/wait-value cases, then the round kernels' PMC traffic
# (tools/r04/gpu_r04_pmc_round.sh's second step).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4o
mkdir -p $O
timeout -k 10 200 python3 -u tools/round_gap_r04.py > $O/gap.log 2>&1
timeout -k 10 900 python3 -u tools/pmc_round.py --out $O/pmc_round_r04.json --workdir $O/pmc > $O/pmc_round.log 2>&1
