# Round 4: the in-process world-1 round (communicator first; no torch group / a torch group; null / created stream)
# at 4 (the box default) and 16 hardware queues per process (GPU_MAX_HW_QUEUES).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4z2
mkdir -p $O
export MASTER_ADDR=127.0.0.1 RANK=0 LOCAL_RANK=0 WORLD_SIZE=1
k=0
for q in 4 16; do
  k=$((k + 1))
  GPU_MAX_HW_QUEUES=$q timeout -k 10 150 python3 -u tools/round_inproc_r04.py --comm-first > $O/nogroup_hwq$q.log 2>&1
  GPU_MAX_HW_QUEUES=$q MASTER_PORT=$((29920 + k)) timeout -k 10 150 python3 -u tools/round_inproc_r04.py --comm-first \
    --torch-group > $O/group_hwq$q.log 2>&1
done
