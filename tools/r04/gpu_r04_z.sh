# Round 4: is the in-process world-1 round's 2x a hardware-queue share between the caller's stream and the round's
# plan / communication streams?  The in-process round (communicator first), with and without a torch group, on the
# null stream and on a created stream, with the side streams as usual and with OMR_SIDE_QUEUES=1 (full-CU-mask
# streams: a hardware queue each); then the bench child's round both ways.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4z
mkdir -p $O
export MASTER_ADDR=127.0.0.1 RANK=0 LOCAL_RANK=0 WORLD_SIZE=1
k=0
for q in 0 1; do
  k=$((k + 1))
  OMR_SIDE_QUEUES=$q timeout -k 10 150 python3 -u tools/round_inproc_r04.py --comm-first > $O/nogroup_q$q.log 2>&1
  OMR_SIDE_QUEUES=$q MASTER_PORT=$((29900 + k)) timeout -k 10 150 python3 -u tools/round_inproc_r04.py --comm-first \
    --torch-group > $O/group_q$q.log 2>&1
  OMR_SIDE_QUEUES=$q MASTER_PORT=$((29910 + k)) timeout -k 10 240 python3 bench.py --force-dist --no-cpu --steps 200 \
    --dist-pipe defer > $O/w1_q$q.json 2> $O/w1_q$q.err
done
