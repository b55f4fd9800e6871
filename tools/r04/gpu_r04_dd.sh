# Round 4: one side stream at world 1 by default: the whole -m gpu suite, config 5 at its shape and smoke
# (tools/r04/gpu_r04_final.sh), then the world-1 round (3 runs) and the in-process configurations.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/r04/gpu_r04_final.sh r04final5
O=gpurun_out/r4dd
mkdir -p $O
export MASTER_ADDR=127.0.0.1 RANK=0 LOCAL_RANK=0 WORLD_SIZE=1
for r in 1 2 3; do
  MASTER_PORT=$((29970 + r)) timeout -k 10 240 python3 bench.py --force-dist --no-cpu --steps 200 --dist-pipe defer \
    > $O/w1_$r.json 2> $O/w1_$r.err
done
timeout -k 10 150 python3 -u tools/round_inproc_r04.py --comm-first > $O/nogroup.log 2>&1
MASTER_PORT=29979 timeout -k 10 150 python3 -u tools/round_inproc_r04.py --comm-first --torch-group > $O/group.log 2>&1
