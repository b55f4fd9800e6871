# one world-1 round timeline per pipeline mode (kernel + HIP runtime trace), for tools/round_timeline.py;
# bench.py's distributed path without the torchrun launcher (so the traces are the bench process's own)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export MASTER_ADDR=127.0.0.1 MASTER_PORT=29513 RANK=0 LOCAL_RANK=0 WORLD_SIZE=1
for pipe in ${PIPES:-sync defer}; do
  timeout -k 10 240 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d gpurun_out/tl_$pipe -o tl -- \
    python bench.py --force-dist --no-cpu --steps 100 --dist-pipe $pipe > gpurun_out/tl_$pipe.log 2>&1
done
