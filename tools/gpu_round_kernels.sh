# world-1 round, kernel trace only (no HIP runtime trace, so the host runs at its own speed), per pipeline mode;
# bench.py's distributed path without the torchrun launcher
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export MASTER_ADDR=127.0.0.1 MASTER_PORT=29514 RANK=0 LOCAL_RANK=0 WORLD_SIZE=1
for pipe in ${PIPES:-sync defer}; do
  timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tk_$pipe -o tk -- \
    python bench.py --force-dist --no-cpu --steps 100 --dist-pipe $pipe > gpurun_out/tk_$pipe.log 2>&1
done
