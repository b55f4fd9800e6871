set -e
timeout -k 10 400 python -u -m pytest tests/test_cpp_dist.py -x -v --timeout 120 --timeout-method thread > gpurun_out/cpp_dist.log 2>&1
for pipe in sync async defer; do
  timeout -k 10 180 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --force-dist --no-cpu --steps 300 --dist-pipe $pipe > gpurun_out/bench_w1_$pipe.log 2>&1
done
